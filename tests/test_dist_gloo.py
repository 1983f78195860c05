"""World-size-2 CPU test (gloo) of the replicas-only multi-GPU path used by bench.py --gpus N (config C5).

Each rank builds its own seeded instance (seed 20261015 + rank), does independent work, and the only
collectives are the ones bench.py uses: barrier, MAX of the elapsed time, one gather of {stats, x} to rank 0
(cvx_amd/dist.py).  The per-rank work here is the oracle's Newton direction on a small instance (CPU; the
device engine needs a GPU), so the test checks the sharding bookkeeping, not the kernels.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from cvx_amd import dist as D
    from cvx_amd import problems as Z
    from oracle import cvx_oracle as O

    r, lr, w = D.env_rank()
    assert (r, lr, w) == (rank, rank, world)
    D.init("gloo")
    dev = torch.device("cpu")
    spec = Z.random_qp(24, 48, instance=rank)
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    x = spec["x0"]
    y = O.barrier_gradient(pb, 1.0, x)
    H = O.barrier_hessian(pb, 1.0, x, literal=False)
    dx = O.cholesky_solve(H, -y, 0.1, fast_subst=True)
    D.barrier(dev)
    elapsed = D.max_over_ranks(1.0 + rank, dev)
    stats = np.array([rank, 1, elapsed, 1.0])
    got = D.gather_results(dx, stats, dev)
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), np.stack(got))
    # every rank also records its own direction for the comparison on the parent side
    np.save(os.path.join(outdir, f"dx{rank}.npy"), dx)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_replicas_gather_world2(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = np.load(tmp_path / "gathered.npy")
    assert g.shape == (2, 4 + 24)
    for rank in range(world):
        rec = g[rank]
        assert rec[0] == rank                       # records arrive in rank order
        assert rec[2] == 2.0                        # MAX over ranks of (1 + rank)
        np.testing.assert_array_equal(rec[4:], np.load(tmp_path / f"dx{rank}.npy"))
    # distinct seeded instances per rank (no accidental sharing of the problem)
    assert not np.allclose(g[0, 4:], g[1, 4:])
