"""World-size-2 CPU test (gloo) of the replicas-only multi-GPU path of bench.py --gpus N (config C5).

Both ranks run bench.py's own per-rank body, bench.run_rank, unchanged: process-group init from the torchrun-style
environment, this rank's seeded instance (seed 20261015 + rank), W untimed + K timed steps between barriers, the MAX
of the elapsed time over ranks and one gather of {stats, x} to rank 0 (cvx_amd/dist.py).  Only the device pieces are
swapped for CPU stand-ins: backend gloo, device cpu, and an engine with the cvxg Engine's interface whose Newton
step is the oracle's (the device engine needs a GPU; its kernels are covered by the -m gpu tests).
"""
import os
import socket
import types

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleEngine:
    """Stand-in for cvx_amd.engine.Engine (the methods run_rank uses): one inner Newton iteration of
    UnconstrainedSolver.solve per newton_step, on the CPU oracle."""

    def __init__(self, n, m, p=0, device=0):
        self.n, self.m = n, m
        self.t, self.it = 1.0, 0
        self.radius = float("nan")

    def load_problem(self, spec):
        from oracle import cvx_oracle as O
        self.O = O
        self.pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
        self.pars = O.standard_params()

    def set_x(self, x):
        self.x = np.array(x, dtype=np.float64)

    def get_x(self):
        return self.x.copy()

    def centering_begin(self, t):
        self.t, self.it = float(t), 0

    def newton_step(self, pars):
        O = self.O
        y = O.barrier_gradient(self.pb, self.t, self.x)
        d = O.newton_direction(self.pb, self.t, self.x, y, pars.tolEqSolve)
        q = float(d @ y)
        took = -q / 2 > pars.tolSolver
        st = 0.0
        if took:
            if self.it == 0:
                self.radius = np.sqrt(-q)
            f = O.barrier_value(self.pb, self.t, self.x)
            s, st, _, _ = O.unconstrained_line_search(self.pb, self.t, self.x, d, q, f, self.it, self.radius, pars)
            self.x = self.x + s * st
        self.it += 1
        return types.SimpleNamespace(done=not took, took_step=int(took), step=float(st))

    def set_timing(self, on, all_phases=True):
        pass

    def phase_times(self):
        return np.zeros(8)

    def ruiz_lookahead(self, sweeps=0):
        return 0

    def close(self):
        pass


def _worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    args = types.SimpleNamespace(workload="C3", n=24, m=48, steps=4, warmup=1)
    out, gathered = bench.run_rank(args, engine_cls=OracleEngine, backend="gloo", device=torch.device("cpu"))
    # the same steps on this rank alone, for the comparison on the parent side
    spec = bench.workload_spec(args, rank)[0]
    eng = OracleEngine(24, 48)
    eng.load_problem(spec)
    eng.set_x(spec["x0"])
    eng.centering_begin(1.0)
    for _ in range(args.warmup + args.steps):
        if eng.newton_step(eng.pars).done:
            eng.centering_begin(eng.t * 10.0)
    np.save(os.path.join(outdir, f"x{rank}.npy"), eng.get_x())
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), np.stack(gathered))
        import json
        json.dump(out, open(os.path.join(outdir, "out.json"), "w"))
    else:
        assert out is None and gathered is None
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_rank_body_world2(tmp_path):
    import json

    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = np.load(tmp_path / "gathered.npy")
    out = json.load(open(tmp_path / "out.json"))
    assert g.shape == (2, 4 + 24)
    assert out["n_gpus"] == 2 and out["gathered_ranks"] == 2 and out["scaling"] == "weak"
    assert out["steps"] == 4
    elapsed = max(g[0, 2], g[1, 2])
    assert g[0, 2] == g[1, 2] == elapsed  # every rank reports the MAX over ranks
    assert out["value"] == pytest.approx(2 * 4 / elapsed)  # whole-job steps / max-rank time
    for rank in range(world):
        rec = g[rank]
        assert rec[0] == rank and rec[1] == 4  # records arrive in rank order
        np.testing.assert_array_equal(rec[4:], np.load(tmp_path / f"x{rank}.npy"))
    assert not np.allclose(g[0, 4:], g[1, 4:])  # distinct seeded instances per rank
