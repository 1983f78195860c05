"""The dataflow Cholesky's worker task order (cvxg_chol_schedule: the host-built list k_dataflow.hip's workgroups
claim in order, cvx_amd/csrc/cvxg.cpp build_chol_schedule) -- host-only, no GPU.

Deadlock freedom of the persistent launch rests on two properties checked here for several block counts:
  * coverage: every TRSM / UPDATE of the right-looking tile factorization (MatrixUtils.scala:452-461 as 64 x 64
    tiles) is either listed exactly once (UPDATE4 covering four consecutive panels of one tile) or is a chain task
    (POTRF(k), TRSM(k+1,k), UPDATE(k+1,k+1,k), UPDATE(k+2,k+2,k), UPDATE(k+2,k+1,k): run by the chain workgroups,
    never listed);
  * order: a listed task appears after every listed task it depends on (a claimed task only ever waits on tasks
    claimed before it, or on chain tasks, whose own inputs come earlier in the list).
"""
import ctypes as C

import pytest

from cvx_amd import _lib


def _order(nblk, workers=256):
    lib = _lib.load()
    n = lib.cvxg_chol_schedule(nblk, workers, None, 0)
    assert n >= 0
    buf = (C.c_uint * max(n, 1))()
    assert lib.cvxg_chol_schedule(nblk, workers, buf, n) == n
    out = []
    for v in buf[:n]:
        out.append((v >> 30, (v >> 20) & 1023, (v >> 10) & 1023, v & 1023))  # (type, k, i, j)
    return out


def _is_chain(typ, k, i, j):
    # POTRF(k), TRSM(k+1,k), UPDATE(k+1,k+1,k), and panel k of block row k+2 (UPDATE(k+2,k+2,k), UPDATE(k+2,k+1,k)),
    # which the chain workgroup of block k+2 applies itself (k_dataflow.hip, own_b2)
    return (typ == 1 and i == k + 1) or (typ == 2 and i == j == k + 1) or (typ == 2 and i == k + 2 and j in (i, i - 1))


@pytest.mark.parametrize("nblk", [1, 2, 3, 4, 10, 16, 64])
def test_schedule_covers_every_task_once_in_dependency_order(nblk):
    order = _order(nblk)
    pos_trsm = {}    # (i, k) -> position
    pos_upd = {}     # (i, j, panel) -> position of the task applying that panel to tile (i, j)
    for p, (typ, k, i, j) in enumerate(order):
        assert typ in (1, 2, 3)
        assert not _is_chain(typ, k, i, j), "chain tasks are run by the chain workgroups, not listed"
        if typ == 1:
            assert i > k and (i, k) not in pos_trsm
            pos_trsm[(i, k)] = p
        else:
            cnt = 4 if typ == 3 else 1
            assert k + cnt <= j <= i
            for kk in range(k, k + cnt):
                assert (i, j, kk) not in pos_upd, "a panel applied twice to a tile"
                pos_upd[(i, j, kk)] = p
    # coverage
    for k in range(nblk):
        for i in range(k + 1, nblk):
            assert (i, k) in pos_trsm or i == k + 1
            for j in range(k + 1, i + 1):
                assert (i, j, k) in pos_upd or _is_chain(2, k, i, j), (i, j, k)
    # order: TRSM(i,k) after the update of tile (i,k) with panel k-1; UPDATE(i,j,k) after TRSM(i,k), TRSM(j,k)
    # and after the update of tile (i,j) with panel k-1
    for (i, k), p in pos_trsm.items():
        if k > 0:
            q = pos_upd.get((i, k, k - 1))
            assert q is None or q < p
    for (i, j, k), p in pos_upd.items():
        for r in (i, j):
            q = pos_trsm.get((r, k))
            assert q is None or q <= p  # (<=: a group entry covers later panels than its first)
        if k > 0:
            q = pos_upd.get((i, j, k - 1))
            assert q is None or q <= p
    assert len(order) == len(set(order))
