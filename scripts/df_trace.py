"""Analyse a dataflow-Cholesky task timeline written with CVXG_DF_TRACE=<file> (k_dataflow.hip).

File: int32 ntasks, int32 nblk, uint32 order[ntasks] (encoded queue tasks), uint64 trace[ntasks + 3 nblk][4]
= {claim, ready, done, wg} in s_memrealtime ticks (100 MHz) for the worker tasks; the last 3 nblk records hold the
chain workgroups' stamps (cvxg.cpp writes 4 (ntasks + 3 nblk) words).  Prints per-type durations of the worker tasks and the
fraction of workgroup time spent busy / waiting (the chain's stamps: scripts/chain_offsets.py).
"""
import sys

import numpy as np


def main(path):
    raw = open(path, "rb").read()
    nq, nbk = (int(v) for v in np.frombuffer(raw[:8], dtype=np.int32))
    order = np.frombuffer(raw[8:8 + 4 * nq], dtype=np.uint32)
    n = nq  # worker tasks only (the 6 nbk chain stamp records after them are read by scripts/chain_offsets.py)
    tr = np.frombuffer(raw[8 + 4 * nq:8 + 4 * nq + 32 * n], dtype=np.uint64).reshape(n, 4).astype(np.int64)
    typ = order >> 30
    k = (order >> 20) & 1023
    i = (order >> 10) & 1023
    j = order & 1023
    t0 = tr[:, 0].min()
    claim, ready, done = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0  # us
    span = done.max()
    nwg = int(tr[:, 3].max()) + 1
    print(f"tasks {n}  span {span:.1f} us  workgroups {nwg}")
    for t, name in enumerate(["POTRF", "TRSM", "UPDATE", "UPDATE4"]):
        m = typ == t
        if m.any():
            print(f"{name:7s} n={m.sum():6d} run avg {np.mean(done[m] - ready[m]):7.2f} us  "
                  f"p50 {np.median(done[m] - ready[m]):7.2f}  wait avg {np.mean(ready[m] - claim[m]):7.2f} us")
    busy = np.sum(done - ready)
    wait = np.sum(ready - claim)
    print(f"busy {busy / (span * nwg):.3f} of wg-time, waiting {wait / (span * nwg):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
