"""Analyse a dataflow-Cholesky task timeline written with CVXG_DF_TRACE=<file> (k_dataflow.hip).

File: int32 ntasks, int32 nblk, uint32 order[ntasks] (encoded queue tasks), uint64 trace[ntasks + 3 nblk][4]
= {claim, ready, done, wg} in s_memrealtime ticks (100 MHz); the last 3 nblk records are workgroup 0's
critical chain POTRF(k), TRSM(k+1,k), UPDATE(k+1,k+1,k).  Prints per-type durations, the critical chain per block step, and the
fraction of workgroup time spent busy / waiting.
"""
import sys

import numpy as np


def main(path):
    raw = open(path, "rb").read()
    nq, nbk = (int(v) for v in np.frombuffer(raw[:8], dtype=np.int32))
    order = np.frombuffer(raw[8:8 + 4 * nq], dtype=np.uint32)
    n = nq + 3 * nbk
    tr = np.frombuffer(raw[8 + 4 * nq:8 + 4 * nq + 32 * n], dtype=np.uint64).reshape(n, 4).astype(np.int64)
    chain = []
    for kk in range(nbk):
        chain += [(0 << 30) | (kk << 20) | (kk << 10) | kk, (1 << 30) | (kk << 20) | ((kk + 1) << 10) | kk,
                  (2 << 30) | (kk << 20) | ((kk + 1) << 10) | (kk + 1)]
    order = np.concatenate([order, np.array(chain, dtype=np.uint32)])
    keep = np.ones(n, bool)
    keep[nq + 3 * (nbk - 1) + 1:] = False  # no TRSM / UPDATE after the last POTRF
    order, tr = order[keep], tr[keep]
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
    nb = int(k.max()) + 1
    pot = {int(k[x]): x for x in np.where(typ == 0)[0]}
    trs = {(int(i[x]), int(k[x])): x for x in np.where(typ == 1)[0]}
    upd = {(int(i[x]), int(j[x]), int(k[x])): x for x in np.where(typ == 2)[0]}
    print(" k | potrf ready..done | trsm(k+1,k) ready..done | upd(k+1,k+1,k) ready..done | gap to next potrf ready")
    for kk in list(range(min(nb, 6))) + list(range(max(6, nb - 3), nb)):
        p = pot[kk]
        line = f"{kk:3d} | {ready[p]:8.1f}..{done[p]:8.1f}"
        if kk + 1 < nb:
            tt = trs[(kk + 1, kk)]
            uu = upd[(kk + 1, kk + 1, kk)]
            pn = pot[kk + 1]
            line += (f" | {ready[tt]:8.1f}..{done[tt]:8.1f} | {ready[uu]:8.1f}..{done[uu]:8.1f} |"
                     f" {ready[pn] - done[uu]:6.1f}  (claimed {claim[pn]:8.1f})")
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
