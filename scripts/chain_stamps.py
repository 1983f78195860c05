"""Per-block critical-chain stamps of a CVXG_DF_TRACE file (k_dataflow.hip): POTRF(k) start / last L^-1
row-block published / done, and for block k+1 on the other chain workgroup: operands staged, slice 2 done,
last row-block in hand, TRSM + diagonal update done (us from the first POTRF)."""
import sys

import numpy as np


def main(path, blocks=(2, 3, 10, 30, 50, 61)):
    raw = open(path, "rb").read()
    nq, nb = (int(v) for v in np.frombuffer(raw[:8], dtype=np.int32))
    order = np.frombuffer(raw[8:8 + 4 * nq], dtype=np.uint32)
    # chain records per block, from the file size (k_dataflow.hip writes 3: POTRF(k), the staging of k+1, the fix hook)
    R = ((len(raw) - 8 - 4 * nq) // 32 - nq) // nb
    n = nq + R * nb
    tr = np.frombuffer(raw[8 + 4 * nq:8 + 4 * nq + 32 * n], dtype=np.uint64).reshape(n, 4).astype(np.int64)
    ch = tr[nq:].reshape(nb, R, 4)
    t0 = ch[0, 0, 0]
    us = lambda v: (v - t0) / 100.0
    per = (ch[nb - 1, 0, 0] - ch[1, 0, 0]) / 100.0 / (nb - 2)
    print(f"chain period {per:.2f} us per block")
    for k in blocks:
        if k + 1 >= nb:
            continue
        p, pn = ch[k], ch[k + 1]
        print(f"{k:3d} potrf {us(p[0, 0]):8.1f} pub3 {us(p[0, 3]):8.1f} done {us(p[0, 2]):8.1f} | k+1: staged "
              f"{us(p[1, 1]):8.1f} slice2 {us(pn[0, 1]):8.1f} lastrow {us(p[1, 3]):8.1f} done {us(p[1, 2]):8.1f}")
    # the worker tasks the staging of block k+1 waits on: claimed / dependencies met / done, us from POTRF(k) start
    typ, kk, ii, jj = order >> 30, (order >> 20) & 1023, (order >> 10) & 1023, order & 1023
    rec = {(int(typ[x]), int(ii[x]), int(jj[x]), int(kk[x])): tr[x] for x in range(nq)}
    print("  k | TRSM(k+1,k-1) claim/start/done | UPD(k+1,k,k-1) claim/start/done | UPD(k+1,k+1,k-1) claim/start/done"
          "  (us from POTRF(k) start)")
    for k in blocks:
        if not 1 <= k < nb - 1:
            continue
        s0 = ch[k, 0, 0]
        row = []
        for key in ((1, k + 1, k - 1, k - 1), (2, k + 1, k, k - 1), (2, k + 1, k + 1, k - 1)):
            r = rec.get(key)
            row.append("        --" if r is None else " ".join(f"{(v - s0) / 100.0:6.1f}" for v in r[:3]))
        print(f"{k:3d} | " + " | ".join(row))


if __name__ == "__main__":
    main(sys.argv[1])
