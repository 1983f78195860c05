"""Worker utilisation and chain period of a dataflow Cholesky trace (CVXG_DF_TRACE file): per 100 us window the share of
the worker slots running a task (ready -> done), waiting on its inputs (claim -> ready) or between tasks; then the chain
period (POTRF(k+1) start - POTRF(k) start) by block range."""
import sys

import numpy as np


def load(path):
    raw = open(path, 'rb').read()
    nq, nb = (int(v) for v in np.frombuffer(raw[:8], dtype=np.int32))
    R = ((len(raw) - 8 - 4 * nq) // 32 - nq) // nb
    tr = np.frombuffer(raw[8 + 4 * nq:8 + 4 * nq + 32 * (nq + R * nb)], dtype=np.uint64).reshape(nq + R * nb, 4)
    tr = tr.astype(np.int64)
    return nq, nb, tr[:nq], tr[nq:].reshape(nb, R, 4)


def main(path, W=100.0, workers=254):
    nq, nb, tk, ch = load(path)
    t0 = ch[0, 0, 0]
    T = (tk[:, :3] - t0) / 100.0
    starts = (ch[:, 0, 0] - t0) / 100.0
    end = starts[-1] + 15
    print(f"{path}: {nq} tasks, {nb} blocks, POTRF(last) starts at {starts[-1]:.1f} us")
    print("window(us)  busy  wait  between")
    for w0 in np.arange(0, end, W):
        w1 = w0 + W
        ov = lambda a, b: np.clip(np.minimum(b, w1) - np.maximum(a, w0), 0, None).sum()
        busy, wait = ov(T[:, 1], T[:, 2]), ov(T[:, 0], T[:, 1])
        cap = workers * min(W, end - w0)
        print(f"{w0:6.0f}     {busy / cap:5.2f} {wait / cap:5.2f} {1 - (busy + wait) / cap:5.2f}")
    per = np.diff(starts)
    for a, b in ((0, 8), (8, 24), (24, 40), (40, nb - 1)):
        print(f"period k in [{a},{b}): mean {per[a:b].mean():5.1f} us")
    dur = T[:, 2] - T[:, 1]
    typ = np.frombuffer(open(path, 'rb').read()[8:8 + 4 * nq], dtype=np.uint32) >> 30
    for t, nm in ((1, "TRSM"), (2, "UPDATE"), (3, "UPDATE4")):
        sel = typ == t
        print(f"{nm:8s} n={sel.sum():6d} ready->done median {np.median(dur[sel]):5.2f} us, claim->ready median "
              f"{np.median((T[:, 1] - T[:, 0])[sel]):5.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
