"""Per-sweep timeline of the one-launch Ruiz loop from a CVXG_RUIZ_TRACE file (k_ruiz.hip): for each sweep, over the
workgroups that ran it, the median / max of batch start, d in hand, tiles done and reductions done (us from the
first workgroup's start)."""
import sys

import numpy as np


def main(path):
    raw = open(path, "rb").read()
    nwg = int(np.frombuffer(raw[:4], dtype=np.int32)[0])
    tr = np.frombuffer(raw[4:], dtype=np.uint64).reshape(nwg, -1, 4).astype(np.int64)
    t0 = tr[:, 0, 0][tr[:, 0, 0] > 0].min()
    print("sweep  n_wg | start med/max | d_in med/max | tiles med/max | reduced med/max (us)")
    for k in range(tr.shape[1]):
        m = tr[:, k, 0] > 0
        if not m.any():
            break
        cols = []
        for f in range(4):
            v = tr[m, k, f]
            v = v[v > 0]
            cols.append(f"{np.median(v - t0) / 100:7.2f} {np.max(v - t0) / 100:7.2f}" if len(v) else "    -       -")
        print(f"{k:5d} {m.sum():5d} | " + " | ".join(cols))


if __name__ == "__main__":
    main(sys.argv[1])
