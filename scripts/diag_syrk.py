"""Diagnostic: per-tile comparison of the assembled barrier Hessian against torch fp64 (C2 shape)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cvx_amd import problems as Z  # noqa: E402
from cvx_amd.engine import Engine  # noqa: E402

n, m = int(sys.argv[1]), int(sys.argv[2])
spec = Z.random_qp(n, m, instance=0)
eng = Engine(n, m, 0, device=0)
eng.load_problem(spec)
x = spec["x0"]
f, g, H = eng.barrier_eval(1.0, x, want_grad=True, want_hess=True)
dev = torch.device("cuda:0")
A = torch.from_numpy(spec["A"]).to(dev)
P = torch.from_numpy(spec["P"]).to(dev)
d = torch.from_numpy(spec["ub"]).to(dev) - A @ torch.from_numpy(x).to(dev)
Href = (P + A.T @ (A / (d * d)[:, None])).cpu().numpy()
T = 128
nt = (n + T - 1) // T
bad = []
for I in range(nt):
    for J in range(I + 1):
        a = H[I * T:(I + 1) * T, J * T:(J + 1) * T]
        b = Href[I * T:(I + 1) * T, J * T:(J + 1) * T]
        e = np.linalg.norm(a - b) / np.linalg.norm(b)
        if e > 1e-12:
            bad.append((I, J, float(e), float(np.linalg.norm(a))))
print("bad tiles", len(bad), bad[:40])
eng.close()
