"""Bitwise fingerprint of the engine's Newton direction and step on fixed states (GPU): for the library CVXG_LIB
selects, print one line per state with SHA-256 of dx, min diag(L), the regularization flag, the accepted step and a
hash of x after the step.  Two builds that must give the same bits (a scheduling change, a re-ordered instruction
stream) print the same lines:  CVXG_LIB=a.so python scripts/lib_fingerprint.py > a.txt; ... ; diff a.txt b.txt"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cvx_amd import problems as Z  # noqa: E402
from cvx_amd.api import SolverParams  # noqa: E402
from cvx_amd.engine import Engine  # noqa: E402

H = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def run(n, m, states, instance):
    spec = Z.random_qp(n, m, instance=instance)
    eng = Engine(n, m, 0)
    eng.load_problem(spec)
    pars = SolverParams.standardParams()
    for t, x, g, it_n, radius in states:
        x = spec["x0"] if x is None else x
        dx, _, info = eng.newton_direction(pars, t, x, grad=g)
        eng.set_x(x)
        eng.centering_resume(t, it_n, radius, grad=g)
        st = eng.newton_step(pars)
        print(f"n={n} t={t:.3g} dx={H(dx)} min_diag={info.min_diag!r} reg={info.regularized} step={st.step!r} "
              f"x={H(eng.get_x())}", flush=True)
    eng.close()


def main():
    nan = float("nan")
    run(1000, 2000, [(1.0, None, None, 0, nan), (1e6, None, None, 0, nan)], 3)
    fx = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "big",
                                   "C3late_n4096_m8192.npz")))
    st = [(1.0, None, None, 0, nan)] + [(float(fx["t"][k]), fx["x"][k], fx["grad"][k], int(fx["it_n"][k]),
                                         float(fx["radius"][k])) for k in (2, 5, 6, 7)]
    run(4096, 8192, st, int(fx["instance"]))


if __name__ == "__main__":
    main()
