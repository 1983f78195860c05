"""GPU: the engine's own C3 barrier solve (random_qp(4096, 8192, instance 0), standard parameters, the t-loop of
BarrierSolver.scala:70-117) from x0, recording late-path states as inputs for the oracle fixture
tests/golden/big/C3late_n4096_m8192.npz (tests/golden/make_golden_big.py C3LATE): in each centering at t = 1e10, 1e11
and 1e12 the iterate entering inner iterations 0 and 1 and the first REGULARIZED steps (regularizedCholesky's
Q + 1e-10 I branch, MatrixUtils.scala:452-461), with the centering's frozen trust radius and the engine's step record.
Writes gpurun_out/c3_late_states.npz."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LATE = (1e10, 1e11, 1e12)
REG_PER_CENTERING = 2


def main():
    import torch
    from cvx_amd import problems as Z
    from cvx_amd.api import SolverParams
    from cvx_amd.engine import Engine
    torch.cuda.set_device(0)
    n, m = 4096, 8192
    spec = Z.random_qp(n, m, instance=0)
    pars = SolverParams.standardParams()
    eng = Engine(n, m, 0, device=0)
    eng.load_problem(spec)
    eng.set_x(spec["x0"])
    fields = ("step", "backtracks_c", "backtracks_armijo", "ruiz_sweeps", "regularized", "min_diag", "rel_err", "q",
              "ls_ties", "ls_fresh", "small_pivot", "trust_radius")
    rec = {k: [] for k in ("t", "it_n", "radius", "x") + fields}
    t, t0 = 1.0, time.perf_counter()
    while True:
        eng.centering_begin(t)
        it, nreg, radius = 0, 0, float("nan")
        while True:
            x = eng.get_x() if t in LATE else None
            st = eng.newton_step(pars)
            if it == 0:
                radius = st.trust_radius
            keep = t in LATE and (it <= 1 or (st.regularized and nreg < REG_PER_CENTERING))
            if keep:
                nreg += int(st.regularized and it > 1)
                rec["t"].append(t)
                rec["it_n"].append(it)
                rec["radius"].append(radius)
                rec["x"].append(x)
                for f in fields:
                    rec[f].append(getattr(st, f))
                print(f"t={t:g} it={it}: step {st.step:g} kc {st.backtracks_c} ka {st.backtracks_armijo} ruiz "
                      f"{st.ruiz_sweeps} reg {st.regularized} (stop row {st.small_pivot}) min diag {st.min_diag:.3e} "
                      f"rel err {st.rel_err:.2e} ties {st.ls_ties}", flush=True)
            it += 1
            if st.done:
                break
        print(f"centering t={t:g}: {it} steps ({time.perf_counter() - t0:.1f} s)", flush=True)
        if m / t < pars.tolSolver:
            break
        t *= 10.0
    eng.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "c3_late_states.npz"),
                        **{k: np.array(v) for k, v in rec.items()})


if __name__ == "__main__":
    main()
