"""Diagnostic (GPU): the direct KL solves kl_1 / kl_2 at n = 2048 (OptimizationProblems.scala:167-210, 271-320;
MinimizationTests.scala:23,35) through OptimizationProblem.withoutFeasiblePoint, centering by centering, under the
KKT right-hand-side variants that give the Newton direction different bits (CVXG_KKT_FUSED_RHS=1: the many-column
solves, 9: the columns fused into the factorization).  Prints per-centering step counts, the final error against the
analytic optimum and, on a failure, the engine's line-search diagnostics; writes the phase-I point and the final x
to gpurun_out/kl_diag_<kind>_<variant>.npz."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(kind, n, variant, sparse="1"):
    os.environ["CVXG_KKT_FUSED_RHS"] = variant
    os.environ["CVXG_SPARSE_ROWS"] = sparse
    from cvx_amd import problems as Z
    from cvx_amd.api import (ConstraintSet, Dist_KL, EqualityConstraint, LinearConstraint, OptimizationProblem,
                             SolverParams)
    pars = SolverParams.standardParams()
    spec = Z.kl_primal_spec(n, kind)
    cnts = [LinearConstraint(f"row{i}", n, spec["ub"][i], spec["r"][i], spec["A"][i]) for i in range(spec["A"].shape[0])]
    ineqs = ConstraintSet(n, cnts, np.full(n, 1.0 / n))
    t0 = time.perf_counter()
    prob = OptimizationProblem.withoutFeasiblePoint(kind, Dist_KL.objectiveFunction(n), ineqs,
                                                    EqualityConstraint(spec["Aeq"], spec["beq"]), "BR", pars)
    solver = prob.solver
    eng = solver.engine
    x0 = np.array(solver.startingPoint, dtype=np.float64)
    m = spec["A"].shape[0]
    eng.set_x(x0)
    t, per, err = 1.0, [], None
    while True:
        try:
            ci = eng.centering(pars, t)
        except Exception as e:  # the reference throws NotConvergedException here too (EqualityConstrainedSolver:90)
            err = f"{type(e).__name__}: {e}"
            break
        per.append(ci.iter)
        if m / t < pars.tolSolver and ci.equality_gap < pars.tolSolver:
            break
        t *= 10.0
        if len(per) >= 100:
            break
    x = eng.get_x()
    dt = time.perf_counter() - t0
    print(f"{kind} n={n} KKT_FUSED_RHS={variant} SPARSE_ROWS={sparse}: per-centering {per} (t at end {t:g}), "
          f"max|x - x_opt| {np.max(np.abs(x - spec['x_opt'])):.3e}, {dt:.1f} s" + (f"\n  FAILED: {err}" if err else ""),
          flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    if n == 2048:
        np.savez(os.path.join(ROOT, "gpurun_out", f"kl_diag_{kind}_{variant}_{sparse}.npz"), x0=x0, x=x,
                 per=np.array(per), t_end=t, failed=err is not None)
    eng.close()


if __name__ == "__main__":
    ns = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2048]
    kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["kl_1", "kl_2"]
    import torch  # noqa: F401  (one HIP runtime, shared with the engine)
    for n in ns:
        for variant in ("1", "9"):
            for sparse in ("1", "0"):
                for kind in kinds:
                    run(kind, n, variant, sparse)
