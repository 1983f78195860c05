"""Golden fixture of the direct (primal) KL solves at n = 2048 from the CPU oracle (oracle/cvx_oracle.py).

What MinimizationTests.runProblems does first with every KL problem (MinimizationTests.scala:23,35): kl_1 / kl_2
(OptimizationProblems.scala:167-210, 271-320) through OptimizationProblem.withoutFeasiblePoint -- phase I
(ConstraintSet.withFeasiblePoint, :556-575), then BarrierSolver.solveWithEQs (BarrierSolver.scala:124-177) over
Dist_KL.objectiveFunction (Dist_KL.scala:223-239) with the EqualityConstrainedSolver inner loop
(EqualityConstrainedSolver.scala:37-107).  The reference cannot run here; these are outputs of the
restatement, which the reference's known-answer tests pin (tests/test_oracle_known_answers.py).

Per kind: the phase-I point x0, the Newton steps per centering, the final x and duality gap, for every Newton step
of the solve (t, f, q, accepted step, the two backtracking counters), and the iterate entering each centering at
t >= 1e10.  Late in the path one ulp of f = t f0 - sum log d (~2e-4 at t = 1e12) exceeds the Armijo decrease
alpha t q (< 1e-8), so those decisions are rounding noise: with 4 OpenBLAS threads (the recorded run)
the kl_1 centerings take [2, 3, 4, 6, 6, 7, 7, 7, 8, 8, 6, 6, 8] steps, with 3 threads (a different dpotrf / dtrtrs
summation) the last one runs to maxIter = 1000.  The BLAS thread count is pinned and stored.  4-20 min of CPU.
  python tests/golden/make_golden_kl.py  ->  tests/golden/kl/kl_direct_n2048.npz
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cvx_amd import problems as Z  # noqa: E402
from oracle import cvx_oracle as O  # noqa: E402


def solve(kind: str, n: int):
    spec = Z.kl_primal_spec(n, kind)
    pb = O.Problem(a0=spec["a0"], r0=0.0, P=None, A=spec["A"], r=spec["r"], ub=spec["ub"], Aeq=spec["Aeq"],
                   beq=spec["beq"], klp_n=n)
    pars = O.standard_params()
    t0 = time.time()
    x0 = O.with_feasible_point(pb, spec["x_where_defined"], pars)
    sol = O.barrier_solve(pb, x0, pars, record=True)
    ts = np.array([r.t for r in sol.records])
    late_t, late_x = [], []
    for r in sol.records:
        if r.t >= 1e10 and r.t not in late_t:
            late_t.append(r.t)
            late_x.append(r.x)
    per = [int(np.sum(ts == t)) for t in sorted(set(ts.tolist()))]
    print(f"{kind} n={n}: {sol.newton_steps} Newton steps {per}, gap {sol.dualityGap:.3e}, "
          f"max|x - x_opt| {np.max(np.abs(sol.x - spec['x_opt'])):.3e}, {time.time() - t0:.0f} s", flush=True)
    return {f"{kind}_x0": x0, f"{kind}_x": sol.x, f"{kind}_per_centering": np.array(per),
            f"{kind}_gap": np.array(sol.dualityGap), f"{kind}_eqgap": np.array(sol.equalityGap),
            f"{kind}_t": ts, f"{kind}_f": np.array([r.f for r in sol.records]),
            f"{kind}_q": np.array([r.q for r in sol.records]),
            f"{kind}_step": np.array([r.step for r in sol.records]),  # NaN: no step (decrement below tol)
            f"{kind}_kc": np.array([r.backtracks_c for r in sol.records]),
            f"{kind}_ka": np.array([r.backtracks_armijo for r in sol.records]),
            # the iterate entering each centering at t >= 1e10 (replay starting points of the late path)
            f"{kind}_late_t": np.array(late_t), f"{kind}_late_x": np.array(late_x)}


if __name__ == "__main__":
    from threadpoolctl import threadpool_limits
    n = 2048
    threads = int(os.environ.get("GOLDEN_BLAS_THREADS", "4"))
    out = {"n": np.array(n), "blas_threads": np.array(threads)}
    with threadpool_limits(threads):
        for kind in ("kl_1", "kl_2"):
            out.update(solve(kind, n))
    np.savez_compressed(os.path.join(HERE, "kl", "kl_direct_n2048.npz"), **out)
