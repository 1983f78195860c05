"""Generate the per-Newton-step golden fixtures from the CPU oracle (oracle/cvx_oracle.py).

The reference (Scala/Breeze) cannot run here, so these vectors are outputs of the
restatement on seeded inputs; the restatement itself is pinned by the reference's known-answer tests
(tests/test_oracle_known_answers.py).  Run:  python tests/golden/make_golden.py [name ...]
Each fixture: the packed problem + every inner Newton step of a full barrier solve
(t, x, grad, f, dx, q, accepted step, backtrack counters, Ruiz sweeps, regularisation flag).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cvx_amd import problems as Z  # noqa: E402
from oracle import cvx_oracle as O  # noqa: E402


def _problem(spec):
    if spec.get("kl_B") is not None and np.size(spec["kl_R"]) == 1:  # vec_R = fill(n)(1/(n e)) (Dist_KL.scala:116)
        spec = dict(spec, kl_R=np.full(spec["kl_B"].shape[1], float(np.ravel(spec["kl_R"])[0])))
    return O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"],
                     Aeq=spec.get("Aeq"), beq=spec.get("beq"), qrows=spec.get("qrows"), qP=spec.get("qP"),
                     kl_B=spec.get("kl_B"), kl_R=spec.get("kl_R"))


def trajectory(spec, x0):
    pb = _problem(spec)
    spec = dict(spec, kl_R=pb.kl_R)
    pars = O.standard_params()
    sol = O.barrier_solve(pb, x0, pars, record=True)
    recs = sol.records
    out = dict(
        a0=spec["a0"], r0=np.array(spec["r0"]), A=spec["A"], r=spec["r"], ub=spec["ub"], x0=x0,
        t=np.array([rc.t for rc in recs]), x=np.array([rc.x for rc in recs]), grad=np.array([rc.grad for rc in recs]),
        f=np.array([rc.f for rc in recs]), dx=np.array([rc.dx for rc in recs]), q=np.array([rc.q for rc in recs]),
        step=np.array([rc.step for rc in recs]), kc=np.array([rc.backtracks_c for rc in recs]),
        ka=np.array([rc.backtracks_armijo for rc in recs]), ruiz=np.array([rc.ruiz_sweeps for rc in recs]),
        reg=np.array([rc.regularized for rc in recs]), fallback=np.array([rc.fallback for rc in recs]),
        x_final=sol.x, gap=np.array(sol.dualityGap), newton_steps=np.array(sol.newton_steps),
    )
    if spec.get("P") is not None:
        out["P"] = spec["P"]
    if spec.get("Aeq") is not None:
        out["Aeq"], out["beq"] = spec["Aeq"], spec["beq"]
    for k in ("qrows", "qP", "kl_B", "kl_R"):  # QuadraticConstraint rows; the KL dual objective
        if spec.get(k) is not None:
            out[k] = spec[k]
    return out


def main(names=None):
    pars = O.standard_params()
    fixtures = {}
    # dense QP, inequalities only (path A), n not a multiple of the 128 tile (padding)
    spec = Z.random_qp(40, 96, instance=5)
    fixtures["qp_n40_m96"] = trajectory(spec, spec["x0"])
    # linear objective (phase-I-shaped problem: f = s, rows (a_i, -1))
    base = Z.random_qp(24, 60, instance=6)
    A1 = np.hstack([base["A"], -np.ones((60, 1))])
    a0 = np.zeros(25)
    a0[24] = 1.0
    x1 = np.zeros(25)
    x1[24] = 1.0 + max(-base["ub"])
    lin = dict(a0=a0, r0=0.0, P=None, A=A1, r=np.zeros(60), ub=base["ub"], Aeq=None, beq=None)
    pb = _problem(lin)
    sol = O.barrier_solve(pb, x1, pars, tc=O.phase_I_termination, record=True)
    recs = sol.records
    fixtures["phase1_n25_m60"] = dict(
        a0=a0, r0=np.array(0.0), A=A1, r=lin["r"], ub=lin["ub"], x0=x1,
        t=np.array([rc.t for rc in recs]), x=np.array([rc.x for rc in recs]), grad=np.array([rc.grad for rc in recs]),
        f=np.array([rc.f for rc in recs]), dx=np.array([rc.dx for rc in recs]), q=np.array([rc.q for rc in recs]),
        step=np.array([rc.step for rc in recs]), kc=np.array([rc.backtracks_c for rc in recs]),
        ka=np.array([rc.backtracks_armijo for rc in recs]), ruiz=np.array([rc.ruiz_sweeps for rc in recs]),
        reg=np.array([rc.regularized for rc in recs]), fallback=np.array([rc.fallback for rc in recs]),
        x_final=sol.x, gap=np.array(sol.dualityGap), newton_steps=np.array(sol.newton_steps), phase1=np.array(1))
    # equality-constrained KKT path (path B): rankOneProblemSimplex(10) from its phase-I point
    spec = Z.rank_one_problem_simplex(10)
    pbe = _problem(spec)
    x0 = O.with_feasible_point(pbe, spec["x_where_defined"], pars)
    fixtures["simplex_rank1_n10_p1"] = trajectory(spec, x0)
    # QuadraticConstraint rows (QuadraticConstraint.scala:8-40) in the barrier path: the line search's quadratic
    # trial expansion g + t e + t^2 f / 2 against the reference's fresh valueAt(x + s t)
    spec = Z.random_qp_quad(30, 50, 3, instance=12)
    fixtures["quad_n30_m50_q3"] = trajectory(spec, spec["x0"])
    # the KL dual (Duality.dualProblem over Dist_KL, Duality.scala:99-112): exp terms in every trial
    spec = Z.kl_dual_spec(300, 12, instance=3)
    fixtures["kldual_n300_k12"] = trajectory(spec, spec["x0"])
    for name, fx in fixtures.items():
        if names and name not in names:
            continue
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **fx)
        print(name, {k: np.shape(v) for k, v in fx.items() if k in ("A", "x", "dx")}, "steps", int(fx["newton_steps"]))


if __name__ == "__main__":
    main(sys.argv[1:] or None)
