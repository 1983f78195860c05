"""Problem generators (synthetic inputs for the barrier path).

Plain numpy arrays in the packing the engine consumes: objective r0 + a0.x + x'Px/2
(P None => LinearObjectiveFunction), linear inequalities r_i + a_i.x <= ub_i with A row i = a_i in
constraint LIST order, optional equalities Aeq x = beq.

* ``random_qp`` — the seeded dense QP of SURVEY.md §8(d) used for configs C2/C3/C5, following the
  reference generator patterns (Constraints.scala:158-171 random a_i in [-1,1]; ConstraintSets.scala:67-89;
  MatrixUtils.scala:57-74): a_i ~ U[-1,1]^n, r_i = 0, ub_i ~ U[0.1,0.2], x0 = 0 strictly feasible,
  P = R'R/n + I, a0 = -P x_tgt with x_tgt ~ 10 U[-1,1]^n.
* known-answer problems of SimpleOptimizationProblems.scala that fit the linear-constraint engine.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

SEED_BASE = 20261015


def random_qp(n: int, m: int, instance: int = 0, dtype=np.float64) -> Dict[str, np.ndarray]:
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + instance))
    A = rng.uniform(-1.0, 1.0, size=(m, n)).astype(dtype)
    ub = rng.uniform(0.1, 0.2, size=m)
    R = rng.uniform(-1.0, 1.0, size=(n, n))
    P = (R.T @ R) / n + np.eye(n)
    P = 0.5 * (P + P.T)  # exactly symmetric (the reference's Breeze cholesky checks symmetry)
    x_tgt = 10.0 * rng.uniform(-1.0, 1.0, size=n)
    a0 = -(P @ x_tgt)
    return dict(id=f"random_qp(n={n},m={m},instance={instance})", a0=a0, r0=0.0, P=P, A=A,
                r=np.zeros(m), ub=ub, Aeq=None, beq=None, x0=np.zeros(n))


def random_qp_eq(n: int, m: int, p: int, instance: int = 0) -> Dict[str, np.ndarray]:
    """random_qp plus p dense equality rows Aeq x = beq (entries U[-1,1]) with beq = Aeq x0 at a small x0 that is
    strictly inside the inequalities: the workload of the affine reduction x = z0 + F u
    (BarrierSolver.reduced over SolutionSpace(Aeq, beq)) and of the wide KKT path (p + 1 > MAX_RHS)."""
    spec = random_qp(n, m, instance)
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 104729 + instance))
    x0 = 0.01 * rng.uniform(-1.0, 1.0, size=n)
    A = spec["A"]
    ub = A @ x0 + rng.uniform(0.1, 0.2, size=m)
    Aeq = rng.uniform(-1.0, 1.0, size=(p, n))
    beq = Aeq @ x0
    spec.update(id=f"random_qp_eq(n={n},m={m},p={p},instance={instance})", ub=ub, Aeq=Aeq, beq=beq, x0=x0)
    return spec


def random_qp_bounds(n: int, m: int, instance: int = 0) -> Dict[str, np.ndarray]:
    """random_qp plus sparse constraint rows interleaved with the dense ones, x0 = 0 strictly feasible:
    lower bounds -x_j <= 1 (the Constraints.singleCoordinatePositive shape, Constraints.scala:26-35, shifted),
    upper bounds x_j <= 2, difference rows x_j - x_k <= 0.5 and phase-I style rows x_j - x_k - x_l <= 1
    (ConstraintSet.scala:153-168: a constraint row with the extra -1 column).  Exercises the engine's split of
    the Hessian into a dense-row SYRK and per-entry sums over the sparse rows."""
    spec = random_qp(n, m, instance)
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 7919 + instance))
    rows, ubs = [], []
    for j in range(n):
        a = np.zeros(n)
        a[j] = -1.0
        rows.append(a)
        ubs.append(1.0)
    for j in rng.choice(n, size=n // 2, replace=False):
        a = np.zeros(n)
        a[j] = 1.0
        rows.append(a)
        ubs.append(2.0)
    for _ in range(n // 2):
        j, k = rng.choice(n, size=2, replace=False)
        a = np.zeros(n)
        a[j], a[k] = 1.0, -1.0
        rows.append(a)
        ubs.append(0.5)
    for _ in range(n // 4):
        j, k, l = rng.choice(n, size=3, replace=False)
        a = np.zeros(n)
        a[j], a[k], a[l] = 1.0, -1.0, -1.0
        rows.append(a)
        ubs.append(1.0)
    S = np.array(rows)
    order = rng.permutation(m + S.shape[0])  # sparse rows interleaved with the dense rows (list order matters)
    A = np.vstack([spec["A"], S])[order]
    ub = np.concatenate([spec["ub"], np.array(ubs)])[order]
    spec.update(id=f"random_qp_bounds(n={n},m={m},instance={instance})", A=A, ub=ub, r=np.zeros(A.shape[0]))
    return spec


def kl_dual_spec(nout: int, k: int, instance: int = 0) -> Dict[str, np.ndarray]:
    """C4 throughput variant: Dist_KL with k random expectation rows H (entries U[0,1]) over
    nout outcomes, u = row means x U[0.9, 1.1], no equalities, in the packing of its dual barrier problem
    (Duality.dualProblem, Duality.scala:99-112; Dist_KL.scala:104-165): z = (lambda, nu) of dimension k + 1,
    B = (H; 1'), w = (u, 1), R = 1/(nout e) with the reference's e, lambda >= 0 as k bound rows, z0 = 0.001."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 104729 + instance))
    H = rng.uniform(0.0, 1.0, size=(k, nout))
    u = H.mean(axis=1) * rng.uniform(0.9, 1.1, k)
    B = np.vstack([H, np.ones((1, nout))])
    w = np.concatenate([u, np.ones(1)])
    A = np.zeros((k, k + 1))
    A[np.arange(k), np.arange(k)] = -1.0
    return dict(id=f"kl_dual(nout={nout},k={k},instance={instance})", a0=w, r0=0.0, P=None, A=A, r=np.zeros(k),
                ub=np.zeros(k), Aeq=None, beq=None, x0=np.full(k + 1, 0.001), kl_B=B,
                kl_R=np.array([1.0 / (nout * 2.7182811828459045)]))


def kl_primal_spec(n: int, kind: str = "kl_1") -> Dict[str, np.ndarray]:
    """The direct (primal) KL problems of OptimizationProblems.scala on Dist_KL.objectiveFunction(n) (x . log(n x),
    Dist_KL.scala:223-239), n even and > 9:
    * kl_1 (:167-210): rows x_j >= 0 (allCoordinatesPositive) then P(A) >= 0.36 and P(B) <= 0.1 (expectation_lt_r),
      equality sum(x) = 1 (Constraints.sumToOne); A = {0, 1, 2}, B = {n/2, .., n-1};
    * kl_2 (:271-320): the positivity rows, equalities 1'x = 1, P(A) = 0.36, P(B) = 0.1 (probEq.addEqualities(e1)
      .addEqualities(e2)).
    x0 is strictly feasible for the inequalities (P(A) = 0.39, P(B) = 0.09 for kl_1; a positive perturbation of the
    known optimum with sum 1 for kl_2); x_opt = kl1_ / kl2_analyticSolution (:136-141, 249-251, n > 15)."""
    assert n > 9 and n % 2 == 0
    j = np.arange(n)
    I_A = (j < 3).astype(float)
    I_B = (j >= n // 2).astype(float)
    A, r, ub = _positivity(n)
    x_opt = np.where(j < 3, 0.12, np.where(j >= n // 2, 0.2 / n, 1.08 / (n - 6)))
    if kind == "kl_1":
        A = np.vstack([A, -I_A, I_B])
        r = np.zeros(n + 2)
        ub = np.concatenate([ub, [-0.36, 0.1]])
        Aeq, beq = _sum_to_one(n)
        x0 = np.where(j < 3, 0.13, np.where(j >= n // 2, 0.18 / n, 0.52 / (n // 2 - 3)))
    elif kind == "kl_2":
        Aeq = np.vstack([np.ones(n), I_A, I_B])
        beq = np.array([1.0, 0.36, 0.1])
        # the known optimum is the whole central path (its gradient lies in the row space of Aeq), so start off it:
        # a positive perturbation that keeps sum(x) = 1 but not the expectation equalities
        x0 = x_opt * (1.0 + 0.25 * np.sin(1.7 * j + 0.3))
        x0 = x0 / np.sum(x0)
    else:
        raise ValueError(kind)
    return dict(id=f"{kind}(n={n})", a0=np.zeros(n), r0=0.0, P=None, A=A, r=r, ub=ub, Aeq=Aeq, beq=beq, x0=x0,
                klp_n=n, x_opt=x_opt, x_where_defined=np.full(n, 1.0 / n))


def random_constraint_set(x0: np.ndarray, p: int, q: int, instance: int = 0, neq: int = 0) -> Dict[str, np.ndarray]:
    """ConstraintSets.randomConstraintSet (ConstraintSets.scala:67-89), seeded: p linear rows a'(x - x0) <= e, a ~
    U[-1,1]^n, e = 0.1 + 0.1 U (Constraints.randomLinearIneqConstraint / linearIneqConstraint, Constraints.scala:158-171:
    r = -a.x0), then q quadratic rows ||R(x - x0)||^2 / 2 <= e, R ~ U[-1,1]^(n x n), e = 0.2 (1 + U)
    (randomQuadraticIneqConstraint / quadraticIneqConstraint, :177-200: P = R'R, a = -R'R x0, r = ||R x0||^2 / 2);
    pointWhereDefined u = 0.  neq > 0 adds Constraints.randomEqualityConstraint(x0, neq) (:207-214): A ~ U[-1,1],
    b = A x0.  The objective is left to the caller (a0 = 0)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 7919 + instance))
    x0 = np.asarray(x0, dtype=np.float64)
    n = x0.shape[0]
    A, r, ub, qP = [], [], [], []
    for _ in range(p):
        e = 0.1 + 0.1 * rng.uniform()
        a = rng.uniform(-1.0, 1.0, n)
        A.append(a), r.append(-(a @ x0)), ub.append(e)
    for _ in range(q):
        e = 0.2 * (1 + rng.uniform())
        R = rng.uniform(-1.0, 1.0, (n, n))
        Rx0 = R @ x0
        nr = np.linalg.norm(Rx0)
        A.append(-(R.T @ Rx0)), r.append(nr * nr / 2), ub.append(e)
        qP.append(R.T @ R)
    spec = dict(id=f"randomConstraintSet(n={n},p={p},q={q},instance={instance})", a0=np.zeros(n), r0=0.0, P=None,
                A=np.array(A), r=np.array(r), ub=np.array(ub), Aeq=None, beq=None,
                qrows=np.arange(p, p + q, dtype=np.int32) if q else None, qP=np.array(qP) if q else None,
                x_where_defined=np.zeros(n), x_feasible=x0.copy())
    if neq:
        Aeq = rng.uniform(-1.0, 1.0, (neq, n))
        spec.update(Aeq=Aeq, beq=Aeq @ x0)
    return spec


def prob_ab(n: int, pA: float, sgnA: float, pB: float, sgnB: float) -> Dict[str, np.ndarray]:
    """ConstraintSets.probAB (ConstraintSets.scala:39-60) with A = {0, 1, 2}, B = {n/2, .., n-1} (FeasibilityTests.
    runAll, FeasibilityTests.scala:117-124): rows sgnB P(B) <= sgnB pB, sgnA P(A) <= sgnA pA (expectation_lt_r), then
    allCoordinatesPositive; pointWhereDefined 1/n; the equality sum(x) = 1 (Constraints.sumToOne)."""
    j = np.arange(n)
    I_A = (j < 3).astype(float)
    I_B = (j >= n // 2).astype(float)
    Ap, rp, ubp = _positivity(n)
    A = np.vstack([I_B * sgnB, I_A * sgnA, Ap])
    Aeq, beq = _sum_to_one(n)
    return dict(id=f"probAB(n={n})", a0=np.zeros(n), r0=0.0, P=None, A=A, r=np.zeros(n + 2),
                ub=np.concatenate([[pB * sgnB, pA * sgnA], ubp]), Aeq=Aeq, beq=beq, x_where_defined=np.full(n, 1.0 / n))


def _positivity(n: int):
    """Constraints.allCoordinatesPositive (Constraints.scala:26-69): -x_j <= 0, j = 0..n-1."""
    return -np.eye(n), np.zeros(n), np.zeros(n)


def _sum_to_one(n: int):
    """Constraints.sumToOne (Constraints.scala:75-80)."""
    return np.ones((1, n)), np.ones(1)


def joptP2() -> Dict:
    """SimpleOptimizationProblems.scala:384-414 — min x'Px (P=[[1,.4],[.4,1]]) on the simplex; x*=(1/2,1/2)."""
    A, r, ub = _positivity(2)
    Aeq, beq = _sum_to_one(2)
    return dict(id="example_1.5", a0=np.zeros(2), r0=0.0, P=np.array([[1.0, 0.4], [0.4, 1.0]]), A=A, r=r,
                ub=ub, Aeq=Aeq, beq=beq, x_where_defined=np.full(2, 2.0), x_opt=np.array([0.5, 0.5]))


def rank_one_problem_simplex(dim: int) -> Dict:
    """SimpleOptimizationProblems.scala:221-255 — f = x'(aa')x/2 form via QuadraticObjectiveFunction(P=aa'),
    a = linspace(1,2,dim), x >= 0, sum x = 1; x* = e_1."""
    a = np.linspace(1.0, 2.0, dim)
    A, r, ub = _positivity(dim)
    Aeq, beq = _sum_to_one(dim)
    x_opt = np.zeros(dim)
    x_opt[0] = 1.0
    return dict(id="Simplicial rankOneProblem", a0=np.zeros(dim), r0=0.0, P=np.outer(a, a), A=A, r=r, ub=ub,
                Aeq=Aeq, beq=beq, x_where_defined=np.full(dim, 1.0 / dim), x_opt=x_opt)


def probability_simplex_problem(n: int) -> Dict:
    """SimpleOptimizationProblems.scala:425-456 — f = 0.5 - 1'x + x'(11')x/2 on x >= 0; minimisers = simplex."""
    A, r, ub = _positivity(n)
    return dict(id="Probability_simplex_problem", a0=-np.ones(n), r0=0.5, P=np.ones((n, n)), A=A, r=r, ub=ub,
                Aeq=None, beq=None, x_where_defined=np.full(n, 2.0), x_opt=np.full(n, 1.0 / n))


def min_dot_product(a: np.ndarray) -> Dict:
    """SimpleOptimizationProblems.scala:142-169 — min -a'x s.t. |x_j| <= |a_j|
    (Constraints.absoluteValuesBoundedBy: +x_j <= |a_j| then -x_j <= |a_j|); x* = a."""
    n = a.shape[0]
    rows, ubs = [], []
    for j in range(n):
        e = np.zeros(n)
        e[j] = 1.0
        rows += [e, -e]
        ubs += [abs(a[j]), abs(a[j])]
    return dict(id="Min f(x)=a'x subject to |x_j|<=|a_j|", a0=-a, r0=0.0, P=None, A=np.array(rows),
                r=np.zeros(2 * n), ub=np.array(ubs), Aeq=None, beq=None, x_where_defined=2.0 * a, x_opt=a.copy())


def norm_squared_with_free_variables(dim: int) -> Dict:
    """SimpleOptimizationProblems.scala:308-340 — 0.5||x||^2 s.t. x_0 <= -1; x* = (-1,0,...,0)."""
    A = np.zeros((1, dim))
    A[0, 0] = 1.0
    x_opt = np.zeros(dim)
    x_opt[0] = -1.0
    return dict(id="normSquaredWithFreeVariables", a0=np.zeros(dim), r0=0.0, P=np.eye(dim), A=A, r=np.zeros(1),
                ub=np.array([-1.0]), Aeq=None, beq=None, x_where_defined=np.ones(dim), x_opt=x_opt)


# ---- problems with QuadraticConstraint rows (qrows index the (A, r, ub) rows; qP holds their P) -----------------

def rank_one_problem_sphere(dim: int) -> Dict:
    """SimpleOptimizationProblems.scala:266-300 — f = x'(aa')x/2, a = linspace(1,2,dim), constraints
    oneHalfNorm2BoundedBy(dim, 1/2) :: allCoordinatesPositive(dim) (Constraints.scala:299-309, 26-69); x* = 0."""
    a = np.linspace(1.0, 2.0, dim)
    Ap, rp, ubp = _positivity(dim)
    A = np.vstack([np.zeros((1, dim)), Ap])
    return dict(id="Spherical rankOneProblem", a0=np.zeros(dim), r0=0.0, P=np.outer(a, a), A=A,
                r=np.concatenate([[0.0], rp]), ub=np.concatenate([[0.5], ubp]), Aeq=None, beq=None,
                qrows=np.array([0], dtype=np.int32), qP=np.eye(dim)[None], x_where_defined=np.full(dim, 1.0 / dim),
                x_opt=np.zeros(dim))


def jopt_p1(dim: int) -> Dict:
    """SimpleOptimizationProblems.scala:347-377 — f = sum(x) s.t. (x.x)/2 <= 1/2; x* = -1/sqrt(dim)."""
    return dict(id="f(x)=sum(x) with ||x||^2<=1", a0=np.ones(dim), r0=0.0, P=None, A=np.zeros((1, dim)),
                r=np.zeros(1), ub=np.array([0.5]), Aeq=None, beq=None, qrows=np.array([0], dtype=np.int32),
                qP=np.eye(dim)[None], x_where_defined=np.full(dim, 2.0), x_opt=-np.ones(dim) / np.sqrt(dim))


def distance_from_origin(n: int, sliced: bool) -> Dict:
    """SimpleOptimizationProblems.scala:464-561 — min ||x||^2/2 (ObjectiveFunctions.normSquared) over
    x'x/2 - 2 x_n + 3/2 <= 0 (QuadraticConstraint(r = 1.5, a = -2 e_n, P = I)); distanceFromOrigin1 (sliced) adds
    for every j the row -(e_j + e_n).x <= -1 twice (the reference builds lc2_j from -a again, not from b); x* = e_n."""
    N = n + 1
    e = np.zeros(N)
    e[n] = 1.0
    rows, r, ub = [-2.0 * e], [1.5], [0.0]
    if sliced:
        for j in range(n):
            a = np.zeros(N)
            a[j] = 1.0
            a = a + e
            rows += [-a, -a]
            r += [0.0, 0.0]
            ub += [-1.0, -1.0]
    return dict(id="DistanceFromOrigin_1" if sliced else "DistanceFromOrigin_0", a0=np.zeros(N), r0=0.0,
                P=np.eye(N), A=np.array(rows), r=np.array(r), ub=np.array(ub), Aeq=None, beq=None,
                qrows=np.array([0], dtype=np.int32), qP=np.eye(N)[None], x_where_defined=np.zeros(N), x_opt=e.copy())


def random_qp_quad(n: int, m: int, q: int, instance: int = 0) -> Dict:
    """random_qp plus q random convex QuadraticConstraint rows x'P_k x/2 + a_k.x <= ub_k (P_k = R'R/n, a_k small),
    interleaved with the linear rows; x0 = 0 stays strictly feasible (ub_k > 0)."""
    spec = random_qp(n, m, instance)
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 31337 + instance))
    qP = np.empty((q, n, n))
    qa = np.empty((q, n))
    for k in range(q):
        R = rng.uniform(-1.0, 1.0, size=(n, n))
        Pk = (R.T @ R) / n
        qP[k] = 0.5 * (Pk + Pk.T)
        qa[k] = 0.1 * rng.uniform(-1.0, 1.0, size=n)
    qrows = np.sort(rng.choice(m + q, size=q, replace=False)).astype(np.int32)
    A = np.zeros((m + q, n))
    ub = np.zeros(m + q)
    lin = [i for i in range(m + q) if i not in set(qrows.tolist())]
    A[lin], ub[lin] = spec["A"], spec["ub"]
    A[qrows], ub[qrows] = qa, rng.uniform(0.5, 1.0, size=q)
    spec.update(id=f"random_qp_quad(n={n},m={m},q={q},instance={instance})", A=A, ub=ub, r=np.zeros(m + q),
                qrows=qrows, qP=qP)
    return spec


def known_answer_zoo_quadratic():
    """The SimpleOptimizationProblems.standardProblems members with a quadratic constraint."""
    return [rank_one_problem_sphere(10), jopt_p1(5), distance_from_origin(4, False), distance_from_origin(4, True)]


def known_answer_zoo():
    """The SimpleOptimizationProblems.standardProblems subset (:576-598) the linear engine covers."""
    return [joptP2(), rank_one_problem_simplex(10), probability_simplex_problem(10),
            min_dot_product(np.array([1.0, -2.0, 0.5, 3.0, -1.5])), norm_squared_with_free_variables(5)]


def objective_value(spec: Dict, x: np.ndarray) -> float:
    v = spec["r0"] + float(spec["a0"] @ x)
    if spec.get("P") is not None:
        v += float(x @ (spec["P"] @ x)) / 2
    return v
