"""CPU oracle for the barrier Newton-step path of spyqqqdia/cvx — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The shipped path (``cvx_amd`` + ``libcvxg.so``)
never calls into it and fails loudly when its HIP library is missing.

What it is
    A line-by-line numpy/scipy restatement of the reference's hot path (Scala 2.11 + Breeze 0.10):

    * barrier value / gradient / Hessian fold ........ BarrierSolver.scala:280-315
    * objective + linear constraint callbacks ......... QuadraticObjectiveFunction.scala:31-33,
                                                        LinearObjectiveFunction.scala:19-21,
                                                        LinearConstraint.scala:22-32
    * strict feasibility (C.isInSet) .................. Constraint.scala:23, ConstraintSet.scala:32-40,
                                                        ConvexSet.scala:63-72
    * Ruiz equilibration ............................. MatrixUtils.scala:240-268
    * regularized Cholesky ............................ MatrixUtils.scala:452-461 (+ Breeze `cholesky`)
    * forward / back substitution ..................... MatrixUtils.scala:383-430
    * triangularSolve (LAPACK dtrtrs) ................. MatrixUtils.scala:362-376
    * relativeSize / choleskySolve .................... MatrixUtils.scala:437-442, 468-516
    * symSolve / diagonalizationSolve (fallback) ...... MatrixUtils.scala:603-707, 734-751
    * KKTSystem.solve chain ........................... KKTSystem.scala:43-66, 99-246, 253-310
    * UnconstrainedSolver.solve (all quirks) .......... UnconstrainedSolver.scala:34-125
    * EqualityConstrainedSolver.solve ................. EqualityConstrainedSolver.scala:37-107
    * barrier t-loop .................................. BarrierSolver.scala:70-177 with
                                                        CvxUtils.scala:61-87, SolverParams.scala:35-46
    * phase-I feasibility (linear constraints) ........ ConstraintSet.scala:123-168, 326-395, 556-575,
                                                        Constraint.scala:64-89, EqualityConstraint.scala:84-100
    * sum-of-infeasibilities phase I ................. ConstraintSet.scala:233-275, 481-535,
                                                        Constraint.scala:101-159, EqualityConstraint.scala:50-55

Third-party arithmetic the reference reaches but does not vendor: Breeze 0.10 (`cholesky` = symmetry
check + LAPACK dpotrf('L'); `eigSym` = LAPACK dsyevr), netlib-java 1.1.2 `LAPACK.dtrtrs`.  They are
restated through scipy's LAPACK (the same routines; OpenBLAS 0.3.29 here), `numpy.linalg.eigh`
(dsyevd: same eigen-decomposition, possibly different eigenvector signs — the solve is invariant).

Pinning
    The reference cannot be compiled or run here (no JVM/sbt), and its tests hold no
    golden vectors.  This oracle is pinned by the reference's own KNOWN-ANSWER tests, replayed in
    ``tests/test_oracle_known_answers.py``: the analytic minimisers of
    SimpleOptimizationProblems.scala (joptP2, rankOneProblemSimplex, probabilitySimplexProblem,
    minDotProduct, normSquaredWithFreeVariables), the known-solution KKT systems of KktTest.scala:117-272,
    the LA known-solution tests of MatrixUtilsTests.scala:16-198 and the KL analytic optimum of
    OptimizationProblems.scala:136-141.  Per-Newton-step golden vectors (``tests/golden/``) are outputs
    of THIS restatement on seeded inputs (script: ``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import numpy as np
from scipy.linalg import lapack

# ----------------------------------------------------------------------------------------------
# Exceptions mirroring the reference's failure modes
# ----------------------------------------------------------------------------------------------


class LinSolveException(Exception):
    """LinSolveException.scala (thrown by choleskySolve / solveWithCholFactor residual checks)."""


class NotConvergedException(Exception):
    """breeze.linalg.NotConvergedException (dpotrf info>0, line-search failures)."""


class UnsolvableSystemException(Exception):
    """UnsolvableSystemException.scala (diagonalizationSolve)."""


class NotStrictlyFeasible(ValueError):
    """IllegalArgumentException thrown by the barrier oracles when d_i <= 0 (BarrierSolver.scala:284)."""


# ----------------------------------------------------------------------------------------------
# Parameters  (SolverParams.scala:24-46)
# ----------------------------------------------------------------------------------------------


@dataclass
class SolverParams:
    maxIter: int = 1000
    alpha: float = 0.04
    beta: float = 0.8
    tolSolver: float = 1e-8
    tolEqSolve: float = 1e-1
    tolFeas: float = 1e-7
    delta: float = 1e-6


def standard_params() -> SolverParams:
    return SolverParams()


# ----------------------------------------------------------------------------------------------
# Problem model (packing of the reference's callback objects)
# ----------------------------------------------------------------------------------------------


@dataclass
class Problem:
    """Quadratic (P given) or linear (P None) objective r0 + a0.x (+ x'Px/2) with linear
    inequalities r_i + a_i.x <= ub_i (rows of A in constraint LIST order) and optional Aeq x = beq.
    """

    a0: np.ndarray
    r0: float = 0.0
    P: Optional[np.ndarray] = None
    A: np.ndarray = None  # m x n, row i = a_i
    r: np.ndarray = None
    ub: np.ndarray = None
    Aeq: Optional[np.ndarray] = None
    beq: Optional[np.ndarray] = None
    # KL dual objective (Duality.objF over Dist_KL, Duality.scala:74-79): with B = kl_B (dualDim x n_outcomes),
    # w = a0 and R = kl_R:  f(z) = w.z + R.exp(-B'z),  grad = w - B(R o exp(-B'z)),  Hessian = B diag(y) B'.
    kl_B: Optional[np.ndarray] = None
    kl_R: Optional[np.ndarray] = None
    # QuadraticConstraint rows (QuadraticConstraint.scala:8-40): row qrows[k] of (A, r, ub) holds (a, r, ub) of
    # r + a'x + x'P_k x / 2 <= ub with P_k = qP[k]
    qrows: Optional[np.ndarray] = None
    qP: Optional[np.ndarray] = None
    # KL primal objective Dist_KL.objectiveFunction(klp_n) (Dist_KL.scala:223-239): f(x) = x . log(x klp_n),
    # gradient 1 + log x + log klp_n, Hessian diag(1/x); a0 / r0 / P unused (a0 = 0 only sizes the problem)
    klp_n: Optional[int] = None

    def quad_index(self, i: int) -> int:
        if self.qrows is None:
            return -1
        hit = np.nonzero(self.qrows == i)[0]
        return int(hit[0]) if hit.size else -1

    @property
    def n(self) -> int:
        return self.a0.shape[0]

    @property
    def m(self) -> int:
        return self.A.shape[0]


def kl_y(pb: Problem, z: np.ndarray) -> np.ndarray:
    """Dist_KL.scala:163,170 — y = vec_R :* exp(-mat_B.t * z)."""
    return pb.kl_R * np.exp(-(pb.kl_B.T @ z))


def objective_value(pb: Problem, x: np.ndarray) -> float:
    """QuadraticObjectiveFunction.scala:31 — r + (a dot x) + (x dot (P*x))/2;
    LinearObjectiveFunction.scala:19 — r + (a dot x);
    KL dual: -dualObjFAt(z) = (vec_w dot z) + (vec_R dot exp(-B'z)) (Dist_KL.scala:146-147, Duality.scala:76)."""
    if isinstance(pb, AffineView):
        return objective_value(pb.pb, pb.x_of(x))
    if pb.kl_B is not None:
        return float(np.dot(pb.a0, x)) + float(np.dot(pb.kl_R, np.exp(-(pb.kl_B.T @ x))))
    if pb.klp_n is not None:  # Dist_KL.scala:226 — x dot log(x*n.toDouble)
        return float(np.dot(x, np.log(x * float(pb.klp_n))))
    v = pb.r0 + float(np.dot(pb.a0, x))
    if pb.P is not None:
        v = v + float(np.dot(x, pb.P @ x)) / 2
    return v


def objective_gradient(pb: Problem, x: np.ndarray) -> np.ndarray:
    """QuadraticObjectiveFunction.scala:32 — a + P*x; LinearObjectiveFunction.scala:20 — a;
    KL dual: -gradientDualObjFAt(z) = vec_w - B*(vec_R :* exp(-B'z)) (Dist_KL.scala:152-153)."""
    if pb.kl_B is not None:
        return pb.a0 - pb.kl_B @ kl_y(pb, x)
    if pb.klp_n is not None:  # Dist_KL.scala:228-229 — DenseVector.tabulate(n)(j => 1+log(x(j))+log(n))
        return (1.0 + np.log(x)) + math.log(pb.klp_n)
    if pb.P is None:
        return pb.a0.copy()
    return pb.a0 + pb.P @ x


def objective_hessian(pb: Problem, x: Optional[np.ndarray] = None) -> np.ndarray:
    """QuadraticObjectiveFunction.scala:33 — P; LinearObjectiveFunction.scala:21 — zeros(n,n);
    KL dual: -hessianDualObjFAt(z) = (B diag(y)) B' with the i,j loop of Dist_KL.scala:158-165."""
    if pb.kl_B is not None:
        y = kl_y(pb, x)
        Bdy = pb.kl_B * y[None, :]
        return -(-(Bdy @ pb.kl_B.T))
    if pb.klp_n is not None:  # Dist_KL.scala:231-236 — diag(1.0/x(j))
        return np.diag(1.0 / x)
    if pb.P is None:
        return np.zeros((pb.n, pb.n))
    return pb.P


def constraint_value(pb: Problem, i: int, x: np.ndarray) -> float:
    """LinearConstraint.scala:22-24 — r + (a dot x); QuadraticConstraint.scala:30-32 — r + (a dot x) + (x dot (P*x))/2."""
    k = pb.quad_index(i)
    if k >= 0:
        return pb.r[i] + float(np.dot(pb.A[i], x)) + float(np.dot(x, pb.qP[k] @ x)) / 2
    return pb.r[i] + float(np.dot(pb.A[i], x))


def constraint_gradient(pb: Problem, i: int, x: np.ndarray) -> np.ndarray:
    """LinearConstraint.gradientAt = a; QuadraticConstraint.gradientAt = a + P*x (QuadraticConstraint.scala:34-36)."""
    k = pb.quad_index(i)
    return pb.A[i] + pb.qP[k] @ x if k >= 0 else pb.A[i]


def constraint_hessian(pb: Problem, i: int) -> Optional[np.ndarray]:
    """QuadraticConstraint.hessianAt = P; None for a LinearConstraint (its zeros(n,n) adds exact zeros)."""
    k = pb.quad_index(i)
    return pb.qP[k] if k >= 0 else None


def is_satisfied_strictly(pb: Problem, i: int, x: np.ndarray) -> bool:
    """Constraint.scala:23 — valueAt(x)*(1+3e-16) < ub."""
    return constraint_value(pb, i, x) * (1 + 3e-16) < pb.ub[i]


def is_in_set(pb: Problem, x: np.ndarray) -> bool:
    """ConstraintSet.scala:34-38 via ConvexSet.scala:69 — short-circuit forall in list order."""
    if isinstance(pb, AffineView):  # ConvexSet.affineTransformed: isInSet(u) = C.isInSet(z0 + F u) (ConvexSet.scala:47-58)
        return is_in_set(pb.pb, pb.x_of(x))
    for i in range(pb.m):
        if not is_satisfied_strictly(pb, i, x):
            return False
    return True


def active_set(pb: Problem, x: np.ndarray, tol: float = 1e-12) -> np.ndarray:
    """Constraint.scala:26 isActive — |g_i(x) - ub_i| < tol (never called by the reference)."""
    g = np.array([constraint_value(pb, i, x) for i in range(pb.m)])
    return np.nonzero(np.abs(g - pb.ub) < tol)[0]


# ----------------------------------------------------------------------------------------------
# Barrier oracles (BarrierSolver.scala:280-315): left folds over the constraint list
# ----------------------------------------------------------------------------------------------


def barrier_value(pb: Problem, t: float, x: np.ndarray) -> float:
    """BarrierSolver.scala:280-289."""
    if isinstance(pb, AffineView):  # BarrierSolver.scala:226 — self.barrierFunction(t, z0 + F u)
        return barrier_value(pb.pb, t, pb.x_of(x))
    s = t * objective_value(pb, x)
    for i in range(pb.m):
        d = pb.ub[i] - constraint_value(pb, i, x)
        if d <= 0:
            raise NotStrictlyFeasible(f"barrierFunction: x not strictly feasible, d = {d}")
        s = s - math.log(d)
    return s


def barrier_gradient(pb: Problem, t: float, x: np.ndarray) -> np.ndarray:
    """BarrierSolver.scala:291-301 — fold starts at objF.gradientAt(x)*t, adds G/d."""
    if isinstance(pb, AffineView):  # BarrierSolver.scala:227-228 — F.t * self.gradientBarrierFunction(t, z0 + F u)
        return pb.F.T @ barrier_gradient(pb.pb, t, pb.x_of(x))
    s = objective_gradient(pb, x) * t
    for i in range(pb.m):
        d = pb.ub[i] - constraint_value(pb, i, x)
        if d <= 0:
            raise NotStrictlyFeasible(f"gradientBarrierFunction: x not strictly feasible, d = {d}")
        s = s + constraint_gradient(pb, i, x) / d
    return s


def barrier_hessian(pb: Problem, t: float, x: np.ndarray, literal: bool = True) -> np.ndarray:
    """BarrierSolver.scala:303-315 — fold starts at objF.hessianAt(x)*t and adds
    GGt/(d*d) + H/d per constraint, H = LinearConstraint.hessianAt = zeros(n,n) (LinearConstraint.scala:30-32).

    ``literal=True`` keeps every temporary of the reference (G*G.t, /(d*d), zeros, /d, two sums) —
    that is the CPU-baseline cost model.  ``literal=False`` drops only the +zeros/d term, which adds
    exact zeros (bit-identical result for d > 0), and updates a linear row's G*G.t/(d*d) only on the
    row's support: every entry outside it would receive (G_p G_q)/(d*d) = +-0.0, which leaves a finite
    sum bitwise unchanged (0.0 + -0.0 = 0.0), so the result is the dense fold's, bit for bit
    (``tests/test_oracle_known_answers.py::test_support_fold_is_the_dense_fold``).  It makes the fold
    O(sum of squared row supports): the KL primal's positivity rows and phase-I rows touch 1-2 entries.
    """
    if isinstance(pb, AffineView):  # BarrierSolver.scala:229-230 — (F.t * self.hessianBarrierFunction(t, z0 + F u)) * F
        return (pb.F.T @ barrier_hessian(pb.pb, t, pb.x_of(x), literal)) @ pb.F
    if literal == "blas":
        return _barrier_hessian_blas(pb, t, x)
    if literal is False:
        return _barrier_hessian_support(pb, t, x)
    literal = literal is True  # "dense": the literal=False fold over whole n x n outer products
    n = pb.n
    s = objective_hessian(pb, x) * t
    for i in range(pb.m):
        d = pb.ub[i] - constraint_value(pb, i, x)
        if d <= 0:
            raise NotStrictlyFeasible(f"hessianBarrierFunction: x not strictly feasible, d = {d}")
        G = constraint_gradient(pb, i, x)
        GGt = np.outer(G, G)
        Hq = constraint_hessian(pb, i)
        if Hq is not None:
            s = s + GGt / (d * d) + Hq / d
        elif literal:
            Hc = np.zeros((n, n))
            s = s + GGt / (d * d) + Hc / d
        else:
            s = s + GGt / (d * d)
    return s


def _barrier_hessian_support(pb: Problem, t: float, x: np.ndarray) -> np.ndarray:
    """barrier_hessian(literal=False) restricted to each linear row's support (see there): bitwise the same fold."""
    s = np.array(objective_hessian(pb, x) * t, dtype=np.float64, copy=True)
    for i in range(pb.m):
        d = pb.ub[i] - constraint_value(pb, i, x)
        if d <= 0:
            raise NotStrictlyFeasible(f"hessianBarrierFunction: x not strictly feasible, d = {d}")
        G = constraint_gradient(pb, i, x)
        Hq = constraint_hessian(pb, i)
        if Hq is not None:
            s = s + np.outer(G, G) / (d * d) + Hq / d
            continue
        sup = np.flatnonzero(G)
        if sup.size == 0:
            continue
        Gs = G[sup]
        blk = np.ix_(sup, sup)
        s[blk] = s[blk] + np.outer(Gs, Gs) / (d * d)
    return s


def _barrier_hessian_blas(pb: Problem, t: float, x: np.ndarray) -> np.ndarray:
    """The same sum as the fold above in BLAS order, t P + A' diag(1/d^2) A (one dgemm): for the C2/C3-size golden
    fixtures, where the per-constraint fold of n x n outer products would take minutes per Hessian.  Linear rows
    only; the two orders differ by rounding (~n u |H|)."""
    assert pb.qrows is None and pb.kl_B is None
    d = pb.ub - (pb.r + pb.A @ x)
    if np.any(d <= 0):
        raise NotStrictlyFeasible("hessianBarrierFunction: x not strictly feasible")
    W = pb.A / d[:, None]
    H = W.T @ W
    if pb.P is not None:
        H = H + pb.P * t
    return 0.5 * (H + H.T)


# ----------------------------------------------------------------------------------------------
# Affine re-parametrisation x = z0 + F u (BarrierSolver.affineTransformed / reduced)
# ----------------------------------------------------------------------------------------------


def solve_underdetermined(A: np.ndarray, b: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """MatrixUtils.solveUnderdetermined (MatrixUtils.scala:536-550), used by SolutionSpace (SolutionSpace.scala:20-27).

    Breeze ``qr(A.t)`` is LAPACK dgeqrf + dorgqr with the full n x n Q (restated by scipy's qr, the same routines):
    F = Q(::, p until n); y = forwardSolve(R.t, b) (only the leading p x p block of R.t is read); z0 = Q(::, 0 until p) y.
    """
    import scipy.linalg
    p, n = A.shape
    assert p == b.shape[0] and p < n
    Q, R = scipy.linalg.qr(A.T)
    F = Q[:, p:]
    y = forward_solve(np.ascontiguousarray(R.T[:, :p]), b)
    z0 = Q[:, :p] @ y
    return z0, F


def solution_space_parameter(z0: np.ndarray, F: np.ndarray, x0: np.ndarray) -> np.ndarray:
    """SolutionSpace.parameter (SolutionSpace.scala:29-33) — u0 = F.t * (x0 - z0)."""
    return F.T @ (x0 - z0)


class AffineView:
    """The solver returned by BarrierSolver.affineTransformed(z0, F, u0) (BarrierSolver.scala:209-232): a
    BarrierSolver in the variable u whose barrier value, gradient and Hessian are the original ones at
    x = z0 + F u (value; F.t * gradient; (F.t * H) * F), whose feasible set is the preimage of C
    (ConvexSet.scala:47-58) and whose equality constraint is (A F) u = b - A z0 (EqualityConstraint.scala:72-73).
    The oracle functions dispatch on this type, so the inner solvers run unchanged on it."""

    def __init__(self, pb: Problem, z0: np.ndarray, F: np.ndarray):
        self.pb, self.z0, self.F = pb, np.asarray(z0, dtype=np.float64), np.asarray(F, dtype=np.float64)
        self.Aeq = None if pb.Aeq is None else pb.Aeq @ self.F
        self.beq = None if pb.Aeq is None else pb.beq - pb.Aeq @ self.z0

    def x_of(self, u: np.ndarray) -> np.ndarray:
        return self.z0 + self.F @ u

    @property
    def n(self) -> int:
        return self.F.shape[1]

    @property
    def m(self) -> int:
        return self.pb.m


# ----------------------------------------------------------------------------------------------
# Dense linear algebra (MatrixUtils.scala)
# ----------------------------------------------------------------------------------------------


def ruiz_equilibrate(H: np.ndarray) -> Tuple[np.ndarray, np.ndarray, int]:
    """MatrixUtils.scala:240-268. Jacobi-style: every row of one sweep uses the Q computed at the top
    of the sweep; rho measured before the update; <=20 sweeps or rho<=1e-6; zero row -> scale 1.
    Returns (d, Q=(dd')oH, sweeps)."""
    n = H.shape[0]
    d = np.ones(n)
    rho = 1.0
    itermax = 20
    it = 0
    while it < itermax and rho > 1e-6:
        Q = np.outer(d, d) * H
        rho = 0.0
        for i in range(n):
            u = math.sqrt(float(np.linalg.norm(Q[i, :])))
            v = 1.0 / u if u > 0 else 1.0
            d[i] *= v
            r = abs(1 - u)
            if r > rho:
                rho = r
        it += 1
    return d, np.outer(d, d) * H, it


def _require_symmetric(X: np.ndarray, tol: float = 1e-7) -> None:
    """Breeze 0.10 requireSymmetricMatrix (un-vendored): |X_ij - X_ji| <= |X_ij|*tol."""
    diff = np.abs(X - X.T)
    if np.any(diff > np.abs(X) * tol):
        raise ValueError("MatrixNotSymmetricException")


def cholesky(X: np.ndarray) -> np.ndarray:
    """Breeze 0.10 `cholesky`: symmetry check, lowerTriangular copy, LAPACK dpotrf('L');
    info>0 -> NotConvergedException."""
    _require_symmetric(X)
    L, info = lapack.dpotrf(np.tril(X), lower=1, clean=1)
    if info > 0:
        raise NotConvergedException("dpotrf: not positive definite")
    return np.tril(L)


def regularized_cholesky(Q: np.ndarray) -> Tuple[np.ndarray, int]:
    """MatrixUtils.scala:452-461. Returns (L, regularized) where regularized = 1 when Q+1e-10*I was used."""
    Qd = Q + np.eye(Q.shape[0]) * 1e-10
    reg = 0
    try:
        C = cholesky(Q)
    except (NotConvergedException, ValueError):
        C = cholesky(Qd)
        reg = 1
    minD = float(np.min(np.diag(C)))
    if minD > 1e-7:
        return C, reg
    return cholesky(Qd), 1


def forward_solve(L: np.ndarray, b: np.ndarray) -> np.ndarray:
    """MatrixUtils.scala:383-403 — x_i = (b_i - sum_{j<i} L_ij x_j)/L_ii, j ascending."""
    n = L.shape[0]
    assert all(abs(L[i, i]) > 0 for i in range(n)), "Singular lower triangular matrix L"
    x = np.zeros(n)
    for i in range(n):
        s = 0.0
        row = L[i]
        for j in range(i):
            s += row[j] * x[j]
        x[i] = (b[i] - s) / L[i, i]
    return x


def back_solve(U: np.ndarray, b: np.ndarray) -> np.ndarray:
    """MatrixUtils.scala:410-430 — x_i = (b_i - sum_{j>i} U_ij x_j)/U_ii, j descending."""
    n = U.shape[0]
    assert all(abs(U[i, i]) > 0 for i in range(n)), "Singular upper triangular matrix U"
    x = np.zeros(n)
    for i in range(n - 1, -1, -1):
        s = 0.0
        row = U[i]
        for j in range(n - 1, i, -1):
            s += row[j] * x[j]
        x[i] = (b[i] - s) / U[i, i]
    return x


def triangular_solve(A: np.ndarray, ltype: str, B: np.ndarray) -> np.ndarray:
    """MatrixUtils.scala:362-376 — LAPACK dtrtrs(Ltype,'N','N') on the triangular copy."""
    assert ltype in ("L", "U")
    Q = np.tril(A) if ltype == "L" else np.triu(A)
    X, info = lapack.dtrtrs(Q, np.asarray(B, dtype=np.float64), lower=1 if ltype == "L" else 0,
                            trans=0, unitdiag=0)
    return X


def relative_size(a: np.ndarray, b: np.ndarray, tol: float) -> float:
    """MatrixUtils.scala:437-442."""
    norm_b = float(np.linalg.norm(b))
    f = tol if norm_b < tol else tol + norm_b
    return float(np.linalg.norm(a)) / f


@dataclass
class CholSolveInfo:
    d_ruiz: np.ndarray = None
    ruiz_sweeps: int = 0
    diagL: np.ndarray = None
    regularized: int = 0
    rel_err: float = float("nan")


def cholesky_solve(H: np.ndarray, b: np.ndarray, tol: float,
                   info: Optional[CholSolveInfo] = None, fast_subst: bool = False) -> np.ndarray:
    """MatrixUtils.scala:468-516: Ruiz -> regularizedCholesky -> w = fwd(L, d*b) -> u = back(L', w)
    -> x = d*u; LinSolveException when relativeSize(Hx-b, b, tol) > tol.
    ``fast_subst`` replaces the scalar substitutions by dtrtrs (same math, LAPACK order) for the
    large-size CPU baseline."""
    d, Q, sweeps = ruiz_equilibrate(H)
    L, reg = regularized_cholesky(Q)
    if fast_subst:
        w = triangular_solve(L, "L", (d * b)[:, None])[:, 0]
        u = triangular_solve(L.T, "U", w[:, None])[:, 0]
    else:
        w = forward_solve(L, d * b)
        u = back_solve(L.T, w)
    x = d * u
    rel = relative_size(H @ x - b, b, tol)
    if info is not None:
        info.d_ruiz, info.ruiz_sweeps, info.diagL, info.regularized, info.rel_err = (
            d, sweeps, np.diag(L).copy(), reg, rel)
    if rel > tol:
        raise LinSolveException(f"choleskySolve: ||Hx-b||/||b|| = {rel}")
    return x


def diagonalization_solve(A, U, dvals, V, b, tol) -> np.ndarray:
    """MatrixUtils.scala:603-707. Quirk: the regularisation loop shadows relError, so once the plain
    solution misses tol the routine always ends in UnsolvableSystemException."""
    n = U.shape[0]
    nz = np.abs(dvals) > 0
    a = np.where(nz, U.T @ b, 0.0)
    b0 = U @ a
    relDist = relative_size(b - b0, b, tol)
    if relDist > tol:
        raise UnsolvableSystemException(f"min_x||Ax-b||/||b|| = {relDist} > tol")
    z = np.where(nz, (U.T @ b) / np.where(nz, dvals, 1.0), 0.0)
    w = V @ z
    relError = relative_size(A @ w - b, b, tol)
    if relError > tol:
        raise UnsolvableSystemException("system not solvable within tolerance")
    return w


def sym_solve(A: np.ndarray, b: np.ndarray, tol: float) -> np.ndarray:
    """MatrixUtils.scala:734-751 — eigSym then diagonalizationSolve."""
    lam, evs = np.linalg.eigh(A)
    return diagonalization_solve(A, evs, lam, evs, b, tol)


# ----------------------------------------------------------------------------------------------
# KKT system (KKTSystem.scala)
# ----------------------------------------------------------------------------------------------


def kkt_solve_with_chol_factor(L, A, q, b, tol):
    """KKTSystem.scala:99-167."""
    n = L.shape[1]
    p = A.shape[0]
    B = np.zeros((n, p + 1))
    B[:, :p] = A.T
    B[:, p] = q
    Y = triangular_solve(L, "L", B)
    X = triangular_solve(L.T, "U", Y)
    Hinv_At = X[:, :p]
    Hinv_q = X[:, p]
    R = A @ Hinv_At
    S = (R + R.T) * 0.5
    K = cholesky(S)
    z = -(b + A @ Hinv_q)
    u = forward_solve(K, z)
    w = back_solve(K.T, u)
    x = -(Hinv_q + Hinv_At @ w)
    Ltx = L.T @ x
    Hx = L @ Ltx
    residual_1 = Hx + A.T @ w + q
    err1 = relative_size(residual_1, -q, tol)
    residual_2 = A @ x - b
    err2 = relative_size(residual_2, b, tol)
    if err1 > tol or err2 > tol:
        raise LinSolveException("Error in solution exceeds tolerance.")
    return x, w


def kkt_block_solve(H, A, q, b, tol):
    """KKTSystem.scala:178-190."""
    L, _ = regularized_cholesky(H)
    return kkt_solve_with_chol_factor(L, A, q, b, tol)


def kkt_solve_pd(H, A, q, b, tol):
    """KKTSystem.scala:200-246 — Ruiz, B = A diag(d), Dq = d*q, blockSolve, x = d*y."""
    d, Q, _ = ruiz_equilibrate(H)
    B = A * d[None, :]
    Dq = d * q
    y, w = kkt_block_solve(Q, B, Dq, b, tol)
    return d * y, w


def kkt_matrix(H, A):
    """KKTSystem.scala:253-260."""
    p = A.shape[0]
    return np.block([[H, A.T], [A, np.zeros((p, p))]])


def kkt_sym_solve(H, A, g, r, tol):
    """KKTSystem.scala:283-310."""
    n = H.shape[0]
    rhs = np.concatenate([-g, r])
    w = sym_solve(kkt_matrix(H, A), rhs, tol)
    return w[:n], w[n:]


def kkt_solve(H, A, q, b, tol, info: Optional[dict] = None):
    """KKTSystem.scala:43-66 — solvePD(H) -> solvePD(H+A'A, q-A'b) -> kktSymSolve."""
    try:
        res = kkt_solve_pd(H, A, q, b, tol)
        if info is not None:
            info["fallback"] = 0
        return res
    except Exception:
        try:
            K = H + A.T @ A
            z = q - A.T @ b
            res = kkt_solve_pd(K, A, z, b, tol)
            if info is not None:
                info["fallback"] = 1
            return res
        except Exception:
            res = kkt_sym_solve(H, A, q, b, tol)
            if info is not None:
                info["fallback"] = 2
            return res


# ----------------------------------------------------------------------------------------------
# Inner Newton solvers
# ----------------------------------------------------------------------------------------------


@dataclass
class NewtonStepRecord:
    """One inner Newton iteration as the GPU engine reports it (cvxg_step_info)."""

    x: np.ndarray
    grad: np.ndarray
    f: float
    dx: np.ndarray
    q: float
    newton_decrement: float
    step: float = float("nan")
    backtracks_c: int = 0
    backtracks_armijo: int = 0
    fallback: int = 0
    ruiz_sweeps: int = 0
    regularized: int = 0
    rel_err: float = float("nan")
    d_ruiz: Optional[np.ndarray] = None
    diagL: Optional[np.ndarray] = None
    it_n: int = 0                    # iteration within its centering
    radius: float = float("nan")     # trust radius frozen at iteration 0 of the centering


@dataclass
class Solution:
    """Solution.scala:32-43 (subset used by the barrier path)."""

    x: np.ndarray
    newtonDecrement: Optional[float] = None
    dualityGap: Optional[float] = None
    equalityGap: Optional[float] = None
    normGrad: Optional[float] = None
    iter: int = 0
    maxedOut: bool = False
    newton_steps: int = 0  # instrumentation: total inner Newton steps (the reference only keeps the last count)
    records: List[NewtonStepRecord] = field(default_factory=list)


def newton_direction(pb: Problem, t: float, x: np.ndarray, y: np.ndarray, tolEqSolve: float,
                     rec: Optional[NewtonStepRecord] = None, fast_subst: bool = False, hess="fold") -> np.ndarray:
    """UnconstrainedSolver.scala:50-67 — H at x, choleskySolve(H,-y) -> choleskySolve(H+1e-9 I,-y) -> symSolve.
    ``hess="blas"`` forms H in BLAS order (large golden fixtures only, see _barrier_hessian_blas)."""
    H = barrier_hessian(pb, t, x, literal="blas" if hess == "blas" else False)
    info = CholSolveInfo()
    fb = 0
    try:
        d = cholesky_solve(H, -y, tolEqSolve, info, fast_subst)
    except Exception:
        try:
            fb = 1
            M = H + np.eye(H.shape[0]) * 1e-9
            d = cholesky_solve(M, -y, tolEqSolve, info, fast_subst)
        except Exception:
            fb = 2
            d = sym_solve(H, -y, tolEqSolve)
    if rec is not None:
        rec.fallback, rec.ruiz_sweeps, rec.regularized, rec.rel_err = fb, info.ruiz_sweeps, info.regularized, info.rel_err
        rec.d_ruiz, rec.diagL = info.d_ruiz, info.diagL
    return d


def unconstrained_line_search(pb: Problem, t: float, x: np.ndarray, d: np.ndarray, q: float, f: float, it_n: int,
                              trustRadius: float, pars: SolverParams):
    """UnconstrainedSolver.scala:86-113: the trust-region scaling (radius frozen at iteration 0) and the two
    backtracking loops.  Returns (s, t_accepted, k1, it): the direction actually stepped along, the accepted step,
    the halvings into C and the shared counter."""
    alpha, beta = pars.alpha, pars.beta
    hNorm_d = math.sqrt(-q)
    s = d if (it_n == 0 or hNorm_d <= trustRadius) else d * (trustRadius / hNorm_d)
    it = 0
    st = 1.0
    while (not is_in_set(pb, x + s * st)) and it < 200:
        st *= beta
        it += 1
    if it == 100:
        raise NotConvergedException("Line search: backtracking into the set C failed.")
    k1 = it
    # trust-radius update: rho == 1 so both branches are no-ops (the f_new evaluation has no
    # observable effect when x+s is in C, and is skipped).
    while barrier_value(pb, t, x + s * st) > f + alpha * st * q and it < 200:
        st *= beta
        it += 1
    if it == 100:
        raise NotConvergedException("Line search: sufficient decrease not reached")
    return s, st, k1, it


def equality_line_search(pb: Problem, t: float, x: np.ndarray, d: np.ndarray, q: float, f: float,
                         pars: SolverParams):
    """EqualityConstrainedSolver.scala:78-97: no trust region, shared counter bound 100.  Returns (t_accepted, k1,
    it)."""
    alpha, beta = pars.alpha, pars.beta
    it = 0
    st = 1.0
    while (not is_in_set(pb, x + d * st)) and it < 100:
        st *= beta
        it += 1
    if it == 100:
        raise NotConvergedException("Line search: backtracking into the set C failed.")
    k1 = it
    while barrier_value(pb, t, x + d * st) > f + alpha * st * q and it < 100:
        st *= beta
        it += 1
    if it == 100:
        raise NotConvergedException("Line search: sufficient decrease not reached")
    return st, k1, it


def unconstrained_solve(pb: Problem, t: float, x0: np.ndarray, pars: SolverParams,
                        record: bool = False, max_steps: Optional[int] = None, hess="fold",
                        fast_subst: bool = False, on_step: Optional[Callable] = None) -> Solution:
    """UnconstrainedSolver.scala:34-125 with objF = the barrier objective at parameter t.

    Quirks reproduced: rho = 1+1/4 == 1 (integer), so the trust radius stays
    at |d_0|_H; steps longer than it are scaled; Armijo uses the UNSCALED q; both backtracking loops
    share `it` (bound 200) and only throw at it == 100; t *= beta repeatedly."""
    maxIter, alpha, beta, tol, tolEq = pars.maxIter, pars.alpha, pars.beta, pars.tolSolver, pars.tolEqSolve
    it_n = 0
    newtonDecrement = tol + 1
    x = x0.copy()
    y = barrier_gradient(pb, t, x)
    normGrad = float(np.linalg.norm(y))
    trustRadius = float("nan")
    records = []
    while it_n < maxIter and newtonDecrement > tol and normGrad > tol:
        if max_steps is not None and it_n >= max_steps:
            break
        f = barrier_value(pb, t, x)
        rec = NewtonStepRecord(x=x.copy(), grad=y.copy(), f=f, dx=None, q=0.0, newton_decrement=0.0)
        d = newton_direction(pb, t, x, y, tolEq, rec, fast_subst=fast_subst, hess=hess)
        q = float(np.dot(d, y))
        newtonDecrement = -q / 2
        rec.dx, rec.q, rec.newton_decrement = d.copy(), q, newtonDecrement
        rec.it_n = it_n
        if newtonDecrement > tol:
            hNorm_d = math.sqrt(-q)
            if it_n == 0:
                trustRadius = hNorm_d
            rec.radius = trustRadius
            s, st, k1, it = unconstrained_line_search(pb, t, x, d, q, f, it_n, trustRadius, pars)
            x = x + s * st
            y = barrier_gradient(pb, t, x)
            normGrad = float(np.linalg.norm(y))
            rec.step, rec.backtracks_c, rec.backtracks_armijo = st, k1, it - k1
        it_n += 1
        if record:
            records.append(rec)
        if on_step is not None:  # instrumentation (long golden runs): observe each finished step
            on_step(rec)
    return Solution(x=x, newtonDecrement=newtonDecrement, normGrad=normGrad, iter=it_n,
                    maxedOut=it_n >= maxIter, newton_steps=it_n, records=records)


def equality_constrained_solve(pb: Problem, t: float, x0: np.ndarray, pars: SolverParams,
                               record: bool = False) -> Solution:
    """EqualityConstrainedSolver.scala:37-107 — KKT Newton step, no trust region, shared `it`
    bound 100 that throws at it == 100."""
    A, b = pb.Aeq, pb.beq
    maxIter, alpha, beta, tol, tolEq = pars.maxIter, pars.alpha, pars.beta, pars.tolSolver, pars.tolEqSolve
    it_n = 0
    newtonDecrement = tol + 1
    x = x0.copy()
    y = barrier_gradient(pb, t, x)
    normGrad = float(np.linalg.norm(y))
    eqDiff = b - A @ x
    records = []
    while it_n < maxIter and ((newtonDecrement > tol and normGrad > tol) or float(np.linalg.norm(eqDiff)) > tol):
        f = barrier_value(pb, t, x)
        H = barrier_hessian(pb, t, x, literal=False)
        info = {}
        d, _w = kkt_solve(H, A, y, eqDiff, tolEq, info)
        q = float(np.dot(d, y))
        newtonDecrement = -q / 2
        rec = NewtonStepRecord(x=x.copy(), grad=y.copy(), f=f, dx=d.copy(), q=q,
                               newton_decrement=newtonDecrement, fallback=info.get("fallback", 0))
        if newtonDecrement > tol:
            st, k1, it = equality_line_search(pb, t, x, d, q, f, pars)
            x = x + d * st
            y = barrier_gradient(pb, t, x)
            normGrad = float(np.linalg.norm(y))
            eqDiff = b - A @ x
            rec.step, rec.backtracks_c, rec.backtracks_armijo = st, k1, it - k1
        it_n += 1
        if record:
            records.append(rec)
    return Solution(x=x, newtonDecrement=newtonDecrement, equalityGap=float(np.linalg.norm(eqDiff)),
                    normGrad=normGrad, iter=it_n, maxedOut=it_n >= maxIter, newton_steps=it_n,
                    records=records)


# ----------------------------------------------------------------------------------------------
# Barrier t-loop (BarrierSolver.scala:70-177)
# ----------------------------------------------------------------------------------------------


def standard_termination(pars: SolverParams) -> Callable[[dict], bool]:
    """CvxUtils.scala:61-70."""
    def tc(state):
        return state["dualityGap"] < pars.tolSolver and (
            state.get("equalityGap") is None or state["equalityGap"] < pars.tolSolver)
    return tc


def phase_I_termination(state) -> bool:
    """CvxUtils.scala:78-87."""
    return state["objectiveFunctionValue"] < 0 and (
        state.get("equalityGap") is None or state["equalityGap"] < 1e-6)


def barrier_solve(pb: Problem, x0: np.ndarray, pars: SolverParams,
                  tc: Optional[Callable[[dict], bool]] = None, record: bool = False) -> Solution:
    """BarrierSolver.scala:70-117 (no equalities) and :124-177 (with equalities)."""
    if tc is None:
        tc = standard_termination(pars)
    withEqs = pb.Aeq is not None
    mu = 10.0
    t = 1.0
    x = x0.copy()
    state = {"dualityGap": float("inf"), "equalityGap": float("inf") if withEqs else None,
             "objectiveFunctionValue": float("inf")}
    sol = None
    maxIter = 1000 / mu
    it = 0
    total = 0
    records: List[NewtonStepRecord] = []
    gaps = []
    while not tc(state) and it < maxIter:
        if withEqs:
            sol = equality_constrained_solve(pb, t, x, pars, record)
        else:
            sol = unconstrained_solve(pb, t, x, pars, record)
        total += sol.newton_steps
        for r_ in sol.records:
            r_.t = t
        records.extend(sol.records)
        x = sol.x
        f = objective_value(pb, x)
        gap = pb.m / t
        state = {"dualityGap": gap, "equalityGap": sol.equalityGap if withEqs else 0.0,
                 "objectiveFunctionValue": f}
        gaps.append(gap)
        t = mu * t
        it += 1
    return Solution(x=sol.x, newtonDecrement=sol.newtonDecrement, dualityGap=state["dualityGap"],
                    equalityGap=state["equalityGap"], normGrad=sol.normGrad, iter=sol.iter,
                    maxedOut=sol.maxedOut, newton_steps=total, records=records)


# ----------------------------------------------------------------------------------------------
# Phase I (basic method, linear constraints) — ConstraintSet.scala:123-168, 326-395
# ----------------------------------------------------------------------------------------------


def phase_I_problem(pb: Problem, x_where_defined: np.ndarray) -> Tuple[Problem, np.ndarray]:
    """phase_I_ObjectiveFunction (f(x,s)=s) + phase_I_Constraints_noEqs (g_j(x)-s <= ub_j) with the
    feasible point (x0, 1 + max_j(g_j(x0)-ub_j)) (ConstraintSet.scala:129-168; Constraint.scala:64-89)."""
    n, m = pb.n, pb.m
    A1 = np.hstack([pb.A, -np.ones((m, 1))])
    a0 = np.zeros(n + 1)
    a0[n] = 1.0
    y0 = max(constraint_value(pb, j, x_where_defined) - pb.ub[j] for j in range(m))
    fp = np.concatenate([x_where_defined, [1 + y0]])
    qP = None
    if pb.qrows is not None:  # hessianAt of the phase-I constraint: P in the x block, zero row/column for s
        qP = np.zeros((pb.qP.shape[0], n + 1, n + 1))
        qP[:, :n, :n] = pb.qP
    return Problem(a0=a0, r0=0.0, P=None, A=A1, r=pb.r.copy(), ub=pb.ub.copy(), qrows=pb.qrows, qP=qP), fp


def phase_I_analysis(pb: Problem, x_where_defined: np.ndarray, pars: SolverParams):
    """phase_I_Analysis (ConstraintSet.scala:404-413): with equalities the equalities are turned into
    +-1e-6 inequalities (:326-347, EqualityConstraint.scala:84-100), then :355-395.
    Returns (x_feas, s_feas)."""
    if pb.Aeq is not None:
        tolEqs = 1e-6
        rowsA, rowsr, rowsub = [pb.A], [pb.r], [pb.ub]
        for i in range(pb.Aeq.shape[0]):
            rowsA.append(pb.Aeq[i:i + 1]); rowsr.append(np.zeros(1)); rowsub.append(np.array([pb.beq[i] + tolEqs]))
            rowsA.append(-pb.Aeq[i:i + 1]); rowsr.append(np.zeros(1)); rowsub.append(np.array([-pb.beq[i] + tolEqs]))
        base = Problem(a0=pb.a0, A=np.vstack(rowsA), r=np.concatenate(rowsr), ub=np.concatenate(rowsub),
                       qrows=pb.qrows, qP=pb.qP)
    else:
        base = Problem(a0=pb.a0, A=pb.A, r=pb.r, ub=pb.ub, qrows=pb.qrows, qP=pb.qP)
    p1, fp = phase_I_problem(base, x_where_defined)
    sol = barrier_solve(p1, fp, pars, tc=phase_I_termination)
    n = pb.n
    return sol.x[:n], float(sol.x[n])


def phase_I_SOI_problem(pb: Problem, x_where_defined: np.ndarray) -> Tuple[Problem, np.ndarray]:
    """The sum-of-infeasibilities phase-I problem in u = (x, s_1..s_p), p = number of constraints:
    phase_I_SOI_ObjectiveFunction f(x, s) = sum(s) (ConstraintSet.scala:233-248); phase_I_SOI_Constraints
    (ConstraintSet.scala:258-275 -> Constraint.phase_I_SOI_Constraints, Constraint.scala:101-159): row j = g_j(x) - s_j
    <= ub_j (gradient (a_j, -e_j), a quadratic member's P in the x block), then the rows -s_j <= 0 in list order; the
    feasible point (x0, s_j = max(0.5, 1 + g_j(x0) - ub_j)); equalities [A | 0] (EqualityConstraint.scala:50-55)."""
    n, p = pb.n, pb.m
    A1 = np.zeros((2 * p, n + p))
    A1[:p, :n] = pb.A
    A1[np.arange(p), n + np.arange(p)] = -1.0
    A1[p + np.arange(p), n + np.arange(p)] = -1.0
    r1 = np.concatenate([pb.r, np.zeros(p)])
    ub1 = np.concatenate([pb.ub, np.zeros(p)])
    a0 = np.concatenate([np.zeros(n), np.ones(p)])
    s0 = np.array([max(0.5, 1 + constraint_value(pb, j, x_where_defined) - pb.ub[j]) for j in range(p)])
    u0 = np.concatenate([x_where_defined, s0])
    qP = None
    if pb.qrows is not None:
        qP = np.zeros((pb.qP.shape[0], n + p, n + p))
        qP[:, :n, :n] = pb.qP
    Aeq = None if pb.Aeq is None else np.hstack([pb.Aeq, np.zeros((pb.Aeq.shape[0], p))])
    return Problem(a0=a0, r0=0.0, P=None, A=A1, r=r1, ub=ub1, Aeq=Aeq, beq=pb.beq, qrows=pb.qrows, qP=qP), u0


def phase_I_analysis_soi(pb: Problem, x_where_defined: np.ndarray, pars: SolverParams):
    """phase_I_Analysis_SOI (ConstraintSet.scala:503-535): the SOI barrier solver (phase_I_Solver_SOI, :481-490)
    solved to the STANDARD termination (solver.solve), then x_feas = u[:n], s_feas = u[n:], the equality error
    |A x_feas - b| and isStrictlySatisfied = (0 until n).forall(j => s_feas(j) < 0) && eqError < tolSolver -- the
    reference's own expression (it ranges over n, not p; s_j > 0 keeps it false).  Returns (x_feas, s_feas,
    isStrictlySatisfied, eqError or None, the barrier Solution)."""
    pb1, u0 = phase_I_SOI_problem(pb, x_where_defined)
    sol = barrier_solve(pb1, u0, pars)
    n = pb.n
    x_feas, s_feas = sol.x[:n], sol.x[n:]
    eq_err = None if pb.Aeq is None else float(np.linalg.norm(pb.Aeq @ x_feas - pb.beq))
    strict = all(s_feas[j] < 0 for j in range(n)) and (0.0 if eq_err is None else eq_err) < pars.tolSolver
    return x_feas, s_feas, strict, eq_err, sol


def with_feasible_point(pb: Problem, x_where_defined: np.ndarray, pars: SolverParams) -> np.ndarray:
    """ConstraintSet.withFeasiblePoint (:556-575): phase I, then a strictly feasible x0."""
    x_feas, s_feas = phase_I_analysis(pb, x_where_defined, pars)
    tol = pars.tolSolver
    # FeasibilityReport.isFeasible(tol): s < tol (FeasibilityReport.scala)
    if not s_feas < tol:
        raise ValueError(f"InfeasibleProblemException: s = {s_feas}")
    if not is_in_set(pb, x_feas):
        raise ValueError("phase I point not strictly feasible")
    return x_feas


# ----------------------------------------------------------------------------------------------
# Kullback-Leibler distance minimisation via the dual barrier problem (Dist_KL.scala, Duality.scala)
# ----------------------------------------------------------------------------------------------

KL_E = 2.7182811828459045  # Dist_KL.scala:114 — NOT exp(1) = 2.718281828459045 (reference quirk, App. A 11)


def kl_dual_problem(n: int, H: Optional[np.ndarray], u: Optional[np.ndarray], A: Optional[np.ndarray],
                    r: Optional[np.ndarray]) -> Tuple[Problem, int]:
    """Duality.dualProblem (Duality.scala:99-112) for Dist_KL (Dist_KL.scala:104-165): variables
    z = (lambda, nu), dualDim = rows(H) + 1 + rows(A); objective -L_*(z); constraints lambda >= 0 as
    firstCoordinatesPositive (Constraints.scala:26-48: a = -e_j, r = 0, ub = 0).  B = (H; 1'; A),
    w = (u, 1, r), R_j = 1/(n e).  Returns (problem, numInequalities)."""
    rows_B = []
    w = []
    if H is not None:
        rows_B.append(np.asarray(H, dtype=np.float64))
        w.append(np.asarray(u, dtype=np.float64))
    rows_B.append(np.ones((1, n)))
    w.append(np.ones(1))
    if A is not None:
        rows_B.append(np.asarray(A, dtype=np.float64))
        w.append(np.asarray(r, dtype=np.float64))
    B = np.vstack(rows_B)
    wv = np.concatenate(w)
    k = B.shape[0]
    m = 0 if H is None else H.shape[0]
    Ac = np.zeros((max(m, 0), k))
    for j in range(m):
        Ac[j, j] = -1.0
    pb = Problem(a0=wv, r0=0.0, P=None, A=Ac, r=np.zeros(m), ub=np.zeros(m), kl_B=B,
                 kl_R=np.full(n, 1.0 / (n * KL_E)))
    return pb, m


def kl_solve_dual(n: int, H, u, A, r, pars: SolverParams, record: bool = False):
    """Duality.solveDual (Duality.scala:120-133): barrier solve of the dual from z0 = 0.001 (:106), then the
    primal optimum Q = vec_R :* exp(-B'z) (Dist_KL.scala:170)."""
    pb, m = kl_dual_problem(n, H, u, A, r)
    z0 = np.full(pb.n, 0.001)
    sol = barrier_solve(pb, z0, pars, record=record)
    Q = kl_y(pb, sol.x)
    return Q, sol, pb


def kl1_analytic_solution(n: int) -> np.ndarray:
    """OptimizationProblems.scala:136-141 (test fixture: the known minimiser of kl_1 / kl_1A)."""
    j = np.arange(n)
    if n <= 15:
        return np.where(j < n // 2, 1.8 / n, 0.2 / n)
    return np.where(j < 3, 0.12, np.where(j >= n // 2, 0.2 / n, 1.08 / (n - 6)))


def kl1A_data(n: int):
    """OptimizationProblems.scala:217-244: H = (-1_A; 1_B), u = (-0.36, 0.1), A = {0,1,2}, B = {n/2..n-1}."""
    IA = (np.arange(n) < 3).astype(np.float64)
    IB = (np.arange(n) >= n // 2).astype(np.float64)
    return np.vstack([-IA, IB]), np.array([-0.36, 0.1])


def kl2A_data(n: int):
    """OptimizationProblems.scala:341-370: equalities (1_A; 1_B) Q = (0.36, 0.1)."""
    IA = (np.arange(n) < 3).astype(np.float64)
    IB = (np.arange(n) >= n // 2).astype(np.float64)
    return np.vstack([IA, IB]), np.array([0.36, 0.1])


# ----------------------------------------------------------------------------------------------
# Primal-dual interior-point solver (PrimalDualSolver.scala, SymmetricLinearSystem.scala)
# ----------------------------------------------------------------------------------------------


class LineSearchFailedException(Exception):
    """LineSearchFailedException (PrimalDualSolver.scala:371, 540)."""


def check_symmetric(Q: np.ndarray, tol: float) -> bool:
    """MatrixUtils.scala:207-211 — Frobenius norm of Q - Q' below tol."""
    diff = Q - Q.T
    return math.sqrt(float(np.sum(diff * diff))) < tol


@dataclass
class PDStepRecord:
    """One primal-dual iteration (what the GPU engine reports in cvxg_pd_step_info)."""

    t: float
    x: np.ndarray
    lam: np.ndarray
    dx: np.ndarray = None
    dlam: np.ndarray = None
    s0: float = float("nan")
    step: float = float("nan")
    backtracks: int = 0
    fallback: int = 0          # 0 choleskySolve, 2 symSolve
    ruiz_sweeps: int = 0       # SymmetricLinearSystem's Ruiz (the inner choleskySolve runs its own)
    regularized: int = 0


@dataclass
class PDSolution:
    """Solution.scala as filled by PrimalDualSolver.solve_noEQs (:455-459)."""

    x: np.ndarray
    lam: np.ndarray
    dualityGap: float
    normDualResidual: float
    iter: int
    maxedOut: bool
    records: List[PDStepRecord] = field(default_factory=list)


def symmetric_linear_system_solve(H: np.ndarray, r: np.ndarray, tol: float,
                                  rec: Optional[PDStepRecord] = None) -> np.ndarray:
    """SymmetricLinearSystem.scala:15-56 — Ruiz once here (d, Q = (dd')oH, s = d o r), then
    checkSymmetric(Q, 1e-13) ? choleskySolve(Q, s) (which equilibrates Q AGAIN, MatrixUtils.scala:484) :
    svdSolve; any exception of choleskySolve -> symSolve(Q, s); x = d o u."""
    d, Q, sweeps = ruiz_equilibrate(H)
    s = d * r
    if not check_symmetric(Q, 1e-13):
        raise NotImplementedError("svdSolve branch (Q not symmetric): H is assembled exactly symmetric here")
    fb = 0
    info = CholSolveInfo()
    try:
        u = cholesky_solve(Q, s, tol, info)
    except Exception:
        fb = 2
        u = sym_solve(Q, s, tol)
    if rec is not None:
        rec.fallback, rec.ruiz_sweeps, rec.regularized = fb, sweeps, info.regularized
    return d * u


def pd_constraint_function(pb: Problem, x: np.ndarray) -> np.ndarray:
    """ConstraintSet.constraintFunctionAt: h_i = g_i(x) - ub_i."""
    return np.array([constraint_value(pb, i, x) - pb.ub[i] for i in range(pb.m)])


def pd_kkt_matrix(pb: Problem, x: np.ndarray, lam: np.ndarray) -> np.ndarray:
    """PrimalDualSolver.kktMatrix_noEqs (:216-240): hpd = objF.hessianAt(x); per constraint in list order
    hpd += grad2_gi*li - (G G')*(li/fi) (grad2_gi = zeros for a LinearConstraint)."""
    hpd = objective_hessian(pb, x).copy()
    for i in range(pb.m):
        li = lam[i]
        fi = constraint_value(pb, i, x) - pb.ub[i]
        assert fi < 0, "line search did not pull back into strictly feasible region"
        G = constraint_gradient(pb, i, x)
        Hq = constraint_hessian(pb, i)  # QuadraticConstraint.hessianAt = P; zeros for a LinearConstraint
        hpd = hpd + ((Hq if Hq is not None else np.zeros_like(hpd)) * li - np.outer(G, G) * (li / fi))
    return hpd


def pd_rhs1(pb: Problem, t: float, x: np.ndarray) -> np.ndarray:
    """PrimalDualSolver.rhs1 (:162-176): -grad f + sum_i grad g_i / (t f_i)."""
    res = -objective_gradient(pb, x)
    for i in range(pb.m):
        fx = constraint_value(pb, i, x) - pb.ub[i]
        res = res + constraint_gradient(pb, i, x) / (t * fx)
    return res


def pd_central_residual(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray) -> np.ndarray:
    """:97-106 — -lambda_i g_i - 1/t (g = constraintFunctionAt)."""
    g = pd_constraint_function(pb, x)
    return -lam * g - 1.0 / t


def pd_dual_residual(pb: Problem, x: np.ndarray, lam: np.ndarray) -> np.ndarray:
    """:63-71 — grad f + Dg' lambda (Dg = ConstraintSet.gradientMatrixAt, the gradients G_i(x) in rows)."""
    if pb.qrows is None:
        return objective_gradient(pb, x) + pb.A.T @ lam
    Dg = np.array([constraint_gradient(pb, i, x) for i in range(pb.m)])
    return objective_gradient(pb, x) + Dg.T @ lam


def pd_residual(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray) -> np.ndarray:
    """:123-130 — (r_dual, r_central)."""
    return np.concatenate([pd_dual_residual(pb, x, lam), pd_central_residual(pb, t, x, lam)])


def pd_delta_lambda(pb: Problem, t: float, x: np.ndarray, dx: np.ndarray, lam: np.ndarray) -> np.ndarray:
    """:184-209 — dlambda_i = (-lambda_i (Dg dx)_i + r_cent_i) / g_i."""
    r_cent = pd_central_residual(pb, t, x, lam)
    gx = pd_constraint_function(pb, x)
    assert np.all(gx < 0), "line search did not pull back into strictly feasible region"
    w = pb.A @ dx if pb.qrows is None else np.array([constraint_gradient(pb, i, x) @ dx for i in range(pb.m)])
    return (-lam * w + r_cent) / gx


def pd_direction(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray, tolEqSolve: float,
                 rec: Optional[PDStepRecord] = None) -> Tuple[np.ndarray, np.ndarray]:
    """One KKT solve of solve_noEQs (:421-425): kktSystem_noEqs + SymmetricLinearSystem.solve + deltaLambda."""
    H = pd_kkt_matrix(pb, x, lam)
    rhs = pd_rhs1(pb, t, x)
    dx = symmetric_linear_system_solve(H, rhs, tolEqSolve, rec)
    return dx, pd_delta_lambda(pb, t, x, dx, lam)


def pd_line_search(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray, dx: np.ndarray, dlam: np.ndarray,
                   pars: SolverParams, rec: Optional[PDStepRecord] = None):
    """lineSearch_noEQs (:311-374).  C.isInSet is the problem's domain (the whole space for the problems the
    engine accepts); maxIter = -30/log(beta) as a Double; throws when iter >= maxIter."""
    s0 = 1.0
    for i in range(lam.shape[0]):
        if dlam[i] < 0 and -lam[i] / dlam[i] < s0:
            s0 = -lam[i] / dlam[i]
    s = 0.99 * s0
    alpha, beta = pars.alpha, pars.beta
    r_t = pd_residual(pb, t, x, lam)
    x_s = x + dx * s
    lam_s = lam + dlam * s
    norm_rt = float(np.linalg.norm(r_t))
    norm_rts = float(np.linalg.norm(pd_residual(pb, t, x_s, lam_s)))
    feas = all(is_satisfied_strictly(pb, i, x_s) for i in range(pb.m))
    decreased = norm_rts < (1 - alpha * s) * norm_rt
    it = 0
    maxIter = -30 / math.log(beta)
    while not (feas and decreased) and it <= maxIter:
        s *= beta
        x_s = x + dx * s
        lam_s = lam + dlam * s
        norm_rts = float(np.linalg.norm(pd_residual(pb, t, x_s, lam_s)))
        feas = all(is_satisfied_strictly(pb, i, x_s) for i in range(pb.m))
        decreased = norm_rts < (1 - alpha * s) * norm_rt
        it += 1
    if it >= maxIter:
        raise LineSearchFailedException("Line search unsuccessful.")
    if rec is not None:
        rec.s0, rec.step, rec.backtracks = s0, s, it
    return x_s, lam_s


def pd_solve(pb: Problem, x0: np.ndarray, pars: SolverParams, record: bool = False) -> PDSolution:
    """PrimalDualSolver.solve (:628-633) -> solve_noEQs (:381-460): lambda0 = -1/h(x0)
    (ConstraintSet.lambda, ConstraintSet.scala:116-120), t = mu m / gap, stop when gap < tol and
    |r_dual| < tol (the state of the previous iteration), at most 2000/mu iterations."""
    if pb.Aeq is not None:
        raise NotImplementedError("solve_withEQs: see pd_solve_with_eqs")
    tol = pars.tolSolver
    mu = 10.0
    x = x0.copy()
    lam = -1.0 / pd_constraint_function(pb, x)
    gap = -float(np.dot(pd_constraint_function(pb, x), lam))
    normDual = float("inf")
    m = pb.m
    t = mu * m / gap
    maxIter = 2000 / mu
    it = 0
    records = []
    while not (gap < tol and normDual < tol) and it < maxIter:
        rec = PDStepRecord(t=t, x=x.copy(), lam=lam.copy())
        dx, dlam = pd_direction(pb, t, x, lam, pars.tolEqSolve, rec)
        rec.dx, rec.dlam = dx, dlam
        x, lam = pd_line_search(pb, t, x, lam, dx, dlam, pars, rec)
        gap = -float(np.dot(pd_constraint_function(pb, x), lam))
        normDual = float(np.linalg.norm(pd_dual_residual(pb, x, lam)))
        with np.errstate(divide="ignore"):
            t = float(np.float64(mu * m) / np.float64(gap))  # JVM Double semantics: x/0.0 = Infinity
        it += 1
        if record:
            records.append(rec)
    return PDSolution(x=x, lam=lam, dualityGap=gap, normDualResidual=normDual, iter=it - 1,
                      maxedOut=it == maxIter, records=records)


def pd_residual_eq(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray, nu: np.ndarray) -> np.ndarray:
    """residual_withEqs (:133-145) = (r_dual + A'nu (:76-90), r_central, A x - b (:111-120))."""
    A, b = pb.Aeq, pb.beq
    return np.concatenate([pd_dual_residual(pb, x, lam) + A.T @ nu, pd_central_residual(pb, t, x, lam), A @ x - b])


def pd_direction_eq(pb: Problem, t: float, x: np.ndarray, lam: np.ndarray, nu: np.ndarray, tolEqSolve: float,
                    info: Optional[dict] = None):
    """One KKT solve of solve_withEQs (:590-593): kktSystem_withEqs (:271-285) = KKTSystem(H_pd, A, q = rhs1 + A'nu,
    -(A x - b)), KKTSystem.solve (H dx + A'dnu = -q), then deltaLambda.  Returns (dx, dlambda, dnu)."""
    A, b = pb.Aeq, pb.beq
    H = pd_kkt_matrix(pb, x, lam)
    q = pd_rhs1(pb, t, x) + A.T @ nu
    dx, dnu = kkt_solve(H, A, q, -(A @ x - b), tolEqSolve, info)
    return dx, pd_delta_lambda(pb, t, x, dx, lam), dnu


def pd_solve_with_eqs(pb: Problem, x0: np.ndarray, pars: SolverParams, record: bool = False):
    """PrimalDualSolver.solve_withEQs (:550-621) as written: KKTSystem(H, A, q = rhs1 + A'nu, b = -(Ax - b))
    (:271-285, the reference's own 'FIX ME: check this!'); KKTSystem solves H dx + A' w = -q, the OPPOSITE sign
    of the no-equality system H dx = rhs1.  lineSearch_withEQs (:478-543) on the full residual
    (r_dual + A'nu, r_central, Ax - b); normDualResidual is the norm of that full residual; <= 1500/mu
    iterations.  Returns (x, lambda, nu, gap, normResidual, iter, maxedOut[, records]) or raises like the
    reference: LineSearchFailedException, with .records (record=True) and .state = (x, lambda, nu, gap,
    normResidual, equalityGap, completed iterations) of the last accepted iterate."""
    A, b = pb.Aeq, pb.beq
    tol, mu, m = pars.tolSolver, 10.0, pb.m
    x = x0.copy()
    lam = -1.0 / pd_constraint_function(pb, x)
    nu = np.zeros(A.shape[0])
    gap = -float(np.dot(pd_constraint_function(pb, x), lam))
    normRes = float("inf")
    eqGap = float("inf")
    t = mu * m / gap
    maxIter = 1500 / mu
    it = 0
    records = []
    while not (gap < tol and normRes < tol) and it < maxIter:
        info = {}
        dx, dlam, dnu = pd_direction_eq(pb, t, x, lam, nu, pars.tolEqSolve, info)
        rec = dict(t=t, x=x.copy(), lam=lam.copy(), nu=nu.copy(), dx=dx, dlam=dlam, dnu=dnu,
                   fallback=info.get("fallback", 0))
        s0 = 1.0
        for i in range(m):
            if dlam[i] < 0 and -lam[i] / dlam[i] < s0:
                s0 = -lam[i] / dlam[i]
        s = 0.99 * s0
        norm_rt = float(np.linalg.norm(pd_residual_eq(pb, t, x, lam, nu)))
        rec.update(s0=s0, norm_rt=norm_rt)

        def trial(s_):
            x_s, l_s, n_s = x + dx * s_, lam + dlam * s_, nu + dnu * s_
            ok = all(is_satisfied_strictly(pb, i, x_s) for i in range(m))
            dec = float(np.linalg.norm(pd_residual_eq(pb, t, x_s, l_s, n_s))) < (1 - pars.alpha * s_) * norm_rt
            return ok and dec, (x_s, l_s, n_s)

        good, u = trial(s)
        k = 0
        maxLS = -30 / math.log(pars.beta)
        while not good and k <= maxLS:
            s *= pars.beta
            good, u = trial(s)
            k += 1
        rec.update(step=s, backtracks=k)
        if record:
            records.append(rec)
        if k >= maxLS:
            e = LineSearchFailedException("Line search unsuccessful.")
            e.records = records
            e.state = (x, lam, nu, gap, normRes, eqGap, it)
            raise e
        x, lam, nu = u
        gap = -float(np.dot(pd_constraint_function(pb, x), lam))
        normRes = float(np.linalg.norm(pd_residual_eq(pb, t, x, lam, nu)))
        eqGap = float(np.linalg.norm(A @ x - b))
        with np.errstate(divide="ignore"):
            t = float(np.float64(mu * m) / np.float64(gap))
        it += 1
    if record:
        return x, lam, nu, gap, normRes, it - 1, it == maxIter, records
    return x, lam, nu, gap, normRes, it - 1, it == maxIter
