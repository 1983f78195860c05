"""Host-side mirror of the reference's problem-model API for the barrier path.

Same names, argument meaning and error behaviour as spyqqqdia/cvx, so a caller (and the parity tests)
read like the reference:

* ObjectiveFunction family ........ ObjectiveFunction.scala:8-14, QuadraticObjectiveFunction.scala:7-33,
                                    LinearObjectiveFunction.scala:7-21
* LinearConstraint ................ LinearConstraint.scala:7-32 (+ Constraint.scala:22-28 predicates)
* ConstraintSet / FeasiblePoint ... ConstraintSet.scala:8-120, 556-638; FeasiblePoint.scala:6-9
* EqualityConstraint .............. EqualityConstraint.scala:16-27, 84-100
* SolverParams / Solution ......... SolverParams.scala:24-46, Solution.scala:32-43
* BarrierSolver.apply ............. BarrierSolver.scala:269-317 — returns a GpuBarrierSolver whose inner
                                    loop runs on the MI355X engine (libcvxg.so) behind the C-ABI
* OptimizationProblem ............. OptimizationProblem.scala:133-196 (solverType "BR" = this engine)

Eligibility: quadratic or linear objective, linear (and quadratic) inequality constraints, optional
EqualityConstraint (any number of rows p < n).  Anything else raises TypeError — the reference's
CPU BarrierSolver remains the path for general callbacks.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .engine import CvxgError, Engine, NotConvergedException, NotStrictlyFeasible, solution_space

# ------------------------------------------------------------------------------------------------


@dataclass
class SolverParams:
    maxIter: int
    alpha: float
    beta: float
    tolSolver: float
    tolEqSolve: float
    tolFeas: float
    delta: float

    @staticmethod
    def standardParams() -> "SolverParams":
        return SolverParams(1000, 0.04, 0.8, 1e-8, 1e-1, 1e-7, 1e-6)


@dataclass
class Solution:
    x: np.ndarray
    newtonDecrement: Optional[float]
    dualityGap: Optional[float]
    equalityGap: Optional[float]
    normGrad: Optional[float]
    iter: int
    maxedOut: bool
    newtonSteps: int = 0
    outerIters: int = 0
    lambda_: Optional[np.ndarray] = None  # dual solutions (Duality.solveDual, Duality.scala:127-131; PD solver)
    nu: Optional[np.ndarray] = None
    normDualResidual: Optional[float] = None  # PrimalDualSolver (Solution.scala:24)


@dataclass
class OptimizationState:
    """OptimizationState.scala:22-29: what a termination criterion sees after each pass of the t-loop."""
    normGradient: Optional[float]
    newtonDecrement: Optional[float]
    dualityGap: Optional[float]
    equalityGap: Optional[float]
    objectiveFunctionValue: float
    normDualResidual: Optional[float] = None


class CvxUtils:
    """The termination criteria of CvxUtils.scala:61-87."""

    @staticmethod
    def standardTerminationCriterion(pars: "SolverParams"):
        def tc(st: OptimizationState) -> bool:
            assert st.dualityGap is not None, "Nonempty duality gap required, Solver should be Barrier or PrimalDual."
            return st.dualityGap < pars.tolSolver and (st.equalityGap is None or st.equalityGap < pars.tolSolver)
        return tc

    @staticmethod
    def phase_I_TerminationCriterion():
        def tc(st: OptimizationState) -> bool:
            assert st.dualityGap is not None, "Nonempty duality gap required, Solver should be Barrier or PrimalDual."
            return st.objectiveFunctionValue < 0 and (st.equalityGap is None or st.equalityGap < 1e-6)
        return tc


class FeasibilityReport:
    """FeasibilityReport.scala:12-40 (basic phase I: s has one entry)."""

    def __init__(self, x0, s, isStrictlySatisfied: bool, constraintSet, equalityConstraintError=None):
        self.x0 = np.asarray(x0, dtype=np.float64)
        self.s = np.atleast_1d(np.asarray(s, dtype=np.float64))
        self.isStrictlySatisfied = isStrictlySatisfied
        self.constraintSet = constraintSet
        self.equalityConstraintError = equalityConstraintError

    def violatedConstraints(self, tol: float):
        return [c for c in self.constraintSet.constraints if not c.isSatisfiedWithTolerance(self.x0, tol)]

    def isFeasible(self, tol: float) -> bool:
        return float(np.max(self.s)) < tol and (self.equalityConstraintError or 0.0) < tol


class InfeasibleProblemException(Exception):
    """InfeasibleProblemException.scala:6-7: phase I found no feasible point."""

    def __init__(self, report: FeasibilityReport, tol: float):
        super().__init__(f"No feasible point found: phase I ended with s = {report.s}, "
                         f"{len(report.violatedConstraints(tol))} constraint(s) violated at tolerance {tol}")
        self.report = report


class ObjectiveFunction:
    def __init__(self, dim: int):
        self.dim = dim

    def valueAt(self, x):
        raise NotImplementedError

    def gradientAt(self, x):
        raise NotImplementedError

    def hessianAt(self, x):
        raise NotImplementedError


class QuadraticObjectiveFunction(ObjectiveFunction):
    """f(x) = r + x'a + (1/2) x'Px."""

    def __init__(self, dim: int, r: float, a, P):
        super().__init__(dim)
        a = np.asarray(a, dtype=np.float64)
        P = np.asarray(P, dtype=np.float64)
        if a.shape != (dim,):
            raise ValueError(f"Vector a must be of dimension {dim} but length(a) {a.shape[0]}")
        if P.shape != (dim, dim):
            raise ValueError(f"Matrix P must be square of dimension {dim} but is {P.shape[0]}x{P.shape[1]}")
        self.r, self.a, self.P = float(r), a, P

    def valueAt(self, x):
        return self.r + float(self.a @ x) + float(x @ (self.P @ x)) / 2

    def gradientAt(self, x):
        return self.a + self.P @ x

    def hessianAt(self, x):
        return self.P


class LinearObjectiveFunction(ObjectiveFunction):
    """f(x) = r + a'x."""

    def __init__(self, dim: int, r: float, a):
        super().__init__(dim)
        a = np.asarray(a, dtype=np.float64)
        if a.shape != (dim,):
            raise ValueError(f"Vector a must be of dimension {dim} but length(a) {a.shape[0]}")
        self.r, self.a = float(r), a

    def valueAt(self, x):
        return self.r + float(self.a @ x)

    def gradientAt(self, x):
        return self.a

    def hessianAt(self, x):
        return np.zeros((self.dim, self.dim))


class DualKLObjectiveFunction(ObjectiveFunction):
    """Duality.objF over Dist_KL (Duality.scala:74-79, Dist_KL.scala:146-165): the convex form -L_*(z) of the
    KL dual, z = (lambda, nu).  B = mat_B (dualDim x n), w = vec_w, R = vec_R's constant 1/(n e)."""

    def __init__(self, B, w, R: float):
        self.B = np.asarray(B, dtype=np.float64)
        self.w = np.asarray(w, dtype=np.float64)
        self.R = float(R)
        super().__init__(self.B.shape[0])

    def _y(self, z):
        return self.R * np.exp(-(self.B.T @ np.asarray(z, dtype=np.float64)))

    def valueAt(self, z):
        return float(self.w @ z) + float(np.sum(self._y(z)))

    def gradientAt(self, z):
        return self.w - self.B @ self._y(z)

    def hessianAt(self, z):
        return (self.B * self._y(z)[None, :]) @ self.B.T


class KLPrimalObjectiveFunction(ObjectiveFunction):
    """Dist_KL.objectiveFunction(n) (Dist_KL.scala:223-239): the KL distance x . log(n x) from the uniform distribution
    on n outcomes; gradient (1 + log x) + log n, Hessian diag(1/x).  On the engine through
    cvxg_set_objective_kl_primal (barrier solver)."""

    def __init__(self, n: int):
        super().__init__(n)
        self.n = n

    def valueAt(self, x):
        x = np.asarray(x, dtype=np.float64)
        assert x.shape[0] == self.n, f"Dimension mismatch x.length = {x.shape[0]} dim(d_KL) = {self.n}"
        return float(x @ np.log(x * float(self.n)))

    def gradientAt(self, x):
        return (1.0 + np.log(x)) + np.log(self.n)

    def hessianAt(self, x):
        return np.diag(1.0 / np.asarray(x, dtype=np.float64))


class LinearConstraint:
    """Affine inequality r + a'x <= ub (LinearConstraint.scala:7-32)."""

    def __init__(self, id: str, dim: int, ub: float, r: float, a):
        a = np.asarray(a, dtype=np.float64)
        if a.shape != (dim,):
            raise ValueError(f"Vector a must be of dimension {dim} but length(a) {a.shape[0]}")
        self.id, self.dim, self.ub, self.r, self.a = id, dim, float(ub), float(r), a

    def valueAt(self, x):
        return self.r + float(self.a @ x)

    def gradientAt(self, x):
        return self.a

    def hessianAt(self, x):
        return np.zeros((self.dim, self.dim))

    def isSatisfied(self, x):
        return self.valueAt(x) <= self.ub

    def isSatisfiedStrictly(self, x):
        return self.valueAt(x) * (1 + 3e-16) < self.ub

    def isSatisfiedWithTolerance(self, x, tol: float):
        """Constraint.scala:24."""
        return self.valueAt(x) < self.ub + tol

    def isActive(self, x, tol: float = 1e-12):
        return abs(self.valueAt(x) - self.ub) < tol

    def margin(self, x):
        return self.ub - self.valueAt(x)


class QuadraticConstraint(LinearConstraint):
    """r + a'x + x'Px/2 <= ub (QuadraticConstraint.scala:8-63); P symmetric (checkSymmetric(P, 1e-13))."""

    def __init__(self, id: str, dim: int, ub: float, r: float, a, P):
        super().__init__(id, dim, ub, r, a)
        P = np.asarray(P, dtype=np.float64)
        if P.shape != (dim, dim):
            raise ValueError(f"Matrix P must be square of dimension {dim} but is {P.shape[0]}x{P.shape[1]}")
        if not np.sqrt(np.sum((P - P.T) ** 2)) < 1e-13:
            raise ValueError("QuadraticConstraint: P not symmetric")
        self.P = P

    def valueAt(self, x):
        return self.r + float(self.a @ x) + float(x @ (self.P @ x)) / 2

    def gradientAt(self, x):
        return self.a + self.P @ x

    def hessianAt(self, x):
        return self.P


class Constraints:
    """The constraint factories of Constraints.scala used by the reference's test problems."""

    @staticmethod
    def singleCoordinatePositive(n: int, j: int) -> LinearConstraint:
        """Constraints.scala:26-35: -x_j <= 0."""
        a = np.zeros(n)
        a[j] = -1.0
        return LinearConstraint(f"x_{j}>0", n, 0.0, 0.0, a)

    @staticmethod
    def allCoordinatesPositive(n: int) -> List[LinearConstraint]:
        return [Constraints.singleCoordinatePositive(n, j) for j in range(n)]

    @staticmethod
    def oneHalfNorm2BoundedBy(n: int, ub: float) -> QuadraticConstraint:
        """Constraints.scala:299-309: (x dot x)/2 <= ub (gradient x, Hessian I) — the QuadraticConstraint
        (r = 0, a = 0, P = I): (x dot (I x))/2 is the same number."""
        return QuadraticConstraint(f"x dot x <= {ub}", n, ub, 0.0, np.zeros(n), np.eye(n))


class EqualityConstraint:
    """Ax = b with A p x n, p < n (EqualityConstraint.scala:16-27)."""

    def __init__(self, A, b):
        A = np.atleast_2d(np.asarray(A, dtype=np.float64))
        b = np.asarray(b, dtype=np.float64).reshape(-1)
        assert A.shape[0] < A.shape[1], f"m=A.rows={A.shape[0]} is not less than n=A.cols={A.shape[1]}"
        assert A.shape[0] == b.shape[0], f"m=A.rows={A.shape[0]} != b.length = {b.shape[0]}"
        self.A, self.b, self.dim = A, b, A.shape[1]

    def errorAt(self, x):
        return float(np.linalg.norm(self.A @ x - self.b))

    def asInequalities(self, tol: float) -> List[LinearConstraint]:
        """EqualityConstraint.scala:84-100."""
        out = []
        for i in range(self.A.shape[0]):
            out.append(LinearConstraint(f"row_{i}(A)'x <= {self.b[i]}", self.dim, self.b[i] + tol, 0.0, self.A[i]))
            out.append(LinearConstraint(f"row_{i}(A)'x >= {self.b[i]}", self.dim, -self.b[i] + tol, 0.0, -self.A[i]))
        return out


class ConstraintSet:
    """ConstraintSet(dim, constraints) (ConstraintSet.scala:8); only LinearConstraint members are eligible."""

    def __init__(self, dim: int, constraints: Sequence[LinearConstraint], pointWhereDefined=None):
        assert all(c.dim == dim for c in constraints)
        self.dim = dim
        self.constraints = list(constraints)
        self.pointWhereDefined = (np.zeros(dim) if pointWhereDefined is None
                                  else np.asarray(pointWhereDefined, dtype=np.float64))
        self.feasiblePoint = None

    @property
    def numConstraints(self):
        return len(self.constraints)

    def packed(self):
        """(A, r, ub) with A row i = a_i in LIST order (fold and forall order)."""
        m = len(self.constraints)
        A = np.zeros((m, self.dim))
        r = np.zeros(m)
        ub = np.zeros(m)
        for i, c in enumerate(self.constraints):
            if not isinstance(c, LinearConstraint):
                raise TypeError("GPU barrier engine supports LinearConstraint only")
            A[i], r[i], ub[i] = c.a, c.r, c.ub
        return A, r, ub

    def quadratic(self):
        """(rows, P stack) of the QuadraticConstraint members in list order, or (None, None)."""
        rows = [i for i, c in enumerate(self.constraints) if isinstance(c, QuadraticConstraint)]
        if not rows:
            return None, None
        return np.array(rows, dtype=np.int32), np.stack([self.constraints[i].P for i in rows])

    def isSatisfiedStrictlyBy(self, x) -> bool:
        return all(c.isSatisfiedStrictly(x) for c in self.constraints)

    def constraintFunctionAt(self, x):
        return np.array([c.valueAt(x) - c.ub for c in self.constraints])

    def addFeasiblePoint(self, x0) -> "ConstraintSet":
        """ConstraintSet.scala:43-54."""
        x0 = np.asarray(x0, dtype=np.float64)
        assert x0.shape[0] == self.dim, "Feasible point does not have the right dimension"
        assert self.isSatisfiedStrictlyBy(x0)
        cs = ConstraintSet(self.dim, self.constraints, x0)
        cs.feasiblePoint = x0
        return cs

    # --- phase I on the same engine (ConstraintSet.scala:123-168, 326-395, 556-575) ------------------
    def phase_I_Analysis(self, eqs: Optional[EqualityConstraint], pars: SolverParams) -> FeasibilityReport:
        """phase_I_Analysis (ConstraintSet.scala:394-404): the basic phase-I barrier problem on the engine, with the
        equalities as inequalities of tolerance 1e-6 (phase_I_Analysis_withEqs, :324-347).  The phase-I objects are
        packed from this list (the Scala glue's GpuBarrierSolver.phaseI): rows (a_i, -1) (Constraint.phase_I,
        Constraint.scala:64-89), quadratic P_k padded with a zero row and column for s, objective f(x, s) = s
        (:129-141), feasible point (x0, 1 + max_j (g_j(x0) - ub_j)) (:161-164); solved under
        CvxUtils.phase_I_TerminationCriterion (:369-372)."""
        cnts = list(self.constraints)
        if eqs is not None:
            cnts = cnts + eqs.asInequalities(1e-6)
        cs = ConstraintSet(self.dim, cnts, self.pointWhereDefined)
        A, r, ub = cs.packed()
        m, n = A.shape
        x0 = self.pointWhereDefined
        A1 = np.hstack([A, -np.ones((m, 1))])
        a0 = np.zeros(n + 1)
        a0[n] = 1.0
        y0 = max(cnts[j].valueAt(x0) - ub[j] for j in range(m))
        fp = np.concatenate([x0, [1 + y0]])
        qrows, qP = cs.quadratic()
        eng = Engine(n + 1, m, 0)
        try:
            eng.set_objective(a0, 0.0, None)
            eng.set_ineq(A1, r, ub)
            if qrows is not None:
                qP1 = np.zeros((len(qrows), n + 1, n + 1))
                qP1[:, :n, :n] = qP
                eng.set_quad(qrows, qP1)
            sol = barrier_t_loop(eng, lambda w: float(w[n]), m, False, CvxUtils.phase_I_TerminationCriterion(), pars,
                                 fp)
        finally:
            eng.close()
        w = sol.x
        x_feas, s_feas = w[:n], float(w[n])
        return FeasibilityReport(x_feas, [s_feas], s_feas < 0.0, cs, 0.0)

    def phase_I_Analysis_SOI(self, eqs: Optional[EqualityConstraint], pars: SolverParams) -> FeasibilityReport:
        """phase_I_Analysis_SOI (ConstraintSet.scala:503-535), the sum-of-infeasibilities method on the engine:
        u = (x, s_1..s_p), objective sum(s) (phase_I_SOI_ObjectiveFunction, :233-248), rows (a_j, -e_j) with r_j, ub_j
        (Constraint.phase_I_SOI, Constraint.scala:101-123; a quadratic member's P padded with zeros for s) followed by
        the rows -s_j <= 0 (:147-158, sparse rows on the engine), feasible point (x0, max(0.5, 1 + g_j(x0) - ub_j))
        (:262-269), equalities [A | 0] (EqualityConstraint.phase_I_SOI_EqualityConstraint, :50-55); solved by
        BarrierSolver.solve, the standard termination (:481-490, 512).  The report keeps the reference's
        isStrictlySatisfied expression, (0 until n).forall(j => s_feas(j) < 0) && eqError < tolSolver."""
        A, r, ub = self.packed()
        p, n = A.shape
        x0 = self.pointWhereDefined
        A1 = np.zeros((2 * p, n + p))
        A1[:p, :n] = A
        A1[np.arange(p), n + np.arange(p)] = -1.0
        A1[p + np.arange(p), n + np.arange(p)] = -1.0
        a0 = np.concatenate([np.zeros(n), np.ones(p)])
        s0 = np.array([max(0.5, 1 + self.constraints[j].valueAt(x0) - self.constraints[j].ub) for j in range(p)])
        u0 = np.concatenate([x0, s0])
        qrows, qP = self.quadratic()
        neq = 0 if eqs is None else eqs.A.shape[0]
        eng = Engine(n + p, 2 * p, neq)
        try:
            eng.set_objective(a0, 0.0, None)
            eng.set_ineq(A1, np.concatenate([r, np.zeros(p)]), np.concatenate([ub, np.zeros(p)]))
            if qrows is not None:
                qP1 = np.zeros((len(qrows), n + p, n + p))
                qP1[:, :n, :n] = qP
                eng.set_quad(qrows, qP1)
            if neq:
                eng.set_eq(np.hstack([eqs.A, np.zeros((neq, p))]), eqs.b)
            sol = barrier_t_loop(eng, lambda u: float(np.sum(u[n:])), 2 * p, neq > 0,
                                 CvxUtils.standardTerminationCriterion(pars), pars, u0)
        finally:
            eng.close()
        w = sol.x
        x_feas, s_feas = w[:n], w[n:]
        eq_err = None if eqs is None else eqs.errorAt(x_feas)
        strict = all(s_feas[j] < 0 for j in range(n)) and (0.0 if eq_err is None else eq_err) < pars.tolSolver
        report = FeasibilityReport(x_feas, s_feas, strict, self, eq_err)
        report.solution = sol
        return report

    def withFeasiblePoint(self, eqs: Optional[EqualityConstraint], pars: SolverParams) -> "ConstraintSet":
        """ConstraintSet.scala:556-575: phase I, InfeasibleProblemException unless the report is feasible at
        pars.tolSolver."""
        if self.feasiblePoint is not None:
            return self
        report = self.phase_I_Analysis(eqs, pars)
        if not report.isFeasible(pars.tolSolver):
            raise InfeasibleProblemException(report, pars.tolSolver)
        return self.addFeasiblePoint(report.x0)


# ------------------------------------------------------------------------------------------------


_DOUBLE_MAX = 1.7976931348623157e308  # Double.MaxValue


def barrier_t_loop(engine: Engine, objF_value, m: int, with_eqs: bool, terminationCriterion, pars: SolverParams,
                   x0) -> Solution:
    """BarrierSolver.solveWithoutEQs / solveWithEQs (BarrierSolver.scala:70-177) on the host, exactly as the Scala glue
    runs it: t = 1, mu = 10, at most 1000/mu passes, the caller's termination criterion on the
    reference's OptimizationState; the inner solver of each pass (UnconstrainedSolver / EqualityConstrainedSolver
    .solve, :97-98, :154-155) is one cvxg_centering on the device-resident iterate."""
    mu = 10.0
    t = 1.0
    engine.set_x(x0)
    state = OptimizationState(None, None, _DOUBLE_MAX, _DOUBLE_MAX if with_eqs else None, _DOUBLE_MAX)
    it, total, ci, x = 0, 0, None, np.asarray(x0, dtype=np.float64)
    while not terminationCriterion(state) and it < 1000 / mu:
        ci = engine.centering(pars, t)
        total += ci.iter
        x = engine.get_x()
        state = OptimizationState(None, None, m / t, ci.equality_gap if with_eqs else 0.0, objF_value(x))
        t = mu * t
        it += 1
    if ci is None:  # the criterion held before the first pass: the reference would dereference a null Solution
        raise AssertionError("termination criterion satisfied before the first centering")
    return Solution(x, ci.newton_decrement, state.dualityGap, state.equalityGap if with_eqs else None, ci.norm_grad,
                    ci.iter, bool(ci.maxed_out), total, it)


class GpuBarrierSolver:
    """BarrierSolver with the inner Newton loop on the MI355X engine (BarrierSolver.scala:22-49, 269-317)."""

    def __init__(self, objF: ObjectiveFunction, cnts: ConstraintSet, eqs: Optional[EqualityConstraint],
                 pars: SolverParams, device: int = 0):
        if not isinstance(objF, (QuadraticObjectiveFunction, LinearObjectiveFunction, DualKLObjectiveFunction,
                                 KLPrimalObjectiveFunction)):
            raise TypeError("GPU barrier engine: objective must be Quadratic-, Linear-, DualKL- or "
                            "KLPrimalObjectiveFunction")
        if cnts.feasiblePoint is None:
            raise ValueError("ConstraintSet with FeasiblePoint required (use withFeasiblePoint)")
        p = 0 if eqs is None else eqs.A.shape[0]
        self.objF, self.cnts, self.eqs, self.pars = objF, cnts, eqs, pars
        self.device = device
        self.dim = cnts.dim
        self.startingPoint = cnts.feasiblePoint
        A, r, ub = cnts.packed()
        self.engine = Engine(cnts.dim, A.shape[0], p, device)
        if isinstance(objF, DualKLObjectiveFunction):
            self.engine.set_objective_kl(objF.B, objF.w, objF.R)
        elif isinstance(objF, KLPrimalObjectiveFunction):
            self.engine.set_objective_kl_primal(objF.n)
        else:
            self.engine.set_objective(objF.a, objF.r, getattr(objF, "P", None))
        self.engine.set_ineq(A, r, ub)
        qrows, qP = cnts.quadratic()
        if qrows is not None:
            self.engine.set_quad(qrows, qP)
        if p:
            self.engine.set_eq(eqs.A, eqs.b)

    @property
    def numConstraints(self):
        return self.cnts.numConstraints

    def barrierFunction(self, t, x):
        return self.engine.barrier_eval(t, x, want_grad=False)[0]

    def gradientBarrierFunction(self, t, x):
        return self.engine.barrier_eval(t, x, want_grad=True)[1]

    def hessianBarrierFunction(self, t, x):
        return self.engine.barrier_eval(t, x, want_grad=False, want_hess=True)[2]

    def solveSpecial(self, terminationCriterion, debugLevel: int = 0) -> Solution:
        """BarrierSolver.solveSpecial (BarrierSolver.scala:178-180) with any criterion (host t-loop)."""
        return barrier_t_loop(self.engine, self.objF.valueAt, self.numConstraints, self.eqs is not None,
                              terminationCriterion, self.pars, self.startingPoint)

    def solve(self, debugLevel: int = 0) -> Solution:
        """BarrierSolver.solve (BarrierSolver.scala:183-187): the standard criterion."""
        return self.solveSpecial(CvxUtils.standardTerminationCriterion(self.pars), debugLevel)

    # --- affine re-parametrisation (BarrierSolver.scala:191-256) -------------------------------------
    def affineTransformed(self, z0, F, u0=None) -> "AffineGpuBarrierSolver":
        """This solver in the variable u with x = z0 + F u; results are reported in u (BarrierSolver.scala:209-232).
        u0 None: u0 = F'(x0 - z0) on the device — svdSolve(F, x0 - z0) of :237-243 for an F with orthonormal
        columns (SolutionSpace's F); the reference's assertion |x0 - (z0 + F u0)| < tolEqSolve catches any other."""
        return AffineGpuBarrierSolver(self, z0, F, u0)

    def reduced(self, sol: "SolutionSpace") -> "AffineGpuBarrierSolver":
        """BarrierSolver.reduced (BarrierSolver.scala:249-256): affineTransformed(sol.z0, sol.F, sol.parameter(x0))."""
        return AffineGpuBarrierSolver(self, sol.z0, sol.F, None)


class AffineGpuBarrierSolver(GpuBarrierSolver):
    """The BarrierSolver returned by affineTransformed: the source problem pulled back to u on its own device context
    (cvxg_affine_from), so every Newton step runs in dimension F.cols on the engine's kernels."""

    def __init__(self, parent: GpuBarrierSolver, z0, F, u0=None):
        z0 = np.asarray(z0, dtype=np.float64)
        F = np.asarray(F, dtype=np.float64)
        if F.ndim != 2 or F.shape[0] != parent.dim or z0.shape != (parent.dim,):
            raise ValueError(f"affineTransformed: F must be {parent.dim} x k and z0 of length {parent.dim}")
        self.parent, self.z0, self.F = parent, z0, F
        self.objF, self.eqs, self.pars = parent.objF, parent.eqs, parent.pars
        self.cnts = parent.cnts
        self.dim = F.shape[1]
        p = 0 if parent.eqs is None else parent.eqs.A.shape[0]
        self.engine = Engine(self.dim, parent.engine.m, p, parent.device)
        self.engine.affine_from(parent.engine, z0, F)
        x0 = parent.startingPoint
        u0 = self.engine.affine_parameter(x0) if u0 is None else np.asarray(u0, dtype=np.float64)
        if not np.linalg.norm(x0 - self.engine.affine_map(u0)) < self.pars.tolEqSolve:  # BarrierSolver.scala:217-219
            raise AssertionError("u0 does not map to x0 under the variable transform.")
        self.startingPoint = u0

    def x_of(self, u) -> np.ndarray:
        """x = z0 + F u on the device (cvxg_affine_map)."""
        return self.engine.affine_map(u)

    def solveSpecial(self, terminationCriterion, debugLevel: int = 0) -> Solution:
        """The t-loop in u; the objective value is objF.affineTransformed(z0, F) (BarrierSolver.scala:221)."""
        return barrier_t_loop(self.engine, lambda u: self.objF.valueAt(self.z0 + self.F @ u), self.numConstraints,
                              self.eqs is not None, terminationCriterion, self.pars, self.startingPoint)


class SolutionSpace:
    """SolutionSpace(A, b) (SolutionSpace.scala:20-37): {x : Ax = b} = {z0 + F u}, F with orthonormal columns spanning
    ker A, z0 the minimum-norm solution — MatrixUtils.solveUnderdetermined's QR of A' on the device
    (cvxg_solution_space)."""

    def __init__(self, A, b, device: int = 0):
        A = np.asarray(A, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        assert A.shape[0] == b.shape[0]
        assert A.shape[0] < A.shape[1]
        self.A, self.b = A, b
        self.z0, self.F = solution_space(A, b, device)

    @staticmethod
    def apply(A, b, device: int = 0) -> "SolutionSpace":
        return SolutionSpace(A, b, device)


class BarrierSolver:
    @staticmethod
    def apply(objF, cnts, eqs, pars, device: int = 0) -> GpuBarrierSolver:
        return GpuBarrierSolver(objF, cnts, eqs, pars, device)


class LineSearchFailedException(NotConvergedException):
    """LineSearchFailedException (PrimalDualSolver.scala:369-372, 538-541): the residual line search did not
    terminate.  .solution holds the last accepted iterate."""

    def __init__(self, code: int, msg: str, solution: Optional[Solution] = None):
        super().__init__(code, msg)
        self.solution = solution


class GpuPrimalDualSolver:
    """PrimalDualSolver (PrimalDualSolver.scala:18-621) on the MI355X engine: each iteration's KKT matrix, its
    solve, dlambda and the residual line-search trials run on the device (cvxg_pd_solve).  Quadratic, linear or KL
    primal objective, LinearConstraint and QuadraticConstraint members; with equality constraints solve_withEQs as the
    reference writes it (its KKT right-hand side "FIX ME", :284), whose line search fails like the reference's
    (LineSearchFailedException, see include/cvxg.h)."""

    def __init__(self, objF: ObjectiveFunction, cnts: ConstraintSet, eqs: Optional[EqualityConstraint],
                 pars: SolverParams, device: int = 0):
        if not isinstance(objF, (QuadraticObjectiveFunction, LinearObjectiveFunction, KLPrimalObjectiveFunction)):
            raise TypeError("GPU primal-dual engine: objective must be Quadratic-, Linear- or KLPrimalObjectiveFunction")
        if cnts.feasiblePoint is None:
            raise ValueError("ConstraintSet with FeasiblePoint required (use withFeasiblePoint)")
        self.objF, self.cnts, self.eqs, self.pars = objF, cnts, eqs, pars
        self.device = device
        self.dim = cnts.dim
        self.startingPoint = cnts.feasiblePoint
        A, r, ub = cnts.packed()
        p = eqs.A.shape[0] if eqs is not None else 0
        self.engine = Engine(cnts.dim, A.shape[0], p, device)
        if isinstance(objF, KLPrimalObjectiveFunction):  # Dist_KL.objectiveFunction (Dist_KL.scala:223-239)
            self.engine.set_objective_kl_primal(objF.n)
        else:
            self.engine.set_objective(objF.a, objF.r, getattr(objF, "P", None))
        self.engine.set_ineq(A, r, ub)
        if eqs is not None:
            self.engine.set_eq(eqs.A, eqs.b)
        qrows, qP = cnts.quadratic()
        if qrows is not None:  # kktMatrix_noEqs adds grad2_gi * lambda_i (PrimalDualSolver.scala:224-238)
            self.engine.set_quad(qrows, qP)

    def solve(self, debugLevel: int = 0) -> Solution:
        """PrimalDualSolver.solve (:628-641): standard criterion gap < tol and |r| < tol; solve_noEQs or, with
        equality constraints, solve_withEQs (:550-621)."""
        self.engine.set_x(self.startingPoint)
        rc, s = self.engine.pd_solve(self.pars, partial=True)
        eqs = self.eqs is not None
        sol = Solution(self.engine.get_x(), None, s.duality_gap, s.equality_gap if eqs else None, None, s.iter,
                       bool(s.maxed_out), s.newton_steps, 0, lambda_=self.engine.get_lambda(),
                       nu=self.engine.get_nu() if eqs else None, normDualResidual=s.norm_dual_residual)
        if rc == _lib.CVXG_E_LINESEARCH:
            raise LineSearchFailedException(rc, self.engine.lib.cvxg_last_error(self.engine.h).decode(), sol)
        self.engine._check(rc)
        return sol


class PrimalDualSolver:
    @staticmethod
    def apply(objF, cnts, eqs, pars, device: int = 0) -> GpuPrimalDualSolver:
        """PrimalDualSolver.apply (PrimalDualSolver.scala:718-728)."""
        return GpuPrimalDualSolver(objF, cnts, eqs, pars, device)


class OptimizationProblem:
    def __init__(self, id: str, objectiveFunction, solver):
        self.id, self.objectiveFunction, self.solver = id, objectiveFunction, solver

    def solve(self, debugLevel: int = 0) -> Solution:
        return self.solver.solve(debugLevel)

    @staticmethod
    def apply(id, objF, ineqs: ConstraintSet, eqs, solverType: str, pars, device: int = 0):
        """OptimizationProblem.scala:133-157: solverType "BR" (barrier) or "PD" (primal-dual), both on the engine."""
        if solverType not in ("BR", "GPU", "PD"):
            raise ValueError(f"Unknown solverType = {solverType}")
        if solverType == "PD":
            return OptimizationProblem(id, objF, PrimalDualSolver.apply(objF, ineqs, eqs, pars, device))
        return OptimizationProblem(id, objF, BarrierSolver.apply(objF, ineqs, eqs, pars, device))

    @staticmethod
    def withoutFeasiblePoint(id, objF, ineqs: ConstraintSet, eqs, solverType: str, pars, device: int = 0):
        """OptimizationProblem.scala:174-196: phase I, then the barrier solver."""
        return OptimizationProblem.apply(id, objF, ineqs.withFeasiblePoint(eqs, pars), eqs, solverType, pars, device)


class Dist_KL(OptimizationProblem):
    """Dist_KL (Dist_KL.scala:68-177) with Duality (Duality.scala): argmin_Q dist_KL(Q, uniform) s.t. HQ <= u,
    AQ = r.  Both solves run on the MI355X engine: the direct one (solve: the barrier solver over the KL primal
    objective with the equalities, Dist_KL.scala:309-312) and the dual one (solveDual)."""

    E = 2.7182811828459045  # Dist_KL.scala:114 (reference constant, not exp(1))

    def __init__(self, id: str, n: int, H=None, u=None, A=None, r=None, device: int = 0):
        assert n > 0, f"n={n} is not positive."
        assert H is not None or A is not None, "Must have some inequality or equality constraints"
        assert (H is None) == (u is None) and (A is None) == (r is None)
        self.id, self.n, self.device = id, n, device
        self.H = None if H is None else np.asarray(H, dtype=np.float64)
        self.u = None if u is None else np.asarray(u, dtype=np.float64)
        self.A = None if A is None else np.asarray(A, dtype=np.float64)
        self.r = None if r is None else np.asarray(r, dtype=np.float64)
        self.numInequalities = 0 if self.H is None else self.H.shape[0]
        ones = np.ones((1, n))
        self.mat_B = np.vstack(([self.H] if self.H is not None else []) + [ones] + ([self.A] if self.A is not None else []))
        self.vec_w = np.concatenate(([self.u] if self.u is not None else []) + [np.ones(1)] +
                                    ([self.r] if self.r is not None else []))
        self.dualDim = self.mat_B.shape[0]
        self.R = 1.0 / (n * Dist_KL.E)
        super().__init__(id, None, None)

    @staticmethod
    def objectiveFunction(n: int) -> "KLPrimalObjectiveFunction":
        """Dist_KL.objectiveFunction (Dist_KL.scala:223-239): x . log(n x), on the engine's KL primal objective."""
        return KLPrimalObjectiveFunction(n)

    @staticmethod
    def equalityConstraint(n: int, A=None, r=None) -> EqualityConstraint:
        """Dist_KL.scala:245-256: E_Q[A] = r stacked above sum(Q) = 1 (EqualityConstraint.addEqualities)."""
        ones = np.ones((1, n))
        if A is None:
            return EqualityConstraint(ones, np.ones(1))
        return EqualityConstraint(np.vstack([np.atleast_2d(A), ones]),
                                  np.concatenate([np.asarray(r, dtype=np.float64).reshape(-1), np.ones(1)]))

    @staticmethod
    def apply(id, n, H, u, A, r, solverType: str = "BR", pars=None, device: int = 0) -> "Dist_KL":
        """Dist_KL.apply (Dist_KL.scala:270-315), including its construction-time phase I on the engine
        (ineqs.withFeasiblePoint(Some(eqs), ...), :303-307): the rows of H (ConstraintSet(H, u, C), ConstraintSet.scala:
        621-638) followed by x_j >= 0 for all j (Constraints.allCoordinatesPositive), the equalities A; 1' as
        inequalities of tolerance 1e-6, from x = 1/n; raises InfeasibleProblemException when phase I fails.  The
        solver itself then runs on the dual (solveDual); "PD" is accepted as in the reference, but the engine's
        primal-dual solver has no KL dual objective (dualProblem("PD") raises TypeError)."""
        if solverType not in ("BR", "PD", "GPU"):
            raise ValueError(f"Unknown solver: {solverType}")
        if H is None and A is None:
            raise ValueError("Must have some inequality or equality constraints")
        pars = pars or SolverParams.standardParams()
        eqs = Dist_KL.equalityConstraint(n, A, r)
        cnts = []
        if H is not None:
            Hm = np.atleast_2d(np.asarray(H, dtype=np.float64))
            uv = np.asarray(u, dtype=np.float64).reshape(-1)
            cnts += [LinearConstraint(f"row_{i}(H)x<=u({i})", n, uv[i], 0.0, Hm[i]) for i in range(Hm.shape[0])]
        cnts += Constraints.allCoordinatesPositive(n)
        ineqs = ConstraintSet(n, cnts, np.full(n, 1.0 / n))
        prob = Dist_KL(id, n, H, u, A, r, device)
        prob.ineqsWithFeasiblePoint = ineqs.withFeasiblePoint(eqs, pars)  # phase I
        prob.solverType = solverType
        prob.eqs, prob.pars = eqs, pars
        prob.objectiveFunction = Dist_KL.objectiveFunction(n)
        return prob

    def primalOptimum(self, z):
        """Dist_KL.scala:170: Q = vec_R :* exp(-mat_B.t * z)."""
        return self.R * np.exp(-(self.mat_B.T @ np.asarray(z, dtype=np.float64)))

    def dualProblem(self, solverType: str, pars: SolverParams) -> OptimizationProblem:
        """Duality.scala:99-112: min -L_*(z) s.t. lambda = z[:numInequalities] >= 0, from z0 = 0.001."""
        k = self.dualDim
        cnts = []
        for j in range(self.numInequalities):  # Constraints.firstCoordinatesPositive (Constraints.scala:26-48)
            a = np.zeros(k)
            a[j] = -1.0
            cnts.append(LinearConstraint(f"x_{j}>0", k, 0.0, 0.0, a))
        ineqs = ConstraintSet(k, cnts, np.zeros(k)).addFeasiblePoint(np.full(k, 0.001))
        objF = DualKLObjectiveFunction(self.mat_B, self.vec_w, self.R)
        if solverType == "PD":
            raise TypeError("GPU primal-dual engine: the KL dual objective is not supported (barrier solver only)")
        return OptimizationProblem.apply(self.id + " dual problem", objF, ineqs, None, solverType, pars, self.device)

    def solveDual(self, solverType: str = "BR", pars: Optional[SolverParams] = None) -> Solution:
        """Duality.scala:120-133: solve the dual, map z to the primal optimum."""
        pars = pars or SolverParams.standardParams()
        solD = self.dualProblem(solverType, pars).solve()
        z = solD.x
        solD.x = self.primalOptimum(z)
        solD.lambda_ = z[:self.numInequalities]
        solD.nu = z[self.numInequalities:] if self.dualDim > self.numInequalities else None
        return solD

    def solve(self, debugLevel: int = 0) -> Solution:
        """The direct solve (Dist_KL.scala:309-315) on the engine's KL primal objective: "BR" builds
        BarrierSolver(objF, ineqsWithFeasiblePoint, Some(eqs)), "PD" PrimalDualSolver(C, objF, ineqsWithFeasiblePoint,
        Some(eqs)), whose solve_withEQs raises LineSearchFailedException like the reference's (include/cvxg.h)."""
        if self.solver is None:
            build = PrimalDualSolver.apply if self.solverType == "PD" else BarrierSolver.apply
            self.solver = build(self.objectiveFunction, self.ineqsWithFeasiblePoint, self.eqs, self.pars, self.device)
        return self.solver.solve(debugLevel)


def problem_from_spec(spec: dict):
    """(objF, ConstraintSet, EqualityConstraint|None) from a cvx_amd.problems spec dict."""
    n = spec["a0"].shape[0]
    objF = (QuadraticObjectiveFunction(n, spec["r0"], spec["a0"], spec["P"]) if spec.get("P") is not None
            else LinearObjectiveFunction(n, spec["r0"], spec["a0"]))
    qrows = [] if spec.get("qrows") is None else [int(v) for v in spec["qrows"]]
    cnts = []
    for i in range(spec["A"].shape[0]):
        if i in qrows:
            cnts.append(QuadraticConstraint(f"QuadCnt{i}", n, spec["ub"][i], spec["r"][i], spec["A"][i],
                                            spec["qP"][qrows.index(i)]))
        else:
            cnts.append(LinearConstraint(f"LinCnt{i}", n, spec["ub"][i], spec["r"][i], spec["A"][i]))
    cs = ConstraintSet(n, cnts, spec.get("x_where_defined", spec.get("x0")))
    eqs = EqualityConstraint(spec["Aeq"], spec["beq"]) if spec.get("Aeq") is not None else None
    return objF, cs, eqs


__all__ = ["SolverParams", "Solution", "OptimizationState", "CvxUtils", "FeasibilityReport",
           "InfeasibleProblemException", "barrier_t_loop", "ObjectiveFunction", "QuadraticObjectiveFunction", "LinearObjectiveFunction",
           "DualKLObjectiveFunction", "KLPrimalObjectiveFunction", "Dist_KL",
           "LinearConstraint", "QuadraticConstraint", "Constraints", "EqualityConstraint", "ConstraintSet", "GpuBarrierSolver", "BarrierSolver",
           "GpuPrimalDualSolver", "PrimalDualSolver",
           "OptimizationProblem", "problem_from_spec", "CvxgError", "NotStrictlyFeasible", "LineSearchFailedException"]
