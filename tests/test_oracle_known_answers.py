"""Pin the CPU oracle against the reference's own known-answer tests (CPU only, no GPU).

The reference holds no golden vectors; what it does hold are known-answer tests:
MatrixUtilsTests.scala (Ruiz zero row, substitutions, dtrtrs, choleskySolve), KktTest.scala
(known-solution KKT systems) and the analytic minimisers of SimpleOptimizationProblems.scala.
Each test below replays one of them against oracle/cvx_oracle.py with a fixed seed (the reference's
own RNG is unseeded, so the random draws are ours; the checks are the reference's).
"""
import math

import numpy as np
import pytest

from oracle import cvx_oracle as O
from cvx_amd import problems as Z

RNG = lambda s: np.random.Generator(np.random.PCG64(1234 + s))  # noqa: E731


def _problem(spec):
    return O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"],
                     Aeq=spec.get("Aeq"), beq=spec.get("beq"))


# --- MatrixUtilsTests.scala -----------------------------------------------------------------------

def test_ruiz_zero_row():
    """MatrixUtilsTests.scala:16-26: equilibration of a matrix with a zero row. Analytic answer:
    rows 0 and 2 end with unit 2-norm, so d0 = d2 = 2^(1/4), d1 = 1 (zero row keeps scale 1)."""
    A = np.array([[0.5, 0.0, 0.5], [0.0, 0.0, 0.0], [-0.5, 0.0, -0.5]])
    d, Q, sweeps = O.ruiz_equilibrate(A)
    np.testing.assert_allclose(d, [2 ** 0.25, 1.0, 2 ** 0.25], rtol=1e-6)
    s = 1 / math.sqrt(2)
    np.testing.assert_allclose(Q, [[s, 0, s], [0, 0, 0], [-s, 0, -s]], atol=1e-6)
    assert sweeps <= 20


@pytest.mark.parametrize("dim", [5, 40])
def test_forward_back_solve_known_solution(dim):
    """MatrixUtilsTests.scala:107-158: U = triu(rand)+delta*I, b = U x0 -> x0."""
    rng = RNG(dim)
    x0 = rng.uniform(size=dim)
    U = np.triu(rng.uniform(size=(dim, dim))) + np.eye(dim) * 1.0
    np.testing.assert_allclose(O.back_solve(U, U @ x0), x0, rtol=1e-10)
    L = np.tril(rng.uniform(size=(dim, dim))) + np.eye(dim) * 1.0
    np.testing.assert_allclose(O.forward_solve(L, L @ x0), x0, rtol=1e-10)


def test_triangular_solve_known_solution():
    """MatrixUtilsTests.scala:36-93: H = KK', B = HX; two dtrtrs recover X (forward+backward error < tol)."""
    rng = RNG(7)
    n, p = 30, 4
    L = np.tril(rng.uniform(-5, 5, size=(n, n))) + np.eye(n) * 20.0
    X = rng.uniform(size=(n, p))
    B = (L @ L.T) @ X
    Y = O.triangular_solve(L, "L", B)
    X1 = O.triangular_solve(L.T, "U", Y)
    assert np.linalg.norm(X - X1) / np.linalg.norm(X) < 1e-10
    assert np.linalg.norm(B - (L @ L.T) @ X1) / np.linalg.norm(B) < 1e-10


@pytest.mark.parametrize("dim", [8, 30])
def test_cholesky_solve_known_solution(dim):
    """MatrixUtilsTests.scala:165-198: H = S+S', S = A'A, b = Hx, tolEqSolve = 1e-8."""
    rng = RNG(100 + dim)
    x = rng.uniform(size=dim)
    A = rng.uniform(size=(dim, dim))
    S = A.T @ A
    H = S + S.T
    info = O.CholSolveInfo()
    u = O.cholesky_solve(H, H @ x, 1e-8, info)
    assert np.linalg.norm(u - x) / np.linalg.norm(x) < 1e-6
    assert info.rel_err < 1e-8


def test_cholesky_solve_raises_on_indefinite():
    """choleskySolve -> LinSolveException / NotConverged on an indefinite matrix (MatrixUtils.scala:452-516)."""
    H = np.diag([1.0, -1.0, 2.0])
    with pytest.raises(Exception):
        O.cholesky_solve(H, np.ones(3), 1e-1)


def test_regularized_cholesky_small_pivot():
    """MatrixUtils.scala:452-461: min diag(L) <= 1e-7 -> refactor Q + 1e-10 I."""
    Q = np.diag([1.0, 1e-16, 1.0])
    L, reg = O.regularized_cholesky(Q)
    assert reg == 1
    np.testing.assert_allclose(np.diag(L) ** 2, [1.0, 1e-10 + 1e-16, 1.0], rtol=1e-6)


# --- KktTest.scala ---------------------------------------------------------------------------------

@pytest.mark.parametrize("n,p", [(10, 1), (25, 3), (40, 6)])
def test_kkt_with_chol_factor_known_solution(n, p):
    """KktTest.scala:117-184: L = tril(U(-5,5)) + sqrt(n) I, A = rand + I, q and b from known (x, w)."""
    rng = RNG(n * 10 + p)
    L = np.tril(rng.uniform(-5, 5, size=(n, n)))
    L[np.diag_indices(n)] += math.sqrt(n)
    A = rng.uniform(size=(p, n))
    A[np.arange(p), np.arange(p)] += 1.0
    x = rng.uniform(-1, 1, size=n)
    w = rng.uniform(-2, 2, size=p)
    H = L @ L.T
    q = -(H @ x + A.T @ w)
    b = A @ x
    x1, w1 = O.kkt_solve_with_chol_factor(L, A, q, b, O.standard_params().tolEqSolve)
    # KktTest.scala:134-146 passes when forward and backward relative errors are < tolEqSolve (0.1 in
    # Runner.scala:29); the random L has near-zero pivots by design, so we bound by conditioning instead.
    fwd = np.linalg.norm(-(H @ x1 + A.T @ w1) - q) / np.linalg.norm(q) + np.linalg.norm(A @ x1 - b) / np.linalg.norm(b)
    cond = np.linalg.cond(H)
    assert fwd < max(1e-10, cond * 1e-15)
    assert np.linalg.norm(x1 - x) / np.linalg.norm(x) < max(1e-10, cond * 1e-14)


@pytest.mark.parametrize("n,p", [(10, 1), (25, 3), (40, 6)])
def test_kkt_positive_definite_known_solution(n, p):
    """KktTest.scala:197-272: full KKTSystem.solve (Ruiz + solvePD chain) on H = (M+M')/2, M = LL'."""
    rng = RNG(n * 100 + p)
    L = np.tril(rng.uniform(-5, 5, size=(n, n)))
    L[np.diag_indices(n)] += math.sqrt(n)
    M = L @ L.T
    H = (M + M.T) * 0.5
    A = rng.uniform(-5, 5, size=(p, n))
    A[np.arange(p), np.arange(p)] += 20.0
    x = rng.uniform(-1, 1, size=n)
    w = rng.uniform(-2, 2, size=p)
    q = -(H @ x + A.T @ w)
    b = A @ x
    info = {}
    x1, w1 = O.kkt_solve(H, A, q, b, O.standard_params().tolEqSolve, info)
    assert info["fallback"] == 0
    assert np.linalg.norm(x1 - x) / np.linalg.norm(x) + np.linalg.norm(w1 - w) / np.linalg.norm(w) < 1e-6


# --- SimpleOptimizationProblems.scala (known minimisers; Runner tolSolution = 1e-2) ----------------

@pytest.mark.parametrize("spec", Z.known_answer_zoo(), ids=lambda s: s["id"])
def test_known_minimizers_barrier_with_phase_I(spec):
    """OptimizationProblem.withoutFeasiblePoint (OptimizationProblem.scala:174-196): phase I, then BR.
    KnownMinimizer.isMinimizer: |f(x) - f(x*)| < tol (KnownMinimizer.scala:59-63), tol = 1e-2 (Runner.scala:30);
    for the uniquely determined minimisers we also check |x - x*| (isEqualToSpecifiedMinimizer)."""
    pb = _problem(spec)
    pars = O.standard_params()
    x0 = O.with_feasible_point(pb, spec["x_where_defined"], pars)
    sol = O.barrier_solve(pb, x0, pars)
    fx = O.objective_value(pb, sol.x)
    fopt = O.objective_value(pb, spec["x_opt"])
    assert abs(fx - fopt) < 1e-2
    if spec["id"] != "Probability_simplex_problem":
        assert np.linalg.norm(sol.x - spec["x_opt"]) < 1e-2
    assert sol.dualityGap < pars.tolSolver


def test_barrier_path_random_qp_small():
    """Random dense QP (SURVEY.md §8d generator) at a small size: the barrier path terminates with gap<tol,
    the final point is strictly feasible and satisfies the KKT stationarity of the barrier problem."""
    spec = Z.random_qp(24, 48, instance=3)
    pb = _problem(spec)
    pars = O.standard_params()
    sol = O.barrier_solve(pb, spec["x0"], pars, record=True)
    assert sol.dualityGap < pars.tolSolver
    assert O.is_in_set(pb, sol.x)
    assert sol.newton_steps == len(sol.records) > 10


# ---- Dist_KL via the dual barrier problem (Dist_KL.scala, Duality.scala) --------------------------------

@pytest.mark.parametrize("n", [20, 2048])
def test_kl1A_dual_known_minimizer(n):
    """OptimizationProblems.kl_1A + MinimizationTests 'Solution via Duality with BarrierSolver': the primal
    optimum from the dual matches kl1_analyticSolution (reference tolerance 1e-2; the restatement reaches ~1e-9)."""
    H, u = O.kl1A_data(n)
    Q, sol, pb = O.kl_solve_dual(n, H, u, None, None, O.standard_params())
    assert pb.n == 3 and pb.m == 2
    assert np.max(np.abs(Q - O.kl1_analytic_solution(n))) < 1e-6
    assert abs(Q.sum() - 1.0) < 1e-8


@pytest.mark.parametrize("n", [20, 2048])
def test_kl2A_dual_known_minimizer(n):
    """OptimizationProblems.kl_2A: equality-only KL problem, dual has no inequalities (one centering)."""
    A, r = O.kl2A_data(n)
    Q, sol, pb = O.kl_solve_dual(n, None, None, A, r, O.standard_params())
    assert pb.m == 0
    assert np.max(np.abs(Q - O.kl1_analytic_solution(n))) < 1e-6


def test_kl_dual_oracles_are_consistent():
    """Gradient and Hessian of the KL dual objective against central differences."""
    rng = np.random.default_rng(4)
    n = 50
    H = rng.uniform(0, 1, size=(4, n))
    pb, m = O.kl_dual_problem(n, H, rng.uniform(0.3, 0.6, 4), None, None)
    z = rng.uniform(0.0, 0.5, pb.n)
    g = O.objective_gradient(pb, z)
    Hs = O.objective_hessian(pb, z)
    h = 1e-6
    for i in range(pb.n):
        e = np.zeros(pb.n)
        e[i] = h
        assert abs((O.objective_value(pb, z + e) - O.objective_value(pb, z - e)) / (2 * h) - g[i]) < 1e-7
        dg = (O.objective_gradient(pb, z + e) - O.objective_gradient(pb, z - e)) / (2 * h)
        assert np.max(np.abs(dg - Hs[:, i])) < 1e-7
    assert O.KL_E != np.e  # the reference's constant (Dist_KL.scala:114) is kept, not exp(1)


# ---- PrimalDualSolver (PrimalDualSolver.scala; Runner.scala:31 runs the known-answer problems with "PD") ------

@pytest.mark.parametrize("spec", [s for s in Z.known_answer_zoo() if s["Aeq"] is None and
                                  s["id"] != "normSquaredWithFreeVariables"], ids=lambda s: s["id"])
def test_known_minimizers_primal_dual_with_phase_I(spec):
    """OptimizationProblem.withoutFeasiblePoint(..., "PD"): phase I, then PrimalDualSolver.solve; the known
    minimiser within the Runner tolerance 1e-2, gap and dual residual below tolSolver.  (normSquaredWithFreeVariables
    is left out: its phase I is unbounded below in the slack and returns x_0 ~ -5e11, from which the primal-dual
    iteration leaves the strictly feasible region — kktMatrix_noEqs asserts.)"""
    pb = _problem(spec)
    pars = O.standard_params()
    x0 = O.with_feasible_point(pb, spec["x_where_defined"], pars)
    sol = O.pd_solve(pb, x0, pars)
    assert abs(O.objective_value(pb, sol.x) - O.objective_value(pb, spec["x_opt"])) < 1e-2
    if spec["id"] != "Probability_simplex_problem":
        assert np.linalg.norm(sol.x - spec["x_opt"]) < 1e-2
    assert sol.dualityGap < pars.tolSolver and sol.normDualResidual < pars.tolSolver
    assert np.all(sol.lam > 0)


def test_primal_dual_agrees_with_barrier_on_random_qp():
    """Both solvers of the reference reach the same minimiser of a random dense QP (strictly convex)."""
    spec = Z.random_qp(30, 60, instance=3)
    pb = _problem(spec)
    pars = O.standard_params()
    pd = O.pd_solve(pb, spec["x0"], pars, record=True)
    br = O.barrier_solve(pb, spec["x0"], pars)
    assert np.linalg.norm(pd.x - br.x) < 1e-7 * max(1.0, np.linalg.norm(br.x))
    assert pd.iter + 1 == len(pd.records) and not pd.maxedOut
    # KKT: lambda_i g_i(x) ~ -1/t at the end, and stationarity
    assert np.linalg.norm(O.pd_dual_residual(pb, pd.x, pd.lam)) < pars.tolSolver


@pytest.mark.parametrize("spec", [Z.joptP2(), Z.rank_one_problem_simplex(10)], ids=lambda s: s["id"])
def test_primal_dual_with_equalities_fails_like_the_reference(spec):
    """solve_withEQs as written passes q = rhs1 + A'nu to KKTSystem (H dx + A'dnu = -q): the opposite sign of the
    no-equality system (the reference marks it 'FIX ME', PrimalDualSolver.scala:284).  On the reference's own
    equality-constrained known-answer problems its line search fails; the engine does not build this path
    (CVXG_E_UNSUPPORTED)."""
    pb = _problem(spec)
    pars = O.standard_params()
    x0 = O.with_feasible_point(pb, spec["x_where_defined"], pars)
    with pytest.raises(O.LineSearchFailedException):
        O.pd_solve_with_eqs(pb, x0, pars)


@pytest.mark.parametrize("kind", ["kl_1", "kl_2"])
def test_primal_dual_with_equalities_on_the_kl_primal_fails_like_the_reference(kind):
    """Dist_KL with solverType "PD" (Dist_KL.scala:313-314, the reference Runner's configuration, Runner.scala:31, 48)
    runs solve_withEQs over the KL primal objective: its line search fails there too (a trial's log of a negative
    coordinate gives NaN, which no acceptance test passes)."""
    n = 20
    spec = Z.kl_primal_spec(n, kind)
    pb = O.Problem(a0=spec["a0"], r0=0.0, P=None, A=spec["A"], r=spec["r"], ub=spec["ub"], Aeq=spec["Aeq"],
                   beq=spec["beq"], klp_n=n)
    with np.errstate(invalid="ignore"), pytest.raises(O.LineSearchFailedException) as ei:
        O.pd_solve_with_eqs(pb, spec["x0"], O.standard_params(), record=True)
    assert ei.value.state[6] >= 1 and len(ei.value.records) == ei.value.state[6] + 1


# ---- QuadraticConstraint problems (SimpleOptimizationProblems.scala:266-300, 347-377, 464-561) ------------------

def _qproblem(spec):
    return O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"],
                     qrows=spec["qrows"], qP=spec["qP"])


@pytest.mark.parametrize("spec", Z.known_answer_zoo_quadratic(), ids=lambda s: s["id"])
def test_known_minimizers_quadratic_constraints(spec):
    """Phase I + BR on the reference's quadratic-constraint problems: the known minimiser within the Runner's
    tolerance (1e-2), duality gap below tolSolver."""
    pb = _qproblem(spec)
    pars = O.standard_params()
    x0 = O.with_feasible_point(pb, spec["x_where_defined"], pars)
    sol = O.barrier_solve(pb, x0, pars)
    assert abs(O.objective_value(pb, sol.x) - O.objective_value(pb, spec["x_opt"])) < 1e-2
    assert np.linalg.norm(sol.x - spec["x_opt"]) < 1e-2
    assert sol.dualityGap < pars.tolSolver


def test_quadratic_constraint_oracles_are_consistent():
    """The barrier gradient / Hessian with quadratic rows against central differences of the barrier value."""
    spec = Z.random_qp_quad(12, 20, 3, instance=2)
    pb = _qproblem(spec)
    x = 1e-3 * np.linspace(-1, 1, 12)
    t = 3.0
    g = O.barrier_gradient(pb, t, x)
    H = O.barrier_hessian(pb, t, x)
    h = 1e-6
    for i in range(12):
        e = np.zeros(12)
        e[i] = h
        assert abs((O.barrier_value(pb, t, x + e) - O.barrier_value(pb, t, x - e)) / (2 * h) - g[i]) < 1e-6
        dg = (O.barrier_gradient(pb, t, x + e) - O.barrier_gradient(pb, t, x - e)) / (2 * h)
        assert np.max(np.abs(dg - H[:, i])) < 1e-5 * max(1.0, np.max(np.abs(H)))


# ---- affine re-parametrisation x = z0 + F u (BarrierSolver.affineTransformed / reduced) -----------------------

@pytest.mark.parametrize("p,n", [(1, 10), (12, 30), (40, 64)])
def test_solution_space_properties(p, n):
    """SolutionSpace.scala:8-18 contract: A F = 0, F'F = I (orthonormal columns spanning ker A), A z0 = b, and z0 is
    the minimum-norm solution (orthogonal to ker A); parameter(x0) recovers u0 from x0 = z0 + F u0."""
    rng = RNG(500 + p)
    A = rng.uniform(-1, 1, size=(p, n))
    b = rng.uniform(-1, 1, size=p)
    z0, F = O.solve_underdetermined(A, b)
    assert F.shape == (n, n - p)
    assert np.abs(A @ F).max() < 1e-13
    assert np.abs(F.T @ F - np.eye(n - p)).max() < 1e-13
    assert np.abs(A @ z0 - b).max() < 1e-12
    assert np.abs(F.T @ z0).max() < 1e-12
    u0 = rng.uniform(-1, 1, size=n - p)
    np.testing.assert_allclose(O.solution_space_parameter(z0, F, z0 + F @ u0), u0, atol=1e-13)


@pytest.mark.parametrize("spec", [Z.rank_one_problem_simplex(10), Z.joptP2()], ids=lambda s: s["id"])
def test_reduced_barrier_known_minimizers(spec):
    """The known-answer simplex problems of SimpleOptimizationProblems.scala solved by dimension reduction
    (BarrierSolver.reduced over the sumToOne SolutionSpace, no equality constraint left): the reference's
    isMinimizer tolerance 1e-2 (Runner.scala:30), and the same optimum as the KKT (EqualityConstrainedSolver) path."""
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    z0, F = O.solve_underdetermined(spec["Aeq"], spec["beq"])
    n = spec["a0"].shape[0]
    x0 = np.full(n, 1.0 / n)  # strictly feasible point of the simplex
    view = O.AffineView(pb, z0, F)
    pars = O.standard_params()
    sol = O.barrier_solve(view, O.solution_space_parameter(z0, F, x0), pars)
    x = view.x_of(sol.x)
    assert abs(O.objective_value(pb, x) - O.objective_value(pb, spec["x_opt"])) < 1e-2
    assert np.linalg.norm(x - spec["x_opt"]) < 1e-2
    sol_kkt = O.barrier_solve(_problem(spec), x0, pars)
    assert np.linalg.norm(x - sol_kkt.x) < 1e-6


def test_reduced_barrier_matches_kkt_path_many_equalities():
    """p = 12 equality rows (more than the engine's on-device KKT Schur path takes): the reduced barrier solve
    reaches the optimum of the EqualityConstrainedSolver path, and the composed oracles are the transforms of the
    original ones (gradient F'g, Hessian (F'H)F)."""
    spec = Z.random_qp_eq(30, 60, 12, instance=1)
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    z0, F = O.solve_underdetermined(spec["Aeq"], spec["beq"])
    view = O.AffineView(pb, z0, F)
    u0 = O.solution_space_parameter(z0, F, spec["x0"])
    assert np.linalg.norm(view.x_of(u0) - spec["x0"]) < 1e-12
    x = spec["x0"]
    np.testing.assert_allclose(O.barrier_gradient(view, 3.0, u0), F.T @ O.barrier_gradient(pb, 3.0, x), rtol=1e-12)
    pars = O.standard_params()
    sol = O.barrier_solve(view, u0, pars)
    sol_kkt = O.barrier_solve(_problem(spec), spec["x0"], pars)
    assert sol.dualityGap < pars.tolSolver
    xr = view.x_of(sol.x)
    assert np.linalg.norm(xr - sol_kkt.x) / np.linalg.norm(sol_kkt.x) < 1e-8
    assert np.abs(spec["Aeq"] @ xr - spec["beq"]).max() < 1e-12


@pytest.mark.parametrize("case", ["kl_1", "kl_2", "qp", "phase_I", "quad"])
def test_support_fold_is_the_dense_fold(case):
    """The oracle's Hessian fold (BarrierSolver.scala:303-315) updates a linear row's G G'/(d d) only on the row's
    support: every other entry would receive +-0.0, which leaves the sum's bits unchanged.  Bitwise (as int64) the
    dense fold over whole n x n outer products, on the KL primal rows, a random QP, its phase-I problem (dense rows plus
    a -1 column) and a problem with QuadraticConstraint rows (dense update kept for those)."""
    if case in ("kl_1", "kl_2"):
        spec = Z.kl_primal_spec(40, case)
        pb = O.Problem(a0=spec["a0"], A=spec["A"], r=spec["r"], ub=spec["ub"], Aeq=spec["Aeq"], beq=spec["beq"],
                       klp_n=40)
        xs = [spec["x0"]]
    elif case == "quad":
        spec = Z.random_qp_quad(12, 20, 3, instance=5)
        pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"],
                       qrows=spec["qrows"], qP=spec["qP"])
        xs = [spec["x0"]]
    else:
        spec = Z.random_qp(30, 60, instance=3)
        pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
        xs = [spec["x0"]]
        if case == "phase_I":
            pb, fp = O.phase_I_problem(pb, np.zeros(30))
            xs = [fp]
    for x in xs:
        for t in (1.0, 1e4, 1e12):
            a = O.barrier_hessian(pb, t, x, literal=False)
            b = O.barrier_hessian(pb, t, x, literal="dense")
            assert np.array_equal(a.view(np.int64), b.view(np.int64)), (case, t)
