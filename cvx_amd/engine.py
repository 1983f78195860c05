"""Thin Python handle over one ``cvxg_ctx`` (one context per GPU; see include/cvxg.h)."""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib as L


class CvxgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{L.STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


class LinSolveException(CvxgError):
    """LinSolveException.scala"""


class NotConvergedException(CvxgError):
    """breeze NotConvergedException (cholesky / line search)"""


class NotStrictlyFeasible(CvxgError, ValueError):
    """IllegalArgumentException 'x not strictly feasible' (BarrierSolver.scala:285)"""


class UnsolvableSystemException(CvxgError):
    """UnsolvableSystemException.scala"""


_EXC = {L.CVXG_E_LINSOLVE_TOL: LinSolveException, L.CVXG_E_NOT_PD: NotConvergedException,
        L.CVXG_E_LINESEARCH: NotConvergedException, L.CVXG_E_INFEASIBLE_X: NotStrictlyFeasible,
        L.CVXG_E_UNSOLVABLE: UnsolvableSystemException}


def _dp(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def params_struct(pars) -> L.cvxg_params:
    return L.cvxg_params(int(pars.maxIter), float(pars.alpha), float(pars.beta), float(pars.tolSolver),
                         float(pars.tolEqSolve), float(pars.tolFeas), float(pars.delta))


class Engine:
    """One device context holding the packed problem (P, a, r; A, r_i, ub_i; A_eq, b_eq) and the iterate."""

    def __init__(self, n: int, m: int, p: int = 0, device: int = 0, **options):
        """options: cvxg_set_option settings applied right after creation (before any problem data), e.g.
        Engine(n, m, early_abort=0); see _lib.OPTIONS."""
        self.lib = L.lib()
        self.n, self.m, self.p = n, m, p
        h = C.c_void_p()
        rc = self.lib.cvxg_create(device, n, m, p, C.byref(h))
        self.h = h
        if rc != 0:
            msg = self.lib.cvxg_last_error(h).decode() if h.value else ""
            if h.value:
                self.lib.cvxg_destroy(h)
                self.h = C.c_void_p()
            raise CvxgError(rc, f"cvxg_create(n={n}, m={m}, p={p}) failed: {msg}")
        for name, value in options.items():
            self.set_option(name, value)

    def set_option(self, name: str, value: int):
        """cvxg_set_option (include/cvxg.h): name is a key of _lib.OPTIONS."""
        self._check(self.lib.cvxg_set_option(self.h, L.OPTIONS[name], int(value)))

    def close(self):
        if self.h is not None and self.h.value:
            self.lib.cvxg_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != 0:
            msg = self.lib.cvxg_last_error(self.h).decode()
            raise _EXC.get(rc, CvxgError)(rc, msg)

    # --- packing ---------------------------------------------------------------------------------
    def set_objective(self, a0, r0: float = 0.0, P=None):
        a0 = _f64(a0)
        if P is not None:
            P = _f64(P)
            self._check(self.lib.cvxg_set_objective(self.h, _dp(P), P.shape[1], _dp(a0), float(r0)))
        else:
            self._check(self.lib.cvxg_set_objective(self.h, None, 0, _dp(a0), float(r0)))
        self._keep_obj = (a0, P)

    def set_objective_kl(self, B, w, R: float):
        """KL dual objective of Duality.dualProblem over Dist_KL: B = mat_B (n x nout, row-major), w = vec_w,
        R = 1/(nout e) (cvxg_set_objective_kl)."""
        B, w = _f64(B), _f64(w)
        assert B.shape[0] == self.n and w.shape[0] == self.n
        self._check(self.lib.cvxg_set_objective_kl(self.h, _dp(B), B.shape[1], 1, B.shape[1], _dp(w), float(R)))
        self._keep_obj = (B, w)

    def set_objective_kl_primal(self, nout: int):
        """Dist_KL.objectiveFunction(nout): x . log(nout x) (cvxg_set_objective_kl_primal)."""
        self._check(self.lib.cvxg_set_objective_kl_primal(self.h, int(nout)))
        self._keep_obj = None

    def set_ineq(self, A, r, ub):
        A, r, ub = _f64(A), _f64(r), _f64(ub)
        self._check(self.lib.cvxg_set_ineq(self.h, _dp(A), A.shape[1] if A.ndim == 2 else self.n, 1, _dp(r), _dp(ub)))

    def set_quad(self, rows, P):
        """QuadraticConstraint rows (cvxg_set_quad): rows ascending indices into the set_ineq list, P (q, n, n)."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        P = _f64(np.asarray(P).reshape(len(rows), self.n, self.n)) if len(rows) else np.zeros((0, self.n, self.n))
        self._keep_quad = (rows, P)
        self._check(self.lib.cvxg_set_quad(self.h, len(rows), rows.ctypes.data_as(C.POINTER(C.c_int)), _dp(P),
                                           self.n))

    def set_eq(self, Aeq, beq):
        Aeq, beq = _f64(Aeq), _f64(beq)
        self._check(self.lib.cvxg_set_eq(self.h, _dp(Aeq), Aeq.shape[1], 1, _dp(beq)))

    def load_problem(self, spec: dict):
        if spec.get("kl_B") is not None:
            self.set_objective_kl(spec["kl_B"], spec["a0"], float(np.asarray(spec["kl_R"]).ravel()[0]))
        elif spec.get("klp_n") is not None:
            self.set_objective_kl_primal(int(np.asarray(spec["klp_n"]).ravel()[0]))
        else:
            self.set_objective(spec["a0"], spec.get("r0", 0.0), spec.get("P"))
        self.set_ineq(spec["A"], spec["r"], spec["ub"])
        if spec.get("qrows") is not None and len(spec["qrows"]) > 0:
            self.set_quad(spec["qrows"], spec["qP"])
        if self.p > 0:
            self.set_eq(spec["Aeq"], spec["beq"])

    def set_x(self, x):
        x = _f64(x)
        self._check(self.lib.cvxg_set_x(self.h, _dp(x)))

    def get_x(self) -> np.ndarray:
        x = np.zeros(self.n)
        self._check(self.lib.cvxg_get_x(self.h, _dp(x)))
        return x

    # --- affine re-parametrisation x = z0 + F u -------------------------------------------------------
    def affine_from(self, src: "Engine", z0, F):
        """Load src's problem pulled back to u (cvxg_affine_from; BarrierSolver.affineTransformed). F: n x k."""
        z0 = _f64(z0)
        Fc = np.ascontiguousarray(np.asarray(F, dtype=np.float64).T)  # column-major n x k = row-major k x n
        assert Fc.shape == (self.n, src.n) and z0.shape == (src.n,)
        self._check(self.lib.cvxg_affine_from(self.h, src.h, _dp(z0), _dp(Fc), src.n))
        self.n_x = src.n

    def affine_parameter(self, x0) -> np.ndarray:
        """SolutionSpace.parameter: u0 = F'(x0 - z0) (cvxg_affine_parameter)."""
        x0 = _f64(x0)
        u0 = np.zeros(self.n)
        self._check(self.lib.cvxg_affine_parameter(self.h, _dp(x0), _dp(u0)))
        return u0

    def affine_map(self, u=None) -> np.ndarray:
        """x = z0 + F u (cvxg_affine_map); u None = the current iterate."""
        x = np.zeros(self.n_x)
        self._check(self.lib.cvxg_affine_map(self.h, None if u is None else _dp(_f64(u)), _dp(x)))
        return x

    # --- oracles ---------------------------------------------------------------------------------
    def barrier_eval(self, t: float, x, want_grad=True, want_hess=False):
        x = _f64(x)
        f = C.c_double()
        g = np.zeros(self.n) if want_grad else None
        H = np.zeros((self.n, self.n)) if want_hess else None
        self._check(self.lib.cvxg_barrier_eval(self.h, float(t), _dp(x), C.byref(f), _dp(g), _dp(H)))
        return f.value, g, H

    def constraint_values(self, x) -> np.ndarray:
        x = _f64(x)
        g = np.zeros(self.m)
        self._check(self.lib.cvxg_constraint_values(self.h, _dp(x), _dp(g)))
        return g

    def active_set(self, x, tol: float = 1e-12) -> np.ndarray:
        x = _f64(x)
        idx = np.zeros(max(self.m, 1), dtype=np.int32)
        cnt = C.c_int()
        self._check(self.lib.cvxg_active_set(self.h, _dp(x), float(tol),
                                             idx.ctypes.data_as(C.POINTER(C.c_int)), C.byref(cnt)))
        return idx[:cnt.value].copy()

    # --- hot path --------------------------------------------------------------------------------
    def newton_direction(self, pars, t: float, x, grad=None):
        x = _f64(x)
        g = None if grad is None else _f64(grad)
        dx = np.zeros(self.n)
        w = np.zeros(max(self.p, 1))
        info = L.cvxg_step_info()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_newton_direction(self.h, C.byref(ps), float(t), _dp(x), _dp(g), _dp(dx), _dp(w),
                                                   C.byref(info)))
        return dx, w[:self.p], info

    def centering_begin(self, t: float):
        self._check(self.lib.cvxg_centering_begin(self.h, float(t)))

    def centering_resume(self, t: float, iter_: int, trust_radius: float = float("nan"), grad=None):
        """cvxg_centering_resume: the inner loop's state before iteration `iter_` (trust radius frozen at
        iteration 0; grad = the host's y, or None for the engine's own)."""
        g = None if grad is None else _f64(grad)
        self._check(self.lib.cvxg_centering_resume(self.h, float(t), int(iter_), float(trust_radius), _dp(g)))

    def newton_step(self, pars) -> L.cvxg_step_info:
        info = L.cvxg_step_info()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_newton_step(self.h, C.byref(ps), C.byref(info)))
        return info

    def centering(self, pars, t: float) -> L.cvxg_centering_info:
        info = L.cvxg_centering_info()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_centering(self.h, C.byref(ps), float(t), C.byref(info)))
        return info

    # --- primal-dual solver (PrimalDualSolver.scala) ------------------------------------------------
    def pd_direction(self, pars, t: float, x, lam):
        """(dx, dlambda, info) of one primal-dual KKT solve at (t, x, lambda) (cvxg_pd_direction)."""
        x, lam = _f64(x), _f64(lam)
        dx, dlam = np.zeros(self.n), np.zeros(self.m)
        info = L.cvxg_pd_step_info()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_pd_direction(self.h, C.byref(ps), float(t), _dp(x), _dp(lam), _dp(dx), _dp(dlam),
                                               C.byref(info)))
        return dx, dlam, info

    def pd_direction_eq(self, pars, t: float, x, lam, nu):
        """(dx, dlambda, dnu, info) of one solve_withEQs KKT solve at (t, x, lambda, nu) (cvxg_pd_direction_eq)."""
        x, lam, nu = _f64(x), _f64(lam), _f64(nu)
        dx, dlam, dnu = np.zeros(self.n), np.zeros(self.m), np.zeros(max(self.p, 1))
        info = L.cvxg_pd_step_info()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_pd_direction_eq(self.h, C.byref(ps), float(t), _dp(x), _dp(lam), _dp(nu), _dp(dx),
                                                  _dp(dlam), _dp(dnu), C.byref(info)))
        return dx, dlam, dnu[:self.p], info

    def pd_solve(self, pars, partial: bool = False):
        """cvxg_pd_solve.  partial=True returns (status, solution) instead of raising: the solution then describes
        the last accepted iterate (solve_withEQs fails in its line search like the reference)."""
        sol = L.cvxg_pd_solution()
        ps = params_struct(pars)
        rc = self.lib.cvxg_pd_solve(self.h, C.byref(ps), C.byref(sol))
        if partial:
            return rc, sol
        self._check(rc)
        return sol

    def get_lambda(self) -> np.ndarray:
        lam = np.zeros(self.m)
        self._check(self.lib.cvxg_get_lambda(self.h, _dp(lam)))
        return lam

    def get_nu(self) -> np.ndarray:
        nu = np.zeros(self.p)
        self._check(self.lib.cvxg_get_nu(self.h, _dp(nu)))
        return nu

    def barrier_solve(self, pars, termination: int = 0) -> L.cvxg_solution:
        sol = L.cvxg_solution()
        ps = params_struct(pars)
        self._check(self.lib.cvxg_barrier_solve(self.h, C.byref(ps), int(termination), C.byref(sol)))
        return sol

    def set_timing(self, on: bool, all_phases: bool = True):
        """cvxg_set_timing: all_phases=False records only the assembly and Cholesky phases (fewer event markers)."""
        self._check(self.lib.cvxg_set_timing(self.h, (1 if all_phases else 2) if on else 0))

    def ruiz_lookahead(self, sweeps: int = 0) -> int:
        """cvxg_set_ruiz_lookahead: the Ruiz sweeps the next Newton step launches (0 keeps the setting); returns how
        often a lookahead has fallen short on this context (the remaining sweeps and the factorization re-ran)."""
        n = C.c_longlong()
        self._check(self.lib.cvxg_set_ruiz_lookahead(self.h, int(sweeps), C.byref(n)))
        return n.value

    def last_error(self) -> str:
        """cvxg_last_error: the message of this context's last failing call."""
        return self.lib.cvxg_last_error(self.h).decode()

    def phase_times(self) -> np.ndarray:
        """cvxg_get_phase_times: per phase, the mean device time (ms) over the steps since set_timing(True) that
        recorded it (a per-occurrence mean: a phase not every step runs is not averaged over the steps)."""
        return self.phase_stats()[0]

    def phase_stats(self):
        """cvxg_get_phase_stats: (per-occurrence mean ms, occurrence count) per phase since set_timing(True)."""
        ms = np.zeros(8)
        cnt = (C.c_int * 8)()
        self._check(self.lib.cvxg_get_phase_stats(self.h, _dp(ms), cnt, 8))
        return ms, np.array(list(cnt), dtype=np.int64)

    def counters(self):
        """cvxg_get_counters: {ruiz_extensions, spec_pairs, spec_pairs_used, factor_attempts, regularized}."""
        out = (C.c_longlong * 5)()
        self._check(self.lib.cvxg_get_counters(self.h, out, 5))
        return dict(zip(("ruiz_extensions", "spec_pairs", "spec_pairs_used", "factor_attempts", "regularized"),
                        (int(v) for v in out)))


def batch_barrier_solve(engines, pars, termination: int = 0):
    """cvxg_batch_barrier_solve: the barrier solves of independent engines (one per GPU, config C5) concurrently from
    one process, one host thread per context.  Returns ([cvxg_solution], [status])."""
    lib = L.lib()
    k = len(engines)
    hs = (C.c_void_p * k)(*[e.h.value for e in engines])
    sols = (L.cvxg_solution * k)()
    st = (C.c_int * k)()
    ps = params_struct(pars)
    rc = lib.cvxg_batch_barrier_solve(k, hs, C.byref(ps), int(termination), sols, st)
    if rc == L.CVXG_E_ARG:  # rejected before any instance ran (NULL or repeated context)
        raise CvxgError(rc, "cvxg_batch_barrier_solve: NULL or repeated context")
    return list(sols), list(st)


def batch_newton_step(engines, pars):
    """cvxg_batch_newton_step: one inner Newton iteration on each engine concurrently.  Returns ([info], [status])."""
    lib = L.lib()
    k = len(engines)
    hs = (C.c_void_p * k)(*[e.h.value for e in engines])
    infos = (L.cvxg_step_info * k)()
    st = (C.c_int * k)()
    ps = params_struct(pars)
    rc = lib.cvxg_batch_newton_step(k, hs, C.byref(ps), infos, st)
    if rc == L.CVXG_E_ARG:
        raise CvxgError(rc, "cvxg_batch_newton_step: NULL or repeated context")
    return list(infos), list(st)


def solution_space(A, b, device: int = 0):
    """SolutionSpace(A, b) on the device (cvxg_solution_space; MatrixUtils.solveUnderdetermined): returns (z0, F)
    with F n x (n-p) column-orthonormal, A F = 0 and A z0 = b."""
    lib = L.lib()
    A, b = _f64(A), _f64(b)
    p, n = A.shape
    z0 = np.zeros(n)
    Fc = np.zeros((max(n - p, 0), n))  # column-major n x (n-p)
    rc = lib.cvxg_solution_space(device, p, n, _dp(A), n, 1, _dp(b), _dp(z0), _dp(Fc), n)
    if rc != 0:
        raise _EXC.get(rc, CvxgError)(rc, lib.cvxg_last_error(None).decode())
    return z0, Fc.T.copy()
