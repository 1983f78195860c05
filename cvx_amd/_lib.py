"""ctypes binding of ``libcvxg.so`` (the C-ABI declared in include/cvxg.h).

The HIP library is the product: there is no CPU fallback.  Importing this module on a machine without
the built library raises immediately; calling into it without a GPU returns CVXG_E_HIP.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CVXG_LIB", os.path.join(_HERE, "libcvxg.so"))  # override: experiment builds

CVXG_OK = 0
CVXG_E_NOT_PD = 1
CVXG_E_LINSOLVE_TOL = 2
CVXG_E_INFEASIBLE_X = 3
CVXG_E_LINESEARCH = 4
CVXG_E_UNSOLVABLE = 5
CVXG_E_DIM = 6
CVXG_E_HIP = 7
CVXG_E_ARG = 8
CVXG_E_UNSUPPORTED = 9
CVXG_MAX_EQ = 8

STATUS_NAMES = {
    0: "CVXG_OK", 1: "CVXG_E_NOT_PD", 2: "CVXG_E_LINSOLVE_TOL", 3: "CVXG_E_INFEASIBLE_X",
    4: "CVXG_E_LINESEARCH", 5: "CVXG_E_UNSOLVABLE", 6: "CVXG_E_DIM", 7: "CVXG_E_HIP", 8: "CVXG_E_ARG",
    9: "CVXG_E_UNSUPPORTED",
}


class cvxg_params(C.Structure):
    _fields_ = [("maxIter", C.c_int), ("alpha", C.c_double), ("beta", C.c_double), ("tolSolver", C.c_double),
                ("tolEqSolve", C.c_double), ("tolFeas", C.c_double), ("delta", C.c_double)]


class cvxg_step_info(C.Structure):
    _fields_ = [("t", C.c_double), ("f", C.c_double), ("norm_grad", C.c_double), ("q", C.c_double),
                ("newton_decrement", C.c_double), ("hnorm", C.c_double), ("trust_radius", C.c_double),
                ("step", C.c_double), ("rel_err", C.c_double), ("min_diag", C.c_double),
                ("norm_grad_new", C.c_double), ("equality_gap", C.c_double),
                ("backtracks_c", C.c_int), ("backtracks_armijo", C.c_int), ("fallback", C.c_int),
                ("ruiz_sweeps", C.c_int), ("regularized", C.c_int), ("took_step", C.c_int), ("done", C.c_int),
                ("iter", C.c_int), ("ls_fresh", C.c_int), ("ls_ties", C.c_int),
                ("small_pivot", C.c_int)]


class cvxg_centering_info(C.Structure):
    _fields_ = [("iter", C.c_int), ("maxed_out", C.c_int), ("newton_decrement", C.c_double),
                ("norm_grad", C.c_double), ("equality_gap", C.c_double)]


class cvxg_solution(C.Structure):
    _fields_ = [("duality_gap", C.c_double), ("equality_gap", C.c_double), ("newton_decrement", C.c_double),
                ("norm_grad", C.c_double), ("objective", C.c_double), ("iter", C.c_int), ("maxed_out", C.c_int),
                ("outer_iters", C.c_int), ("newton_steps", C.c_int)]


_P = C.c_void_p
class cvxg_pd_step_info(C.Structure):
    _fields_ = [("t", C.c_double), ("s0", C.c_double), ("step", C.c_double), ("norm_residual", C.c_double),
                ("rel_err", C.c_double), ("backtracks", C.c_int), ("fallback", C.c_int), ("ruiz_sweeps", C.c_int),
                ("regularized", C.c_int)]


class cvxg_pd_solution(C.Structure):
    _fields_ = [("duality_gap", C.c_double), ("norm_dual_residual", C.c_double), ("objective", C.c_double),
                ("iter", C.c_int), ("maxed_out", C.c_int), ("newton_steps", C.c_int), ("equality_gap", C.c_double)]


_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int)

# name -> (restype, argtypes)   (every symbol of include/cvxg.h)
SIGNATURES = {
    "cvxg_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "cvxg_destroy": (None, [_P]),
    "cvxg_last_error": (C.c_char_p, [_P]),
    "cvxg_version": (C.c_char_p, []),
    "cvxg_set_objective": (C.c_int, [_P, _D, C.c_int, _D, C.c_double]),
    "cvxg_set_objective_kl": (C.c_int, [_P, _D, C.c_int, C.c_int, C.c_int, _D, C.c_double]),
    "cvxg_set_objective_kl_primal": (C.c_int, [_P, C.c_int]),
    "cvxg_set_ineq": (C.c_int, [_P, _D, C.c_int, C.c_int, _D, _D]),
    "cvxg_set_eq": (C.c_int, [_P, _D, C.c_int, C.c_int, _D]),
    "cvxg_set_quad": (C.c_int, [_P, C.c_int, _I, _D, C.c_int]),
    "cvxg_set_x": (C.c_int, [_P, _D]),
    "cvxg_get_x": (C.c_int, [_P, _D]),
    "cvxg_barrier_eval": (C.c_int, [_P, C.c_double, _D, _D, _D, _D]),
    "cvxg_constraint_values": (C.c_int, [_P, _D, _D]),
    "cvxg_active_set": (C.c_int, [_P, _D, C.c_double, _I, _I]),
    "cvxg_newton_direction": (C.c_int, [_P, C.POINTER(cvxg_params), C.c_double, _D, _D, _D, _D,
                                        C.POINTER(cvxg_step_info)]),
    "cvxg_centering_begin": (C.c_int, [_P, C.c_double]),
    "cvxg_centering_resume": (C.c_int, [_P, C.c_double, C.c_int, C.c_double, _D]),
    "cvxg_newton_step": (C.c_int, [_P, C.POINTER(cvxg_params), C.POINTER(cvxg_step_info)]),
    "cvxg_centering": (C.c_int, [_P, C.POINTER(cvxg_params), C.c_double, C.POINTER(cvxg_centering_info)]),
    "cvxg_barrier_solve": (C.c_int, [_P, C.POINTER(cvxg_params), C.c_int, C.POINTER(cvxg_solution)]),
    "cvxg_batch_barrier_solve": (C.c_int, [C.c_int, C.POINTER(_P), C.POINTER(cvxg_params), C.c_int,
                                           C.POINTER(cvxg_solution), C.POINTER(C.c_int)]),
    "cvxg_batch_newton_step": (C.c_int, [C.c_int, C.POINTER(_P), C.POINTER(cvxg_params), C.POINTER(cvxg_step_info),
                                         C.POINTER(C.c_int)]),
    "cvxg_pd_direction": (C.c_int, [_P, C.POINTER(cvxg_params), C.c_double, _D, _D, _D, _D,
                                    C.POINTER(cvxg_pd_step_info)]),
    "cvxg_pd_solve": (C.c_int, [_P, C.POINTER(cvxg_params), C.POINTER(cvxg_pd_solution)]),
    "cvxg_pd_direction_eq": (C.c_int, [_P, C.POINTER(cvxg_params), C.c_double, _D, _D, _D, _D, _D, _D,
                                       C.POINTER(cvxg_pd_step_info)]),
    "cvxg_get_lambda": (C.c_int, [_P, _D]),
    "cvxg_get_nu": (C.c_int, [_P, _D]),
    "cvxg_solution_space": (C.c_int, [C.c_int, C.c_int, C.c_int, _D, C.c_int, C.c_int, _D, _D, _D, C.c_int]),
    "cvxg_affine_from": (C.c_int, [_P, _P, _D, _D, C.c_int]),
    "cvxg_affine_parameter": (C.c_int, [_P, _D, _D]),
    "cvxg_affine_map": (C.c_int, [_P, _D, _D]),
    "cvxg_set_timing": (C.c_int, [_P, C.c_int]),
    "cvxg_get_phase_times": (C.c_int, [_P, _D, C.c_int]),
    "cvxg_get_phase_stats": (C.c_int, [_P, _D, C.POINTER(C.c_int), C.c_int]),
    "cvxg_get_counters": (C.c_int, [_P, C.POINTER(C.c_longlong), C.c_int]),
    "cvxg_chol_schedule": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_uint), C.c_int]),
    "cvxg_set_ruiz_lookahead": (C.c_int, [_P, C.c_int, C.POINTER(C.c_longlong)]),
    "cvxg_set_option": (C.c_int, [_P, C.c_int, C.c_longlong]),
}

# cvxg_set_option's options (include/cvxg.h)
OPTIONS = {"sparse_rows": 1, "early_abort": 2, "h_lower": 3, "kkt_fused_rhs": 4, "spec_reg": 5, "ruiz_loop": 6,
           "ruiz_wg": 7}


def load(path: str = LIB_PATH) -> C.CDLL:
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7).  Loading torch
    # first lets libcvxg.so bind to that same runtime, so torch tensors, RCCL and the engine share devices.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise ImportError(f"cvx_amd: HIP library {path} is not built (run __graft_entry__.build()); "
                          "there is no CPU fallback")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = load()
    return _lib
