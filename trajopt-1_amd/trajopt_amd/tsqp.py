"""ctypes binding of the trajopt_sqp front end (include/trajopt_host.h, tsqp_*).

trajopt's second SQP front end (trajopt_optimizers/trajopt_sqp: TrustRegionSQPSolver
over a TrajOptQPProblem of trajopt_ifopt constraint sets)
keeps one QP sparsity pattern for the whole solve and updates it in place; here
the QP lives in thip_qp's resident GPU workspace (trajopt_sqp::GpuQPSolver).
`Spec` mirrors tsqp_spec: a joint trajectory of n_nodes nodes with joint
position / velocity / acceleration / jerk terms, as constraints or as squared /
absolute / hinge costs.  `solve` runs the C++ product path on a HIP device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, host

MAX_NODES = 64
MAX_TERMS = 16
JOINT_POS, JOINT_VEL, JOINT_ACC, JOINT_JERK = 0, 1, 2, 3
CONSTRAINT, SQUARED, ABSOLUTE, HINGE = 0, 1, 2, 3
STATUS = {0: "SQP_RUNNING", 1: "SQP_CONVERGED", 2: "SQP_ITERATION_LIMIT", 3: "SQP_PENALTY_ITERATION_LIMIT",
          4: "SQP_TIME_LIMIT", 5: "SQP_FAILED", 6: "SQP_STOPPED_BY_CALLBACK"}
D_MAX = abi.MAX_DOF


class Term(C.Structure):
    _fields_ = [("kind", C.c_int), ("penalty", C.c_int), ("first", C.c_int), ("last", C.c_int),
                ("n_coeffs", C.c_int), ("coeffs", C.c_double * D_MAX), ("lower", C.c_double * D_MAX),
                ("upper", C.c_double * D_MAX)]


class Spec(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("n_dof", C.c_int), ("init", C.c_double * (MAX_NODES * D_MAX)),
                ("var_lower", C.c_double * D_MAX), ("var_upper", C.c_double * D_MAX), ("n_terms", C.c_int),
                ("terms", Term * MAX_TERMS),
                ("improve_ratio_threshold", C.c_double), ("min_trust_box_size", C.c_double),
                ("min_approx_improve", C.c_double), ("min_approx_improve_frac", C.c_double),
                ("max_iterations", C.c_int), ("trust_shrink_ratio", C.c_double), ("trust_expand_ratio", C.c_double),
                ("cnt_tolerance", C.c_double), ("max_merit_coeff_increases", C.c_double),
                ("max_qp_solver_failures", C.c_int), ("merit_coeff_increase_ratio", C.c_double),
                ("max_time", C.c_double), ("initial_merit_error_coeff", C.c_double),
                ("inflate_constraints_individually", C.c_int), ("initial_trust_box_size", C.c_double),
                ("osqp", abi.OsqpSettings)]


class Result(C.Structure):
    _fields_ = [("status", C.c_int), ("overall_iteration", C.c_int), ("penalty_iteration", C.c_int),
                ("qp_setups", C.c_int), ("qp_updates", C.c_int), ("qp_solves", C.c_int),
                ("admm_iters", C.c_longlong), ("best_exact_merit", C.c_double)]


def _lib():
    L = host.load_host()
    if not hasattr(L, "_tsqp_ready"):
        L.thost_tsqp_defaults.argtypes = [C.POINTER(Spec)]
        L.thost_tsqp_defaults.restype = None
        L.thost_tsqp_solve.argtypes = [C.POINTER(Spec), C.c_int, C.POINTER(C.c_double), C.POINTER(Result),
                                       C.c_char_p, C.c_int]
        L.thost_tsqp_solve.restype = C.c_int
        L.thost_tsqp_sizeof_spec.restype = C.c_int
        L.thost_tsqp_sizeof_result.restype = C.c_int
        if L.thost_tsqp_sizeof_spec() != C.sizeof(Spec) or L.thost_tsqp_sizeof_result() != C.sizeof(Result):
            raise RuntimeError("tsqp_spec / tsqp_result layout mismatch between Python and the host library")
        L._tsqp_ready = True
    return L


def make_spec(init, terms, var_lower=None, var_upper=None, **params):
    """init [n_nodes, n_dof]; terms: dicts with kind, penalty, first, last (default
    first), coeffs (list), lower, upper (per-dof lists); params: SQPParameters /
    `osqp` (dict of thip_osqp_settings fields) overrides.  SQPParameters and OSQP
    settings default to the reference's (types.h, OSQPEigenSolver::setDefaultOSQPSettings)."""
    init = np.asarray(init, dtype=np.float64)
    n, d = init.shape
    if n > MAX_NODES or d > D_MAX or len(terms) > MAX_TERMS:
        raise ValueError("spec exceeds TSQP_MAX_NODES / THIP_MAX_DOF / TSQP_MAX_TERMS")
    s = Spec()
    _lib().thost_tsqp_defaults(C.byref(s))
    s.n_nodes, s.n_dof = n, d
    for i, v in enumerate(init.reshape(-1)):
        s.init[i] = float(v)
    for k in range(d):
        s.var_lower[k] = -np.inf if var_lower is None else float(var_lower[k])
        s.var_upper[k] = np.inf if var_upper is None else float(var_upper[k])
    s.n_terms = len(terms)
    for i, t in enumerate(terms):
        T = s.terms[i]
        T.kind, T.penalty = int(t["kind"]), int(t.get("penalty", CONSTRAINT))
        T.first = int(t.get("first", 0))
        T.last = int(t.get("last", T.first))
        co = list(t.get("coeffs", []))
        T.n_coeffs = len(co)
        for k, v in enumerate(co):
            T.coeffs[k] = float(v)
        lo = list(t.get("lower", [0.0] * d))
        up = list(t.get("upper", lo))
        for k in range(d):
            T.lower[k] = float(lo[k])
            T.upper[k] = float(up[k])
    osqp = params.pop("osqp", {})
    for k, v in params.items():
        if not hasattr(s, k):
            raise KeyError(k)
        setattr(s, k, v)
    for k, v in osqp.items():
        if not hasattr(s.osqp, k):
            raise KeyError(k)
        setattr(s.osqp, k, v)
    return s


def solve(spec: Spec, device: int = 0):
    """-> (x [n_nodes, n_dof], Result) through trajopt_sqp::TrustRegionSQPSolver with
    trajopt_sqp::GpuQPSolver on HIP device `device`."""
    L = _lib()
    x = np.zeros((spec.n_nodes, spec.n_dof))
    res = Result()
    err = C.create_string_buffer(4096)
    rc = L.thost_tsqp_solve(C.byref(spec), device, x.ctypes.data_as(C.POINTER(C.c_double)), C.byref(res), err, 4096)
    if rc != 0:
        raise host.HostError(err.value.decode())
    return x, res
