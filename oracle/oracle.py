"""ORACLE binding — test infrastructure only.

ctypes access to oracle/build/liboracle.so, the CPU restatement of the
reference's trajopt_sco / OSQP / trajopt hot path. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module:
it is the checker (and the timed CPU baseline), never the thing measured or
shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
REPO = ROOT.parent
sys.path.insert(0, str(REPO / "trajopt-1_amd"))
from trajopt_amd import abi  # noqa: E402

LIB = ROOT / "build" / "liboracle.so"
KAT = ROOT / "build" / "kat"
_libs = {}


def _has_avx512():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("flags"):
                    return " avx512f " in ln + " "
    except OSError:
        pass
    return False


def variant_path(variant="exact"):
    """exact: the parity checker (no FMA contraction).  fast: the same sources at
    -O3 with FMA contraction for the highest x86-64 ISA level this host runs
    (v4 with AVX-512, else v3) -- the timed CPU baseline, and a second rounding
    of the same algorithm for the parity gate's stability proofs."""
    if variant == "exact":
        return LIB
    if variant == "fast":
        return ROOT / "build" / ("liboracle_fast_v4.so" if _has_avx512() else "liboracle_fast_v3.so")
    if variant == "san":
        return ROOT / "build" / "liboracle_san.so"
    raise ValueError(variant)


def build(quiet=True):
    """make -C oracle (called by __graft_entry__.build())."""
    out = subprocess.run(["make", "-C", str(ROOT), "-j8"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def lib(variant="exact"):
    if variant not in _libs:
        path = variant_path(variant)
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        P = C.POINTER
        dp = P(C.c_double)
        L.oracle_solve_batch.argtypes = [P(abi.ProblemDesc), C.c_int, dp, dp, dp, dp, dp, P(abi.Result), C.c_int]
        L.oracle_solve_batch.restype = C.c_int
        L.oracle_linearize.argtypes = [P(abi.ProblemDesc), C.c_int, dp, dp, dp, dp]
        L.oracle_linearize.restype = C.c_int
        L.oracle_fwd_kin.argtypes = [P(abi.Chain), C.c_int, dp, dp]
        L.oracle_fwd_kin.restype = C.c_int
        L.oracle_transform_error.argtypes = [dp, dp, dp, dp]
        L.oracle_transform_error.restype = None
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_sizeof_desc.restype = C.c_int
        assert L.oracle_sizeof_desc() == C.sizeof(abi.ProblemDesc), "descriptor layout mismatch"
        L.oracle_sizeof_result.restype = C.c_int
        assert L.oracle_sizeof_result() == C.sizeof(abi.Result), "result layout mismatch (rebuild the oracle)"
        _libs[variant] = L
    return _libs[variant]


def set_jitter(jac_abs=0.0, kkt_rel=0.0, sol_rel=0.0, seed=0, variant="exact"):
    """Rounding jitter of the next solves (oracle/src/jitter.hpp): +-jac_abs on
    every FD Jacobian entry, a relative +-kkt_rel on every KKT solution entry, a
    relative +-sol_rel on every returned QP solution; all 0 turns it off.  Test
    infrastructure: the parity gate's stability proofs."""
    L = lib(variant)
    L.oracle_set_jitter.argtypes = [C.c_double, C.c_double, C.c_double, C.c_ulonglong]
    L.oracle_set_jitter.restype = None
    L.oracle_set_jitter(float(jac_abs), float(kkt_rel), float(sol_rel), int(seed))


def set_jitter_coll(coll_abs=0.0, variant="exact"):
    """+-coll_abs on every linearised contact expression's coefficients and
    constant in the next solves (jitter.hpp), with set_jitter's seed; 0 = off."""
    L = lib(variant)
    L.oracle_set_jitter_coll.argtypes = [C.c_double]
    L.oracle_set_jitter_coll.restype = None
    L.oracle_set_jitter_coll(float(coll_abs))


SCO_CASES = {0: "setup_problem", 1: "ExprMult_test2", 2: "ExprMult_test3", 3: "QuadraticSeparable",
             4: "QuadraticNonseparable", 5: "TP1", 6: "TP3", 7: "TP6", 8: "TP7"}


def sco_case(case_id, variant="exact"):
    """One of the reference's trajopt_sco unit problems (src/sco_cases.cpp) on the
    oracle's OSQPModel / BasicTrustRegionSQP -> dict(x, status, n_qp, n_sqp,
    n_vars_after, n_admm)."""
    L = lib(variant)
    L.oracle_sco_case.argtypes = [C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int),
                                  C.POINTER(C.c_longlong)]
    L.oracle_sco_case.restype = C.c_int
    x = np.zeros(8)
    counts = (C.c_int * 5)()
    admm = C.c_longlong(0)
    if L.oracle_sco_case(case_id, _dp(x), 8, counts, C.byref(admm)) != 0:
        raise RuntimeError(f"oracle_sco_case({case_id}) failed")
    return {"x": x[: counts[0]].copy(), "status": counts[1], "n_qp": counts[2], "n_sqp": counts[3],
            "n_vars_after": counts[4], "n_admm": admm.value}


def _dp(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _jpos(wl, b=None):
    jt = getattr(wl, "jpos_targets", None)
    if jt is None:
        return None
    return np.ascontiguousarray(jt if b is None else jt[b], dtype=np.float64)


def solve(wl, n_threads=1, variant="exact"):
    """BasicTrustRegionSQP::optimize for every problem of the workload.
    Returns (x [B,N,D], list of abi.Result)."""
    L = lib(variant)
    B = wl.batch
    init = np.ascontiguousarray(wl.init, dtype=np.float64)
    tg = np.ascontiguousarray(wl.targets, dtype=np.float64) if wl.targets.size else None
    sc = np.ascontiguousarray(wl.scene, dtype=np.float64) if wl.scene.size else None
    jt = _jpos(wl)
    # [B][N][D], and the dt column after the joints with use_time
    x = np.zeros((B, init.shape[1], init.shape[2] + (1 if wl.desc.use_time else 0)))
    res = (abi.Result * B)()
    rc = L.oracle_solve_batch(C.byref(wl.desc), B, _dp(init), _dp(tg), _dp(sc), _dp(jt), _dp(x), res, n_threads)
    if rc != 0:
        raise RuntimeError("oracle_solve_batch: " + L.oracle_last_error().decode())
    return x, list(res)


def solve_trace(wl, b, cap=2048):
    """Problem b with its per-QP trace records (see oracle_solve_trace)."""
    L = lib()
    L.oracle_solve_trace.argtypes = [C.POINTER(abi.ProblemDesc), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(abi.Result), C.POINTER(C.c_double), C.c_int]
    L.oracle_solve_trace.restype = C.c_int
    init = np.ascontiguousarray(wl.init[b], dtype=np.float64)
    tg = np.ascontiguousarray(wl.targets[b], dtype=np.float64) if wl.targets.size else None
    sc = np.ascontiguousarray(wl.scene[b], dtype=np.float64) if wl.scene.size else None
    x = np.zeros_like(init)
    res = abi.Result()
    rec = np.zeros((cap, 12))
    n = L.oracle_solve_trace(C.byref(wl.desc), _dp(init), _dp(tg), _dp(sc), _dp(_jpos(wl, b)), _dp(x), C.byref(res),
                             _dp(rec), cap)
    if n < 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return x, res, rec[:n]


def linearize(wl, x):
    L = lib()
    B = wl.batch
    D = wl.n_dof
    x = np.ascontiguousarray(x, dtype=np.float64)
    tg = np.ascontiguousarray(wl.targets, dtype=np.float64)
    err = np.zeros((B, wl.desc.n_cart, 6))
    jac = np.zeros((B, wl.desc.n_cart, 6, D))
    L.oracle_linearize(C.byref(wl.desc), B, _dp(x), _dp(tg), _dp(err), _dp(jac))
    return err, jac


def fwd_kin(chain, q):
    L = lib()
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    out = np.zeros((q.shape[0], chain.n_links, 12))
    L.oracle_fwd_kin(C.byref(chain), q.shape[0], _dp(q), _dp(out))
    return out


def collision_rows(wl, b, x=None, cap=8192, term=0):
    """Linearised collision rows of problem b at trajectory x (default: the
    initial trajectory) for collision term `term` (0: the descriptor's coll_*
    term, k: coll_extra[k - 1]); see oracle_collision_rows_term.  Returns an
    array [n, 8 + 2 D + 1]."""
    L = lib()
    L.oracle_collision_rows_term.argtypes = [C.POINTER(abi.ProblemDesc), C.c_int, C.POINTER(C.c_double),
                                             C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int]
    L.oracle_collision_rows_term.restype = C.c_int
    D = wl.n_dof
    W = 8 + 2 * D + 1
    xb = np.ascontiguousarray(wl.init[b] if x is None else x, dtype=np.float64)
    sc = np.ascontiguousarray(wl.scene[b], dtype=np.float64)
    out = np.zeros((cap, W))
    n = L.oracle_collision_rows_term(C.byref(wl.desc), term, _dp(sc), _dp(xb), _dp(out), cap)
    if n < 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return out[:min(n, cap)]


def qp_solve(P, q, A, l, u, settings):
    """One QP (scipy CSC P upper triangular, A) through the OSQP restatement with
    thip_osqp_settings `settings`: (status, x, y, iterations)."""
    L = lib()
    ip = C.POINTER(C.c_int)
    dp = C.POINTER(C.c_double)
    L.oracle_qp_solve.argtypes = [C.c_int, C.c_int, ip, ip, dp, dp, ip, ip, dp, dp, dp, C.c_void_p, dp, dp, ip]
    L.oracle_qp_solve.restype = C.c_int
    n, m = P.shape[0], A.shape[0]
    arrs = [np.ascontiguousarray(v, dtype=np.int32) for v in (P.indptr, P.indices, A.indptr, A.indices)]
    vals = [np.ascontiguousarray(v, dtype=np.float64) for v in (P.data, q, A.data, l, u)]
    x, y, it = np.zeros(n), np.zeros(max(m, 1)), C.c_int(0)
    st = L.oracle_qp_solve(n, m, arrs[0].ctypes.data_as(ip), arrs[1].ctypes.data_as(ip), _dp(vals[0]), _dp(vals[1]),
                           arrs[2].ctypes.data_as(ip), arrs[3].ctypes.data_as(ip), _dp(vals[2]), _dp(vals[3]),
                           _dp(vals[4]), C.cast(C.pointer(settings), C.c_void_p), _dp(x), _dp(y), C.byref(it))
    return st, x, y[:m], it.value


def swept_sphere_prim(a, b, r, prim):
    """(dist, normal, p_robot, t_star) of the sphere swept a -> b vs a primitive."""
    L = lib()
    dp = C.POINTER(C.c_double)
    L.oracle_swept_sphere_prim.argtypes = [dp, dp, C.c_double, dp, dp]
    L.oracle_swept_sphere_prim.restype = None
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    prim = np.ascontiguousarray(prim, dtype=np.float64)
    out = np.zeros(9)
    L.oracle_swept_sphere_prim(_dp(a), _dp(b), r, _dp(prim), _dp(out))
    return out[0], out[1:4], out[4:7], out[7]


def sphere_prim(c, r, prim):
    L = lib()
    L.oracle_sphere_prim.argtypes = [C.POINTER(C.c_double), C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.oracle_sphere_prim.restype = None
    c = np.ascontiguousarray(c, dtype=np.float64)
    prim = np.ascontiguousarray(prim, dtype=np.float64)
    out = np.zeros(8)
    L.oracle_sphere_prim(_dp(c), float(r), _dp(prim), _dp(out))
    return out[0], out[1:4], out[4:7]


def run_kats():
    if not KAT.exists():
        build()
    p = subprocess.run([str(KAT)], capture_output=True, text=True)
    return p.returncode, p.stdout


def tsqp_solve(spec, variant="exact"):
    """The trajopt_sqp front end (src/trajopt_sqp.cpp: TrustRegionSQPSolver over
    TrajOptQPProblem with OSQPEigenSolver's update-in-place QP) on one
    trajopt_amd.tsqp.Spec -> (x [n_nodes, n_dof], tsqp.Result)."""
    from trajopt_amd import tsqp  # the spec layout (include/trajopt_host.h)

    L = lib(variant)
    if not hasattr(L, "_tsqp_ready"):
        L.oracle_tsqp_solve.argtypes = [C.POINTER(tsqp.Spec), C.POINTER(C.c_double), C.POINTER(tsqp.Result)]
        L.oracle_tsqp_solve.restype = C.c_int
        L._tsqp_ready = True
    x = np.zeros((spec.n_nodes, spec.n_dof))
    res = tsqp.Result()
    if L.oracle_tsqp_solve(C.byref(spec), _dp(x), C.byref(res)) != 0:
        raise RuntimeError("oracle_tsqp_solve: " + L.oracle_last_error().decode())
    return x, res
