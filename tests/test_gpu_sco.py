"""GPU tests of the generic trajopt_sco path: sco::BasicTrustRegionSQP's host
loop with every convex subproblem solved on the GPU by the GpuModel (OSQP 1.0
in qp_csc.hip through thip_qp_*), against the oracle's OSQPModel on the same
problems.

* The reference's trajopt_sco unit problems (solver-interface-unit.cpp,
  small-problems-unit.cpp; drivers trajopt-1_amd/host/tests/sco_cases.cpp and
  oracle/src/sco_cases.cpp): identical status, QP / SQP counts and solutions
  within 1e-5.
* The joint-term problems of joint_costs_unit.cpp through the front door's
  single-problem entry (thost_solve_json -> trajopt::BasicTrustRegionSQP):
  the lowerable ones run the fused kernel as a batch of one, the others (JointVel
  equality constraint, JointAcc, JointJerk) the host loop with GpuModel QPs; both
  through the parity gate of tests/parity.py.
"""
import ctypes as C

import numpy as np
import pytest

import joint_terms
from parity import TOL_X, check_parity
from trajopt_amd import abi, host

pytestmark = pytest.mark.gpu

SCO_LIB = abi.LIB_DIR / "libsco_cases.so"


@pytest.fixture(scope="module")
def sco_lib():
    abi.load_hip()
    import torch

    assert torch.cuda.is_available(), "gpu tests need an AMD GPU"
    host.load_host()
    L = C.CDLL(str(SCO_LIB))
    L.sco_case_run.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int),
                               C.POINTER(C.c_longlong), C.c_char_p, C.c_int]
    L.sco_case_run.restype = C.c_int
    return L


def run_case(L, case_id):
    x = np.zeros(8)
    counts = (C.c_int * 5)()
    admm = C.c_longlong(0)
    err = C.create_string_buffer(2048)
    rc = L.sco_case_run(case_id, 0, x.ctypes.data_as(C.POINTER(C.c_double)), 8, counts, C.byref(admm), err, 2048)
    assert rc == 0, err.value.decode()
    return {"x": x[: counts[0]].copy(), "status": counts[1], "n_qp": counts[2], "n_sqp": counts[3],
            "n_vars_after": counts[4], "n_admm": admm.value}


# the reference's own assertions (small-problems-unit.cpp)
SOLUTIONS = {3: ([0, 1, 2], 1e-3), 4: ([1, 7, 2], 0.01), 5: ([1, 1], 0.01), 6: ([0, 0], 0.01), 7: ([1, 1], 0.01),
             8: ([0, np.sqrt(3.0)], 0.01)}


def _same(a, b):
    return (a["status"], a["n_qp"], a["n_sqp"], a["n_vars_after"]) == (b["status"], b["n_qp"], b["n_sqp"],
                                                                        b["n_vars_after"]) and \
        np.abs(a["x"] - b["x"]).max() <= TOL_X


@pytest.mark.parametrize("case", range(9))
def test_sco_cases_gpu_model(sco_lib, oracle_mod, case):
    """Bar: the oracle's status, QP / SQP counts and solution within 1e-5.  A
    miss passes only if the oracle's second rounding (liboracle_fast_*, the same
    algorithm with FMA contraction) reaches the GPU's outcome, or itself leaves
    the exact build's outcome while the GPU meets the reference's assertion: the
    reference algorithm does not determine that problem's path at double
    precision.  (TP3's numerical Hessian of 1e-5 (x1 - x0)^2 is a second
    difference at eps = 1e-5: rounding-dominated.)"""
    name = oracle_mod.SCO_CASES[case]
    g = run_case(sco_lib, case)
    o = oracle_mod.sco_case(case)
    print(f"{name}: gpu {g} | oracle {o}")
    if _same(g, o):
        return
    f = oracle_mod.sco_case(case, variant="fast")
    print(f"{name}: oracle fast build {f}")
    if _same(g, f):
        return  # reach
    assert not _same(f, o), f"{name}: the GPU misses the bar and the oracle's outcome is stable"
    sol, tol = SOLUTIONS[case]
    assert g["status"] == o["status"] == 0, name
    np.testing.assert_allclose(g["x"], sol, rtol=0, atol=tol, err_msg=name)


@pytest.mark.parametrize("name", sorted(joint_terms.PROBLEMS))
def test_joint_terms_single_problem(sco_lib, oracle_mod, name):
    text, check = joint_terms.PROBLEMS[name]
    x, res, native = host.solve_json(text)
    assert native == (name in joint_terms.LOWERABLE)
    assert check(x) == [], (name, check(x))
    wl = joint_terms.workload(text, host)
    check_parity(wl, oracle_mod, x[None], [res], label=f"json-{name}", min_strict=0.0)
