"""CPU tests of the trajopt_sco surface and the joint-difference terms.

* The oracle's restatements of the reference's trajopt_sco unit problems
  (oracle/src/sco_cases.cpp: solver-interface-unit.cpp setup_problem /
  ExprMult_test2 / ExprMult_test3, small-problems-unit.cpp QuadraticSeparable /
  QuadraticNonseparable / TP1 / TP3 / TP6 / TP7) meet the reference's own
  assertions -- the known answers the GPU path is then compared against
  (tests/test_gpu_sco.py).
* The joint-term problems of joint_costs_unit.cpp (tests/joint_terms.py), lowered
  by the host front door (JointPos / JointVel terms into the kernel's tables,
  JointVel equality constraints / JointAcc / JointJerk into the jdt table), solved
  by the oracle, meet the reference's assertions (KATs).
"""
import numpy as np
import pytest

import joint_terms
from trajopt_amd import host

SOLUTIONS = {3: ([0, 1, 2], 1e-3), 4: ([1, 7, 2], 0.01), 5: ([1, 1], 0.01), 6: ([0, 0], 0.01), 7: ([1, 1], 0.01),
             8: ([0, np.sqrt(3.0)], 0.01)}


@pytest.fixture(scope="module")
def built():
    import __graft_entry__

    __graft_entry__.build()


@pytest.mark.parametrize("case", range(9))
def test_oracle_sco_cases_meet_reference_assertions(oracle_mod, case):
    r = oracle_mod.sco_case(case)
    if case == 0:
        assert abs(r["x"].sum() - 3) < 1e-6  # aff(soln) == 0
        assert r["n_vars_after"] == 2       # removeVar
    elif case in (1, 2):
        c1, c2, k1, k2 = (2, 1, 0, 0) if case == 1 else (3, 2, -3, -5)
        v = (c1 * r["x"][0] + k1) * (c2 * r["x"][1] + k2)
        assert abs(v - (400 if case == 1 else 945)) < 1e-6
    else:
        sol, tol = SOLUTIONS[case]
        assert r["status"] == 0, oracle_mod.SCO_CASES[case]
        np.testing.assert_allclose(r["x"], sol, rtol=0, atol=tol)


@pytest.mark.parametrize("name", sorted(joint_terms.PROBLEMS))
def test_joint_term_kats(built, oracle_mod, name):
    text, check = joint_terms.PROBLEMS[name]
    wl = joint_terms.workload(text, host)
    assert joint_terms.lowerable(wl.desc) == (name in joint_terms.LOWERABLE)
    x, res = oracle_mod.solve(wl)
    assert res[0].status == 0, (name, res[0].status)
    assert check(x[0]) == [], (name, check(x[0]))


def test_joint_acc_lowering_clamps_like_the_reference(built):
    """JointAccTermInfo::hatch (problem_description.cpp:1423-1440): first_step is
    clamped to n_steps - 3, last_step == first_step becomes first + 2; the jdt
    table holds the clamped steps, costs before constraints."""
    text, _ = joint_terms.PROBLEMS["equality_jointAcc"]
    d, _, _, _ = host.lower_json(text)
    assert d.n_jdt == 2
    assert (d.jdt_order[0], d.jdt_is_cnt[0], d.jdt_first_step[0], d.jdt_last_step[0]) == (2, 0, 0, 9)
    assert (d.jdt_order[1], d.jdt_is_cnt[1], d.jdt_first_step[1], d.jdt_last_step[1]) == (2, 1, 0, 2)
    text, _ = joint_terms.PROBLEMS["equality_jointJerk"]
    d, _, _, _ = host.lower_json(text)
    assert (d.jdt_order[1], d.jdt_first_step[1], d.jdt_last_step[1]) == (3, 0, 4)
    text, _ = joint_terms.PROBLEMS["equality_jointVel"]
    d, _, _, _ = host.lower_json(text)
    assert d.jv_enabled == 1 and d.n_jdt == 1
    assert (d.jdt_order[0], d.jdt_is_cnt[0], d.jdt_first_step[0], d.jdt_last_step[0]) == (1, 1, 0, 1)


def test_generic_path_evaluates_kinematic_terms_on_the_device_only(built):
    """A problem mixing a CartPose term with one the kernel does not lower
    (JointAcc) runs the host loop, whose CartPose error and jacobian come from
    the device (thip_eval_cart_pose): without a GPU it fails loudly at the
    evaluator, never computing FK on the CPU (the -m gpu twin solves it,
    tests/test_gpu_dropin.py)."""
    import json

    doc = json.loads(joint_terms.PROBLEMS["equality_jointAcc"][0])
    doc["costs"].append({"type": "cart_pose", "params": {
        "timestep": 9, "source_frame": "r_gripper_tool_frame", "target_frame": "torso_lift_link",
        "target_frame_offset_xyz": [0.6, -0.2, 0.1]}})
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the -m gpu tests solve this problem")
    with pytest.raises(host.HostError) as ei:
        host.solve_json(json.dumps(doc))
    assert "thip_eval_create" in str(ei.value)


def test_time_and_fixed_dof_lowering(built):
    """use_time adds the dt column (TrajOptProb ctor, problem_description.cpp:557-598)
    with the init dt appended (:372-379); time JointVel terms fill the jvt table
    with the JointVel clamping; TotalTime and fixed dofs fill theirs."""
    text, _ = joint_terms.PROBLEMS["inequality_jointVel_time"]
    d, init, _, _ = host.lower_json(text)
    assert d.use_time == 1 and (d.dt_lower, d.dt_upper) == (0.01234, 3.5678)
    assert abs(d.init_dt - (3.5678 - 0.01234)) < 1e-15
    assert init.shape == (joint_terms.STEPS, 7) and d.n_jdt == 0
    assert d.n_jvt == 3 and [d.jvt_is_cnt[k] for k in range(3)] == [0, 0, 1]
    assert [(d.jvt_first_step[k], d.jvt_last_step[k]) for k in range(3)] == [(0, 4), (5, 9), (0, 9)]
    text, _ = joint_terms.PROBLEMS["equality_jointVel_time"]
    d, _, _, _ = host.lower_json(text)
    assert (d.jvt_first_step[1], d.jvt_last_step[1]) == (0, 1)  # last == first -> first + 1
    text, _ = joint_terms.PROBLEMS["total_time_cnt"]
    d, _, _, _ = host.lower_json(text)
    assert d.n_ttt == 1 and d.ttt_is_cnt[0] == 1 and d.ttt_limit[0] == 5.8 and d.ttt_coeff[0] == 1.0
    text, _ = joint_terms.PROBLEMS["fixed_dofs"]
    d, _, _, _ = host.lower_json(text)
    assert d.n_fixed_dofs == 2 and list(d.fixed_dofs)[:2] == [2, 5] and d.use_time == 0


@pytest.mark.parametrize("edit, msg", [
    (lambda doc: doc["basic_info"].update(use_time=True), "No terms use time"),
    (lambda doc: doc["basic_info"].update(fixed_dofs=[7]), "greater than the number of DOF"),
    (lambda doc: doc["costs"].append({"type": "total_time", "params": {"coeff": 1, "limit": 1, "bogus": 0}}),
     "bogus"),
])
def test_time_front_door_errors(built, edit, msg):
    """ConstructProblem's use_time consistency checks (problem_description.cpp:419-456)
    and the fixed-dof range check (:515-520); TotalTime's params whitelist (:1868)."""
    import json

    doc = json.loads(joint_terms.PROBLEMS["equality_jointVel"][0])
    edit(doc)
    with pytest.raises(host.HostError) as ei:
        host.lower_json(json.dumps(doc))
    assert msg in str(ei.value)



def test_gpu_model_capacity_is_a_failed_solve(built, capfd):
    """GpuModel answers a convex subproblem beyond the KKT capacity
    (n + m > THIP_QP_MAX_KKT) with CVX_FAILED before touching the device, the
    limit named on stderr: the reference's failure handling (trust-box shrink
    and retry, then /tmp/fail.lp and OPT_FAILED, optimizers.cpp:790-822) then
    applies to that problem alone, and a batch's other problems go on."""
    import ctypes as C

    from trajopt_amd import abi

    L = C.CDLL(str(abi.LIB_DIR / "libsco_cases.so"))
    L.sco_case_run.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int),
                               C.POINTER(C.c_longlong), C.c_char_p, C.c_int]
    x = np.zeros(8)
    counts = (C.c_int * 5)()
    err = C.create_string_buffer(2048)
    rc = L.sco_case_run(9, 0, x.ctypes.data_as(C.POINTER(C.c_double)), 8, counts, None, err, 2048)
    assert rc == 0, err.value.decode()
    assert counts[1] == 2  # sco::CVX_FAILED
    assert "THIP_QP_MAX_KKT" in capfd.readouterr().err
