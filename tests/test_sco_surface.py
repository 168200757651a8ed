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
    assert (wl.desc.n_jdt == 0) == (name in joint_terms.LOWERABLE)
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


def test_generic_path_refuses_device_only_terms(built):
    """A problem mixing a kernel-only term (CartPose: FK on the device) with one
    the kernel does not lower (JointAcc) runs the host loop, which refuses to
    evaluate the CartPose term on the CPU: it fails loudly, before any QP."""
    import json

    doc = json.loads(joint_terms.PROBLEMS["equality_jointAcc"][0])
    doc["costs"].append({"type": "cart_pose", "params": {
        "timestep": 9, "source_frame": "r_gripper_tool_frame", "target_frame": "torso_lift_link",
        "target_frame_offset_xyz": [0.6, -0.2, 0.1]}})
    with pytest.raises(host.HostError) as ei:
        host.solve_json(json.dumps(doc))
    assert "evaluated by the batched GPU kernel only" in str(ei.value)
