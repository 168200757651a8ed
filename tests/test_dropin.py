"""CPU checks of the drop-in boundary beyond the batched kernel (tests/dropin_cases.py):
the reference's own single-waypoint configs and mixed problems lower through the
host front door (ConstructProblem, unchanged JSON), and the oracle solving the
lowered problems meets the reference's own assertions -- the known answers the
GPU path is then held to (tests/test_gpu_dropin.py)."""
import numpy as np
import pytest

import dropin_cases as dc
from trajopt_amd import host


@pytest.fixture(scope="module", autouse=True)
def built():
    if not host.HOST_LIB.exists():
        import __graft_entry__

        __graft_entry__.build()
    host.load_host()


def test_numerical_ik1_lowers_unchanged():
    """numerical_ik1.json: one waypoint, left_arm, a CartPose constraint to
    base_footprint (problem_description.cpp:919-1005); AUTO_SOLVER accepted."""
    d, init, tgt, jpt = host.lower_json(dc.text("numerical_ik1.json"))
    assert d.n_steps == 1 and d.chain.n_dof == 7 and d.n_cart == 1 and d.cart_is_cnt[0] == 1
    assert d.chain.joint_axis[1][2] == 1 and d.chain.joint_origin[1][7] == 0.188  # l_shoulder_pan
    assert not init.any() and d.coll_enabled == 0 and d.n_coll_extra == 0
    # the target pose (base_footprint * offset) in the chain root (torso_lift_link)
    T = np.asarray(tgt[0]).reshape(3, 4)
    np.testing.assert_allclose(T[:, :3], dc.IK_GOAL[:, :3], atol=1e-15)
    np.testing.assert_allclose(T[:, 3], [0.4 + 0.05, 0.0, 0.8 - 0.051 - 0.739675], atol=1e-15)


def test_simple_collision_lowers_unchanged():
    """simple_collision_test.json on spherebot: the collision cost is the first
    collision term (coll_*), the collision constraint the second (coll_extra[0]),
    both DISCRETE; the scene is the URDF's three static spheres."""
    d, init, _, jpt, scene = host.lower_json(dc.text("simple_collision_test.json"), with_scene=True)
    assert d.n_steps == 1 and d.chain.n_dof == 2 and d.chain.joint_type[1] == 3 and d.chain.joint_type[2] == 3
    np.testing.assert_array_equal(init, [[-0.75, 0.75]])
    assert d.coll_enabled == 1 and d.coll_is_cnt == 0 and d.coll_continuous == 2
    assert (d.coll_margin, d.coll_coeff, d.coll_first_step, d.coll_last_step) == (0.3, 1.0, 0, 0)
    assert d.n_coll_extra == 1
    x = d.coll_extra[0]
    assert (x.is_cnt, x.continuous, x.margin, x.coeff, x.first_step, x.last_step) == (1, 2, 0.2, 1.0, 0, 0)
    assert d.n_jpos == 1 and d.jpos_is_cnt[0] == 0 and not jpt.any()
    assert d.n_spheres == 1 and d.sphere_radius[0] == 0.5 and d.sphere_link[0] == 3
    np.testing.assert_array_equal(scene[:, [0, 1, 2, 3, 4]], [[0, 0, 0, 0, .5], [0, -.75, 0, 0, .5], [0, 0, .75, 0, .5]])


@pytest.mark.parametrize("name", ["numerical_ik1.json", "simple_collision_test.json"])
def test_oracle_meets_reference_assertions(oracle_mod, name):
    """The oracle on the lowered reference config meets the reference test's own
    EXPECTs: numerical_ik_unit.cpp:119-125 (final pose within 1e-3 of the goal),
    simple_collision_unit.cpp:88-91, 121-124 (initial state in collision, final
    state collision-free, contact margin 0.2)."""
    wl = dc.json_workload(dc.text(name), host)
    x, res = oracle_mod.solve(wl)
    assert res[0].status == 0, res[0].status
    if name.startswith("numerical_ik"):
        assert dc.ik_pose_error(wl.desc, x[0], oracle_mod) < 1e-3
    else:
        assert dc.spherebot_min_distance(wl.init[0, 0], wl.scene[0]) < 0.2
        assert dc.spherebot_min_distance(x[0, 0], wl.scene[0]) >= 0.2


def test_mixed_problems_lower_for_the_generic_path(oracle_mod):
    """CartPose + JointAcc and collision + JointJerk: the kernel-lowered terms keep
    their descriptor records, the others the jdt table; the oracle solves both."""
    d, *_ = host.lower_json(dc.cartpose_jointacc())
    assert d.n_cart == 1 and d.n_jdt == 2
    d, *_ = host.lower_json(dc.collision_jointjerk(), scene=dc.table_scene())
    assert d.coll_enabled == 1 and d.n_jdt == 1 and d.n_prims == 1
    for text in (dc.cartpose_jointacc(), dc.collision_jointjerk()):
        sc = dc.table_scene() if "collision" in text else None
        wl = dc.json_workload(text, host) if sc is None else _with_scene(text, sc)
        x, res = oracle_mod.solve(wl)
        assert res[0].status in (0, 1), res[0].status


def _with_scene(text, scene):
    from trajopt_amd.problems import Workload

    desc, init, tgt, jpt, sc = host.lower_json(text, scene=scene, with_scene=True)
    return Workload("json", desc, init[None].copy(), tgt[None].copy(), sc[None].copy(), init[None].copy(),
                    jpt[None].copy() if desc.n_jpos else None)


def test_collision_term_limits():
    """At most 1 + THIP_MAX_COLL_EXTRA collision terms; further terms of one
    problem must share the environment's robot model and scene."""
    import json

    doc = json.loads(dc.text("simple_collision_test.json"))
    extra = doc["constraints"][0]
    doc["constraints"] = [extra] * 4
    with pytest.raises(host.HostError) as ei:
        host.lower_json(json.dumps(doc))
    assert "collision terms" in str(ei.value)


def test_oracle_meets_planning_unit_assertions(oracle_mod):
    """arm_around_table.json with the table as its exact box (dropin_cases):
    the oracle meets planning_unit.cpp's EXPECTs -- the initial trajectory in
    collision (:101), OPT_CONVERGED (:125), the final trajectory collision-free
    (:148) -- under this build's sphere model of the PR2 arm."""
    text = dc.text("arm_around_table.json")
    scene = dc.arm_around_table_scene()
    wl = _with_scene(text, scene)
    assert dc.continuous_check_found(wl.desc, wl.init[0], wl.scene[0], oracle_mod)
    x, res = oracle_mod.solve(wl)
    assert res[0].status == 0
    assert not dc.continuous_check_found(wl.desc, x[0], wl.scene[0], oracle_mod)
