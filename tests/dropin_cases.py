"""Problems that exercise the drop-in boundary beyond the batched kernel, shared
by tests/test_dropin.py (CPU: lowering, oracle KATs) and tests/test_gpu_dropin.py
(GPU parity):

* the reference's own test configs, unchanged (data fixtures under
  tests/golden/json/):
  - numerical_ik1.json (trajopt/test/numerical_ik_unit.cpp:61-136): one
    waypoint, a CartPose constraint on the PR2 left arm; the reference asserts
    the final l_gripper_tool_frame pose within 1e-3 of the goal (:113-125);
  - simple_collision_test.json (trajopt/test/simple_collision_unit.cpp:62-126):
    one waypoint on spherebot, a DISCRETE collision cost (dist_pen 0.3) and a
    DISCRETE collision constraint (0.2) plus a JointPos cost; the reference
    asserts the initial state in collision and the final one collision-free
    under a 0.2 m contact margin (:88-91, :121-124);
* mixed problems: CartPose next to JointAcc (a term the kernel does not lower),
  collision next to JointJerk.
"""
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden" / "json"


def text(name):
    return (GOLDEN / name).read_text()


def json_batch_workload(texts, host):
    """JSON problems of one structure (every problem lowers to the same
    description; targets and initial trajectories differ) as one Workload."""
    from trajopt_amd.problems import Workload

    low = [host.lower_json(t) for t in texts]
    init = np.stack([v[1] for v in low])
    return Workload("json-batch", low[0][0], init, np.stack([v[2] for v in low]), np.zeros((len(texts), 0, 16)),
                    init.copy(), None)


def json_workload(text_, host, prims=None):
    """The JSON problem lowered by the host front door as a one-problem Workload
    (scene = the built-in environment's primitives, then `prims`)."""
    from trajopt_amd.problems import Workload

    desc, init, tgt, jpt, scene = host.lower_json(text_, prims, with_scene=True)
    return Workload("json", desc, init[None].copy(), tgt[None].copy(), scene[None].copy(), init[None].copy(),
                    jpt[None].copy() if desc.n_jpos else None)


# numerical_ik_unit.cpp:114-117: translation (0.4, 0, 0.8), quaternion (w, x, y, z) = (0, 0, 1, 0)
IK_GOAL = np.array([[-1.0, 0.0, 0.0, 0.4], [0.0, 1.0, 0.0, 0.0], [0.0, 0.0, -1.0, 0.8]])


def ik_pose_error(desc, x, oracle_mod):
    """max |goal - final pose| over the 3x4 pose entries (the reference checks the
    4x4 matrix, whose last row is exact) of l_gripper_tool_frame (the group's last
    link), in base_footprint = world."""
    poses = oracle_mod.fwd_kin(desc.chain, np.asarray(x).reshape(1, -1))
    T = poses[0, desc.chain.n_links - 1].reshape(3, 4)
    return float(np.abs(T - IK_GOAL).max())


def spherebot_min_distance(x, scene):
    """Smallest signed distance between spherebot's 0.5 m sphere at (x, y, 0) and
    the scene's spheres (tesseract's contact test on spheres is this closed form)."""
    c = np.array([x[0], x[1], 0.0])
    return min(float(np.linalg.norm(c - p[1:4]) - 0.5 - p[4]) for p in scene)


def cartpose_jointacc():
    """joint_costs_unit's equality_jointAcc (a JointAcc cost on every step, a
    zero-acceleration constraint on the first) plus a CartPose cost on the last
    waypoint: the kernel does not lower JointAcc, so the CartPose term runs in
    the host loop with its FK on the device."""
    import joint_terms

    doc = json.loads(joint_terms.PROBLEMS["equality_jointAcc"][0])
    doc["costs"].append({"type": "cart_pose", "name": "tool_goal", "params": {
        "timestep": joint_terms.STEPS - 1, "source_frame": "r_gripper_tool_frame", "target_frame": "torso_lift_link",
        "pos_coeffs": [5, 5, 5], "rot_coeffs": [1, 1, 0],
        "target_frame_offset_xyz": [0.55, -0.35, 0.05], "target_frame_offset_wxyz": [0.7071068, 0, 0.7071068, 0]}})
    return json.dumps(doc)


def collision_jointjerk(evaluator=2):
    """A 10-waypoint right-arm move over a table-top scene: JointVel cost, a
    collision cost (evaluator 1 DISCRETE / 2 LVS_DISCRETE / 4 LVS_CONTINUOUS,
    lvs 0.2) against table_scene(), a JointJerk cost (not lowered) and a
    JointPos goal constraint."""
    n = 10
    start = [-0.9, 0.2, -1.2, -1.4, 0.3, -0.6, 0.1]
    end = [0.4, 0.3, -0.8, -0.9, -0.2, -0.4, 0.5]
    doc = {
        "basic_info": {"n_steps": n, "manip": "right_arm", "fixed_timesteps": [0]},
        "costs": [
            {"type": "joint_vel", "params": {"coeffs": [1] * 7, "targets": [0] * 7}},
            {"type": "collision", "name": "coll", "params": {
                "coeffs": 20, "dist_pen": 0.025, "evaluator_type": evaluator, "longest_valid_segment_length": 0.2}},
            {"type": "joint_jerk", "params": {"coeffs": [0.5] * 7, "targets": [0] * 7}},
        ],
        "constraints": [
            {"type": "joint_pos", "params": {"targets": end, "first_step": n - 1, "last_step": n - 1}},
        ],
        "init_info": {"type": "given_traj",
                      "data": [list(np.linspace(start, end, n)[i]) for i in range(n)]},
    }
    return json.dumps(doc)


# the obstacle of collision_jointjerk (THIP_PRIM_* record, world frame): a 0.1 m
# sphere near the arm's path -- 50-90 contacts per QP with the JSON's 0.5 m buffer,
# a size the generic path's dense-KKT QP solver runs in seconds
def table_scene():
    sph = np.zeros(16)
    sph[0] = 0  # SPHERE
    sph[1:5] = [0.8, -0.5, 1.2, 0.1]
    return sph[None, :]


# arm_around_table.urdf:71-94: table_link at (1.11, 0, 0.635) off base_footprint; its
# collision mesh Table.stl is 12 triangles spanning [-0.85, 0.85] x [-0.55, 0.55] x
# [-0.01, 0.0095] -- a box, so this primitive is the table exactly (data read from the
# mesh, vertex bounds rounded to float32 as stored)
def arm_around_table_scene():
    lo = np.array([-0.85000038, -0.55000061, -0.00999997])
    hi = np.array([0.8500005, 0.55000037, 0.00951481])
    table = np.zeros(16)
    table[0] = 1  # BOX
    table[1:4] = np.array([1.11, 0.0, 0.635]) + 0.5 * (lo + hi)
    table[4:13] = np.eye(3).reshape(9)
    table[13:16] = 0.5 * (hi - lo)
    return table[None, :]


def continuous_check_found(desc, x, scene, oracle_mod):
    """planning_unit.cpp:92-101, 143-148: checkTrajectory with a CONTINUOUS contact
    manager, collision margin 0 over the whole trajectory -- True when some step
    pair's cast touches the scene (distance < 0), evaluated by the oracle's
    CastCollisionEvaluator restatement (one cast per step pair)."""
    from trajopt_amd import abi
    from trajopt_amd.problems import Workload

    d = abi.ProblemDesc.from_buffer_copy(desc)
    d.coll_enabled, d.coll_continuous, d.coll_lvs = 1, 1, 1.7976931348623157e308
    d.coll_margin, d.coll_buffer = 0.0, 0.0
    d.coll_first_step, d.coll_last_step, d.coll_n_fixed = 0, d.n_steps - 1, 0
    x = np.asarray(x, dtype=float)
    w = Workload("check", d, x[None], np.zeros((1, max(d.n_cart, 0), 12)), np.asarray(scene)[None], x[None], None)
    return len(oracle_mod.collision_rows(w, 0, x)) > 0
