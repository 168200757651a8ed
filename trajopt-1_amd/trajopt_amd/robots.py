"""Robot kinematic chains used by the synthetic workloads.

PR2 right arm: the reference's `right_arm` group (chain torso_lift_link ->
r_gripper_tool_frame, trajopt_common/data/pr2.srdf:15-17) with the joint data
of trajopt_common/data/arm_around_table.urdf (shoulder_pan 1479-1485,
shoulder_lift 1513-1523, upper_arm_roll 1545-1550, elbow_flex 1702-1712,
forearm_roll 1655-1664, wrist_flex 1779-1788, wrist_roll 1811-1820, tool
1908-1911; base chain base_footprint->base_link 121-124, torso 735-744 with
the torso joint at 0).  Continuous joints get +-4 pi variable bounds.

PR2 both arms (config E, 14 DoF): the reference's left_arm and right_arm
groups (pr2.srdf:12-17) as one joint group branching at torso_lift_link, left
arm joints first (l_shoulder_pan 2396-2402, l_shoulder_lift 2430-2436,
l_upper_arm_roll 2462-2468, l_elbow_flex 2619-2625, l_forearm_roll
2572-2578, l_wrist_flex 2696-2702, l_wrist_roll 2728-2733, tool 2825-2828:
the right arm mirrored in y, with its own limits).  The reference's SRDF has
no 14-joint group (full_body adds the torso, pr2.srdf:54-70), so the group is
named "both_arms" here.
"""
from __future__ import annotations

import math

import numpy as np

from .abi import JOINT_CONTINUOUS, JOINT_FIXED, JOINT_PRISMATIC, JOINT_REVOLUTE, Chain


def _pose(xyz=(0.0, 0.0, 0.0)):
    p = np.zeros(12)
    p[0] = p[5] = p[10] = 1.0
    p[3], p[7], p[11] = xyz
    return p


# (name, type, origin xyz, axis, (lower, upper))
PR2_RIGHT_ARM = [
    ("r_shoulder_pan_joint", JOINT_REVOLUTE, (0.0, -0.188, 0.0), (0, 0, 1), (-2.2853981634, 0.714601836603)),
    ("r_shoulder_lift_joint", JOINT_REVOLUTE, (0.1, 0.0, 0.0), (0, 1, 0), (-0.5236, 1.3963)),
    ("r_upper_arm_roll_joint", JOINT_REVOLUTE, (0.0, 0.0, 0.0), (1, 0, 0), (-3.9, 0.8)),
    ("r_upper_arm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("r_elbow_flex_joint", JOINT_REVOLUTE, (0.4, 0.0, 0.0), (0, 1, 0), (-2.3213, 0.0)),
    ("r_forearm_roll_joint", JOINT_CONTINUOUS, (0.0, 0.0, 0.0), (1, 0, 0), (-4 * math.pi, 4 * math.pi)),
    ("r_forearm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("r_wrist_flex_joint", JOINT_REVOLUTE, (0.321, 0.0, 0.0), (0, 1, 0), (-2.18, 0.0)),
    ("r_wrist_roll_joint", JOINT_CONTINUOUS, (0.0, 0.0, 0.0), (1, 0, 0), (-4 * math.pi, 4 * math.pi)),
    ("r_gripper_palm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("r_gripper_tool_joint", JOINT_FIXED, (0.18, 0.0, 0.0), None, None),
]
PR2_LEFT_ARM = [
    ("l_shoulder_pan_joint", JOINT_REVOLUTE, (0.0, 0.188, 0.0), (0, 0, 1), (-0.714601836603, 2.2853981634)),
    ("l_shoulder_lift_joint", JOINT_REVOLUTE, (0.1, 0.0, 0.0), (0, 1, 0), (-0.5236, 1.3963)),
    ("l_upper_arm_roll_joint", JOINT_REVOLUTE, (0.0, 0.0, 0.0), (1, 0, 0), (-0.8, 3.9)),
    ("l_upper_arm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("l_elbow_flex_joint", JOINT_REVOLUTE, (0.4, 0.0, 0.0), (0, 1, 0), (-2.3213, 0.0)),
    ("l_forearm_roll_joint", JOINT_CONTINUOUS, (0.0, 0.0, 0.0), (1, 0, 0), (-4 * math.pi, 4 * math.pi)),
    ("l_forearm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("l_wrist_flex_joint", JOINT_REVOLUTE, (0.321, 0.0, 0.0), (0, 1, 0), (-2.18, 0.0)),
    ("l_wrist_roll_joint", JOINT_CONTINUOUS, (0.0, 0.0, 0.0), (1, 0, 0), (-4 * math.pi, 4 * math.pi)),
    ("l_gripper_palm_joint", JOINT_FIXED, (0.0, 0.0, 0.0), None, None),
    ("l_gripper_tool_joint", JOINT_FIXED, (0.18, 0.0, 0.0), None, None),
]
# world pose of torso_lift_link: base_footprint -> base_link (0,0,0.051) -> torso (-0.05,0,0.739675), q_torso = 0
PR2_TORSO_WORLD = (-0.05, 0.0, 0.051 + 0.739675)
PR2_TOOL_LINK = 11  # r_gripper_tool_frame
# torso_lift_joint (arm_around_table.urdf:735-745): prismatic along z, base_link -> torso_lift_link
PR2_TORSO_JOINT = ("torso_lift_joint", JOINT_PRISMATIC, (-0.05, 0.0, 0.739675), (0, 0, 1), (0.0, 0.33))
PR2_BASE_LINK_WORLD = (0.0, 0.0, 0.051)

# Robots the synthetic workloads can use: name -> (chain builder, tool link, link offset of the arm links).
# "right_arm" is the reference's right_arm group (7 DoF); "torso_right_arm" prepends the prismatic torso
# joint (8 DoF, the full_body group's torso + right arm joints, pr2.srdf:51-70); "right_arm_6dof" is a
# synthetic 6-DoF variant with r_wrist_roll_joint held fixed at 0.


def pr2_right_arm() -> Chain:
    return _chain(PR2_TORSO_WORLD, PR2_RIGHT_ARM)


def pr2_torso_right_arm() -> Chain:
    return _chain(PR2_BASE_LINK_WORLD, [PR2_TORSO_JOINT] + PR2_RIGHT_ARM)


def pr2_both_arms() -> Chain:
    """14-DoF tree: links 1-11 the left arm (l_gripper_tool_frame = 11), links
    12-22 the right arm (r_gripper_tool_frame = 22), both off the root."""
    return _chain(PR2_TORSO_WORLD, PR2_LEFT_ARM + PR2_RIGHT_ARM,
                  parents=[0] + list(range(1, 11)) + [0] + list(range(12, 22)))


def pr2_right_arm_6dof() -> Chain:
    joints = [(n, JOINT_FIXED, xyz, None, None) if n == "r_wrist_roll_joint" else (n, t, xyz, ax, lim)
              for n, t, xyz, ax, lim in PR2_RIGHT_ARM]
    return _chain(PR2_TORSO_WORLD, joints)


ROBOTS = {
    "right_arm": (pr2_right_arm, PR2_TOOL_LINK, 0),
    "torso_right_arm": (pr2_torso_right_arm, PR2_TOOL_LINK + 1, 1),
    "right_arm_6dof": (pr2_right_arm_6dof, PR2_TOOL_LINK, 0),
    "both_arms": (pr2_both_arms, 22, 0),  # config E; its CartPose terms use both tool links
}
# both_arms (config E): tool links of the two arms
PR2_BOTH_TOOL_LINKS = (11, 22)


def _chain(base_xyz, joints, parents=None) -> Chain:
    """Joint k (1-based) attaches link k to link parents[k - 1] (default k - 1)."""
    c = Chain()
    c.n_links = len(joints) + 1
    c.is_tree = 0 if parents is None else 1
    for k in range(1, c.n_links):
        c.parent[k] = (k - 1) if parents is None else parents[k - 1]
    base = _pose(base_xyz)
    for i in range(12):
        c.base_pose[i] = base[i]
    dof = 0
    for k, (_, jtype, xyz, axis, lim) in enumerate(joints, start=1):
        c.joint_type[k] = jtype
        o = _pose(xyz)
        for i in range(12):
            c.joint_origin[k][i] = o[i]
        if jtype == JOINT_FIXED:
            c.joint_dof[k] = -1
        else:
            c.joint_dof[k] = dof
            for i in range(3):
                c.joint_axis[k][i] = axis[i]
            c.lower[dof], c.upper[dof] = lim
            dof += 1
    c.n_dof = dof
    c.joint_dof[0] = -1
    return c


def chain_limits(c: Chain):
    lo = np.array([c.lower[i] for i in range(c.n_dof)])
    hi = np.array([c.upper[i] for i in range(c.n_dof)])
    types = []
    for k in range(1, c.n_links):
        if c.joint_type[k] != JOINT_FIXED:
            types.append(c.joint_type[k])
    return lo, hi, np.array(types)


# ---------------------------------------------------------------- numpy FK
def _axis_angle(axis, angle):
    """Eigen AngleAxis::toRotationMatrix."""
    ax = np.asarray(axis, dtype=float)
    s, c = math.sin(angle), math.cos(angle)
    sa = s * ax
    ca = (1 - c) * ax
    R = np.zeros((3, 3))
    t = ca[0] * ax[1]
    R[0, 1] = t - sa[2]
    R[1, 0] = t + sa[2]
    t = ca[0] * ax[2]
    R[0, 2] = t + sa[1]
    R[2, 0] = t - sa[1]
    t = ca[1] * ax[2]
    R[1, 2] = t - sa[0]
    R[2, 1] = t + sa[0]
    R[0, 0] = ca[0] * ax[0] + c
    R[1, 1] = ca[1] * ax[1] + c
    R[2, 2] = ca[2] * ax[2] + c
    return R


def _to44(p12):
    T = np.eye(4)
    T[:3, :] = np.asarray(p12, dtype=float).reshape(3, 4)
    return T


def fwd_kin(c: Chain, q):
    """World pose (4x4) of every link at joint values q (host-side helper for
    data generation only)."""
    T = [_to44(list(c.base_pose))]
    for k in range(1, c.n_links):
        t = T[c.parent[k]] @ _to44(list(c.joint_origin[k]))
        jt = c.joint_type[k]
        if jt in (JOINT_REVOLUTE, JOINT_CONTINUOUS):
            M = np.eye(4)
            M[:3, :3] = _axis_angle(list(c.joint_axis[k]), q[c.joint_dof[k]])
            t = t @ M
        elif jt != JOINT_FIXED:
            M = np.eye(4)
            M[:3, 3] = np.asarray(list(c.joint_axis[k])) * q[c.joint_dof[k]]
            t = t @ M
        T.append(t)
    return T
