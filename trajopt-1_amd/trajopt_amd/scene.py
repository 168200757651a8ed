"""Config C collision model and synthetic scenes.

Robot collision model: 2 spheres on each of the 7 moving links of the PR2
right arm (radii 0.06-0.09 m), a committed fixture (PR2_ARM_SPHERES).  Scene:
10 primitives per problem, 4 spheres (r ~ U(0.05, 0.12)), 3 boxes (half
extents ~ U(0.04, 0.1), random orientation) and 3 capsules (r ~ U(0.03,
0.06), half length ~ U(0.05, 0.15)), each placed next to a robot sphere of
q_ref(t) for a random waypoint t, in a random direction, with a clearance of
U(0.08, 0.2) m between the robot sphere and the primitive's bounding sphere
(SURVEY.md's "offset by U(0.08, 0.2) m" read as surface clearance).  A
placement is redrawn (at most 64 times, same splitmix64 stream) until every
robot sphere at every waypoint of q_ref is farther than the contact distance
(dist_pen + buffer = 0.075 m) from it: the reference path is collision free,
contacts come from the interpolated initial trajectory deviating toward the
obstacles, and only part of the problems start in collision.  Robot self-collision: the arm link pairs pr2.srdf's allowed-collision
matrix leaves enabled (arm_self_pairs).  The collision term is the reference's LVS_DISCRETE cost with
dist_pen 0.025, coeffs 20, safety_margin_buffer 0.05, lvs 0.05 and
fixed_steps [0] (CollisionTermInfo, problem_description.cpp:1636-1733).
Primitive record layout: include/trajopt_hip.h (THIP_PRIM_*).
"""
from __future__ import annotations

import math

import numpy as np

from . import abi
from .robots import fwd_kin

# (link index, center in the link frame, radius); link indices of
# robots.pr2_right_arm(): 1 shoulder_pan, 2 shoulder_lift, 3 upper_arm_roll,
# 5 elbow_flex, 6 forearm_roll, 8 wrist_flex, 9 wrist_roll
PR2_ARM_SPHERES = [
    (1, (0.0, 0.0, 0.0), 0.09),
    (1, (0.1, 0.0, 0.0), 0.08),
    (2, (0.0, 0.0, 0.0), 0.08),
    (2, (0.1, 0.0, 0.0), 0.07),
    (3, (0.15, 0.0, 0.0), 0.07),
    (3, (0.3, 0.0, 0.0), 0.07),
    (5, (0.0, 0.0, 0.0), 0.07),
    (5, (0.08, 0.0, 0.0), 0.06),
    (6, (0.12, 0.0, 0.0), 0.06),
    (6, (0.24, 0.0, 0.0), 0.06),
    (8, (0.0, 0.0, 0.0), 0.06),
    (8, (0.08, 0.0, 0.0), 0.06),
    (9, (0.12, 0.0, 0.0), 0.06),
    (9, (0.18, 0.0, 0.0), 0.06),
]

N_PRIMS = 10
MARGIN, COEFF, BUFFER, LVS = 0.025, 20.0, 0.05, 0.05

# names of the sphere-carrying links of PR2_ARM_SPHERES (without the l_ / r_ prefix)
ARM_SPHERE_LINK_NAMES = {1: "shoulder_pan_link", 2: "shoulder_lift_link", 3: "upper_arm_roll_link",
                         5: "elbow_flex_link", 6: "forearm_roll_link", 8: "wrist_flex_link", 9: "wrist_roll_link"}
# pr2.srdf <disable_collisions> between those links (trajopt_common/data/pr2.srdf:752-1036): the
# allowed-collision matrix.  The pairs it leaves enabled are tested as robot self-collision: each
# arm's shoulder_pan vs its wrist links, and 33 of the 49 left-vs-right pairs.
PR2_ARM_ACM = frozenset(frozenset(p) for p in [
    ("l_elbow_flex_link", "l_forearm_roll_link"), ("l_elbow_flex_link", "l_shoulder_lift_link"),
    ("l_elbow_flex_link", "l_shoulder_pan_link"), ("l_elbow_flex_link", "l_upper_arm_roll_link"),
    ("l_elbow_flex_link", "l_wrist_flex_link"), ("l_elbow_flex_link", "l_wrist_roll_link"),
    ("l_elbow_flex_link", "r_shoulder_lift_link"), ("l_elbow_flex_link", "r_shoulder_pan_link"),
    ("l_elbow_flex_link", "r_upper_arm_roll_link"), ("l_forearm_roll_link", "l_shoulder_lift_link"),
    ("l_forearm_roll_link", "l_shoulder_pan_link"), ("l_forearm_roll_link", "l_upper_arm_roll_link"),
    ("l_forearm_roll_link", "l_wrist_flex_link"), ("l_forearm_roll_link", "l_wrist_roll_link"),
    ("l_forearm_roll_link", "r_shoulder_lift_link"), ("l_forearm_roll_link", "r_shoulder_pan_link"),
    ("l_forearm_roll_link", "r_upper_arm_roll_link"), ("l_shoulder_lift_link", "l_shoulder_pan_link"),
    ("l_shoulder_lift_link", "l_upper_arm_roll_link"), ("l_shoulder_lift_link", "l_wrist_flex_link"),
    ("l_shoulder_lift_link", "l_wrist_roll_link"), ("l_shoulder_lift_link", "r_elbow_flex_link"),
    ("l_shoulder_lift_link", "r_forearm_roll_link"), ("l_shoulder_lift_link", "r_shoulder_lift_link"),
    ("l_shoulder_lift_link", "r_upper_arm_roll_link"), ("l_shoulder_pan_link", "l_upper_arm_roll_link"),
    ("l_shoulder_pan_link", "r_elbow_flex_link"), ("l_shoulder_pan_link", "r_forearm_roll_link"),
    ("l_upper_arm_roll_link", "l_wrist_flex_link"), ("l_upper_arm_roll_link", "l_wrist_roll_link"),
    ("l_upper_arm_roll_link", "r_elbow_flex_link"), ("l_upper_arm_roll_link", "r_forearm_roll_link"),
    ("l_upper_arm_roll_link", "r_shoulder_lift_link"), ("l_upper_arm_roll_link", "r_upper_arm_roll_link"),
    ("l_wrist_flex_link", "l_wrist_roll_link"), ("r_elbow_flex_link", "r_forearm_roll_link"),
    ("r_elbow_flex_link", "r_shoulder_lift_link"), ("r_elbow_flex_link", "r_shoulder_pan_link"),
    ("r_elbow_flex_link", "r_upper_arm_roll_link"), ("r_elbow_flex_link", "r_wrist_flex_link"),
    ("r_elbow_flex_link", "r_wrist_roll_link"), ("r_forearm_roll_link", "r_shoulder_lift_link"),
    ("r_forearm_roll_link", "r_shoulder_pan_link"), ("r_forearm_roll_link", "r_upper_arm_roll_link"),
    ("r_forearm_roll_link", "r_wrist_flex_link"), ("r_forearm_roll_link", "r_wrist_roll_link"),
    ("r_shoulder_lift_link", "r_shoulder_pan_link"), ("r_shoulder_lift_link", "r_upper_arm_roll_link"),
    ("r_shoulder_lift_link", "r_wrist_flex_link"), ("r_shoulder_lift_link", "r_wrist_roll_link"),
    ("r_shoulder_pan_link", "r_upper_arm_roll_link"), ("r_upper_arm_roll_link", "r_wrist_flex_link"),
    ("r_upper_arm_roll_link", "r_wrist_roll_link"), ("r_wrist_flex_link", "r_wrist_roll_link"),
])


def arm_self_pairs(link_offsets=(0,), sides=("r_",)):
    """Self-collision link pairs of the arms (ascending link index, the lower first): every pair of
    sphere-carrying links the ACM does not disable -- what the host front door derives from the
    environment for the same group (problem_description.cpp CollisionTermInfo::hatch)."""
    links = sorted((link + off, side + name) for off, side in zip(link_offsets, sides)
                   for link, name in ARM_SPHERE_LINK_NAMES.items())
    return [(la, lb) for a, (la, na) in enumerate(links) for lb, nb in links[a + 1:]
            if frozenset((na, nb)) not in PR2_ARM_ACM]


def arm_spheres(link_offsets=(0,)):
    """PR2_ARM_SPHERES once per arm, the arm's links shifted by its offset (both_arms: the left arm at
    links 1-11, the right arm at 12-22, offsets (0, 11))."""
    return [(link + off, c, r) for off in link_offsets for link, c, r in PR2_ARM_SPHERES]


def desc_spheres(d: abi.ProblemDesc):
    """The (link, center, radius) spheres of a descriptor."""
    return [(d.sphere_link[s], tuple(d.sphere_center[s][i] for i in range(3)), d.sphere_radius[s])
            for s in range(d.n_spheres)]


def add_collision_model(d: abi.ProblemDesc, link_offset: int = 0, link_offsets=None):
    """LVS_DISCRETE collision cost over all step pairs, step 0 fixed.  link_offset shifts the sphere links
    for chains with extra links before the arm (robots.ROBOTS); link_offsets lists one offset per arm."""
    d.coll_enabled = 1
    d.coll_is_cnt = 0
    d.coll_first_step = 0
    d.coll_last_step = d.n_steps - 1
    d.coll_n_fixed = 1
    d.coll_fixed_steps[0] = 0
    d.coll_margin = MARGIN
    d.coll_coeff = COEFF
    d.coll_buffer = BUFFER
    d.coll_lvs = LVS
    spheres = arm_spheres(link_offsets if link_offsets is not None else (link_offset,))
    d.n_spheres = len(spheres)
    for s, (link, c, r) in enumerate(spheres):
        d.sphere_link[s] = link
        for i in range(3):
            d.sphere_center[s][i] = c[i]
        d.sphere_radius[s] = r
    d.n_prims = N_PRIMS
    # both_arms: left arm links first (l_), then the right arm (r_); one arm: the right arm
    pairs = (arm_self_pairs(link_offsets, ("l_", "r_")) if link_offsets is not None
             else arm_self_pairs((link_offset,), ("r_",)))
    d.n_self_pairs = len(pairs)
    for k, (a, b) in enumerate(pairs):
        d.self_pair[k][0], d.self_pair[k][1] = a, b


def _unit(rng):
    v = np.array([rng.normal(), rng.normal(), rng.normal()])
    n = np.linalg.norm(v)
    return v / n if n > 1e-12 else np.array([0.0, 0.0, 1.0])


def _rotation(rng):
    q = np.array([rng.normal(), rng.normal(), rng.normal(), rng.normal()])
    q = q / max(np.linalg.norm(q), 1e-12)
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def sphere_centers(chain, q, link_offset: int = 0, spheres=None):
    """World centers of the robot spheres at joint values q (spheres: (link, center, radius) with chain
    link indices; default PR2_ARM_SPHERES shifted by link_offset)."""
    T = fwd_kin(chain, q)
    if spheres is None:
        spheres = arm_spheres((link_offset,))
    return np.array([T[link][:3, :3] @ np.array(c) + T[link][:3, 3] for link, c, _ in spheres])


def make_scene(rng, chain, q_ref, d, link_offset: int = 0) -> np.ndarray:
    """10 primitive records near the reference path of one problem (near the descriptor's robot spheres)."""
    N = q_ref.shape[0]
    prims = np.zeros((N_PRIMS, 16))
    spheres = desc_spheres(d)
    path = [sphere_centers(chain, q_ref[t], spheres=spheres) for t in range(N)]
    radii = [r for _, _, r in spheres]
    for k in range(N_PRIMS):
        for _attempt in range(64):
            rec = _draw_prim(rng, k, N, path, radii)
            if all(sphere_prim_distance(c[s], radii[s], rec)[0] > MARGIN + BUFFER
                   for c in path for s in range(len(radii))):
                break
        prims[k] = rec
    return prims


def _draw_prim(rng, k, N, path, radii):
    rec = np.zeros(16)
    if True:  # one placement draw
        t = min(int(rng.uniform() * N), N - 1)
        s = min(int(rng.uniform() * len(radii)), len(radii) - 1)
        anchor = path[t][s]
        direction = _unit(rng)
        if k < 4:
            radius = rng.uniform(0.05, 0.12)
            bound = radius
        elif k < 7:
            R = _rotation(rng)
            h = np.array([rng.uniform(0.04, 0.1) for _ in range(3)])
            bound = float(np.linalg.norm(h))
        else:
            axis = _unit(rng)
            half = rng.uniform(0.05, 0.15)
            cap_r = rng.uniform(0.03, 0.06)
            bound = half + cap_r
        center = anchor + direction * (radii[s] + bound + rng.uniform(0.08, 0.2))
        if k < 4:
            rec[0] = abi.PRIM_SPHERE
            rec[1:4] = center
            rec[4] = radius
        elif k < 7:
            rec[0] = abi.PRIM_BOX
            rec[1:4] = center
            rec[4:13] = R.reshape(9)
            rec[13:16] = h
        else:
            rec[0] = abi.PRIM_CAPSULE
            rec[1:4] = center - half * axis
            rec[4:7] = center + half * axis
            rec[7] = cap_r
    return rec


def sphere_prim_distance(c, r, prim):
    """numpy restatement of the closed-form signed distance (test helper)."""
    c = np.asarray(c, dtype=float)
    typ = int(prim[0])

    def sph(s, rs):
        v = s - c
        L = math.sqrt(float(v @ v))
        n = v / L if L >= 1e-12 else np.array([0.0, 0.0, 1.0])
        return L - r - rs, n

    if typ == abi.PRIM_SPHERE:
        return sph(prim[1:4], prim[4])
    if typ == abi.PRIM_CAPSULE:
        a, b = prim[1:4], prim[4:7]
        ab = b - a
        den = float(ab @ ab)
        t = float((c - a) @ ab) / den if den > 1e-24 else 0.0
        t = min(max(t, 0.0), 1.0)
        return sph(a + t * ab, prim[7])
    ctr, R, h = prim[1:4], prim[4:13].reshape(3, 3), prim[13:16]
    cl = R.T @ (c - ctr)
    if np.any(np.abs(cl) > h):
        ql = np.clip(cl, -h, h)
        vl = ql - cl
        L = float(np.linalg.norm(vl))
        return L - r, R @ vl / L
    depth = h - np.abs(cl)
    k = int(np.argmin(depth))
    sgn = -1.0 if cl[k] < 0 else 1.0
    return -depth[k] - r, -sgn * R[:, k]
