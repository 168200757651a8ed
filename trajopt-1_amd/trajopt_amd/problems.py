"""Synthetic batched workloads, deterministic per problem.

Each problem b draws from splitmix64 seeded with 20261015 + b:
  * a reference joint path q_ref(t) = q_mid + a * sin(2 pi t / (N-1) + phi),
    a ~ U(0.1, 0.4) * range, phi ~ U(0, 2 pi), clipped 0.05 inside the limits
    (continuous joints use [-pi, pi] as their range);
  * CartPose targets = FK(q_ref(t)) of the tool frame expressed in the chain
    root (torso_lift_link, static), i.e. the target-frame offset pose;
  * the initial trajectory: joint-interpolated q_ref(0) -> q_ref(N-1) plus
    N(0, 0.02) noise on interior steps; fixed_timesteps = [0].

Configs (BASELINE.json):
  A  7-DoF PR2 right arm, 10 steps, JointVel cost + one CartPose EQ constraint
     at the last step (target = FK(q_ref(mid-horizon)), a reaching problem).
  B  30 steps, JointVel cost + CartPose ABS costs at t = 1..29 (tracking).
  C  B + 10-primitive scene + LVS-discrete collision cost.
  J  joint-space planning (arm_around_table.json's term set without the
     collision cost, trajopt_common/data/config/arm_around_table.json:2-36):
     10 steps, JointVel cost, a JointPos EQ constraint at the last step with a
     per-problem goal q_ref(N-1), a JointPos EQ cost (coeff 0.1) on the
     interior steps toward the joint-range midpoint; the initial trajectory
     interpolates q_ref(0) -> goal + U(-goal_offset, goal_offset) like
     planning_unit.cpp's given_traj (which ends at the goal).  With an offset
     the goal starts violated; the constraint's exact violation is the
     *squared* error (trajectory_costs.cpp:162-171) while the model's is
     linear, so the trust region shrinks and the penalty loop runs out in the
     reference too (OPT_PENALTY_ITERATION_LIMIT).
  E  14-DoF PR2 dual arm (robots.pr2_both_arms: both arms as one joint group,
     a tree branching at torso_lift_link), 50 steps, JointVel cost, CartPose
     ABS costs for both tool frames at t = 1..49, 10-primitive scene near the
     reference path of either arm and the LVS_CONTINUOUS (swept-volume)
     collision cost on 2 x 14 arm spheres (BASELINE.json configs[4]).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import abi
from .robots import PR2_BOTH_TOOL_LINKS, PR2_TOOL_LINK, ROBOTS, _to44, chain_limits, fwd_kin, pr2_both_arms

SEED_BASE = 20261015
_MASK = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & _MASK

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & _MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
        return z ^ (z >> 31)

    def uniform(self, lo=0.0, hi=1.0) -> float:
        return lo + (hi - lo) * ((self.next() >> 11) * (1.0 / 9007199254740992.0))

    def normal(self, sigma=1.0) -> float:
        u1 = self.uniform()
        u2 = self.uniform()
        u1 = max(u1, 1e-300)
        return sigma * math.sqrt(-2.0 * math.log(u1)) * math.cos(2.0 * math.pi * u2)


@dataclass
class Workload:
    name: str
    desc: abi.ProblemDesc
    init: np.ndarray      # [B, N, D]
    targets: np.ndarray   # [B, n_cart, 12]
    scene: np.ndarray     # [B, n_prims, 16]
    q_ref: np.ndarray     # [B, N, D]
    jpos_targets: np.ndarray | None = None  # [B, n_jpos, D]; None: desc.jpos_targets for every problem

    @property
    def batch(self):
        return self.init.shape[0]

    @property
    def n_steps(self):
        return self.init.shape[1]

    @property
    def n_dof(self):
        return self.init.shape[2]

    def slice(self, lo, hi):
        return Workload(self.name, self.desc, self.init[lo:hi].copy(), self.targets[lo:hi].copy(),
                        self.scene[lo:hi].copy(), self.q_ref[lo:hi].copy(),
                        None if self.jpos_targets is None else self.jpos_targets[lo:hi].copy())


def _ref_path(rng: SplitMix64, lo, hi, types, n_steps):
    D = len(lo)
    q_lo = np.where(types == abi.JOINT_CONTINUOUS, -math.pi, lo)
    q_hi = np.where(types == abi.JOINT_CONTINUOUS, math.pi, hi)
    mid = 0.5 * (q_lo + q_hi)
    rng_ = q_hi - q_lo
    a = np.array([rng.uniform(0.1, 0.4) for _ in range(D)]) * rng_
    phi = np.array([rng.uniform(0.0, 2 * math.pi) for _ in range(D)])
    t = np.arange(n_steps)[:, None]
    q = mid[None, :] + a[None, :] * np.sin(2 * math.pi * t / (n_steps - 1) + phi[None, :])
    return np.clip(q, q_lo + 0.05, q_hi - 0.05)


def _pose12_in_root(chain, q, link):
    T = fwd_kin(chain, q)
    rel = np.linalg.inv(T[0]) @ T[link]
    return rel[:3, :].reshape(12)


def base_desc(n_steps: int, robot: str = "right_arm") -> abi.ProblemDesc:
    d = abi.ProblemDesc()
    d.n_steps = n_steps
    d.chain = ROBOTS[robot][0]()
    d.n_fixed = 1
    d.fixed_steps[0] = 0
    d.jv_enabled = 1
    d.jv_first_step = 0
    d.jv_last_step = -1
    for j in range(d.chain.n_dof):
        d.jv_coeffs[j] = 1.0
        d.jv_targets[j] = 0.0
    d.sqp = abi.default_sqp_params()
    d.osqp = abi.default_osqp_settings()
    return d


def _add_cart(d, k, step, is_cnt, tool=PR2_TOOL_LINK):
    d.cart_step[k] = step
    d.cart_is_cnt[k] = 1 if is_cnt else 0
    d.cart_source_link[k] = tool
    eye = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    for i in range(12):
        d.cart_source_offset[k][i] = eye[i]
    for i in range(3):
        d.cart_pos_coeffs[k][i] = 1.0
        d.cart_rot_coeffs[k][i] = 1.0


def make_workload(config: str, batch: int, first_problem: int = 0, n_steps: int | None = None,
                  goal_offset: float = 0.0, robot: str = "right_arm") -> Workload:
    """Synthetic workload of SURVEY.md §8d config A/B/C (or J: JointPos terms).  robot picks the chain
    (robots.ROBOTS); the default is the reference's PR2 right_arm group."""
    config = config.upper()
    if config == "HA":
        # config B plus joint_costs_unit's JointAcc cost on every step (coefficient 1,
        # zero targets): the fused kernel's waypoint-pair solve (bench.py --config HA)
        return with_joint_acc(make_workload("B", batch, first_problem=first_problem, n_steps=n_steps,
                                            goal_offset=goal_offset, robot=robot))
    if config == "A":
        N = n_steps or 10
    elif config in ("B", "C"):
        N = n_steps or 30
    elif config == "J":
        N = n_steps or 10
    elif config == "E":
        N = n_steps or 50
        robot = "both_arms"
    else:
        raise ValueError(f"unknown config {config}")
    d = base_desc(N, robot)
    chain = d.chain
    _, tool, link_offset = ROBOTS[robot]
    lo, hi, types = chain_limits(chain)
    D = chain.n_dof
    if config == "A":
        d.n_cart = 1
        _add_cart(d, 0, N - 1, True, tool)
    elif config == "J":
        d.n_cart = 0
    elif config == "E":
        # both tool frames at every step after the first (cost_infos order: left, then right, per step)
        d.n_cart = 2 * (N - 1)
        for k, t in enumerate(range(1, N)):
            for a, tl in enumerate(PR2_BOTH_TOOL_LINKS):
                _add_cart(d, 2 * k + a, t, False, tl)
    else:
        d.n_cart = N - 1
        for k, t in enumerate(range(1, N)):
            _add_cart(d, k, t, False, tool)
    if config == "C":
        from .scene import add_collision_model
        add_collision_model(d, link_offset)
    if config == "E":
        from .scene import add_collision_model
        add_collision_model(d, link_offsets=(0, PR2_BOTH_TOOL_LINKS[0]))
        d.coll_continuous = 1  # LVS_CONTINUOUS (CastCollisionEvaluator)
    jpos_targets = None
    if config == "J":
        q_lo = np.where(types == abi.JOINT_CONTINUOUS, -math.pi, lo)
        q_hi = np.where(types == abi.JOINT_CONTINUOUS, math.pi, hi)
        d.n_jpos = 2
        # term 0: JointPosEqCost on the interior steps toward the range midpoint
        # (costs are hatched before constraints, so a JSON problem lowers in this order)
        d.jpos_is_cnt[0] = 0
        d.jpos_first_step[0] = 1
        d.jpos_last_step[0] = N - 2
        # term 1: JointPosEqConstraint at the last step (goal, per problem)
        d.jpos_is_cnt[1] = 1
        d.jpos_first_step[1] = N - 1
        d.jpos_last_step[1] = N - 1
        for j in range(D):
            d.jpos_coeffs[0][j] = 0.1
            d.jpos_targets[0][j] = 0.5 * (q_lo[j] + q_hi[j])
            d.jpos_coeffs[1][j] = 1.0
        jpos_targets = np.zeros((batch, 2, D))

    init = np.zeros((batch, N, D))
    targets = np.zeros((batch, d.n_cart, 12))
    q_refs = np.zeros((batch, N, D))
    scene = np.zeros((batch, max(d.n_prims, 0), 16))
    for b in range(batch):
        rng = SplitMix64(SEED_BASE + first_problem + b)
        q_ref = _ref_path(rng, lo, hi, types, N)
        q_refs[b] = q_ref
        start, end = q_ref[0], q_ref[N - 1]
        if config == "J":
            end = q_ref[N - 1] + np.array([rng.uniform(-goal_offset, goal_offset) for _ in range(D)])
            jpos_targets[b, 0] = [d.jpos_targets[0][j] for j in range(D)]
            jpos_targets[b, 1] = q_ref[N - 1]
        for t in range(N):
            init[b, t] = start + (end - start) * (t / (N - 1))
        for t in range(1, N - 1):
            for j in range(D):
                init[b, t, j] += rng.normal(0.02)
        if config == "A":
            targets[b, 0] = _pose12_in_root(chain, q_ref[(N - 1) // 2], tool)
        else:
            for k in range(d.n_cart):
                targets[b, k] = _pose12_in_root(chain, q_ref[d.cart_step[k]], d.cart_source_link[k])
        if config in ("C", "E"):
            from .scene import make_scene
            scene[b] = make_scene(rng, chain, q_ref, d, link_offset)
    return Workload(config, d, init, targets, scene, q_refs, jpos_targets)


def make_reference_unit(name: str, batch: int = 1) -> Workload:
    """Problems of the reference's own unit tests, replicated `batch` times.

    joint_pos_eq    trajopt/test/joint_costs_unit.cpp:63-150 (equality_jointPos):
                    10 steps, STATIONARY init at the zero state, JointPos EQ
                    constraint x_0 = 0 (coeff 10), JointPos EQ cost x_t = -0.1
                    on every step (coeff 10); no JointVel, no fixed steps.
    joint_pos_ineq  joint_costs_unit.cpp:152-262 (inequality_jointPos): JointPos
                    constraint 0 with tolerances [-0.1, 0.2] on all steps, hinge
                    costs toward +0.5 / -0.5 (tolerance 0.01) on each half.
    joint_vel_ineq  joint_costs_unit.cpp:354-463 (inequality_jointVel): JointVel
                    constraint 0 with tolerances [-0.1, 0.2] on all steps
                    (JointVelIneqConstraint, a jvx term), hinge costs toward
                    +0.5 (tolerances [-0.01, 0]) on steps 0..4 (the jv_* term) and
                    -0.5 (+-0.01) on steps 5..9 (a jvx term).
    """
    N = 10
    d = base_desc(N)
    D = d.chain.n_dof
    d.n_fixed = 0
    d.jv_enabled = 0
    d.n_cart = 0
    if name == "joint_pos_eq":
        d.n_jpos = 2
        d.jpos_is_cnt[0], d.jpos_first_step[0], d.jpos_last_step[0] = 1, 0, 0
        d.jpos_is_cnt[1], d.jpos_first_step[1], d.jpos_last_step[1] = 0, 0, N - 1
        for j in range(D):
            d.jpos_coeffs[0][j] = 10.0
            d.jpos_targets[0][j] = 0.0
            d.jpos_coeffs[1][j] = 10.0
            d.jpos_targets[1][j] = -0.1
    elif name == "joint_pos_ineq":
        d.n_jpos = 3
        d.jpos_is_cnt[0], d.jpos_first_step[0], d.jpos_last_step[0] = 1, 0, N - 1
        d.jpos_is_cnt[1], d.jpos_first_step[1], d.jpos_last_step[1] = 0, 0, (N - 1) // 2
        d.jpos_is_cnt[2], d.jpos_first_step[2], d.jpos_last_step[2] = 0, (N - 1) // 2 + 1, N - 1
        for j in range(D):
            for k in range(3):
                d.jpos_coeffs[k][j] = 1.0
            d.jpos_lower_tols[0][j], d.jpos_upper_tols[0][j] = -0.1, 0.2
            d.jpos_targets[1][j], d.jpos_lower_tols[1][j], d.jpos_upper_tols[1][j] = 0.5, -0.01, 0.01
            d.jpos_targets[2][j], d.jpos_lower_tols[2][j], d.jpos_upper_tols[2][j] = -0.5, -0.01, 0.01
    elif name == "joint_vel_ineq":
        d.jv_enabled = 1
        d.jv_first_step, d.jv_last_step = 0, (N - 1) // 2
        d.n_jvx = 2
        d.jvx_is_cnt[0], d.jvx_first_step[0], d.jvx_last_step[0] = 0, (N - 1) // 2 + 1, N - 1
        d.jvx_is_cnt[1], d.jvx_first_step[1], d.jvx_last_step[1] = 1, 0, N - 1
        for j in range(D):
            d.jv_coeffs[j], d.jv_targets[j], d.jv_lower_tols[j], d.jv_upper_tols[j] = 1.0, 0.5, -0.01, 0.0
            d.jvx_coeffs[0][j], d.jvx_targets[0][j] = 1.0, -0.5
            d.jvx_lower_tols[0][j], d.jvx_upper_tols[0][j] = -0.01, 0.01
            d.jvx_coeffs[1][j], d.jvx_targets[1][j] = 1.0, 0.0
            d.jvx_lower_tols[1][j], d.jvx_upper_tols[1][j] = -0.1, 0.2
    else:
        raise ValueError(f"unknown reference unit {name}")
    init = np.zeros((batch, N, D))
    return Workload(name, d, init, np.zeros((batch, 0, 12)), np.zeros((batch, 0, 16)), init.copy())


def with_cart_tolerances(wl, pos=0.02, rot=0.1, axes=range(6)):
    """Give every CartPose term of wl a symmetric tolerance band (CartPoseErrCalculator
    with lower/upper tolerances, kinematic_terms.cpp:209-247): +-pos on x, y, z and
    +-rot on rx, ry, rz, for the components in axes (the others get a [0, 0] band)."""
    d = wl.desc
    for k in range(d.n_cart):
        d.cart_has_tol[k] = 1
        for i in range(6):
            b = (pos if i < 3 else rot) if i in axes else 0.0
            d.cart_lower_tol[k][i] = -b
            d.cart_upper_tol[k][i] = b
    return wl


def with_joint_acc(wl, coeff=1.0, target=0.0, first_step=0, last_step=-1):
    """Add a JointAccEqCost to every problem of wl (JointAccTermInfo, coefficient and
    target per joint, zero tolerances: joint_costs_unit.cpp's acceleration cost), with
    JointAccTermInfo::hatch's step clamping (problem_description.cpp:1412-1440).  On an
    even number of waypoints with 2 n_dof <= 16 the fused kernel lowers it (waypoint
    pairs, thip_jdt_fused); otherwise only the generic path runs it."""
    d = wl.desc
    N, D = d.n_steps, d.chain.n_dof
    f, l = first_step, last_step
    if l <= -1:
        l = N - 1
    if N - 3 <= f:
        f = N - 3
    if N - 1 <= l:
        l = N - 1
    if l == f:
        l += 2
    if l < f:
        f, l = l, f
    k = d.n_jdt
    d.jdt_order[k] = 2
    d.jdt_is_cnt[k] = 0
    d.jdt_first_step[k] = f
    d.jdt_last_step[k] = l
    for j in range(D):
        d.jdt_coeffs[k][j] = coeff
        d.jdt_targets[k][j] = target
        d.jdt_upper_tols[k][j] = 0.0
        d.jdt_lower_tols[k][j] = 0.0
    d.n_jdt = k + 1
    return wl


def with_dynamic_target(wl, link=3):
    """Make every CartPose term of wl a DynamicCartPose term (both frames active,
    DynamicCartPoseTermInfo, problem_description.cpp:683-842): the target is chain link
    `link`, and each problem's target offset (in that link's frame) is the source
    frame's pose relative to it along the problem's reference path, so the term holds
    the tool at a fixed pose relative to the arm link."""
    d = wl.desc
    for k in range(d.n_cart):
        d.cart_target_link[k] = link
    for b in range(wl.batch):
        for k in range(d.n_cart):
            T = fwd_kin(d.chain, wl.q_ref[b, d.cart_step[k]])
            src = T[d.cart_source_link[k]] @ _to44(list(d.cart_source_offset[k]))
            rel = np.linalg.inv(T[link]) @ src
            wl.targets[b, k] = rel[:3, :].reshape(12)
    return wl


def add_coll_pair(desc, link, other, margin, coeff, term=0):
    """One CollisionTermInfo "pairs" entry (problem_description.cpp:1686-1719)
    in the descriptor: robot link `link` against scene primitive `other` (>= 0)
    or robot link `-1 - other`, with its own margin (dist_pen) and coefficient."""
    k = desc.n_coll_pairs
    assert k < abi.MAX_COLL_PAIRS
    e = desc.coll_pairs[k]
    e.term, e.link, e.other, e.margin, e.coeff = term, link, other, margin, coeff
    desc.n_coll_pairs = k + 1
    return desc


def with_pair_data(wl, self_pairs=True):
    """Config C with per link-pair data on the collision term, on the pairs
    config C's contacts concentrate on (the wrist links against primitives 5
    and 8, the upper arm against 9, the forearm against 7): a wider margin and
    heavier coefficient, a zero coefficient (that pair's contacts are dropped),
    a narrower margin, and -- when the group has self-collision pairs -- one
    self pair with its own data."""
    d = wl.desc
    links = sorted({d.sphere_link[s] for s in range(d.n_spheres)})
    add_coll_pair(d, links[-1], 5, 0.06, 35.0)           # replaced below (insert_or_assign)
    add_coll_pair(d, links[-1], 8, 0.0, 0.0)             # dropped (hasZeroCoeff)
    add_coll_pair(d, links[2], 9, 0.01, 4.0)             # narrower, lighter
    add_coll_pair(d, links[4], 7, 0.04, 60.0)
    add_coll_pair(d, links[-1], 5, 0.05, 30.0)           # the wrist against primitive 5: wider, heavier
    if self_pairs and d.n_self_pairs > 0:
        a, b = d.self_pair[0][0], d.self_pair[0][1]
        add_coll_pair(d, b, -1 - a, 0.03, 12.0)          # unordered: (b, a) names the pair (a, b)
    return wl


def pair_overrides(desc, term=0):
    """{(link, other): (margin, coeff)} of a term's pair entries, last entry
    winning; `other` is a primitive index or -1 - link (both orders listed)."""
    out = {}
    for k in range(desc.n_coll_pairs):
        e = desc.coll_pairs[k]
        if e.term != term:
            continue
        out[(e.link, e.other)] = (e.margin, e.coeff)
        if e.other < 0:
            out[(-1 - e.other, -1 - e.link)] = (e.margin, e.coeff)
    return out
