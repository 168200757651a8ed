"""The reference's joint-term unit problems (trajopt/test/joint_costs_unit.cpp)
as TrajOptRequest JSON on the PR2 right_arm, plus jerk, TotalTime and fixed-dof
problems, shared by
tests/test_sco_surface.py (oracle KATs) and tests/test_gpu_sco.py (GPU parity).

Each entry: name -> (json text, check(traj) -> list of failed assertions).  The
reference builds its ProblemConstructionInfo in code; cost_infos hatch before
cnt_infos (problem_description.cpp:414-546), which the JSON "costs" /
"constraints" sections reproduce.  STATIONARY init at the environment's zero
state, 10 steps, no fixed timesteps.
"""
import json

import numpy as np

STEPS = 10


def _term(kind, coeff, targ, first, last, lower=None, upper=None, name=None):
    p = {"coeffs": [coeff] * 7, "targets": [targ] * 7, "first_step": first, "last_step": last}
    if lower is not None:
        p["lower_tols"] = [lower] * 7
        p["upper_tols"] = [upper] * 7
    return {"type": kind, "name": name or kind, "params": p}


def _doc(costs, cnts, basic=None, init=None):
    bi = {"n_steps": STEPS, "manip": "right_arm"}
    bi.update(basic or {})
    ii = {"type": "stationary"}
    ii.update(init or {})
    return json.dumps({"basic_info": bi, "costs": costs, "constraints": cnts, "init_info": ii})


def _timed(term):
    """The term with TT_USE_TIME (the JSON entry's "use_time", problem_description.cpp:173-215)."""
    return dict(term, use_time=True)


def _vel_time(traj):
    """vel_i = (x[i+1] - x[i]) * dt[i+1] over the joint columns (joint_costs_unit.cpp:533-548):
    the reference's dt column holds the inverse time step."""
    t = np.asarray(traj)
    return (t[1:, :-1] - t[:-1, :-1]) * t[1:, -1:]


def _diff(traj, order):
    d = np.asarray(traj)
    for _ in range(order):
        d = d[1:] - d[:-1]
    return d


def _equality(kind, order):
    """equality_joint{Pos,Vel,Acc}: a conflicting single-step constraint to 0
    (coeff 10) and a cost to cost_targ on every step."""
    cost_targ = -0.1 if order == 0 else 0.1
    text = _doc([_term(kind, 10.0, cost_targ, 0, STEPS - 1, name=kind + "_all")],
                [_term(kind, 10.0, 0.0, 0, 0, name=kind + "_single")])

    def check(traj):
        d = _diff(traj, order)
        bad = []
        if np.abs(d[0]).max() > 1e-4:
            bad.append(f"constraint: max |d0| {np.abs(d[0]).max():.2e}")
        if np.abs(d[1:] - cost_targ).max() > 0.01:
            bad.append(f"cost: max |d - {cost_targ}| {np.abs(d[1:] - cost_targ).max():.2e}")
        return bad

    return text, check


def _inequality(kind, order):
    """inequality_joint{Pos,Vel,Acc}: a [-0.1, 0.2] band constraint on every step
    and conflicting +-0.5 tolerance costs on the two halves."""
    lower_tol, upper_tol = -0.1, 0.2
    half = (STEPS - 1) // 2
    cost1_up = 0.0 if kind == "joint_vel" else 0.01  # inequality_jointVel's jv2 upper tolerance is 0
    text = _doc([_term(kind, 1.0, 0.5, 0, half, -0.01, cost1_up, kind + "_targ_1"),
                 _term(kind, 1.0, -0.5, half + 1, STEPS - 1, -0.01, 0.01, kind + "_targ_2")],
                [_term(kind, 1.0, 0.0, 0, STEPS - 1, lower_tol, upper_tol, kind + "_limits")])

    def check(traj):
        d = _diff(traj, order)
        bad = []
        if d.max() >= upper_tol + 1e-4 or d.min() <= lower_tol - 1e-4:
            bad.append(f"band: d in [{d.min():.4f}, {d.max():.4f}]")
        return bad

    return text, check


def _jerk():
    """A jerk cost to 0.02 over the trajectory with a zero-jerk constraint from the
    first step (JointJerkTermInfo, problem_description.cpp:1514-1634)."""
    text = _doc([_term("joint_jerk", 10.0, 0.02, 0, STEPS - 1, name="jerk_all")],
                [_term("joint_jerk", 10.0, 0.0, 0, 0, name="jerk_single")])

    def check(traj):
        # last_step == first_step becomes first + 4: the constraint covers the jerks at steps 0 and 1
        d = _diff(traj, 3)
        bad = []
        if np.abs(d[:2]).max() > 1e-4:
            bad.append(f"constraint: max |j0|, |j1| {np.abs(d[:2]).max():.2e}")
        if np.abs(d[2:] - 0.02).max() > 0.01:
            bad.append(f"cost: max |j - 0.02| {np.abs(d[2:] - 0.02).max():.2e}")
        return bad

    return text, check


def _equality_vel_time():
    """equality_jointVel_time (joint_costs_unit.cpp:465-551): a zero-velocity
    constraint on the first step and a cost to 0.1 on every step, with the dt
    column in [0.01234, 1.5678]."""
    dt_lower, dt_upper = 0.01234, 1.5678
    text = _doc([_timed(_term("joint_vel", 1.0, 0.1, 0, STEPS - 1, name="joint_vel_all"))],
                [_timed(_term("joint_vel", 1.0, 0.0, 0, 0, 0.0, 0.0, name="joint_vel_single"))],
                basic={"use_time": True, "dt_lower_lim": dt_lower, "dt_upper_lim": dt_upper})

    def check(traj):
        v, dt = _vel_time(traj), np.asarray(traj)[:, -1]
        bad = []
        if np.abs(v[0]).max() > 1e-4:
            bad.append(f"constraint: max |v0| {np.abs(v[0]).max():.2e}")
        if dt[1:-1].max() > dt_upper or dt[1:-1].min() < dt_lower:
            bad.append(f"dt limits: [{dt.min():.4f}, {dt.max():.4f}]")
        if np.abs(v[1:] - 0.1).max() > 0.01:
            bad.append(f"cost: max |v - 0.1| {np.abs(v[1:] - 0.1).max():.2e}")
        return bad

    return text, check


def _inequality_vel_time():
    """inequality_jointVel_time (joint_costs_unit.cpp:562-665): a [-0.1, 0.2]
    velocity band on every step, conflicting +-0.5 costs on the two halves, the
    dt column in [0.01234, 3.5678] initialised to their difference."""
    dt_lower, dt_upper, lower_tol, upper_tol = 0.01234, 3.5678, -0.1, 0.2
    half = (STEPS - 1) // 2
    text = _doc([_timed(_term("joint_vel", 1.0, 0.5, 0, half, -0.01, 0.01, "joint_vel_targ_1")),
                 _timed(_term("joint_vel", 1.0, -0.5, half + 1, STEPS - 1, -0.01, 0.01, "joint_vel_targ_2"))],
                [_timed(_term("joint_vel", 1.0, 0.0, 0, STEPS - 1, lower_tol, upper_tol, "joint_vel_limits"))],
                basic={"use_time": True, "dt_lower_lim": dt_lower, "dt_upper_lim": dt_upper},
                init={"dt": dt_upper - dt_lower})

    def check(traj):
        v = _vel_time(traj)
        rows = list(range(0, STEPS // 2)) + list(range(STEPS // 2 + 1, STEPS - 1))
        bad = []
        if v[rows].max() >= upper_tol + 1e-4 or v[rows].min() <= lower_tol - 1e-4:
            bad.append(f"band: v in [{v[rows].min():.4f}, {v[rows].max():.4f}]")
        return bad

    return text, check


def _total_time(is_cnt):
    """TotalTimeTermInfo (problem_description.cpp:1860-1913) over the dt column of
    equality_jointVel_time: as a constraint sum(1/dt[1:]) <= 5.8 (9 at the init
    dt of 1; 9 / 1.5678 = 5.7405 at the upper limit), as a squared cost (limit 0)
    that drives dt to its upper limit."""
    dt_lower, dt_upper, limit = 0.01234, 1.5678, 5.8
    tt = {"type": "total_time", "name": "total_time", "use_time": True,
          "params": {"coeff": 1.0, "limit": limit if is_cnt else 0.0}}
    costs = [_timed(_term("joint_vel", 1.0, 0.1, 0, STEPS - 1, name="joint_vel_all"))]
    cnts = []
    (cnts if is_cnt else costs).append(tt)
    text = _doc(costs, cnts, basic={"use_time": True, "dt_lower_lim": dt_lower, "dt_upper_lim": dt_upper})

    def check(traj):
        v, dt = _vel_time(traj), np.asarray(traj)[:, -1]
        total = (1.0 / dt[1:]).sum()
        bad = []
        if is_cnt and total > limit + 1e-4:
            bad.append(f"total time {total:.5f} > {limit}")
        if not is_cnt and dt[1:].min() < dt_upper - 1e-3:
            bad.append(f"dt below its upper limit: min {dt[1:].min():.5f}")
        if np.abs(v - 0.1).max() > 0.01:
            bad.append(f"cost: max |v - 0.1| {np.abs(v - 0.1).max():.2e}")
        return bad

    return text, check


def _fixed_dofs():
    """basic_info.fixed_dofs (problem_description.cpp:512-534): joints 2 and 5 held
    at the initial trajectory on every step, under the equality_jointVel cost."""
    text = _doc([_term("joint_vel", 10.0, 0.1, 0, STEPS - 1, name="joint_vel_all")], [],
                basic={"fixed_dofs": [2, 5]})

    def check(traj):
        t = np.asarray(traj)
        bad = []
        if np.abs(t[:, [2, 5]]).max() > 1e-4:
            bad.append(f"fixed dofs moved: max {np.abs(t[:, [2, 5]]).max():.2e}")
        free = _diff(t, 1)[:, [0, 1, 3, 4, 6]]
        if np.abs(free - 0.1).max() > 0.01:
            bad.append(f"cost: max |v - 0.1| {np.abs(free - 0.1).max():.2e}")
        return bad

    return text, check


PROBLEMS = {
    "equality_jointPos": _equality("joint_pos", 0),
    "inequality_jointPos": _inequality("joint_pos", 0),
    "equality_jointVel": _equality("joint_vel", 1),
    "inequality_jointVel": _inequality("joint_vel", 1),
    "equality_jointAcc": _equality("joint_acc", 2),
    "inequality_jointAcc": _inequality("joint_acc", 2),
    "equality_jointJerk": _jerk(),
    "equality_jointVel_time": _equality_vel_time(),
    "inequality_jointVel_time": _inequality_vel_time(),
    "total_time_cnt": _total_time(True),
    "total_time_cost": _total_time(False),
    "fixed_dofs": _fixed_dofs(),
}
# those the batched kernel runs (the rest take the generic path: GpuModel QPs)
LOWERABLE = {"equality_jointPos", "inequality_jointPos", "inequality_jointVel"}


def jdt_fused(desc):
    """thip_jdt_fused (trajopt_hip.h): every jdt term a JointAccEqCost on an even
    number of waypoints with 2 n_dof <= 16 (waypoint-pair blocks)."""
    D = desc.chain.n_dof
    if desc.n_jdt == 0:
        return True
    if desc.n_steps % 2 or 2 * D > 16 or desc.use_time:
        return False
    return all(desc.jdt_order[k] == 2 and not desc.jdt_is_cnt[k] and
               all(abs(desc.jdt_upper_tols[k][j]) < 1e-5 and abs(desc.jdt_lower_tols[k][j]) < 1e-5 for j in range(D))
               for k in range(desc.n_jdt))


def lowerable(desc):
    """TrajOptProb::lowerable(): no term or variable the kernel does not lower."""
    return jdt_fused(desc) and desc.n_jvt == 0 and desc.n_ttt == 0 and not desc.use_time and desc.n_fixed_dofs == 0


def workload(text, host):
    """The JSON problem lowered by the host front door as a one-problem Workload."""
    from trajopt_amd.problems import Workload

    desc, init, tgt, jpt = host.lower_json(text)
    return Workload("json", desc, init[None].copy(), tgt[None].copy(), np.zeros((1, 0, 16)), init[None].copy(),
                    jpt[None].copy() if desc.n_jpos else None)
