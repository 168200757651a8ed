"""The reference's joint-term unit problems (trajopt/test/joint_costs_unit.cpp)
as TrajOptRequest JSON on the PR2 right_arm, plus a jerk problem, shared by
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


def _doc(costs, cnts):
    return json.dumps({"basic_info": {"n_steps": STEPS, "manip": "right_arm"},
                       "costs": costs, "constraints": cnts, "init_info": {"type": "stationary"}})


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


PROBLEMS = {
    "equality_jointPos": _equality("joint_pos", 0),
    "inequality_jointPos": _inequality("joint_pos", 0),
    "equality_jointVel": _equality("joint_vel", 1),
    "inequality_jointVel": _inequality("joint_vel", 1),
    "equality_jointAcc": _equality("joint_acc", 2),
    "inequality_jointAcc": _inequality("joint_acc", 2),
    "equality_jointJerk": _jerk(),
}
# those the batched kernel runs (the rest take the generic path: GpuModel QPs)
LOWERABLE = {"equality_jointPos", "inequality_jointPos", "inequality_jointVel"}


def workload(text, host):
    """The JSON problem lowered by the host front door as a one-problem Workload."""
    from trajopt_amd.problems import Workload

    desc, init, tgt, jpt = host.lower_json(text)
    return Workload("json", desc, init[None].copy(), tgt[None].copy(), np.zeros((1, 0, 16)), init[None].copy(),
                    jpt[None].copy() if desc.n_jpos else None)
