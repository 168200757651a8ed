"""Generate the committed golden fixtures (tests/golden/*.npz).

    python tests/golden/make_golden.py

The reference (C++ over Eigen/Boost/tesseract/OSQP) cannot be built in this
image, so these vectors are outputs of the oracle -- the CPU
restatement under oracle/, itself pinned by the 45 reference KATs in
oracle/tests/kat_main.cpp -- on small seeded inputs.  They pin the oracle
against drift and give the GPU tests a fixed target; the reference-pinned
anchors are the KATs.

Contents (all fp64):
  fk_pr2.npz        PR2 right-arm FK of 16 seeded joint vectors (oracle), and
                    the independent numpy FK of trajopt_amd.robots
  cartpose_A.npz    CartPose error + forward-difference Jacobian at the init
                    trajectories of config A (4 problems)
  cartpose_B.npz    same for config B (2 problems, 29 terms each)
  sqp_A.npz         converged x, status, counters, cost, max violation for
                    config A problems 0..7
  sqp_B.npz         the same for config B problems 0..1
  sqp_jv.npz        JointVel-only (no CartPose) variant, 12 steps, 4 problems
  sqp_C.npz         config C (B + LVS-discrete collision cost, 10-primitive
                    scene) problems 0..2
  collision_rows_C_cont.npz  LVS_CONTINUOUS rows of 3 config C problems at init
  collision_rows_C.npz  linearised collision rows of those problems at their
                    converged trajectories (oracle_collision_rows)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "trajopt-1_amd"))
sys.path.insert(0, str(REPO))

from oracle import oracle  # noqa: E402
from trajopt_amd import problems, robots  # noqa: E402


def jointvel_only(batch, n_steps=12):
    """Config B structure without CartPose terms (JointVel + fixed step 0)."""
    wl = problems.make_workload("B", batch, n_steps=n_steps)
    wl.desc.n_cart = 0
    wl.targets = np.zeros((batch, 0, 12))
    wl.name = "JV"
    return wl


def result_arrays(res):
    keys = ["status", "n_sqp_iters", "n_qp_solves", "n_func_evals", "n_merit_increases"]
    out = {k: np.array([getattr(r, k) for r in res], dtype=np.int64) for k in keys}
    out["total_cost"] = np.array([r.total_cost for r in res])
    out["max_cnt_viol"] = np.array([r.max_cnt_viol for r in res])
    return out


def main():
    oracle.build()
    chain = robots.pr2_right_arm()
    lo, hi, _ = robots.chain_limits(chain)
    rng = problems.SplitMix64(20261015)
    q = np.array([[lo[j] + (hi[j] - lo[j]) * rng.uniform() for j in range(len(lo))] for _ in range(16)])
    q = np.clip(q, -3.0, 3.0)
    np.savez(HERE / "fk_pr2.npz", q=q, poses=oracle.fwd_kin(chain, q),
             poses_numpy=np.stack([[T[:3, :].reshape(12) for T in robots.fwd_kin(chain, qi)] for qi in q]))

    for cfg, B in (("A", 4), ("B", 2)):
        wl = problems.make_workload(cfg, B)
        err, jac = oracle.linearize(wl, wl.init)
        np.savez(HERE / f"cartpose_{cfg}.npz", x=wl.init, targets=wl.targets, err=err, jac=jac)

    for name, wl in (("sqp_A", problems.make_workload("A", 8)), ("sqp_B", problems.make_workload("B", 2)),
                     ("sqp_jv", jointvel_only(4)), ("sqp_C", problems.make_workload("C", 3))):
        x, res = oracle.solve(wl, n_threads=8)
        np.savez(HERE / f"{name}.npz", init=wl.init, targets=wl.targets, scene=wl.scene, x=x, **result_arrays(res))
    wl = problems.make_workload("C", 3)
    x, _ = oracle.solve(wl, n_threads=3)
    np.savez(HERE / "collision_rows_C.npz", x=x,
             **{f"rows{b}": oracle.collision_rows(wl, b, x[b]) for b in range(3)})
    continuous_fixture()
    discrete_fixture()
    tolerance_fixture()
    print("golden fixtures written to", HERE)


def continuous_fixture():
    """collision_rows_C_cont.npz: LVS_CONTINUOUS rows (swept-sphere casts) of
    3 config C problems at their initial trajectories."""
    wl = problems.make_workload("C", 3)
    wl.desc.coll_continuous = 1
    np.savez(HERE / "collision_rows_C_cont.npz", x=wl.init,
             **{f"rows{b}": oracle.collision_rows(wl, b, wl.init[b]) for b in range(3)})


def tolerance_fixture():
    """cartpose_B_tol.npz: toleranced CartPose rows (+-0.02 m, +-0.1 rad bands) of 2
    config B problems at their initial trajectories."""
    wl = problems.with_cart_tolerances(problems.make_workload("B", 2))
    err, jac = oracle.linearize(wl, wl.init)
    np.savez(HERE / "cartpose_B_tol.npz", x=wl.init, targets=wl.targets, err=err, jac=jac)


def discrete_fixture():
    """collision_rows_C_single.npz: DISCRETE (single-timestep) rows of 3
    config C problems at their initial trajectories."""
    wl = problems.make_workload("C", 3)
    wl.desc.coll_continuous = 2
    wl.desc.coll_buffer = 0.1
    np.savez(HERE / "collision_rows_C_single.npz", x=wl.init,
             **{f"rows{b}": oracle.collision_rows(wl, b, wl.init[b]) for b in range(3)})


if __name__ == "__main__":
    main()
