"""GPU vs oracle parity summary for a config/batch (diagnostic).

    python tools/parity.py A 64 [B 64 ...]
    PARITY_ROOTS=".:r6nc" python tools/parity.py C 256   (several build trees, one oracle run)

Workload names: the configs of trajopt_amd.problems.make_workload (A, B, C, J) and
the variants C-disc (DISCRETE evaluator, buffer 0.1), C-cont (LVS_CONTINUOUS),
C-cnt (collision constraint), B-tol / A-tol (CartPose tool-axis tolerance band),
C50-cont (50 waypoints, LVS_CONTINUOUS).
"""
import importlib
import os
import sys
import time

ROOTS = os.environ.get("PARITY_ROOTS", ".").split(":")
sys.path.insert(0, ".")
import numpy as np

from oracle import oracle


def load_tree(root):
    """the trajopt_amd package (and its HIP library) of one build tree"""
    for k in [k for k in sys.modules if k == "trajopt_amd" or k.startswith("trajopt_amd.")]:
        del sys.modules[k]
    sys.path.insert(0, os.path.join(root, "trajopt-1_amd"))
    try:
        return importlib.import_module("trajopt_amd.problems"), importlib.import_module("trajopt_amd.runtime")
    finally:
        sys.path.pop(0)


import trajopt_amd.problems as problems  # the oracle's own import (its ctypes types)



def make(name, B, problems=problems):
    base, _, var = name.partition("-")
    n_steps = 50 if base == "C50" else None
    wl = problems.make_workload("C" if base == "C50" else base, B, **({"n_steps": n_steps} if n_steps else {}))
    if var == "disc":
        wl.desc.coll_continuous = 2
        wl.desc.coll_buffer = 0.1
    elif var == "cont":
        wl.desc.coll_continuous = 1
    elif var == "cnt":
        wl.desc.coll_is_cnt = 1
    elif var == "tol":
        problems.with_cart_tolerances(wl, rot=0.2, axes=(3,))
    elif var == "acc":
        problems.with_joint_acc(wl)
    return wl


args = sys.argv[1:]
def report(tag, cfg, B, wl, xg, rg, xo, ro, tg, to):
    d = np.abs(xg - xo).reshape(B, -1).max(1)
    st = np.array([a.status == b.status for a, b in zip(rg, ro)])
    tol = wl.desc.sqp.cnt_tolerance
    fl = np.array([(a.max_cnt_viol < tol) == (b.max_cnt_viol < tol) for a, b in zip(rg, ro)])
    ok = (d <= 1e-5) & st & fl
    cost_rel = np.array([abs(a.total_cost - b.total_cost) / max(1.0, abs(b.total_cost)) for a, b in zip(rg, ro)])
    print(f"[{tag}] config {cfg} batch {B}: x within 1e-5 {np.sum(d <= 1e-5)}/{B}, status equal {st.sum()}/{B}, "
          f"cnt-flag equal {fl.sum()}/{B}, all three {ok.sum()}/{B}; gpu {tg:.2f}s oracle {to:.2f}s (16 thr)")
    print(f"   max|dx| quantiles 50/90/100%: {np.quantile(d, 0.5):.2e} {np.quantile(d, 0.9):.2e} {d.max():.2e}; "
          f"cost rel diff of mismatches: {np.round(cost_rel[~ok], 6).tolist()[:12]}")
    print(f"   mismatching problems: {np.nonzero(~ok)[0].tolist()[:20]}  statuses gpu/cpu: "
          f"{[(rg[b].status, ro[b].status) for b in np.nonzero(~ok)[0][:8]]}", flush=True)


for i in range(0, len(args), 2):
    cfg, B = args[i], int(args[i + 1])
    wl = make(cfg, B)
    t = time.time()
    xo, ro = oracle.solve(wl, n_threads=16)
    to = time.time() - t
    for root in ROOTS:
        prob_r, runtime = load_tree(root)
        s = runtime.BatchTrustRegionSQP(make(cfg, B, prob_r))
        t = time.time()
        xg, rg = s.optimize()
        tg = time.time() - t
        s.close()
        report(root, cfg, B, wl, xg, rg, xo, ro, tg, to)
