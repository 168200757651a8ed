"""GPU vs oracle trajectories with and without the self-collision pairs
(diagnostic): config E on the wide path, config C continuous.

    python tools/selfoff_parity.py
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "trajopt-1_amd", REPO / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402  (diagnostic tool: the checker)
from trajopt_amd import abi, problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402


def run(wl, wide=False):
    hip = abi.load_hip()
    if wide:
        hip.thip_debug_set_path(abi.DEBUG_NO_BRANCH)
    try:
        s = BatchTrustRegionSQP(wl)
        x, res = s.optimize()
        s.close()
    finally:
        hip.thip_debug_set_path(0)
    xo, ro = oracle.solve(wl, n_threads=16)
    dx = np.abs(x - xo).reshape(wl.batch, -1).max(1)
    same = [(a.n_sqp_iters == b.n_sqp_iters and a.n_qp_solves == b.n_qp_solves) for a, b in zip(res, ro)]
    return dx, same


for label, mk, wide in (("E", lambda: problems.make_workload("E", 4), True),
                        ("Ccont", lambda: problems.make_workload("C", 16, first_problem=200), False)):
    for self_on in (False, True):
        wl = mk()
        if label == "Ccont":
            wl.desc.coll_continuous = 1
        if not self_on:
            wl.desc.n_self_pairs = 0
        dx, same = run(wl, wide)
        print(f"{label} self pairs {'on ' if self_on else 'off'}: max dx per problem {np.array2string(dx, precision=1)}; "
              f"same iteration counts {sum(same)}/{len(same)}", flush=True)
