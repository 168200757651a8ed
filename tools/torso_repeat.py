"""torso_arm_8dof_C (config C on the 8-dof torso arm, 8 problems) repeated on one
build tree: problem statuses and costs per run, and bitwise agreement with run 0
(diagnostic for an intermittent OPT_FAILED).

    python tools/torso_repeat.py <root> <runs>
"""
import sys

root, runs = sys.argv[1], int(sys.argv[2])
sys.path.insert(0, root + "/trajopt-1_amd")
import numpy as np  # noqa: E402

from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

x0 = None
for rep in range(runs):
    wl = problems.make_workload("C", 8, robot="torso_right_arm")
    s = BatchTrustRegionSQP(wl)
    x, res = s.optimize()
    s.close()
    same = "" if x0 is None else f" bitwise {'equal' if np.array_equal(x, x0) else 'DIFFERENT'}"
    x0 = x if x0 is None else x0
    print(f"{root} run {rep}: statuses {[r.status for r in res]} cost[2] {res[2].total_cost:.6f}{same}", flush=True)
