"""torso_arm_8dof_C (config C on the 8-dof torso arm, 8 problems) repeated on one
build tree: problem statuses and costs per run, and bitwise agreement with run 0
(diagnostic for an intermittent OPT_FAILED).

    python tools/torso_repeat.py <root> <runs> [problem [static]]

(problem: that problem alone, a batch of one; static: one workgroup per problem
instead of the persistent dispatch -- a deterministic outcome that holds in
every arrangement points at the code, one that moves at a race)
"""
import sys

root, runs = sys.argv[1], int(sys.argv[2])
only = int(sys.argv[3]) if len(sys.argv) > 3 else None
static = len(sys.argv) > 4 and sys.argv[4] == "static"
sys.path.insert(0, root + "/trajopt-1_amd")
sys.path.insert(1, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tests"))
import numpy as np  # noqa: E402

from trajopt_amd import abi, problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

x0 = None
for rep in range(runs):
    wl = problems.make_workload("C", 8, robot="torso_right_arm")
    if only is not None:
        from parity import subset

        wl = subset(wl, [only])
    if static:
        abi.load_hip().thip_debug_set_path(abi.DEBUG_STATIC_DISPATCH)
    s = BatchTrustRegionSQP(wl)
    x, res = s.optimize()
    s.close()
    if static:
        abi.load_hip().thip_debug_set_path(0)
    same = "" if x0 is None else f" bitwise {'equal' if np.array_equal(x, x0) else 'DIFFERENT'}"
    x0 = x if x0 is None else x0
    print(f"{root} run {rep}{'' if only is None else f' problem {only} alone'}{' static' if static else ''}: "
          f"statuses {[r.status for r in res]} cost {res[0 if only is not None else 2].total_cost:.6f}{same}", flush=True)
