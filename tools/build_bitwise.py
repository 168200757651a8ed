"""Run the hinge-heavy workloads on one build tree's GPU library and save the
trajectories and results (diagnostic: a restructured kernel must reproduce the
previous build bit for bit).

    python tools/build_bitwise.py <root with trajopt-1_amd/> <tag>
    python tools/build_bitwise.py --compare <tagA> <tagB>
"""
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = (np.load(f"gpurun_out/bitwise_{t}.npz") for t in sys.argv[2:4])
    bad = 0
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        bad += not same
        print(f"{k:24s} {'bitwise equal' if same else 'DIFFERENT, max |d| %.3e' % np.abs(a[k] - b[k]).max()}")
    sys.exit(1 if bad else 0)

root, tag = sys.argv[1], sys.argv[2]
sys.path.insert(0, root + "/trajopt-1_amd")
from trajopt_amd import abi, problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

print(abi.__file__, flush=True)
out = {}


def run(name, wl, path=0):
    hip = abi.load_hip()
    if path:
        assert hip.thip_debug_set_path(path) == 0
    try:
        s = BatchTrustRegionSQP(wl)
        x, res = s.optimize()
        s.close()
    finally:
        if path:
            hip.thip_debug_set_path(0)
    out[name + "_x"] = x
    out[name + "_r"] = np.array([[r.status, r.n_sqp_iters, r.n_qp_solves, r.n_admm_iters, r.total_cost] for r in res])
    print(name, "done", flush=True)


run("E8", problems.make_workload("E", 8))
wl = problems.make_workload("C", 16, first_problem=200)
wl.desc.coll_continuous = 1
run("Ccont_generic", wl, abi.DEBUG_NO_SEGMENT)
run("C_wide", problems.make_workload("C", 16), abi.DEBUG_FORCE_WIDE)
run("C_seg", problems.make_workload("C", 64))
run("torso_C", problems.make_workload("C", 8, robot="torso_right_arm"))
np.savez(f"gpurun_out/bitwise_{tag}.npz", **out)
