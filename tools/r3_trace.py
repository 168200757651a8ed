"""Per-QP traces and contact rows of config C continuous on a given build tree
(diagnostic: bitwise comparison of two builds on the same box).

    python tools/r3_trace.py <root> <tag>
"""
import sys

root, tag = sys.argv[1], sys.argv[2]
sys.path.insert(0, root)
sys.path.insert(0, root + "/trajopt-1_amd")
import numpy as np  # noqa: E402

from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

wl = problems.make_workload("C", 16, first_problem=200)
wl.desc.coll_continuous = 1
if hasattr(wl.desc, "n_self_pairs"):
    wl.desc.n_self_pairs = 0
s = BatchTrustRegionSQP(wl)
s.enable_trace(256)
x, res = s.optimize()
tr = s.get_trace()
s.close()
np.savez(f"gpurun_out/tr_{tag}.npz", *[np.asarray(t) for t in tr])
np.save(f"gpurun_out/x_{tag}.npy", x)
s = BatchTrustRegionSQP(wl)
rows = s.collision_rows(wl.init)
rows2 = s.collision_rows(x)
s.close()
np.save(f"gpurun_out/rows_init_{tag}.npy", np.concatenate(rows))
np.save(f"gpurun_out/rows_x_{tag}.npy", np.concatenate(rows2))
np.save(f"gpurun_out/rows_n_{tag}.npy", np.array([len(r) for r in rows] + [len(r) for r in rows2]))
print(tag, "done")
