"""Run config C continuous twice on one build and compare bitwise (diagnostic).

    python tools/determinism.py <root>
"""
import sys

root = sys.argv[1]
sys.path.insert(0, root)
sys.path.insert(0, root + "/trajopt-1_amd")
import numpy as np  # noqa: E402

from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

xs = []
for rep in range(3):
    wl = problems.make_workload("C", 16, first_problem=200)
    wl.desc.coll_continuous = 1
    if hasattr(wl.desc, "n_self_pairs"):
        wl.desc.n_self_pairs = 0
    s = BatchTrustRegionSQP(wl)
    x, res = s.optimize()
    s.close()
    xs.append(x)
for rep in (1, 2):
    d = np.abs(xs[rep] - xs[0]).reshape(16, -1).max(1)
    print(root.split("/")[-1], f"run {rep} vs run 0: max dx per problem", np.array2string(d, precision=1))
