"""Config C continuous on a given build tree's GPU library and oracle
(diagnostic: round-3 tree vs the current one on the same box).

    python tools/r3_ccont.py <root with trajopt-1_amd/ and oracle/>
"""
import sys

root = sys.argv[1]
sys.path.insert(0, root)
sys.path.insert(0, root + "/trajopt-1_amd")
import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402  (diagnostic tool: the checker)
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

print(oracle.__file__)
wl = problems.make_workload("C", 16, first_problem=200)
wl.desc.coll_continuous = 1
if hasattr(wl.desc, "n_self_pairs"):
    wl.desc.n_self_pairs = 0
s = BatchTrustRegionSQP(wl)
x, res = s.optimize()
s.close()
xo, ro = oracle.solve(wl, n_threads=16)
np.save(f"gpurun_out/ccont_x_{'r3' if 'r3cmp' in root else 'now'}.npy", x)
dx = np.abs(x - xo).reshape(wl.batch, -1).max(1)
print("max dx per problem", np.array2string(dx, precision=1))
