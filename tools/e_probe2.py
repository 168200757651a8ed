"""Config E variants probe (diagnostic): which ingredient breaks the 14-DoF solve."""
import sys

sys.path.insert(0, "trajopt-1_amd")
sys.path.insert(0, ".")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP
from oracle import oracle


def run(label, wl):
    s = BatchTrustRegionSQP(wl)
    s.enable_trace(256)
    x, res = s.optimize()
    tr = s.get_trace()
    s.close()
    xo, ro = oracle.solve(wl, n_threads=16)
    for b in range(wl.batch):
        qs = [(int(r[3]), int(r[2])) for r in tr[b][:12]]
        print(f"{label} b{b}: gpu {res[b].status} orc {ro[b].status} sqp {res[b].n_sqp_iters}/{ro[b].n_sqp_iters} "
              f"dx {float(np.abs(x[b] - xo[b]).max()):.2e} qp(status,iters) {qs}", flush=True)


wl = problems.make_workload("E", 2, n_steps=12)
wl.desc.coll_enabled = 0
wl.desc.n_prims = 0
run("E-nocoll", wl)
wl = problems.make_workload("E", 2, n_steps=12)
wl.desc.coll_enabled = 0
wl.desc.n_prims = 0
wl.desc.n_cart = 0
wl.targets = wl.targets[:, :0]
run("E-jv-only", wl)
wl = problems.make_workload("E", 2, n_steps=12)
run("E-full", wl)
