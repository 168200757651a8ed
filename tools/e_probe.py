"""Config E probe (diagnostic): GPU solve of a few dual-arm problems, timed,
against the oracle.  python tools/e_probe.py [n_steps] [batch]"""
import sys
import time

sys.path.insert(0, "trajopt-1_amd")
sys.path.insert(0, ".")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
wl = problems.make_workload("E", B, n_steps=N)
s = BatchTrustRegionSQP(wl)
t = time.time()
x, res = s.optimize()
print(f"GPU E N={N} B={B}: {time.time() - t:.2f} s, kernel {s.kernel_ms():.1f} ms", flush=True)
for r in res:
    print("  gpu", r.status, r.n_sqp_iters, r.n_qp_solves, r.n_admm_iters, r.total_cost, r.max_cnt_viol, flush=True)
from oracle import oracle  # noqa: E402

t = time.time()
xo, ro = oracle.solve(wl, n_threads=16)
print(f"oracle: {time.time() - t:.2f} s", flush=True)
for b, r in enumerate(ro):
    print("  orc", r.status, r.n_sqp_iters, r.n_qp_solves, r.n_admm_iters, r.total_cost, r.max_cnt_viol,
          float(np.abs(x[b] - xo[b]).max()), flush=True)
