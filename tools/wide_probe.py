"""Wide-block solve probe (diagnostic): config B/C problems with the wide
(D > 8) block solve forced (THIP_FORCE_WIDE=1) against the oracle."""
import os
import sys
import time

sys.path.insert(0, "trajopt-1_amd")
sys.path.insert(0, ".")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP
from oracle import oracle

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wl = problems.make_workload(cfg, B)
s = BatchTrustRegionSQP(wl)
t = time.time()
x, res = s.optimize()
print(f"GPU {cfg} B={B} wide={os.environ.get('THIP_FORCE_WIDE')}: {time.time() - t:.2f} s", flush=True)
xo, ro = oracle.solve(wl, n_threads=16)
for b in range(B):
    print(" ", res[b].status, ro[b].status, res[b].n_sqp_iters, ro[b].n_sqp_iters, res[b].n_admm_iters,
          ro[b].n_admm_iters, float(np.abs(x[b] - xo[b]).max()), flush=True)
