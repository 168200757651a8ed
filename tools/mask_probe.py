"""Where do the HIP path's and the oracle's CartPose Jacobians disagree about
cleanupAff's 1e-7 threshold (the warm-start pattern, quirk Q2)?  Diagnostic.

    python tools/mask_probe.py <config> <batch> <problem>

Walks the oracle's own iterates of one problem (the oracle rerun with
max_iter = 1, 2, ...), linearises each on the GPU (thip_linearize) and in the
oracle, and prints per iterate the entries whose |J| lies on different sides
of 1e-7, plus the largest |J_gpu - J_oracle| anywhere.
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "trajopt-1_amd", REPO / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from parity import subset  # noqa: E402
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

cfg, B, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
wl = subset(problems.make_workload(cfg, B), [b])
_, r = oracle.solve(wl, n_threads=1)
n_it = r[0].n_sqp_iters
s = BatchTrustRegionSQP(wl)
worst = 0.0
for k in range(1, n_it + 1):
    w = subset(wl, [0])
    w.desc.sqp.max_iter = k
    x, _ = oracle.solve(w, n_threads=1)
    eg, jg = s.linearize(x)
    eo, jo = oracle.linearize(wl, x)
    d = np.abs(jg - jo)
    worst = max(worst, float(d.max()))
    flips = np.argwhere((np.abs(jg) > 1e-7) != (np.abs(jo) > 1e-7))
    msg = f"iterate {k:3d}: max|dJ| {d.max():.2e}, max|de| {np.abs(eg - eo).max():.2e}"
    for f in flips:
        f = tuple(int(v) for v in f)
        msg += f"\n    flip at {f}: gpu {jg[f]:.12e} oracle {jo[f]:.12e}"
    print(msg, flush=True)
s.close()
print(f"largest |J_gpu - J_oracle| over all iterates: {worst:.3e}")
