"""Along the HIP path's own iterates of one problem (max_iter = 1, 2, ...):
which CartPose Jacobian entries cross cleanupAff's 1e-7 between consecutive
iterates, on the GPU and in the oracle at the same points (diagnostic).

    python tools/mask_walk.py <config> <batch> <problem>
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
s = BatchTrustRegionSQP(wl)
x, r = s.optimize()
n_it = r[0].n_sqp_iters
prev_g = prev_o = None
for k in range(1, n_it + 1):
    w = subset(wl, [0])
    w.desc.sqp.max_iter = k
    sk = BatchTrustRegionSQP(w)
    xk, rk = sk.optimize()
    sk.close()
    _, jg = s.linearize(xk)
    _, jo = oracle.linearize(wl, xk)
    mg, mo = np.abs(jg) > 1e-7, np.abs(jo) > 1e-7
    line = f"iterate {k:3d} (qp {rk[0].n_qp_solves}): gpu/oracle masks differ at {int((mg != mo).sum())} entries"
    if prev_g is not None:
        cg, co = np.argwhere(mg != prev_g), np.argwhere(mo != prev_o)
        line += f"; changed since k-1: gpu {len(cg)} oracle {len(co)}"
        for f in cg:
            f = tuple(int(v) for v in f)
            line += f"\n    gpu change {f}: {jg[f]:.10e} (oracle {jo[f]:.10e})"
    print(line, flush=True)
    prev_g, prev_o = mg, mo
s.close()
