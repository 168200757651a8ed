"""Debug: per-QP traces, GPU vs oracle, for one problem of a tests/test_gpu.py variant."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "trajopt-1_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402

from test_gpu import _variant  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402
from oracle import oracle  # noqa: E402

name, b = sys.argv[1], int(sys.argv[2])
lo, hi = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (0, 40)
wl = _variant(name)
s = BatchTrustRegionSQP(wl)
s.enable_trace(512)
x, res = s.optimize()
tr = s.get_trace()[b]
xo, ro, to = oracle.solve_trace(wl, b, cap=512)
print("gpu", res[b].status, res[b].n_sqp_iters, res[b].total_cost, "orc", ro.status, ro.n_sqp_iters, ro.total_cost)
np.set_printoptions(precision=10, linewidth=220)
for k in range(lo, min(hi, max(len(tr), len(to)))):
    if k < len(tr):
        print(f"g{k:3d}", tr[k])
    if k < len(to):
        print(f"o{k:3d}", to[k])
