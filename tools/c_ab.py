"""Config C lone-batch timing of one build tree (A/B of kernel variants):
one warm-up launch, then `reps` timed launches of the same batch (HIP events),
SQP / ADMM iterations, and the trajectories saved for a bitwise comparison.

    python tools/c_ab.py <root with trajopt-1_amd/> <tag> [batch] [reps] [config]
    python tools/c_ab.py --compare <tagA> <tagB>
"""
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = (np.load(f"gpurun_out/c_ab_{t}.npz") for t in sys.argv[2:4])
    same = np.array_equal(a["x"], b["x"])
    d = np.abs(a["x"] - b["x"]).reshape(a["x"].shape[0], -1).max(1)
    print(f"{sys.argv[2]} vs {sys.argv[3]}: bitwise {same}, problems differing {(d > 0).sum()}, max |dx| {d.max():.2e}")
    sys.exit(0)

root, tag = sys.argv[1], sys.argv[2]
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
cfg = sys.argv[5] if len(sys.argv) > 5 else "C"
sys.path.insert(0, root + "/trajopt-1_amd")
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

wl = problems.make_workload(cfg, B)
s = BatchTrustRegionSQP(wl)
s.upload()
s.run()
s.sync()
ms = []
for _ in range(reps):
    s.run()
    s.sync()
    ms.append(s.kernel_ms())
x, res = s.download()
s.close()
it = sum(r.n_sqp_iters for r in res)
admm = sum(r.n_admm_iters for r in res)
np.savez(f"gpurun_out/c_ab_{tag}.npz", x=x)
print(f"{tag}: {cfg} x{B} kernel {' '.join(f'{m:.1f}' for m in ms)} ms, {it} SQP iters, {admm} ADMM iters, "
      f"{it / (min(ms) * 1e-3):.0f} SQP it/s lone", flush=True)
