"""A/B of the fused kernel's two builds on a workload whose QPs never take the
register-resident segment (config E by default): the generic-step build
(sqp_kernel_gen, layout.hpp kGenBlock threads; the default for such QPs since
round 6) against the main build's generic step (THIP_DEBUG_MAIN_BUILD).  Per
build: one batch alone (HIP-event ms), SQP iterations, statuses; then whether
the two builds agree to the parity bar.

    python tools/gen_ab.py [config] [batch] [n_steps] [root]

(root: another build tree with a trajopt-1_amd/ directory; the segment is
switched off in both runs, so segment-capable configs run the generic step too)
"""
import sys
import time
from pathlib import Path

ROOT = Path(sys.argv[4]).resolve() if len(sys.argv) > 4 else Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "trajopt-1_amd"))

import numpy as np  # noqa: E402

from trajopt_amd import abi, problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "E"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
N = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) > 0 else None
hip = abi.load_hip()
out = {}
print(abi.__file__, flush=True)
for name, flags in (("gen", abi.DEBUG_GEN_BUILD | abi.DEBUG_NO_SEGMENT),
                    ("main", abi.DEBUG_NO_SEGMENT | abi.DEBUG_MAIN_BUILD)):
    assert hip.thip_debug_set_path(flags) == 0
    wl = problems.make_workload(cfg, B, n_steps=N) if N else problems.make_workload(cfg, B)
    s = BatchTrustRegionSQP(wl)
    s.upload()
    t0 = time.perf_counter()
    s.run()
    s.sync()
    wall = time.perf_counter() - t0
    ms = s.kernel_ms()
    x, res = s.download()
    s.close()
    hip.thip_debug_set_path(0)
    it = sum(r.n_sqp_iters for r in res)
    admm = sum(r.n_admm_iters for r in res)
    out[name] = (x, res)
    print(f"{cfg} x{B} {name}: kernel {ms:.1f} ms (wall {wall:.2f} s), {it} SQP iters -> {it / (ms * 1e-3):.0f} it/s, "
          f"{admm} ADMM iters, {admm / (ms * 1e-3) / B:.0f} ADMM it/s per problem, statuses "
          f"{np.bincount([r.status for r in res], minlength=6).tolist()}", flush=True)
xg, rg = out["gen"]
xm, rm = out["main"]
dx = np.abs(xg - xm).reshape(B, -1).max(1)
same = sum(a.status == b.status for a, b in zip(rg, rm))
print(f"builds agree: status {same}/{B}, |dx| <= 1e-5 on {(dx <= 1e-5).sum()}/{B}, median |dx| {np.median(dx):.1e}, "
      f"max {dx.max():.1e}, bitwise {np.array_equal(xg, xm)}", flush=True)
