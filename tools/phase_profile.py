"""Per-phase cycle breakdown of sqp_kernel (thip_debug_profile), diagnostic.

    python tools/phase_profile.py B 1024
    PP_ROOT=r6nc python tools/phase_profile.py C 1024   (another build tree)
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.environ.get("PP_ROOT", "."), "trajopt-1_amd"))
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP

os.makedirs("gpurun_out", exist_ok=True)
cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
wl = problems.make_workload(cfg, B)
s = BatchTrustRegionSQP(wl)
s.upload()
s.run()
s.download()
s.enable_profile(True)
t = time.time()
s.run()
x, res = s.download()
print(f"config {cfg} batch {B}: kernel {s.kernel_ms():.1f} ms (wall {time.time() - t:.2f}s)")
pf = s.get_profile().astype(np.float64)
admm = np.array([r.n_admm_iters for r in res], dtype=np.float64)
qps = np.array([r.n_qp_solves for r in res], dtype=np.float64)
sqp = np.array([r.n_sqp_iters for r in res], dtype=np.float64)
subs = np.array([r.n_substates for r in res], dtype=np.float64)
fev = np.array([r.n_func_evals for r in res], dtype=np.float64)
print(f"LVS sub-state passes per problem {subs.mean():.0f}; per scan call and step pair "
      f"{subs.sum() / max(1.0, (fev + sqp).sum() * (wl.n_steps - 1)):.2f}")
mhz = pf[:, 13].sum() / pf[:, 14].sum() * 100.0
print(f"shader clock ~{mhz:.0f} MHz; per problem: admm {admm.mean():.0f} (max {admm.max():.0f}), "
      f"qp {qps.mean():.1f}, sqp {sqp.mean():.1f}")
# per-problem wall time (10 ns units) for the dispatch simulation (tools/dispatch_sim.py)
np.save(f"gpurun_out/pp_{cfg}_{B}_wall.npy", pf[:, 14])
slowest = int(np.argmax(pf[:, 14]))
print(f"slowest problem {slowest}: {pf[slowest, 14] / 100:.0f} us wall, admm {admm[slowest]:.0f}")
tot = pf[:, 13].sum()
for k, name in [kv for kv in enumerate(BatchTrustRegionSQP.PROFILE_SLOTS) if kv[0] != 14 and not kv[1].startswith('unused') and not kv[1].startswith('n_')]:
    v = pf[:, k].sum()
    per_admm = v / admm.sum()
    print(f"  {k:2d} {name:<16} {100 * v / tot:6.1f}%   {per_admm:10.0f} cyc/admm-iter   "
          f"{v / qps.sum():12.0f} cyc/qp")

# the slowest problems: per-ADMM breakdown and contact-row load
print("slowest problems (per-ADMM cycles by phase):")
nh_avg = np.array([r.n_hinge_admm for r in res], dtype=np.float64) / np.maximum(admm, 1)
for b in np.argsort(-pf[:, 14])[:4]:
    parts = "  ".join(f"{BatchTrustRegionSQP.PROFILE_SLOTS[k]}={pf[b, k] / max(admm[b], 1):.0f}"
                      for k in (0, 1, 3, 5, 6, 8, 9, 10, 11, 15, 16, 17, 18, 34, 19, 20, 21, 22, 23, 24, 25, 35, 36, 26, 30, 31, 32, 33))
    print(f"  problem {b}: {pf[b, 14] / 100:.0f} us, admm {admm[b]:.0f}, qp {qps[b]:.0f}, sqp {sqp[b]:.0f}, "
          f"mean hinge rows {nh_avg[b]:.0f}, contact rows {res[b].n_contact_rows}\n    {parts}")
print(f"mean hinge rows per ADMM iteration (all): {nh_avg.mean():.1f}, max {nh_avg.max():.0f}")
print(f"per QP: full primal-infeasibility checks {pf[:, 27].sum() / qps.sum():.2f}, "
      f"full dual-infeasibility checks {pf[:, 28].sum() / qps.sum():.2f}, factorisations {pf[:, 29].sum() / qps.sum():.2f}")
