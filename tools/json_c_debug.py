"""Debug: JSON-lowered config C (safety_margin_buffer 0.5) on the GPU vs the oracle, per-QP traces."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "trajopt-1_amd"), str(ROOT)]
import numpy as np  # noqa: E402

from trajopt_amd import host, problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402
from oracle import oracle  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
wl0 = problems.make_workload("C", B)
texts = [host.workload_to_json(wl0, b) for b in range(B)]
parts = [host.lower_json(t, wl0.scene[b]) for b, t in enumerate(texts)]
desc = parts[0][0]
wl = problems.Workload("json", desc, np.stack([p[1] for p in parts]), np.stack([p[2] for p in parts]), wl0.scene,
                       wl0.q_ref, None)
s = BatchTrustRegionSQP(wl)
s.enable_trace(256)
x, res = s.optimize()
tr = s.get_trace()
for b in range(B):
    r = res[b]
    print(f"gpu {b}: status {r.status} flags {r.flags} sqp {r.n_sqp_iters} qp {r.n_qp_solves} admm {r.n_admm_iters} "
          f"rows {r.n_contact_rows} cost {r.total_cost}")
    for k, rec in enumerate(tr[b][:12]):
        print("   qp", k, np.array2string(rec, precision=4, max_line_width=200))
    xo, ro, to = oracle.solve_trace(wl, b, cap=256)
    print(f"orc {b}: status {ro.status} sqp {ro.n_sqp_iters} qp {ro.n_qp_solves} admm {ro.n_admm_iters} cost {ro.total_cost}")
    for k, rec in enumerate(to[:12]):
        print("   qp", k, np.array2string(rec, precision=4, max_line_width=200))
print("h_cap probe:")
for b in range(B):
    d = np.linalg.norm(np.diff(x[b], axis=0), axis=1)
    print(f"  problem {b}: max LVS sub-states {int(np.ceil(d.max() / desc.coll_lvs)) + 1}")
rows = s.collision_rows(x, cap=20000)
print("  contacts at final x:", [len(r) for r in rows])
