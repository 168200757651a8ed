"""Per-QP traces of torso_arm_8dof_C (config C on the 8-dof torso arm, 8
problems) from one build tree, saved for a side-by-side comparison of two
builds (diagnostic for the a.x-reuse OPT_FAILED, round 5).

    python tools/ax_trace.py <root> <tag>          # on the GPU box
    python tools/ax_trace.py --compare <tagA> <tagB> [problem]
"""
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = (np.load(f"gpurun_out/axtrace_{t}.npz") for t in sys.argv[2:4])
    probs = [int(sys.argv[4])] if len(sys.argv) > 4 else range(a["counts"].shape[0])
    for p in probs:
        na, nb = int(a["counts"][p]), int(b["counts"][p])
        first = None
        for q in range(min(na, nb)):
            ra, rb = a["trace"][p, q], b["trace"][p, q]
            if not np.array_equal(ra, rb):
                first = q
                break
        print(f"problem {p}: QPs {na} / {nb}, status {a['status'][p]} / {b['status'][p]}, "
              f"x bitwise {'equal' if np.array_equal(a['x'][p], b['x'][p]) else 'DIFFERENT'}, first differing QP {first}")
        if first is not None:
            for q in range(max(0, first - 1), min(first + 3, na, nb)):
                for tag, r in (("A", a["trace"][p, q]), ("B", b["trace"][p, q])):
                    print(f"  qp {q:3d} {tag}: ws{int(r[0])} rho {r[1]:.17e}->{r[5]:.17e} it {int(r[2])} st {int(r[3])} "
                          f"pol {int(r[4])} pr {r[6]:.17e} dr {r[7]:.17e} |x| {r[8]:.17e} tb {r[9]:.3e}")
    sys.exit(0)

root, tag = sys.argv[1], sys.argv[2]
sys.path.insert(0, root + "/trajopt-1_amd")
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

wl = problems.make_workload("C", 8, robot="torso_right_arm")
s = BatchTrustRegionSQP(wl)
s.enable_trace(2048)
x, res = s.optimize()
recs = s.get_trace()
s.close()
cnt = np.array([len(r) for r in recs])
tr = np.zeros((len(recs), max(cnt.max(), 1), recs[0].shape[1]))
for p, r in enumerate(recs):
    tr[p, : len(r)] = r
np.savez(f"gpurun_out/axtrace_{tag}.npz", trace=tr, counts=cnt, x=x, status=np.array([r.status for r in res]))
print(tag, [r.status for r in res], flush=True)
