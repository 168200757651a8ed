"""Scratch: compare per-QP traces GPU vs oracle for the first problems that diverge."""
import sys
sys.path.insert(0, "trajopt-1_amd"); sys.path.insert(0, ".")
import numpy as np
from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP
from oracle import oracle
np.set_printoptions(linewidth=200, precision=6)
cfg = sys.argv[1] if len(sys.argv) > 1 else "A"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wl = problems.make_workload(cfg, B)
s = BatchTrustRegionSQP(wl)
s.enable_trace(1024)
xg, rg = s.optimize()
tr = s.get_trace()
for b in range(B):
    xo, ro, to = oracle.solve_trace(wl, b)
    tg = tr[b]
    d = np.abs(xg[b] - xo).max()
    print(f"== problem {b}: max|dx| {d:.3e}  nqp gpu {len(tg)} cpu {len(to)}")
    n = min(len(tg), len(to))
    first = None
    for i in range(n):
        a, o = tg[i], to[i]
        same = (a[0] == o[0]) and (a[2] == o[2]) and (a[3] == o[3]) and (a[4] == o[4]) and abs(a[8] - o[8]) <= 1e-6 * max(1, abs(o[8]))
        if not same:
            first = i
            break
    if first is None and len(tg) == len(to):
        print("   identical traces")
        continue
    f0 = n if first is None else first
    lo = max(0, f0 - 2)
    for i in range(lo, min(n, f0 + 3)):
        print("  qp", i, "gpu", tg[i][[0,1,2,3,4,5]], "xs %.10g tb %.3g pr %.2e dr %.2e" % (tg[i][8], tg[i][9], tg[i][6], tg[i][7]))
        print("  qp", i, "cpu", to[i][[0,1,2,3,4,5]], "xs %.10g tb %.3g pr %.2e dr %.2e" % (to[i][8], to[i][9], to[i][6], to[i][7]))
