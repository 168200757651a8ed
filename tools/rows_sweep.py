"""Contact rows of the fused kernel vs the oracle along the straight path from
each problem's initial trajectory to the oracle's solution (diagnostic).

    python tools/rows_sweep.py <C|Ccont|Ccnt|E> [n_problems] [first_problem] [steps]
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "trajopt-1_amd", REPO / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402  (diagnostic tool: the checker)
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

name = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
first = int(sys.argv[3]) if len(sys.argv) > 3 else 200
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 21
wl = problems.make_workload("E" if name == "E" else "C", B, first_problem=first)
if name == "Ccont":
    wl.desc.coll_continuous = 1
if name == "Ccnt":
    wl.desc.coll_is_cnt = 1
xo, _ = oracle.solve(wl, n_threads=16)
s = BatchTrustRegionSQP(wl)
worst = 0.0
for k in range(steps):
    a = k / (steps - 1)
    x = (1 - a) * wl.init + a * xo
    rows = s.collision_rows(x)
    for b in range(B):
        rc = oracle.collision_rows(wl, b, x[b])
        rg = rows[b]
        if rg.shape != rc.shape or not np.array_equal(rg[:, [0, 1, 2, 3, 4, 7]], rc[:, [0, 1, 2, 3, 4, 7]]):
            print(f"step {k} problem {b}: {len(rg)} GPU rows vs {len(rc)} oracle rows")
            gk = {tuple(r[[0, 1, 2, 3, 4]].astype(int)): r for r in rg}
            ok = {tuple(r[[0, 1, 2, 3, 4]].astype(int)): r for r in rc}
            for key in sorted(set(gk) ^ set(ok)):
                r = gk.get(key, ok.get(key))
                print(f"   only in {'GPU' if key in gk else 'oracle'}: t,link,prim,sphere,sub {key} dist {r[5]:.17g}")
            continue
        d = np.abs(rg[:, 5:] - rc[:, 5:]).max() if len(rc) else 0.0
        worst = max(worst, d)
        if d > 1e-10:
            i = int(np.argmax(np.abs(rg[:, 5:] - rc[:, 5:]).max(1)))
            print(f"step {k} problem {b}: row {i} {rg[i, :5]} differs by {d:.3e}")
s.close()
print(f"{name}: worst value difference over matching rows {worst:.3e}")
