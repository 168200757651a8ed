"""Config C diagnostics: GPU collision rows vs oracle, then SQP parity."""
import sys
import time

sys.path.insert(0, "trajopt-1_amd")
sys.path.insert(0, ".")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP
from oracle import oracle

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
wl = problems.make_workload("C", B)
xo, ro = oracle.solve(wl, n_threads=16)
s = BatchTrustRegionSQP(wl)
rows_g = s.collision_rows(xo)
worst = {"count": 0, "meta": 0, "dist": 0.0, "coef": 0.0, "const": 0.0}
for b in range(B):
    rg = rows_g[b]
    rc = oracle.collision_rows(wl, b, xo[b])
    if len(rg) != len(rc):
        print(f"problem {b}: row count gpu {len(rg)} oracle {len(rc)}")
        worst["count"] += 1
        continue
    if len(rc) == 0:
        continue
    meta = np.abs(rg[:, [0, 1, 2, 3, 4, 7]] - rc[:, [0, 1, 2, 3, 4, 7]]).max()
    worst["meta"] = max(worst["meta"], meta)
    worst["dist"] = max(worst["dist"], np.abs(rg[:, 5] - rc[:, 5]).max())
    worst["coef"] = max(worst["coef"], np.abs(rg[:, 8:-1] - rc[:, 8:-1]).max())
    worst["const"] = max(worst["const"], np.abs(rg[:, -1] - rc[:, -1]).max())
print("rows:", [len(r) for r in rows_g], "worst", worst)
t = time.time()
xg, rg = s.optimize()
tg = time.time() - t
s.close()
d = np.abs(xg - xo).reshape(B, -1).max(1)
st = [(a.status, o.status) for a, o in zip(rg, ro)]
print(f"SQP: gpu {tg:.2f}s; within 1e-5 {np.sum(d <= 1e-5)}/{B}; status equal {sum(a == o for a, o in st)}/{B}")
print("max|dx|", np.round(d, 8).tolist())
print("status", st, "flags", [r.flags for r in rg])
print("sqp iters gpu", [r.n_sqp_iters for r in rg], "cpu", [r.n_sqp_iters for r in ro])
print("cost gpu", [round(r.total_cost, 6) for r in rg])
print("cost cpu", [round(r.total_cost, 6) for r in ro])
