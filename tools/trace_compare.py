"""Per-QP traces of the HIP path and the oracle side by side (diagnostic).

    python tools/trace_compare.py <variant> <problem> [<problem> ...]

<variant> is a name from tests/test_gpu.py VARIANTS, or A / B / C / J
(problems.make_workload at its default batch of 32).  For each problem: one
line per QP solve -- warm start, rho in/out, ADMM iterations, OSQP status,
polish status, residuals, sum|x*|, trust box, the step's ratio and decision --
GPU first, oracle second, and the first QP where they part.
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "trajopt-1_amd", REPO / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402  (diagnostic tool: the checker)
from parity import subset  # noqa: E402
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402


def workload(name):
    if "@" in name:  # e.g. C@613: problem 613 of config C alone (the full-batch tests' indexing)
        cfg, first = name.split("@")
        return problems.make_workload(cfg, 1, first_problem=int(first))
    if name in ("A", "B", "C", "J"):
        return problems.make_workload(name, 32)
    if name == "E":
        return problems.make_workload("E", 4)
    if name == "Ccont":
        wl = problems.make_workload("C", 32, first_problem=200)
        wl.desc.coll_continuous = 1
        return wl
    if name == "Ccnt":
        wl = problems.make_workload("C", 32, first_problem=64)
        wl.desc.coll_is_cnt = 1
        return wl
    import test_gpu

    try:
        return test_gpu._variant(name)
    except KeyError:
        return test_gpu._joint_acc_variant(name)  # B-acc, C-acc, ... (JointAccEqCost)


def fmt(r):
    return (f"ws{int(r[0])} rho {r[1]:.3e}->{r[5]:.3e} it {int(r[2]):5d} st {int(r[3]):2d} pol {int(r[4]):2d} "
            f"pr {r[6]:.2e} dr {r[7]:.2e} |x| {r[8]:.12e} tb {r[9]:.3e} ratio {r[14]: .6e} dec {int(r[15])}")


def main():
    name = sys.argv[1]
    probs = [int(a) for a in sys.argv[2:]]
    wl = workload(name)
    s = BatchTrustRegionSQP(wl)
    s.enable_trace(4096)
    x, res = s.optimize()
    tr = s.get_trace()
    s.close()
    for b in probs:
        _, ro, to = oracle.solve_trace(wl, b, cap=4096)
        xo, _ = oracle.solve(subset(wl, [b]), n_threads=1)
        print(f"=== {name} problem {b}: gpu status {res[b].status} cost {res[b].total_cost:.10g} sqp {res[b].n_sqp_iters} "
              f"qp {res[b].n_qp_solves} | oracle status {ro.status} cost {ro.total_cost:.10g} sqp {ro.n_sqp_iters} "
              f"qp {ro.n_qp_solves} | max|dx| {np.abs(x[b] - xo[0]).max():.3e}")
        tg = tr[b]
        split = None
        for k in range(max(len(tg), len(to))):
            g = fmt(tg[k]) if k < len(tg) else "-"
            o = fmt(np.concatenate([to[k], np.zeros(6)]) if len(to[k]) < 16 else to[k]) if k < len(to) else "-"
            if split is None and k < len(tg) and k < len(to) and abs(tg[k][8] - to[k][8]) > 1e-9 * max(1, abs(to[k][8])):
                split = k
            mark = " <== first |x| difference" if split == k else ""
            print(f"{k:3d} G {g}{mark}\n    O {o}")


if __name__ == "__main__":
    main()
