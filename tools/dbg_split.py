"""Side-by-side per-QP traces (GPU vs oracle) of one problem: where do they split?
usage: python tools/dbg_split.py <variant-expr> <problem>"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "trajopt-1_amd"), str(ROOT)]
from oracle import oracle  # noqa: E402  (checker only)
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402


def main():
    cfg, B, first, cont, cnt, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
    wl = problems.make_workload(cfg, B, first_problem=first)
    wl.desc.coll_continuous = cont
    wl.desc.coll_is_cnt = cnt
    s = BatchTrustRegionSQP(wl, device=0)
    s.enable_trace(2048)
    x, res = s.optimize()
    tg = s.get_trace()[b]
    s.close()
    xo, ro = oracle.solve(wl, n_threads=16)
    _, _, to = oracle.solve_trace(wl, b, cap=2048)
    print("gpu status", res[b].status, res[b].max_cnt_viol, "oracle", ro[b].status, ro[b].max_cnt_viol)
    print("n", len(tg), len(to))
    for k in range(max(len(tg), len(to))):
        a = tg[k] if k < len(tg) else None
        o = to[k] if k < len(to) else None
        fa = " ".join(f"{v:.10g}" for v in a) if a is not None else "-"
        fo = " ".join(f"{v:.10g}" for v in o) if o is not None else "-"
        print(k, "G", fa)
        print(k, "O", fo)


main()
