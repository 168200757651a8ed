"""Does a problem's first QP predict its total solve time? (diagnostic)

    python tools/probe_check.py C 1024
"""
import heapq
import sys

sys.path.insert(0, "trajopt-1_amd")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
s = BatchTrustRegionSQP(problems.make_workload(cfg, B))
s.upload()
s.enable_profile(True)
s.enable_trace(512)
s.run()
x, res = s.download()
dur = s.get_profile().astype(np.float64)[:, 14] / 100.0
tr = s.get_trace()


def rank(v):
    o = np.argsort(v, kind="stable")
    r = np.empty_like(o)
    r[o] = np.arange(len(v))
    return r.astype(np.float64)


def makespan(order, n_xcd=8, cus=32):
    heaps = [[0.0] * cus for _ in range(n_xcd)]
    for i, p in enumerate(order):
        h = heaps[i % n_xcd]
        heapq.heappush(h, heapq.heappop(h) + dur[p])
    return max(max(h) for h in heaps) / 1e3


print(f"natural order makespan {makespan(np.arange(B)):.0f} ms, true LPT {makespan(np.argsort(-dur)):.0f} ms, "
      f"max problem {dur.max() / 1e3:.0f} ms")
for k in (1, 2, 3, 5):
    feat = np.array([t[:k, 2].sum() * (1 + t[:k, 8].mean() * 0) if len(t) else 0 for t in tr])
    sp = np.corrcoef(rank(dur), rank(feat))[0, 1]
    print(f"first {k} QPs' ADMM iterations: spearman {sp:.3f}, LPT-by-feature makespan "
          f"{makespan(np.argsort(-feat, kind='stable')):.0f} ms")
