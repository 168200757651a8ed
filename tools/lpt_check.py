"""Dispatch-order study (diagnostic): how well does the initial contact count
predict a problem's solve time, and what would a longest-first dispatch order
give?  Simulates the hardware's in-order workgroup dispatch (workgroup i on
XCD i % 8, each XCD filling its free CUs in order) with the measured
per-problem times.

    python tools/lpt_check.py C 1024
"""
import heapq
import sys

sys.path.insert(0, "trajopt-1_amd")
import numpy as np

from trajopt_amd import problems
from trajopt_amd.runtime import BatchTrustRegionSQP

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
wl = problems.make_workload(cfg, B)
s = BatchTrustRegionSQP(wl)
s.upload()
s.enable_profile(True)
s.run()
x, res = s.download()
pf = s.get_profile().astype(np.float64)
dur = pf[:, 14] / 100.0  # us
rows = s.collision_rows(wl.init)
n0 = np.array([len(r) for r in rows], dtype=np.float64)
# contact depth: sum of (margin + buffer - d)+ over the initial contacts
depth = np.array([float(np.sum(np.maximum(0.075 - r[:, 5], 0.0))) if len(r) else 0.0 for r in rows])
print(f"kernel {s.kernel_ms():.1f} ms; problem time mean {dur.mean():.0f} us, max {dur.max():.0f} us")


def rank(v):
    o = np.argsort(v, kind="stable")
    r = np.empty_like(o)
    r[o] = np.arange(len(v))
    return r.astype(np.float64)


for name, v in (("initial contacts", n0), ("initial depth", depth)):
    print(f"spearman(time, {name}) = {np.corrcoef(rank(dur), rank(v))[0, 1]:.3f}")


def makespan(order, n_xcd=8, cus=32):
    heaps = [[0.0] * cus for _ in range(n_xcd)]
    for i, p in enumerate(order):
        h = heaps[i % n_xcd]
        t = heapq.heappop(h)
        heapq.heappush(h, t + dur[p])
    return max(max(h) for h in heaps)


nat = np.arange(B)
print(f"simulated makespan: natural {makespan(nat) / 1e3:.0f} ms, "
      f"by initial contacts {makespan(np.argsort(-n0, kind='stable')) / 1e3:.0f} ms, "
      f"by depth {makespan(np.argsort(-depth, kind='stable')) / 1e3:.0f} ms, "
      f"by true time {makespan(np.argsort(-dur, kind='stable')) / 1e3:.0f} ms, "
      f"bound max(problem) {dur.max() / 1e3:.0f} ms, mean load {dur.sum() / 256 / 1e3:.0f} ms")
