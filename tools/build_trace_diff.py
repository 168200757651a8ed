"""Per-QP traces of one build tree, and where two builds first part (diagnostic
for build-dependent results of the fused kernel):

    python tools/build_trace_diff.py <root> <tag> [config] [batch]
    python tools/build_trace_diff.py --compare <tagA> <tagB>

The first form solves config (default C) with thip_debug_trace on (env THIP_PATH:
thip_debug_set_path bits, e.g. abi.DEBUG_NO_SEGMENT) and saves x,
statuses, counters and the trace records to gpurun_out/trace_<tag>.npz; the
second prints, per problem whose results differ, the first QP whose record
differs and both records around it (fields: include/trajopt_hip.h THIP_TRACE_W).
"""
import sys

import numpy as np

np.set_printoptions(linewidth=220, precision=9)
NAMES = ["warm", "rho0", "admm", "st", "pol", "rho1", "prim", "dual", "sum|x|", "box", "old", "new", "approx",
         "exact", "ratio", "dec"]

if sys.argv[1] == "--compare":
    a, b = (np.load(f"gpurun_out/trace_{t}.npz") for t in sys.argv[2:4])
    d = np.abs(a["x"] - b["x"]).reshape(a["x"].shape[0], -1).max(1)
    print(f"problems differing {(d > 0).sum()} of {len(d)}; statuses A {np.bincount(a['st'], minlength=8)} "
          f"B {np.bincount(b['st'], minlength=8)}; SQP iters A {a['sqp'].sum()} B {b['sqp'].sum()}")
    shown = 0
    for p in np.nonzero(d > 0)[0]:
        ta, tb = a["tr"][p][: a["cnt"][p]], b["tr"][p][: b["cnt"][p]]
        n = min(len(ta), len(tb))
        first = next((i for i in range(n) if not np.array_equal(ta[i], tb[i])), n)
        print(f"== problem {p}: |dx| {d[p]:.2e}, status {a['st'][p]} / {b['st'][p]}, QPs {len(ta)} / {len(tb)}, "
              f"first differing QP {first}")
        for i in range(max(0, first - 1), min(n, first + 2)):
            print(f"   QP {i} A: " + " ".join(f"{k}={v:.6g}" for k, v in zip(NAMES, ta[i])))
            print(f"   QP {i} B: " + " ".join(f"{k}={v:.6g}" for k, v in zip(NAMES, tb[i])))
        shown += 1
        if shown >= 12:
            break
    sys.exit(0)

root, tag = sys.argv[1], sys.argv[2]
cfg = sys.argv[3] if len(sys.argv) > 3 else "C"
B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
sys.path.insert(0, root + "/trajopt-1_amd")
from trajopt_amd import problems  # noqa: E402
from trajopt_amd.runtime import BatchTrustRegionSQP  # noqa: E402

wl = problems.make_workload(cfg, B)
path = int(__import__("os").environ.get("THIP_PATH", "0"))  # thip_debug_set_path bits (abi.DEBUG_*)
if path:
    from trajopt_amd import abi  # noqa: E402

    assert abi.load_hip().thip_debug_set_path(path) == 0
s = BatchTrustRegionSQP(wl)
s.enable_trace(1024)
x, res = s.optimize()
tr = s.get_trace()
s.close()
cnt = np.array([len(t) for t in tr])
rec = np.zeros((B, max(cnt.max(), 1), 16))
for p, t in enumerate(tr):
    if len(t):
        rec[p, : len(t)] = np.asarray(t)[:, :16]
np.savez(f"gpurun_out/trace_{tag}.npz", x=x, st=np.array([r.status for r in res]),
         sqp=np.array([r.n_sqp_iters for r in res]), admm=np.array([r.n_admm_iters for r in res]), tr=rec, cnt=cnt)
print(f"{tag}: {cfg} x{B} statuses {np.bincount([r.status for r in res], minlength=8)}, "
      f"SQP {sum(r.n_sqp_iters for r in res)}, ADMM {sum(r.n_admm_iters for r in res)}", flush=True)
