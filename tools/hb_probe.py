"""Where a host-loop batch (bench.py --config HB) spends its time: for a few
batch sizes, prepared-batch set-up, solve wall time, SQP iterations, QP
launches / QPs and the wall time inside the QP launches.

    python tools/hb_probe.py [batch ...]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "trajopt-1_amd"))

from trajopt_amd import abi, host, sharding  # noqa: E402

import ctypes as C  # noqa: E402

hip = abi.load_hip()
hip.thip_qp_debug_profile.argtypes = [C.POINTER(C.c_longlong), C.c_int]
for B in [int(a) for a in sys.argv[1:]] or [1, 8, 32]:
    wl = sharding.rank_workload("B", B, 0)
    texts = [host.hostloop_workload_json(wl, b) for b in range(B)]
    hip.thip_qp_debug_profile(None, 1)
    t0 = time.perf_counter()
    pb = host.PreparedBatch(texts)
    t1 = time.perf_counter()
    x, res = pb.solve()
    t2 = time.perf_counter()
    st = pb.stats()
    sh = pb.qp_shape()
    pb.close()
    it = sum(r.n_sqp_iters for r in res)
    print(f"HB x{B}: setup {t1 - t0:.2f} s, solve {t2 - t1:.2f} s, {it} SQP iters ({it / (t2 - t1):.0f} it/s), "
          f"statuses {[r.status for r in res][:16]}, QP launches {st['qp_launches']}, QPs {st['qps']}, "
          f"in launches {st['qp_seconds']:.2f} s, {st['qp_bytes'] / 1e9:.2f} GB; QP shape {sh}", flush=True)
    pf = (C.c_longlong * 8)()
    hip.thip_qp_debug_profile(pf, 1)
    its = max(pf[4], 1)
    print("  first QP of each launch, cycles per ADMM iteration: " + ", ".join(
        f"{k} {pf[i] / its:.0f}" for i, k in enumerate(("copy+rhs", "kkt_solve", "updates", "checks")))
        + f"; iterations {pf[4]}, polish {pf[5]} cycles total; KKT solve level loops: forward "
        f"{pf[6] / its:.0f}, backward {pf[7] / its:.0f} (incl. polish solves)", flush=True)
