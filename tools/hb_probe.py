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

abi.load_hip()
for B in [int(a) for a in sys.argv[1:]] or [1, 8, 32]:
    wl = sharding.rank_workload("B", B, 0)
    texts = [host.hostloop_workload_json(wl, b) for b in range(B)]
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
