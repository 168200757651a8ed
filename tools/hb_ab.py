"""A/B of the generic QP kernel's forward solve (qp_csc.hip): config HB's
host-loop batch solved once, its wall time, SQP iterations and final
trajectories saved under a tag; `compare` checks two tags bitwise.

    python tools/hb_ab.py run <tag> [batch]      (THIP_QP_LEVEL_SOLVE=1: the level-by-level baseline)
    python tools/hb_ab.py compare <tag_a> <tag_b>
"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "trajopt-1_amd"))
OUT = ROOT / "gpurun_out"

if sys.argv[1] == "compare":
    a = np.load(OUT / f"hb_x_{sys.argv[2]}.npy")
    b = np.load(OUT / f"hb_x_{sys.argv[3]}.npy")
    d = np.abs(a - b).max(axis=1)
    print(f"{sys.argv[2]} vs {sys.argv[3]}: bitwise {bool(np.array_equal(a, b))}, max |dx| {d.max():.3e}, "
          f"problems differing {int((d > 0).sum())} / {len(d)}", flush=True)
    sys.exit(0)

from trajopt_amd import host, sharding  # noqa: E402

tag = sys.argv[2]
B = int(sys.argv[3]) if len(sys.argv) > 3 else 16
wl = sharding.rank_workload("B", B, 0)
texts = [host.hostloop_workload_json(wl, b) for b in range(B)]
pb = host.PreparedBatch(texts)
t0 = time.perf_counter()
x, res = pb.solve()
t1 = time.perf_counter()
st = pb.stats()
pb.close()
it = sum(r.n_sqp_iters for r in res)
np.save(OUT / f"hb_x_{tag}.npy", np.asarray(x, dtype=np.float64).reshape(B, -1))
print(f"HB x{B} [{tag}]: solve {t1 - t0:.2f} s, {it} SQP iters ({it / (t1 - t0):.1f} it/s), QP launches "
      f"{st['qp_launches']}, in launches {st['qp_seconds']:.2f} s, statuses {sorted(set(r.status for r in res))}",
      flush=True)
