"""Diagnostic: the trajopt_sqp product (GPU) against the oracle on the synthetic
cases of tests/tsqp_cases.py -- max |dx|, statuses and counters per case."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "trajopt-1_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
import numpy as np  # noqa: E402

import tsqp_cases  # noqa: E402
from oracle import oracle  # noqa: E402
from trajopt_amd import tsqp  # noqa: E402

for kind, seed in tsqp_cases.SYNTHETIC:
    spec = tsqp_cases.synthetic(kind, seed)
    x, r = tsqp.solve(spec)
    xo, ro = oracle.tsqp_solve(spec)
    print(f"{kind:9s} {seed} dx={np.abs(x - xo).max():.2e} {tsqp.STATUS[r.status]} it {r.overall_iteration}/{ro.overall_iteration} "
          f"admm {r.admm_iters}/{ro.admm_iters} merit {r.best_exact_merit:.9e}/{ro.best_exact_merit:.9e}", flush=True)
