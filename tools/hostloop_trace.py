"""Per-QP traces of a host-loop problem (the generic path: sco::BasicTrustRegionSQP
on the host, every QP on the GPU through GpuModel) beside the oracle's, and the
first QP where they part (diagnostic for the parity table's spread excusals of
single-problem drop-in fixtures, e.g. the reference's numerical_ik1.json).

    python tools/hostloop_trace.py <json file> [scene.npy]     # on the GPU box
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "trajopt-1_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

import dropin_cases as dc  # noqa: E402
from oracle import oracle  # noqa: E402  (diagnostic tool: the checker)
from trajopt_amd import abi, host  # noqa: E402


def fmt(r):
    return (f"ws{int(r[0])} rho {r[1]:.6e}->{r[5]:.6e} it {int(r[2]):5d} st {int(r[3]):2d} pol {int(r[4]):2d} "
            f"pr {r[6]:.3e} dr {r[7]:.3e} |x| {r[8]:.15e}")


def main():
    path = Path(sys.argv[1])
    text = path.read_text()
    p = subprocess.run([str(abi.LIB_DIR / "sqp_single"), "--trace", str(path)], capture_output=True, text=True,
                       timeout=300)
    if p.returncode != 0:
        raise SystemExit(p.stderr)
    head = p.stdout.splitlines()[0]
    xg = np.array([[float(v) for v in ln.split()] for ln in p.stdout.splitlines()[1:]])
    tg = np.array([[float(v) for v in ln.split()[1:]] for ln in p.stderr.splitlines() if ln.startswith("qp ")])
    wl = dc.json_workload(text, host)
    xo, ro, to = oracle.solve_trace(wl, 0, cap=4096)
    print(f"=== {path.name}: GPU host loop: {head}\n    oracle: status {ro.status} cost {ro.total_cost:.17g} "
          f"sqp {ro.n_sqp_iters} qp {ro.n_qp_solves}; max|dx| {np.abs(xg - xo).max():.3e}")
    split = None
    for k in range(max(len(tg), len(to))):
        g = fmt(tg[k]) if k < len(tg) else "-"
        o = fmt(to[k]) if k < len(to) else "-"
        if split is None and k < len(tg) and k < len(to) and abs(tg[k][8] - to[k][8]) > 1e-9 * max(1, abs(to[k][8])):
            split = k
        mark = " <== first |x*| difference > 1e-9 relative" if split == k else ""
        print(f"{k:3d} G {g}{mark}\n    O {o}")
    if split is not None:
        rel = abs(tg[split][8] - to[split][8]) / max(1, abs(to[split][8]))
        print(f"first parting: QP {split} (of {len(tg)} / {len(to)}), relative |x*| difference {rel:.2e}; "
              f"before it the largest relative |x*| difference was "
              f"{max([abs(tg[k][8] - to[k][8]) / max(1, abs(to[k][8])) for k in range(split)], default=0):.2e}")


if __name__ == "__main__":
    main()
