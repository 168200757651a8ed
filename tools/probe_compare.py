"""Compare two caller-side probe dumps (tools/r6_segprobe_apply.py): per ADMM
iteration, the largest |difference| in x, z and y, and where the first large
one sits (column / row kind).

    python tools/probe_compare.py <a.bin> <b.bin> [n_fixed_rows n_abs D]
"""
import sys

import numpy as np

REC, NREC = 12288, 64
a = np.fromfile(sys.argv[1]).reshape(NREC, REC)
b = np.fromfile(sys.argv[2]).reshape(NREC, REC)
nfr, nab, D = (int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (7, 174, 7)
nx = 30 * D
for i in range(NREC):
    if a[i, 5] == 0 and b[i, 5] == 0:
        break
    n, m, nh = int(a[i, 1]), int(a[i, 2]), int(a[i, 3])
    xa, xb = a[i, 16:16 + n], b[i, 16:16 + n]
    za, zb = a[i, 4096:4096 + m], b[i, 4096:4096 + m]
    ya, yb = a[i, 8192:8192 + m], b[i, 8192:8192 + m]
    dx, dz, dy = np.abs(xa - xb), np.abs(za - zb), np.abs(ya - yb)
    nr = nfr + nab
    nc_base = nx + 2 * nab
    m_base = nr + nc_base

    def rowkind(r):
        if r < nfr:
            return f"fixed {r}"
        if r < nr:
            return f"cartpose {r - nfr}"
        if r < m_base:
            col = r - nr
            return f"bound of col {col}" + (f" (t {col // D}, j {col % D})" if col < nx else " (aux)")
        h = (r - m_base) // 2
        return f"hinge {h}" + (" bound" if (r - m_base) % 2 else "")

    def colkind(col):
        if col < nx:
            return f"x t {col // D} j {col % D}"
        if col < nc_base:
            return f"aux {col - nx}"
        return f"hinge var {col - nc_base}"

    line = (f"it {int(a[i, 5])}/{int(b[i, 5])} seg {int(a[i, 4])}/{int(b[i, 4])} n {n} m {m} nh {nh}: "
            f"max|dx| {dx.max():.3e} ({colkind(int(dx.argmax()))}) max|dz| {dz.max():.3e} ({rowkind(int(dz.argmax()))}) "
            f"max|dy| {dy.max():.3e} ({rowkind(int(dy.argmax()))})")
    print(line)
    if max(dx.max(), dz.max(), dy.max()) > 1e-6:
        for name, d, kind in (("x", dx, colkind), ("z", dz, rowkind), ("y", dy, rowkind)):
            idx = np.argsort(-d)[:6]
            print("   worst", name, [(kind(int(k)), f"{d[k]:.2e}") for k in idx if d[k] > 1e-9])
        if i > 3:
            break
