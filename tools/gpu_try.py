"""Scratch GPU check: GPU vs oracle on small batches of configs A and B."""
import sys, time
sys.path.insert(0, "trajopt-1_amd"); sys.path.insert(0, ".")
import numpy as np
from trajopt_amd import problems, abi
from trajopt_amd.runtime import BatchTrustRegionSQP
from oracle import oracle

for cfg, B in (("A", 8), ("B", 8)):
    wl = problems.make_workload(cfg, B)
    s = BatchTrustRegionSQP(wl)
    # linearization parity at init
    e_g, j_g = s.linearize(wl.init)
    e_o, j_o = oracle.linearize(wl, wl.init)
    print(cfg, "linearize max|err diff| %.3e max|jac diff| %.3e" % (np.abs(e_g - e_o).max(), np.abs(j_g - j_o).max()))
    t = time.time()
    xg, rg = s.optimize()
    tg = time.time() - t
    print(cfg, "gpu wall %.3f s kernel %.3f ms" % (tg, s.kernel_ms()))
    xo, ro = oracle.solve(wl)
    for b in range(B):
        a, o = rg[b], ro[b]
        print(cfg, b, "gpu", abi.OPT_STATUS[a.status], a.n_sqp_iters, a.n_qp_solves, a.n_admm_iters, "%.6g" % a.total_cost,
              "| cpu", abi.OPT_STATUS[o.status], o.n_sqp_iters, o.n_qp_solves, o.n_admm_iters, "%.6g" % o.total_cost,
              "| max|dx| %.3e" % np.abs(xg[b] - xo[b]).max())
    s.close()
