"""Round 6 diagnostic (scratch trees only): caller-side probe of the ADMM
iterates of one problem's QP (THIP_DBG_PROB, THIP_DBG_QP; file THIP_DBG_OUT).
For that QP the register-resident segment runs one ADMM iteration per call,
and qp_solve (the caller, so the segment's own code is untouched when it is a
separate function) records after every iteration, on either path: x, z and y
(records of 12288 doubles: [0] QP, [1] n, [2] m, [3] hinge rows, [4] segment
path, [5] iteration; x at 16.., z at 4096.., y at 8192..; 64 records).

    python tools/r6_segprobe_apply.py <tree>
"""
import sys

root = sys.argv[1] + "/trajopt-1_amd/csrc/"
REC, NREC = 12288, 64


def edit(f, old, new, count=1):
    p = root + f
    s = open(p).read()
    assert s.count(old) == count, (f, old[:60], s.count(old))
    s = s.replace(old, new)
    open(p, "w").write(s)


edit("layout.hpp", "  int* work;\n};", "  int* work;\n  double* dbg;\n  int dbg_prob, dbg_qp;\n};")
edit("sqp_kernel.hip", "  int hbits_x;                      // the hit bits are those of the last count pass (batched)\n};",
     "  int hbits_x;                      // the hit bits are those of the last count pass (batched)\n"
     "  double* dbg;\n  int dbg_qp, dbg_it;\n};")
edit("sqp_kernel.hip", "    ctl.prof = args.prof ? args.prof + (long long)b * kProfSlots : nullptr;\n",
     "    ctl.prof = args.prof ? args.prof + (long long)b * kProfSlots : nullptr;\n"
     "    ctl.dbg = (args.dbg && b == args.dbg_prob) ? args.dbg : nullptr;\n"
     "    ctl.dbg_qp = args.dbg_qp;\n    ctl.dbg_it = 0;\n")
# one iteration per segment for the probed QP
edit("sqp_kernel.hip", """      if (os.adaptive_rho && interval)
        stop = min(stop, (it + interval - 1) / interval * interval);
      // the segment computes""", """      if (os.adaptive_rho && interval)
        stop = min(stop, (it + interval - 1) / interval * interval);
      const bool probe = c.s->dbg && c.s->n_qp == c.s->dbg_qp;
      if (probe)
        stop = it;
      // the segment computes""")
# the record, after either path's iteration(s)
edit("sqp_kernel.hip", """    can_check = ct && (it % ct == 0);
    const int cur = c.s->cur;
    const double* xc = c.a(cur ? A_XA1 : A_XA0);
    const double* zc = c.a(cur ? A_Z1 : A_Z0);
""", """    can_check = ct && (it %% ct == 0);
    const int cur = c.s->cur;
    const double* xc = c.a(cur ? A_XA1 : A_XA0);
    const double* zc = c.a(cur ? A_Z1 : A_Z0);
    if (c.s->dbg && c.s->n_qp == c.s->dbg_qp && c.s->dbg_it < %d)
    {
      double* rec = c.s->dbg + (long long)c.s->dbg_it * %d;
      if (c.tid == 0)
      {
        rec[0] = c.s->n_qp;
        rec[1] = c.nc();
        rec[2] = c.m();
        rec[3] = c.s->n_h;
        rec[4] = seg ? 1 : 0;
        rec[5] = it;
      }
      for (int k = c.tid; k < c.nc() && k < 4080; k += kBlock)
        rec[16 + k] = xc[k];
      for (int k = c.tid; k < c.m() && k < 4096; k += kBlock)
      {
        rec[4096 + k] = zc[k];
        rec[8192 + k] = Y[k];
      }
      BSYNC();
      if (c.tid == 0)
        c.s->dbg_it++;
      BSYNC();
    }
""" % (NREC, REC))
edit("thip_api.hip", "struct thip_ctx\n{\n  int device = 0;\n", "struct thip_ctx\n{\n  double* dbg = nullptr;\n  int device = 0;\n")
edit("thip_api.hip", "  a.work = nullptr;\n  return a;\n}",
     "  a.work = nullptr;\n  static double* g_dbg = nullptr;\n  a.dbg = nullptr;\n"
     "  if (getenv(\"THIP_DBG_QP\"))\n  {\n"
     "    if (!g_dbg && hipMalloc(&g_dbg, %d * %d * sizeof(double)) == hipSuccess)\n"
     "      hipMemset(g_dbg, 0, %d * %d * sizeof(double));\n"
     "    a.dbg = g_dbg;\n    a.dbg_prob = atoi(getenv(\"THIP_DBG_PROB\"));\n    a.dbg_qp = atoi(getenv(\"THIP_DBG_QP\"));\n"
     "    ctx->dbg = g_dbg;\n  }\n  return a;\n}" % (NREC, REC, NREC, REC))
edit("thip_api.hip", "  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));\n  return THIP_OK;\n}\n\nconst double* thip_device_x",
     "  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));\n"
     "  if (ctx->dbg && getenv(\"THIP_DBG_OUT\"))\n  {\n"
     "    std::vector<double> h((size_t)%d * %d);\n"
     "    hipMemcpy(h.data(), ctx->dbg, h.size() * sizeof(double), hipMemcpyDeviceToHost);\n"
     "    FILE* f = fopen(getenv(\"THIP_DBG_OUT\"), \"wb\");\n"
     "    if (f)\n    {\n      fwrite(h.data(), sizeof(double), h.size(), f);\n      fclose(f);\n    }\n  }\n"
     "  return THIP_OK;\n}\n\nconst double* thip_device_x" % (NREC, REC))
print("segment probe applied to", sys.argv[1])
