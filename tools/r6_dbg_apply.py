"""Round 6 diagnostic (scratch trees only): per-ADMM-iteration dump of one
problem's QP (THIP_DBG_PROB, THIP_DBG_QP; file THIP_DBG_OUT) from the generic
step: after every admm_step of that QP (first 48 steps), x~ over the columns
and z over the rows.  Applied by editing a tree made by tools/mktree.sh:

    python tools/r6_dbg_apply.py <tree>
"""
import sys

root = sys.argv[1] + "/trajopt-1_amd/csrc/"


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
# the dump at the end of admm_step (after its last loop's stores)
edit("sqp_kernel.hip", "  BSYNC();\n  if (pf)\n    pf[31] += clock64() - tq;\n}",
     "  BSYNC();\n  if (pf)\n    pf[31] += clock64() - tq;\n"
     "  if (c.s->dbg && c.s->n_qp == c.s->dbg_qp && c.s->dbg_it < 48)\n  {\n"
     "    double* row = c.s->dbg + (long long)c.s->dbg_it * 8192;\n"
     "    if (tid == 0)\n    {\n      row[0] = c.s->n_qp;\n      row[1] = nc;\n      row[2] = m;\n      row[3] = c.s->n_h;\n"
     "      row[4] = c.L.seg_ok;\n    }\n"
     "    for (int k = tid; k < nc && 8 + k < 4096; k += kBlock)\n      row[8 + k] = XT[k];\n"
     "    for (int k = tid; k < m && 4096 + k < 8192; k += kBlock)\n      row[4096 + k] = z[k];\n"
     "    BSYNC();\n    if (tid == 0)\n      c.s->dbg_it++;\n    BSYNC();\n  }\n}")
edit("thip_api.hip", "struct thip_ctx\n{\n  int device = 0;\n", "struct thip_ctx\n{\n  double* dbg = nullptr;\n  int device = 0;\n")
edit("thip_api.hip", "  a.work = nullptr;\n  return a;\n}",
     "  a.work = nullptr;\n  static double* g_dbg = nullptr;\n  a.dbg = nullptr;\n"
     "  if (getenv(\"THIP_DBG_QP\"))\n  {\n"
     "    if (!g_dbg && hipMalloc(&g_dbg, 48 * 8192 * sizeof(double)) == hipSuccess)\n"
     "      hipMemset(g_dbg, 0, 48 * 8192 * sizeof(double));\n"
     "    a.dbg = g_dbg;\n    a.dbg_prob = atoi(getenv(\"THIP_DBG_PROB\"));\n    a.dbg_qp = atoi(getenv(\"THIP_DBG_QP\"));\n"
     "    ctx->dbg = g_dbg;\n  }\n  return a;\n}")
edit("thip_api.hip", "  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));\n  return THIP_OK;\n}\n\nconst double* thip_device_x",
     "  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));\n"
     "  if (ctx->dbg && getenv(\"THIP_DBG_OUT\"))\n  {\n"
     "    std::vector<double> h(48 * 8192);\n"
     "    hipMemcpy(h.data(), ctx->dbg, h.size() * sizeof(double), hipMemcpyDeviceToHost);\n"
     "    FILE* f = fopen(getenv(\"THIP_DBG_OUT\"), \"wb\");\n"
     "    if (f)\n    {\n      fwrite(h.data(), sizeof(double), h.size(), f);\n      fclose(f);\n    }\n  }\n"
     "  return THIP_OK;\n}\n\nconst double* thip_device_x")
print("dbg patch applied to", sys.argv[1])
