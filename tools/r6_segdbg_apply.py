"""Round 6 diagnostic (scratch trees only): tools/r6_dbg_apply.py's dump of one
problem's QP (THIP_DBG_PROB, THIP_DBG_QP; file THIP_DBG_OUT), extended to the
register-resident segment: after every admm_step and after every segment
(admm_iterations) of that QP, the first 48 records: x over the columns and z
over the rows, record[5] = 1 for a segment record, record[6] = its iterations.

    python tools/r6_segdbg_apply.py <tree>
"""
import runpy
import sys

runpy.run_path(__file__.replace("r6_segdbg_apply.py", "r6_dbg_apply.py"), run_name="__main__")
root = sys.argv[1] + "/trajopt-1_amd/csrc/"
p = root + "sqp_kernel.hip"
s = open(p).read()
old = """__device__ void admm_iterations(Ctx& c, Solver& sv, int n_iter, Norms* res)
{
  admm_segment<1, 1>(c, sv, n_iter, res);
}"""
new = """__device__ void admm_iterations(Ctx& c, Solver& sv, int n_iter, Norms* res)
{
  admm_segment<1, 1>(c, sv, n_iter, res);
  if (c.s->dbg && c.s->n_qp == c.s->dbg_qp && c.s->dbg_it < 48)
  {
    const int tid = c.tid, nc = c.nc(), m = c.m();
    const double* XA = c.a(A_XA0);
    const double* Zs = c.a(A_Z0);
    double* row = c.s->dbg + (long long)c.s->dbg_it * 8192;
    if (tid == 0)
    {
      row[0] = c.s->n_qp;
      row[1] = nc;
      row[2] = m;
      row[3] = c.s->n_h;
      row[4] = c.L.seg_ok;
      row[5] = 1;
      row[6] = n_iter;
    }
    for (int k = tid; k < nc && 8 + k < 4096; k += kBlock)
      row[8 + k] = XA[k];
    for (int k = tid; k < m && 4096 + k < 8192; k += kBlock)
      row[4096 + k] = Zs[k];
    BSYNC();
    if (tid == 0)
      c.s->dbg_it++;
    BSYNC();
  }
}"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
print("segment dump applied to", sys.argv[1])
