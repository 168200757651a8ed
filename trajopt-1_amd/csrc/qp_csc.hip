// Generic sparse QP solve with OSQP 1.0 semantics on gfx950 (the GpuModel
// backend of trajopt_sco::Model, include/trajopt_hip.h "Generic QP").
//
// The reference solves every convexified QP with OSQP 1.0 through
// sco::OSQPModel (trajopt_sco/src/osqp_interface.cpp:283-615).  This kernel
// runs that algorithm for a batch of QPs that share one sparsity pattern, one
// 256-thread workgroup per QP:
//   * modified Ruiz equilibration + cost scaling (settings.scaling passes);
//   * the rho vector (equality rows x1e3, free rows rho_min);
//   * the quasi-definite KKT [P + sigma I, A'; A, -diag(1/rho)] factored as a
//     sparse LDL^T in the QP's HBM workspace (no pivoting: a quasi-definite
//     matrix factors under any symmetric order; the pivot signs give OSQP's
//     convexity check).  The symbolic part runs once per pattern on the host
//     (thip_qp_create): QDLDL's role in OSQP -- a minimum-degree order (the
//     oracle's LdlSolver::order, the AMD role), the elimination tree, the
//     pattern of L -- plus what the GPU needs on top: the tree's levels.  The
//     numeric factor walks the levels bottom-up, one thread per pivot then
//     one per entry of the level's columns of L (each a merge of two rows of
//     L); the solves walk them up (rows of L) and down (columns of L) with
//     the permuted solve vector in LDS.  One __syncthreads per level, where
//     the dense factor needed one per row;
//   * ADMM with over-relaxation, termination on unscaled inf-norm residuals
//     every check_termination iterations, primal / dual infeasibility
//     certificates, iteration-based adaptive rho (refactorisation);
//   * polishing: active set from (z, y), the delta-regularised reduced KKT,
//     polish_refine_iter refinements on the unregularised one, OSQP's
//     acceptance test;
//   * warm start of (x, y, rho) as OSQPModel::createOrUpdateSolver passes it.
// The structured trajectory QPs of a TrajOptProb batch do not come here: they
// run sqp_kernel's block-tridiagonal path.  This path serves arbitrary
// sco::Model users (custom terms, JointAcc / JointJerk terms, the reference's
// small-problem and solver-interface tests, collision QPs with more contacts
// than the fused kernel's table).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/trajopt_hip.h"
#include "kkt_symbolic.hpp"

namespace thip_qp_dev
{
constexpr int kQB = 256;
constexpr long long kQpLdsBudget = 150 * 1024;  // dynamic LDS of a QP workgroup with its factor staged
constexpr double kInf = 1e30;             // OSQP_INFTY
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoTol = 1e-4, kRhoEq = 1e3;
constexpr double kMinScaling = 1e-4, kMaxScaling = 1e4;
constexpr double kDivTol = 1.0 / kInf;

// OSQP 1.0 status values (osqp_api_constants.h)
enum : int
{
  SOLVED = 1,
  SOLVED_INACCURATE = 2,
  PRIMAL_INFEASIBLE = 3,
  PRIMAL_INFEASIBLE_INACCURATE = 4,
  DUAL_INFEASIBLE = 5,
  DUAL_INFEASIBLE_INACCURATE = 6,
  MAX_ITER_REACHED = 7,
  NON_CVX = 9,
  UNSOLVED = 11,
};

// workspace arrays per QP (doubles), sizes n / m / nnz / N = n + m / N*N
enum Arr : int
{
  W_PX, W_AX, W_Q, W_L, W_U, W_D, W_DI, W_E, W_EI, W_TD, W_TE, W_RHO, W_RHOI, W_CT,
  W_X, W_XP, W_Z, W_ZP, W_Y, W_DX, W_DY, W_XT, W_AXV, W_PXV, W_ATY, W_RP, W_RD, W_T1, W_T2,
  W_PXS, W_PZS, W_PYS, W_RHS, W_RES, W_FLG, W_LX, W_DG, W_LV, W_SC, W_COUNT
};
// W_LX / W_DG: the factor (L values in row order, D); W_LV: the permuted solve
// vector when it does not fit LDS.
// W_SC: the scalars a resident workspace keeps between launches (thip_qp_setup ...
// thip_qp_solve_resident): cost scaling c and 1/c, the current rho, setup ok, and
// whether the ADMM KKT factor in W_LX must be rebuilt (polish factors its KKT in
// the same storage; OSQP keeps a separate polish factor)
enum : int
{
  SC_C = 0,
  SC_CINV,
  SC_RHO,
  SC_OK,
  SC_KKT_DIRTY,
  SC_COUNT
};
// resident-workspace operations (qp_resident_kernel), OSQP 1.0 API calls
enum : int
{
  OP_SETUP = 0,    // osqp_setup
  OP_UPDATE_VEC,   // osqp_update_data_vec
  OP_UPDATE_MAT,   // osqp_update_data_mat
  OP_WARM_START,   // osqp_warm_start
  OP_SOLVE,        // osqp_solve
};

struct QpPattern
{
  int n, m, nnz_p, nnz_a, N;  // N = n + m: the KKT dimension
  // P upper triangular CSC and its rows (entries (j, c >= j) of row j -> index into P values)
  const int *Pp, *Pi, *Prp, *Prj, *Prmap;
  // A CSC and its rows (-> index into A values)
  const int *Ap, *Ai, *Arp, *Arj, *Armap;
  // symbolic LDL^T of the permuted KKT (kkt_symbolic): perm[new] = old node
  // (x_j = j, row r = n + r); L rows (lrp, lrj: columns ascending); L columns
  // (lcp; lci = row, lcpos = position in the row order, lksrc = the KKT entry
  // it starts from: 2e = P value e, 2e + 1 = A value e, -1 = fill); dpd = the
  // P diagonal value of an x node (-1 none); nodes by etree level (lvp, lvn);
  // the level's column entries (fip; fik = column, fic = entry)
  const int *perm, *lrp, *lrj, *lcp, *lci, *lcpos, *lksrc, *dpd, *lvp, *lvn, *fip, *fik, *fic;
  int nlev;
  // the forward solve's passes of row segments (kkt_symbolic: fwp, fwk, fwa, fwb)
  const int *fwp, *fwk, *fwa, *fwb;
  int npass;
  int lds_vec;  // the permuted solve vector lives in LDS (else W_LV)
  // the whole factor in LDS (QP_LDS_*, staged at kernel entry): the solve
  // vector, L and D, and the index arrays the factor and the solves walk
  // (16-bit row / column indices)
  int lds_pat;
  long long lds_off[12];
  long long off[W_COUNT];
  long long stride;
};

struct QpArgs
{
  QpPattern pat;
  thip_osqp_settings s;
  const double *Pv, *qv, *Av, *lv, *uv;       // [batch][...]
  const double *x_ws, *y_ws, *rho_ws;         // warm start (null = cold)
  const int* ws_mask;                         // per QP: warm start (1) or cold (0); null = all as x_ws / y_ws
  double *x_out, *y_out;                      // [batch][n], [batch][m]
  thip_qp_info* info;                         // [batch]
  double* ws;                                 // [batch][stride]
  int batch;
};

struct Sh
{
  double red[kQB / 64];
  double c, cinv, rho;
  double prim_res, dual_res;
  int status, polish, iter, npos, fail, nred;
};

#define QFOR(i, n) for (int i = static_cast<int>(threadIdx.x); i < (n); i += kQB)

__device__ __forceinline__ double wave_max(double v)
{
  for (int o = 32; o > 0; o >>= 1)
    v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_sum(double v)
{
  for (int o = 32; o > 0; o >>= 1)
    v += __shfl_xor(v, o);
  return v;
}
__device__ double bmax(Sh& sh, double v)
{
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = sh.red[0];
  for (int w = 1; w < kQB / 64; ++w)
    r = fmax(r, sh.red[w]);
  return r;
}
__device__ double bsum(Sh& sh, double v)
{
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = sh.red[0];
  for (int w = 1; w < kQB / 64; ++w)
    r += sh.red[w];
  return r;
}
__device__ double norm_inf(Sh& sh, const double* v, int n)
{
  double a = 0;
  QFOR(i, n) a = fmax(a, fabs(v[i]));
  return bmax(sh, a);
}
__device__ double scaled_norm_inf(Sh& sh, const double* s, const double* v, int n)
{
  double a = 0;
  QFOR(i, n) a = fmax(a, fabs(s[i] * v[i]));
  return bmax(sh, a);
}
__device__ __forceinline__ double limit_scaling(double a)
{
  a = a < kMinScaling ? 1.0 : a;
  return a > kMaxScaling ? kMaxScaling : a;
}

// The arrays the factorisation and the solves walk: the pattern's (HBM) or
// their LDS copies (QpPattern::lds_pat: 16-bit indices).  The LDS view's
// pointers are address-space-3 typed, so its accesses are ds_* instructions: a
// generic pointer would make each a FLAT access, which pays the vector-memory
// latency even when it lands in LDS (the level loops are chains of dependent
// loads, so that latency is their whole cost).
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(3))) unsigned short lds_u16;
template <typename IX, typename IN, typename DB>
struct FacViewT
{
  const IX *lrj, *lcpos, *lci, *lvn;
  const IN *lrp, *lcp, *lvp;
  DB *LX, *DG;
  const IX *fwk, *fwa, *fwb;
  const IN* fwp;
};
using FacViewG = FacViewT<int, int, double>;
using FacViewL = FacViewT<lds_u16, lds_i32, lds_f64>;
// LDS layout of a staged factor (QpPattern::lds_off)
enum : int
{
  QL_LX = 0, QL_DG, QL_LRJ, QL_LCPOS, QL_LCI, QL_LVN, QL_LRP, QL_LVP,  // (lcp follows lrp)
  QL_FWK, QL_FWA, QL_FWB, QL_FWP, QL_COUNT
};

// phase cycles of workgroup 0's ADMM loop (diagnostic, thip_qp_debug_profile):
// [0] iterate copies + rhs, [1] KKT solves, [2] z / y / x updates, [3] residuals,
// termination and rho updates (incl. refactorisations), [4] iterations, [5] polish.
// Compiled in only with -DTHIP_QP_PROF=1 (csrc/Makefile EXTRA): the shipped
// kernels carry no clock reads or counter traffic on the solve's critical path.
#ifndef THIP_QP_PROF
#define THIP_QP_PROF 0
#endif
__device__ unsigned long long g_qp_prof[8];
__device__ __forceinline__ void qp_prof_add(int k, long long v)
{
  atomicAdd(&g_qp_prof[k], static_cast<unsigned long long>(v));  // concurrent launches on other streams
}


struct Qp
{
  const QpPattern& p;
  const thip_osqp_settings& s;
  double* w;
  Sh& sh;
  double* lv;  // the permuted solve vector [N] (LDS, or W_LV)
  int n, m;
  FacViewG fg;  // HBM
  FacViewL fs;  // LDS (p.lds_pat)
  bool persist;                 // keep W_LX / W_DG current (resident workspaces)
  __device__ double* a(int k) const { return w + p.off[k]; }
};

// Qp's factor views; with lds_pat, stage the index arrays and the current
// factor (W_LX, W_DG) into the dynamic LDS after the solve vector.  All threads.
__device__ void fac_views(Qp& q, char* lds)
{
  const QpPattern& p = q.p;
  q.fg = FacViewG{ p.lrj, p.lcpos, p.lci, p.lvn, p.lrp, p.lcp, p.lvp, q.a(W_LX), q.a(W_DG), p.fwk, p.fwa, p.fwb, p.fwp };
  if (!p.lds_pat)
    return;
  const int N = p.N, nl = static_cast<int>(p.lds_off[QL_DG] - p.lds_off[QL_LX]) / 8;  // entries of L
  double* LX = reinterpret_cast<double*>(lds + p.lds_off[QL_LX]);
  double* DG = reinterpret_cast<double*>(lds + p.lds_off[QL_DG]);
  unsigned short* lrj = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_LRJ]);
  unsigned short* lcpos = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_LCPOS]);
  unsigned short* lci = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_LCI]);
  unsigned short* lvn = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_LVN]);
  int* lrp = reinterpret_cast<int*>(lds + p.lds_off[QL_LRP]);
  int* lcp = lrp + (N + 1);
  int* lvp = reinterpret_cast<int*>(lds + p.lds_off[QL_LVP]);
  unsigned short* fwk = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_FWK]);
  unsigned short* fwa = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_FWA]);
  unsigned short* fwb = reinterpret_cast<unsigned short*>(lds + p.lds_off[QL_FWB]);
  int* fwp = reinterpret_cast<int*>(lds + p.lds_off[QL_FWP]);
  const double *GX = q.a(W_LX), *GD = q.a(W_DG);
  QFOR(e, nl)
  {
    LX[e] = GX[e];
    lrj[e] = static_cast<unsigned short>(p.lrj[e]);
    lcpos[e] = static_cast<unsigned short>(p.lcpos[e]);
    lci[e] = static_cast<unsigned short>(p.lci[e]);
  }
  QFOR(k, N)
  {
    DG[k] = GD[k];
    lvn[k] = static_cast<unsigned short>(p.lvn[k]);
  }
  QFOR(k, N + 1)
  {
    lrp[k] = p.lrp[k];
    lcp[k] = p.lcp[k];
  }
  QFOR(l, p.nlev + 1) lvp[l] = p.lvp[l];
  const int nseg = p.fwp[p.npass];
  QFOR(t, nseg)
  {
    fwk[t] = static_cast<unsigned short>(p.fwk[t]);
    fwa[t] = static_cast<unsigned short>(p.fwa[t]);
    fwb[t] = static_cast<unsigned short>(p.fwb[t]);
  }
  QFOR(l, p.npass + 1) fwp[l] = p.fwp[l];
  q.fs = FacViewL{ (const lds_u16*)lrj, (const lds_u16*)lcpos, (const lds_u16*)lci, (const lds_u16*)lvn,
                   (const lds_i32*)lrp, (const lds_i32*)lcp, (const lds_i32*)lvp, (lds_f64*)LX, (lds_f64*)DG,
                   (const lds_u16*)fwk, (const lds_u16*)fwa, (const lds_u16*)fwb, (const lds_i32*)fwp };
  __syncthreads();
}

// y = A x (rows), y = A' x (columns), y = P x (full symmetric from the upper triangle)
__device__ void a_mul(const Qp& q, const double* x, double* y)
{
  const double* AX = q.a(W_AX);
  QFOR(r, q.m)
  {
    double v = 0;
    for (int e = q.p.Arp[r]; e < q.p.Arp[r + 1]; ++e)
      v += AX[q.p.Armap[e]] * x[q.p.Arj[e]];
    y[r] = v;
  }
}
__device__ void at_mul(const Qp& q, const double* x, double* y)
{
  const double* AX = q.a(W_AX);
  QFOR(j, q.n)
  {
    double v = 0;
    for (int e = q.p.Ap[j]; e < q.p.Ap[j + 1]; ++e)
      v += AX[e] * x[q.p.Ai[e]];
    y[j] = v;
  }
}
__device__ void p_mul(const Qp& q, const double* x, double* y)
{
  const double* PX = q.a(W_PX);
  QFOR(j, q.n)
  {
    double v = 0;
    for (int e = q.p.Pp[j]; e < q.p.Pp[j + 1]; ++e)  // (i, j), i <= j
      v += PX[e] * x[q.p.Pi[e]];
    for (int e = q.p.Prp[j]; e < q.p.Prp[j + 1]; ++e)  // (j, c), c > j
      if (q.p.Prj[e] != j)
        v += PX[q.p.Prmap[e]] * x[q.p.Prj[e]];
    y[j] = v;
  }
}

// inf-norm of the full symmetric P's columns
__device__ void p_col_norm(const Qp& q, double* out)
{
  const double* PX = q.a(W_PX);
  QFOR(j, q.n)
  {
    double v = 0;
    for (int e = q.p.Pp[j]; e < q.p.Pp[j + 1]; ++e)
      v = fmax(v, fabs(PX[e]));
    for (int e = q.p.Prp[j]; e < q.p.Prp[j + 1]; ++e)
      v = fmax(v, fabs(PX[q.p.Prmap[e]]));
    out[j] = v;
  }
}

// modified Ruiz equilibration (OSQP scale_data)
__device__ void scale_data(Qp& q)
{
  const int n = q.n, m = q.m;
  double *PX = q.a(W_PX), *AX = q.a(W_AX), *Q = q.a(W_Q), *D = q.a(W_D), *E = q.a(W_E), *TD = q.a(W_TD),
         *TE = q.a(W_TE);
  if (threadIdx.x == 0)
    q.sh.c = 1.0;
  QFOR(j, n) D[j] = 1.0;
  QFOR(r, m) E[r] = 1.0;
  __syncthreads();
  for (int it = 0; it < q.s.scaling; ++it)
  {
    p_col_norm(q, TD);
    __syncthreads();
    QFOR(j, n)
    {
      double v = 0;
      for (int e = q.p.Ap[j]; e < q.p.Ap[j + 1]; ++e)
        v = fmax(v, fabs(AX[e]));
      TD[j] = 1.0 / sqrt(limit_scaling(fmax(TD[j], v)));
    }
    QFOR(r, m)
    {
      double v = 0;
      for (int e = q.p.Arp[r]; e < q.p.Arp[r + 1]; ++e)
        v = fmax(v, fabs(AX[q.p.Armap[e]]));
      TE[r] = 1.0 / sqrt(limit_scaling(v));
    }
    __syncthreads();
    QFOR(j, n)
    for (int e = q.p.Pp[j]; e < q.p.Pp[j + 1]; ++e)
      PX[e] = (PX[e] * TD[q.p.Pi[e]]) * TD[j];
    QFOR(j, n)
    for (int e = q.p.Ap[j]; e < q.p.Ap[j + 1]; ++e)
      AX[e] = (AX[e] * TE[q.p.Ai[e]]) * TD[j];
    QFOR(j, n)
    {
      Q[j] *= TD[j];
      D[j] *= TD[j];
    }
    QFOR(r, m) E[r] *= TE[r];
    __syncthreads();
    // cost normalisation
    p_col_norm(q, TD);
    __syncthreads();
    double s = 0;
    QFOR(j, n) s += TD[j];
    s = bsum(q.sh, s);
    double c_temp = (n > 0) ? s / static_cast<double>(n) : 0.0;
    const double qn = limit_scaling(norm_inf(q.sh, Q, n));
    c_temp = fmax(c_temp, qn);
    c_temp = 1.0 / limit_scaling(c_temp);
    QFOR(j, n)
    for (int e = q.p.Pp[j]; e < q.p.Pp[j + 1]; ++e)
      PX[e] *= c_temp;
    QFOR(j, n) Q[j] *= c_temp;
    if (threadIdx.x == 0)
      q.sh.c *= c_temp;
    __syncthreads();
  }
  double *DI = q.a(W_DI), *EI = q.a(W_EI), *L = q.a(W_L), *U = q.a(W_U);
  QFOR(j, n) DI[j] = 1.0 / D[j];
  QFOR(r, m)
  {
    EI[r] = 1.0 / E[r];
    L[r] *= E[r];
    U[r] *= E[r];
  }
  if (threadIdx.x == 0)
    q.sh.cinv = 1.0 / q.sh.c;
  __syncthreads();
}

__device__ void set_rho_vec(Qp& q)
{
  double *L = q.a(W_L), *U = q.a(W_U), *RHO = q.a(W_RHO), *RHOI = q.a(W_RHOI), *CT = q.a(W_CT);
  const double rho = q.sh.rho;
  QFOR(r, q.m)
  {
    double ct, rv;
    if (L[r] < -kInf * kMinScaling && U[r] > kInf * kMinScaling)
    {
      ct = -1;
      rv = kRhoMin;
    }
    else if (U[r] - L[r] < kRhoTol)
    {
      ct = 1;
      rv = kRhoEq * rho;
    }
    else
    {
      ct = 0;
      rv = rho;
    }
    CT[r] = ct;
    RHO[r] = rv;
    RHOI[r] = 1.0 / rv;
  }
  __syncthreads();
}

// The KKT entry an L entry starts from (kkt_symbolic's lksrc code).  In polish
// mode the rows outside the active set are decoupled: their A entries read 0.
__device__ __forceinline__ double kkt_entry(const Qp& q, int code, bool pol, const double* FLG)
{
  if (code < 0)
    return 0.0;
  const int e = code >> 1;
  if (!(code & 1))
    return q.a(W_PX)[e];
  if (pol && FLG[q.p.Ai[e]] == 0.0)
    return 0.0;
  return q.a(W_AX)[e];
}

// KKT diagonal of permuted node k: ADMM [P + sigma I; -diag(1/rho)], polish
// [P + delta I; -delta I] on the active rows and -1 on the decoupled ones
// (their solution component is 0: OSQP's reduced KKT, without re-analysis)
__device__ __forceinline__ double kkt_diag(const Qp& q, int k, bool pol, const double* FLG)
{
  const int o = q.p.perm[k];
  if (o < q.n)
  {
    const int e = q.p.dpd[k];
    const double p = (e >= 0) ? q.a(W_PX)[e] : 0.0;
    return p + (pol ? q.s.delta : q.s.sigma);
  }
  const int r = o - q.n;
  if (pol)
    return FLG[r] != 0.0 ? -q.s.delta : -1.0;
  return -q.a(W_RHOI)[r];
}

// numeric LDL^T of the permuted KKT over the symbolic pattern, level by level
// of the elimination tree: first the level's pivots
//     D_k = K_kk - sum_j L_kj^2 D_j                (row k of L is final: its
//                                                   columns are descendants)
// then every entry of the level's columns
//     L_ik = (K_ik - sum_{j < k} L_ij D_j L_kj) / D_k
// as a merge of rows i and k (both ascending).  sh.npos = positive pivots,
// sh.fail = 1 on a zero / non-finite pivot.
// s - sum over e in [e0, e1) of LX[e] w[j[e]], in order (the same expression
// as the plain loop, so the same contraction and rounding), eight entries'
// loads issued before their products: one memory round trip per eight
// entries instead of one per entry (a long row near the tree's root is a
// serial chain otherwise)
template <typename PL, typename PJ, typename PW>
__device__ __forceinline__ double row_sub(double s, PL LX, PJ j, PW w, int e0, int e1)
{
  int e = e0;
  for (; e + 8 <= e1; e += 8)
  {
    double a[8], b[8];
    int jj[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
    {
      a[u] = LX[e + u];
      jj[u] = j[e + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      b[u] = w[jj[u]];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      s -= a[u] * b[u];
  }
  for (; e < e1; ++e)
    s -= LX[e] * w[j[e]];
  return s;
}
// the same over column entries c in [c0, c1): LX[pos[c]] w[i[c]]
template <typename PL, typename PJ, typename PW>
__device__ __forceinline__ double col_sub(double s, PL LX, PJ pos, PJ i, PW w, int c0, int c1)
{
  int c = c0;
  for (; c + 8 <= c1; c += 8)
  {
    double a[8], b[8];
    int pp[8], ii[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
    {
      pp[u] = pos[c + u];
      ii[u] = i[c + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
    {
      a[u] = LX[pp[u]];
      b[u] = w[ii[u]];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      s -= a[u] * b[u];
  }
  for (; c < c1; ++c)
    s -= LX[pos[c]] * w[i[c]];
  return s;
}

template <typename V, typename PW>
__device__ void kkt_factor_v(Qp& q, const V f, PW dense, bool pol)
{
  const QpPattern& p = q.p;
  auto LX = f.LX;
  auto DG = f.DG;
  const double* FLG = q.a(W_FLG);
  double bad = 0, npos = 0;
  // one-node levels (the chain) with the solve vector in LDS: row k of L is
  // scattered into the (otherwise zero) vector LDS, so an entry's merge of
  // rows i and k becomes a branch-free walk of row i's prefix (its entries
  // before column k, lcpos order) -- (L_ij D_j) L_kj for the shared j, exact
  // zeros for the rest: bitwise the merge's sum.  The vector is zero between levels.
  const bool scatter = p.lds_vec;
  if (scatter)
  {
    QFOR(k, p.N) dense[k] = 0.0;
    __syncthreads();
  }
  for (int lev = 0; lev < p.nlev; ++lev)
  {
    const int n0 = f.lvp[lev], n1 = f.lvp[lev + 1];
    for (int t = n0 + static_cast<int>(threadIdx.x); t < n1; t += kQB)
    {
      const int k = f.lvn[t];
      double d = kkt_diag(q, k, pol, FLG);
      for (int e = f.lrp[k]; e < f.lrp[k + 1]; ++e)
      {
        const double l = LX[e];
        d -= (l * DG[f.lrj[e]]) * l;
      }
      DG[k] = d;
      if (d == 0.0 || !isfinite(d))
        bad = 1;
      else if (d > 0)
        npos += 1;
    }
    const int f0 = p.fip[lev], f1 = p.fip[lev + 1];
    if (scatter && n1 - n0 == 1)
    {
      const int k = f.lvn[n0];
      const int r0 = f.lrp[k], r1 = f.lrp[k + 1];
      for (int e = r0 + static_cast<int>(threadIdx.x); e < r1; e += kQB)
        dense[f.lrj[e]] = LX[e];
      __syncthreads();
      const double dk = DG[k];
      for (int t = f0 + static_cast<int>(threadIdx.x); t < f1; t += kQB)
      {
        const int c = p.fic[t], i = f.lci[c];
        double s = kkt_entry(q, p.lksrc[c], pol, FLG);
        const int ae = f.lcpos[c];  // entry (i, k)'s place in row i: the entries before it have j < k
        int a = f.lrp[i];
        for (; a + 4 <= ae; a += 4)
        {
          double la[4], da[4], xa[4];
          int ja[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
          {
            la[u] = LX[a + u];
            ja[u] = f.lrj[a + u];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
          {
            da[u] = DG[ja[u]];
            xa[u] = dense[ja[u]];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            s -= (la[u] * da[u]) * xa[u];
        }
        for (; a < ae; ++a)
        {
          const int ja = f.lrj[a];
          s -= (LX[a] * DG[ja]) * dense[ja];
        }
        LX[ae] = s / dk;
      }
      __syncthreads();
      for (int e = r0 + static_cast<int>(threadIdx.x); e < r1; e += kQB)
        dense[f.lrj[e]] = 0.0;
    }
    else
    {
      __syncthreads();
      for (int t = f0 + static_cast<int>(threadIdx.x); t < f1; t += kQB)
      {
        const int k = p.fik[t], c = p.fic[t], i = f.lci[c];
        double s = kkt_entry(q, p.lksrc[c], pol, FLG);
        int a = f.lrp[i], b = f.lrp[k];
        const int ae = f.lrp[i + 1], be = f.lrp[k + 1];
        while (a < ae && b < be)
        {
          const int ja = f.lrj[a], jb = f.lrj[b];
          if (ja == jb)
          {
            s -= (LX[a] * DG[ja]) * LX[b];
            ++a;
            ++b;
          }
          else if (ja < jb)
            ++a;
          else
            ++b;
        }
        LX[f.lcpos[c]] = s / DG[k];
      }
    }
    __syncthreads();
  }
  bad = bmax(q.sh, bad);
  npos = bsum(q.sh, npos);
  if (threadIdx.x == 0)
  {
    q.sh.fail = bad != 0.0;
    q.sh.npos = static_cast<int>(npos);
  }
  __syncthreads();
}

__device__ void kkt_factor(Qp& q, bool pol)
{
  if (!q.p.lds_pat)
  {
    kkt_factor_v(q, q.fg, q.lv, pol);
    return;
  }
  kkt_factor_v(q, q.fs, (lds_f64*)q.lv, pol);
  if (q.persist)  // the resident workspace's copy (the next launch stages it)
  {
    const int nl = static_cast<int>(q.p.lds_off[QL_DG] - q.p.lds_off[QL_LX]) / 8;
    double *GX = q.a(W_LX), *GD = q.a(W_DG);
    QFOR(e, nl) GX[e] = q.fs.LX[e];
    QFOR(k, q.p.N) GD[k] = q.fs.DG[k];
    __syncthreads();
  }
}

// in place solve K v = b for v[0..N) in the QP's workspace (original order):
// gather into the permuted vector, L forward by levels up the tree (rows of
// L), D, L' backward by levels down the tree (columns of L), scatter back.
// With the factor staged in LDS (QpPattern::lds_pat) every access of a level
// is an LDS access: a level costs a few LDS round trips and a barrier instead
// of a chain of dependent HBM loads (level pointer -> node -> row bounds ->
// entries), which set the pace of the HBM form.
// (the view by value and every pointer in a local: a Qp or view reached through
// a reference lives in scratch, and the stores to w would force a reload of
// each of its pointers from there at every level)
// (the view by value and every pointer in a local: a Qp or view reached through
// a reference lives in scratch)
template <typename V, typename PW>
__device__ void kkt_solve_v(Qp& q, const V f, PW w, double* v)
{
  const QpPattern& p = q.p;
  auto LX = f.LX;
  auto DG = f.DG;
  const auto lvp = f.lvp;
  const auto lvn = f.lvn;
  const auto lrj = f.lrj;
  const auto lcp = f.lcp;
  const auto lcpos = f.lcpos;
  const auto lci = f.lci;
  const int N = p.N, nlev = p.nlev;
  const int* perm = p.perm;
  __syncthreads();
  QFOR(k, N) w[k] = v[perm[k]];
  __syncthreads();
  const bool prof = THIP_QP_PROF && blockIdx.x == 0 && threadIdx.x == 0;
  long long t0 = prof ? clock64() : 0;
  // forward: the passes of row segments (kkt_symbolic), each row still
  // summed in its order -- its segments run in increasing passes -- and a
  // segment's columns final by the end of the pass before it
  const auto fwp = f.fwp;
  const auto fwk = f.fwk;
  const auto fwa = f.fwa;
  const auto fwb = f.fwb;
  for (int ps = 0; ps < p.npass; ++ps)
  {
    const int t1 = fwp[ps + 1];
    for (int t = fwp[ps] + static_cast<int>(threadIdx.x); t < t1; t += kQB)
    {
      const int k = fwk[t];
      w[k] = row_sub(static_cast<double>(w[k]), LX, lrj, w, static_cast<int>(fwa[t]), static_cast<int>(fwb[t]));
    }
    __syncthreads();
  }
  // (npass = 0: the level-by-level forward solve, THIP_QP_LEVEL_SOLVE -- the same sums)
  if (p.npass == 0)
    for (int lev = 0; lev < nlev; ++lev)
    {
      const int n1 = lvp[lev + 1];
      for (int t = lvp[lev] + static_cast<int>(threadIdx.x); t < n1; t += kQB)
      {
        const int k = lvn[t];
        w[k] = row_sub(static_cast<double>(w[k]), LX, lrj, w, f.lrp[k], f.lrp[k + 1]);
      }
      __syncthreads();
    }
  if (prof)
    qp_prof_add(6, clock64() - t0);
  QFOR(k, N) w[k] /= DG[k];
  __syncthreads();
  if (prof)
    t0 = clock64();
  for (int lev = nlev - 1; lev >= 0; --lev)
  {
    const int n1 = lvp[lev + 1];
    for (int t = lvp[lev] + static_cast<int>(threadIdx.x); t < n1; t += kQB)
    {
      const int k = lvn[t];
      w[k] = col_sub(static_cast<double>(w[k]), LX, lcpos, lci, w, lcp[k], lcp[k + 1]);
    }
    __syncthreads();
  }
  if (prof)
    qp_prof_add(7, clock64() - t0);
  QFOR(k, N) v[perm[k]] = w[k];
  __syncthreads();
}

__device__ void kkt_solve(Qp& q, double* v)
{
  if (q.p.lds_pat)
    kkt_solve_v(q, q.fs, (lds_f64*)q.lv, v);
  else if (q.p.lds_vec)
    kkt_solve_v(q, q.fg, (lds_f64*)q.lv, v);
  else
    kkt_solve_v(q, q.fg, q.lv, v);
}

__device__ double prim_res(Qp& q, const double* x, const double* z)
{
  double *AXV = q.a(W_AXV), *RP = q.a(W_RP);
  a_mul(q, x, AXV);
  __syncthreads();
  QFOR(r, q.m) RP[r] = AXV[r] - z[r];
  __syncthreads();
  return q.s.scaling > 0 ? scaled_norm_inf(q.sh, q.a(W_EI), RP, q.m) : norm_inf(q.sh, RP, q.m);
}

__device__ double dual_res(Qp& q, const double* x, const double* y)
{
  double *PXV = q.a(W_PXV), *ATY = q.a(W_ATY), *RD = q.a(W_RD), *Q = q.a(W_Q);
  p_mul(q, x, PXV);
  if (q.m > 0)
    at_mul(q, y, ATY);
  __syncthreads();
  QFOR(j, q.n) RD[j] = (q.m > 0) ? (Q[j] + PXV[j]) + ATY[j] : Q[j] + PXV[j];
  __syncthreads();
  return q.s.scaling > 0 ? q.sh.cinv * scaled_norm_inf(q.sh, q.a(W_DI), RD, q.n) : norm_inf(q.sh, RD, q.n);
}

__device__ bool primal_infeasible(Qp& q, double eps)
{
  double *L = q.a(W_L), *U = q.a(W_U), *DY = q.a(W_DY), *T1 = q.a(W_T1);
  QFOR(r, q.m)
  {
    if (U[r] > kInf * kMinScaling)
      DY[r] = (L[r] < -kInf * kMinScaling) ? 0.0 : fmin(DY[r], 0.0);
    else if (L[r] < -kInf * kMinScaling)
      DY[r] = fmax(DY[r], 0.0);
  }
  __syncthreads();
  const double ndy = q.s.scaling > 0 ? scaled_norm_inf(q.sh, q.a(W_E), DY, q.m) : norm_inf(q.sh, DY, q.m);
  if (!(ndy > kDivTol))
    return false;
  double lhs = 0;
  QFOR(r, q.m) lhs += U[r] * fmax(DY[r], 0.0) + L[r] * fmin(DY[r], 0.0);
  lhs = bsum(q.sh, lhs);
  if (!(lhs < eps * ndy))
    return false;
  at_mul(q, DY, T1);
  __syncthreads();
  if (q.s.scaling > 0)
  {
    const double* DI = q.a(W_DI);
    QFOR(j, q.n) T1[j] *= DI[j];
    __syncthreads();
  }
  return norm_inf(q.sh, T1, q.n) < eps * ndy;
}

__device__ bool dual_infeasible(Qp& q, double eps)
{
  double *DX = q.a(W_DX), *Q = q.a(W_Q), *T1 = q.a(W_T1), *T2 = q.a(W_T2), *L = q.a(W_L), *U = q.a(W_U);
  double ndx, cs;
  if (q.s.scaling > 0)
  {
    ndx = scaled_norm_inf(q.sh, q.a(W_D), DX, q.n);
    cs = q.sh.c;
  }
  else
  {
    ndx = norm_inf(q.sh, DX, q.n);
    cs = 1.0;
  }
  if (!(ndx > kDivTol))
    return false;
  double qdx = 0;
  QFOR(j, q.n) qdx += Q[j] * DX[j];
  qdx = bsum(q.sh, qdx);
  if (!(qdx < cs * eps * ndx))
    return false;
  p_mul(q, DX, T1);
  __syncthreads();
  if (q.s.scaling > 0)
  {
    const double* DI = q.a(W_DI);
    QFOR(j, q.n) T1[j] *= DI[j];
    __syncthreads();
  }
  if (!(norm_inf(q.sh, T1, q.n) < cs * eps * ndx))
    return false;
  a_mul(q, DX, T2);
  __syncthreads();
  if (q.s.scaling > 0)
  {
    const double* EI = q.a(W_EI);
    QFOR(r, q.m) T2[r] *= EI[r];
    __syncthreads();
  }
  double bad = 0;
  QFOR(r, q.m)
  if (((U[r] < kInf * kMinScaling) && (T2[r] > eps * ndx)) || ((L[r] > -kInf * kMinScaling) && (T2[r] < -eps * ndx)))
    bad = 1;
  return bmax(q.sh, bad) == 0.0;
}

// check_termination (OSQP 1.0): sets sh.status, returns true when done
__device__ bool check_termination(Qp& q, bool approximate)
{
  double eps_abs = q.s.eps_abs, eps_rel = q.s.eps_rel, eps_pi = q.s.eps_prim_inf, eps_di = q.s.eps_dual_inf;
  if (approximate)
  {
    eps_abs *= 10;
    eps_rel *= 10;
    eps_pi *= 10;
    eps_di *= 10;
  }
  bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
  const bool sc = q.s.scaling > 0;
  if (q.m == 0)
    prim_ok = true;
  else
  {
    const double* EI = q.a(W_EI);
    const double mr = sc ? fmax(scaled_norm_inf(q.sh, EI, q.a(W_Z), q.m), scaled_norm_inf(q.sh, EI, q.a(W_AXV), q.m))
                         : fmax(norm_inf(q.sh, q.a(W_Z), q.m), norm_inf(q.sh, q.a(W_AXV), q.m));
    const double eps_prim = eps_abs + eps_rel * mr;
    if (q.sh.prim_res < eps_prim)
      prim_ok = true;
    else
      prim_inf = primal_infeasible(q, eps_pi);
  }
  double mr;
  if (sc)
  {
    const double* DI = q.a(W_DI);
    mr = scaled_norm_inf(q.sh, DI, q.a(W_Q), q.n);
    mr = fmax(mr, scaled_norm_inf(q.sh, DI, q.a(W_ATY), q.n));
    mr = fmax(mr, scaled_norm_inf(q.sh, DI, q.a(W_PXV), q.n));
    mr *= q.sh.cinv;
  }
  else
    mr = fmax(fmax(norm_inf(q.sh, q.a(W_Q), q.n), norm_inf(q.sh, q.a(W_ATY), q.n)), norm_inf(q.sh, q.a(W_PXV), q.n));
  const double eps_dual = eps_abs + eps_rel * mr;
  if (q.sh.dual_res < eps_dual)
    dual_ok = true;
  else
    dual_inf = dual_infeasible(q, eps_di);
  int st = 0;
  if (prim_ok && dual_ok)
    st = approximate ? SOLVED_INACCURATE : SOLVED;
  else if (prim_inf)
    st = approximate ? PRIMAL_INFEASIBLE_INACCURATE : PRIMAL_INFEASIBLE;
  else if (dual_inf)
    st = approximate ? DUAL_INFEASIBLE_INACCURATE : DUAL_INFEASIBLE;
  __syncthreads();
  if (threadIdx.x == 0 && st)
    q.sh.status = st;
  __syncthreads();
  return st != 0;
}

// adaptive rho: estimate, and refactor when it moved by more than the tolerance.
// Returns false when the refactorisation is not quasi-definite (OSQP_NON_CVX).
__device__ bool adapt_rho(Qp& q)
{
  double pr = norm_inf(q.sh, q.a(W_RP), q.m);
  double dr = norm_inf(q.sh, q.a(W_RD), q.n);
  const double prn = fmax(norm_inf(q.sh, q.a(W_Z), q.m), norm_inf(q.sh, q.a(W_AXV), q.m));
  pr /= (prn + kDivTol);
  double drn = fmax(norm_inf(q.sh, q.a(W_Q), q.n), norm_inf(q.sh, q.a(W_ATY), q.n));
  drn = fmax(drn, norm_inf(q.sh, q.a(W_PXV), q.n));
  dr /= (drn + kDivTol);
  double est = q.sh.rho * sqrt(pr / (dr + kDivTol));
  est = fmin(fmax(est, kRhoMin), kRhoMax);
  if (!(est > q.sh.rho * q.s.adaptive_rho_tolerance || est < q.sh.rho / q.s.adaptive_rho_tolerance))
    return true;
  __syncthreads();
  if (threadIdx.x == 0)
    q.sh.rho = fmin(fmax(est, kRhoMin), kRhoMax);
  __syncthreads();
  double *RHO = q.a(W_RHO), *RHOI = q.a(W_RHOI), *CT = q.a(W_CT);
  QFOR(r, q.m)
  {
    if (CT[r] == 0.0)
    {
      RHO[r] = q.sh.rho;
      RHOI[r] = 1.0 / q.sh.rho;
    }
    else if (CT[r] == 1.0)
    {
      RHO[r] = kRhoEq * q.sh.rho;
      RHOI[r] = 1.0 / RHO[r];
    }
  }
  __syncthreads();
  kkt_factor(q, false);
  return !q.sh.fail && q.sh.npos >= q.n;
}

__device__ void polish(Qp& q)
{
  const int n = q.n, m = q.m, N = n + m;
  double *Z = q.a(W_Z), *Y = q.a(W_Y), *L = q.a(W_L), *U = q.a(W_U), *FLG = q.a(W_FLG);
  QFOR(r, m)
  {
    double f = 0;
    if (Z[r] - L[r] < -Y[r])
      f = -1;
    else if (U[r] - Z[r] < Y[r])
      f = 1;
    FLG[r] = f;
  }
  __syncthreads();
  // [P + delta I, Aact'; Aact, -delta I] over the full pattern, the inactive
  // rows decoupled (kkt_diag / kkt_entry in polish mode)
  kkt_factor(q, true);
  if (q.sh.fail || q.sh.npos < n)
  {
    if (threadIdx.x == 0)
      q.sh.polish = -1;
    __syncthreads();
    return;
  }
  double *RHS = q.a(W_RHS), *RES = q.a(W_RES), *Q = q.a(W_Q), *T1 = q.a(W_T1), *T2 = q.a(W_T2), *AX = q.a(W_AX);
  double* SOL = q.a(W_XT);  // [x (n), y of the rows (m); 0 on the inactive rows]
  double* SOLY = SOL + n;
  QFOR(j, n) RHS[j] = -Q[j];
  QFOR(r, m) RHS[n + r] = (FLG[r] < 0) ? L[r] : ((FLG[r] > 0) ? U[r] : 0.0);
  __syncthreads();
  QFOR(i, N) SOL[i] = RHS[i];
  kkt_solve(q, SOL);
  for (int itr = 0; itr < q.s.polish_refine_iter; ++itr)
  {
    // RES = RHS - [P, Aact'; Aact, 0] sol
    p_mul(q, SOL, T1);
    QFOR(j, n)
    {
      double t = 0;
      for (int e = q.p.Ap[j]; e < q.p.Ap[j + 1]; ++e)
        if (FLG[q.p.Ai[e]] != 0.0)
          t += AX[e] * SOLY[q.p.Ai[e]];
      T2[j] = t;
    }
    QFOR(r, m)
    {
      double res = 0;
      if (FLG[r] != 0.0)
      {
        double t = 0;
        for (int e = q.p.Arp[r]; e < q.p.Arp[r + 1]; ++e)
          t += AX[q.p.Armap[e]] * SOL[q.p.Arj[e]];
        res = RHS[n + r] - t;
      }
      RES[n + r] = res;
    }
    __syncthreads();
    QFOR(j, n) RES[j] = (RHS[j] - T1[j]) - T2[j];
    kkt_solve(q, RES);
    QFOR(i, N) SOL[i] += RES[i];
    __syncthreads();
  }
  double *PXS = q.a(W_PXS), *PZS = q.a(W_PZS), *PYS = q.a(W_PYS);
  QFOR(j, n) PXS[j] = SOL[j];
  __syncthreads();
  a_mul(q, PXS, PZS);
  __syncthreads();
  QFOR(r, m)
  {
    const double py = (FLG[r] != 0.0) ? SOLY[r] : 0.0;
    const double t = PZS[r] + py;
    PZS[r] = fmin(fmax(t, L[r]), U[r]);
    PYS[r] = t - PZS[r];
  }
  __syncthreads();
  const double pr0 = q.sh.prim_res, dr0 = q.sh.dual_res;
  const double pp = (m > 0) ? prim_res(q, PXS, PZS) : 0.0;
  const double pd = dual_res(q, PXS, PYS);
  const bool ok = (pp < pr0 && pd < dr0) || (pp < pr0 && dr0 < 1e-10) || (pd < dr0 && pr0 < 1e-10);
  __syncthreads();
  if (ok)
  {
    double *X = q.a(W_X);
    QFOR(j, n) X[j] = PXS[j];
    QFOR(r, m)
    {
      Z[r] = PZS[r];
      Y[r] = PYS[r];
    }
  }
  if (threadIdx.x == 0)
  {
    q.sh.polish = ok ? 1 : -1;
    if (ok)
    {
      q.sh.prim_res = pp;
      q.sh.dual_res = pd;
    }
  }
  __syncthreads();
}

// osqp_solve from the current iterates (X, Z, Y in the scaled space): ADMM
// with termination / infeasibility checks and adaptive rho, polish, then the
// unscaled solution and info of problem b.  Shared by the one-shot kernel and
// the resident workspace.
__device__ void admm_solve(Qp& q, const QpArgs& args, int b, thip_qp_info* info)
{
  Sh& sh = q.sh;
  const int n = q.n, m = q.m;
  double *X = q.a(W_X), *XP = q.a(W_XP), *Z = q.a(W_Z), *ZP = q.a(W_ZP), *Y = q.a(W_Y), *DX = q.a(W_DX),
         *DY = q.a(W_DY), *XT = q.a(W_XT), *Q = q.a(W_Q), *L = q.a(W_L), *U = q.a(W_U), *RHO = q.a(W_RHO),
         *RHOI = q.a(W_RHOI);
  int interval = args.s.adaptive_rho_interval;
  if (args.s.adaptive_rho == 1 && interval == 0)
    interval = args.s.check_termination ? 4 * args.s.check_termination : 100;
  const double alpha = args.s.alpha, sigma = args.s.sigma;
  bool can_check = false;
  bool noncvx = false;
  int it;
  const bool prof = THIP_QP_PROF && blockIdx.x == 0 && threadIdx.x == 0;
  long long t0 = prof ? clock64() : 0, t1;
  for (it = 1; it <= args.s.max_iter; ++it)
  {
    // (x_prev, z_prev) <- (x, z): OSQP swaps the buffers; x and z are overwritten below
    QFOR(j, n) XP[j] = X[j];
    QFOR(r, m) ZP[r] = Z[r];
    __syncthreads();
    QFOR(j, n) XT[j] = sigma * XP[j] - Q[j];
    QFOR(r, m) XT[n + r] = ZP[r] - RHOI[r] * Y[r];
    __syncthreads();
    if (prof)
    {
      t1 = clock64();
      qp_prof_add(0, t1 - t0);
      t0 = t1;
    }
    kkt_solve(q, XT);  // (x~, nu) in place
    if (prof)
    {
      t1 = clock64();
      qp_prof_add(1, t1 - t0);
      t0 = t1;
    }
    QFOR(r, m) XT[n + r] = (ZP[r] - RHOI[r] * Y[r]) + RHOI[r] * XT[n + r];  // z~ = rhs + nu / rho
    __syncthreads();
    QFOR(j, n)
    {
      X[j] = alpha * XT[j] + (1.0 - alpha) * XP[j];
      DX[j] = X[j] - XP[j];
    }
    QFOR(r, m)
    {
      double zr = RHOI[r] * Y[r];
      zr = zr + alpha * XT[n + r];
      zr = zr + (1.0 - alpha) * ZP[r];
      Z[r] = fmin(fmax(zr, L[r]), U[r]);
      DY[r] = RHO[r] * (alpha * XT[n + r] + (1.0 - alpha) * ZP[r] - Z[r]);
      Y[r] += DY[r];
    }
    __syncthreads();
    if (prof)
    {
      t1 = clock64();
      qp_prof_add(2, t1 - t0);
      t0 = t1;
    }
    can_check = args.s.check_termination && (it % args.s.check_termination == 0);
    const bool adapt_now = args.s.adaptive_rho && interval && (it % interval == 0);
    bool done = false;
    if (can_check || adapt_now)
    {
      const double pr = (m > 0) ? prim_res(q, X, Z) : 0.0;
      const double dr = dual_res(q, X, Y);
      if (threadIdx.x == 0)
      {
        sh.iter = it;
        sh.prim_res = pr;
        sh.dual_res = dr;
      }
      __syncthreads();
      if (can_check)
        done = check_termination(q, false);
      if (!done && adapt_now && !adapt_rho(q))
      {
        noncvx = true;
        break;
      }
    }
    if (prof)
    {
      t1 = clock64();
      qp_prof_add(3, t1 - t0);
      qp_prof_add(4, 1);
      t0 = t1;
    }
    if (done)
      break;
  }
  if (noncvx)
  {
    if (threadIdx.x == 0)
      sh.status = NON_CVX;
    __syncthreads();
  }
  else
  {
    if (!can_check)
    {
      // the last iterate was not checked: compute and test it
      const double pr = (m > 0) ? prim_res(q, X, Z) : 0.0;
      const double dr = dual_res(q, X, Y);
      if (threadIdx.x == 0)
      {
        sh.iter = it - 1;
        sh.prim_res = pr;
        sh.dual_res = dr;
      }
      __syncthreads();
      check_termination(q, false);
    }
    if (sh.status == UNSOLVED && !check_termination(q, true))
    {
      if (threadIdx.x == 0)
        sh.status = MAX_ITER_REACHED;
      __syncthreads();
    }
    if (args.s.polishing && sh.status == SOLVED)
      polish(q);
    if (prof)
      qp_prof_add(5, clock64() - t0);
  }
  // store_solution (unscaled), NaN on infeasibility
  const int st = sh.status;
  const bool inf = st == PRIMAL_INFEASIBLE || st == PRIMAL_INFEASIBLE_INACCURATE || st == DUAL_INFEASIBLE ||
                   st == DUAL_INFEASIBLE_INACCURATE;
  const double *D = q.a(W_D), *E = q.a(W_E);
  const bool sc = args.s.scaling > 0;
  QFOR(j, n) args.x_out[(long long)b * n + j] = inf ? NAN : (sc ? D[j] * X[j] : X[j]);
  QFOR(r, m) args.y_out[(long long)b * m + r] = inf ? NAN : (sc ? sh.cinv * (E[r] * Y[r]) : Y[r]);
  if (threadIdx.x == 0)
  {
    info->status = st;
    info->setup_error = 0;
    info->polish_status = sh.polish;
    info->iter = sh.iter;
    info->rho = sh.rho;
    info->prim_res = sh.prim_res;
    info->dual_res = sh.dual_res;
  }
}

// one QP of a launch: setup (scaling, rho vector, factor), warm start, ADMM,
// polish, solution out
__device__ __forceinline__ void qp_csc_body(const QpArgs& args, const int b, double* lv, Sh& sh)
{
  const QpPattern& P = args.pat;
  const int n = P.n, m = P.m;
  double* w = args.ws + (long long)b * P.stride;
  Qp q{ P, args.s, w, sh, P.lds_vec ? lv : w + P.off[W_LV], n, m, {}, {}, false };
  fac_views(q, reinterpret_cast<char*>(lv));
  // data (scaled in place)
  {
    double *PX = q.a(W_PX), *AX = q.a(W_AX), *Q = q.a(W_Q), *L = q.a(W_L), *U = q.a(W_U);
    QFOR(e, P.nnz_p) PX[e] = args.Pv[(long long)b * P.nnz_p + e];
    QFOR(e, P.nnz_a) AX[e] = args.Av[(long long)b * P.nnz_a + e];
    QFOR(j, n) Q[j] = args.qv[(long long)b * n + j];
    QFOR(r, m)
    {
      L[r] = args.lv[(long long)b * m + r];
      U[r] = args.uv[(long long)b * m + r];
    }
  }
  if (threadIdx.x == 0)
  {
    sh.c = sh.cinv = 1.0;
    sh.rho = args.rho_ws ? args.rho_ws[b] : args.s.rho;
    sh.rho = fmin(fmax(sh.rho, kRhoMin), kRhoMax);
    sh.status = UNSOLVED;
    sh.polish = 0;
    sh.iter = 0;
    sh.prim_res = sh.dual_res = 0;
  }
  __syncthreads();
  if (args.s.scaling > 0)
    scale_data(q);
  else
  {
    QFOR(j, n) q.a(W_D)[j] = q.a(W_DI)[j] = 1.0;
    QFOR(r, m) q.a(W_E)[r] = q.a(W_EI)[r] = 1.0;
    __syncthreads();
  }
  set_rho_vec(q);
  kkt_factor(q, false);
  thip_qp_info* info = args.info + b;
  if (q.sh.fail || q.sh.npos < n)
  {
    // osqp_setup fails: OSQP_LINSYS_SOLVER_INIT_ERROR / OSQP_NONCVX_ERROR
    if (threadIdx.x == 0)
    {
      info->status = -1;
      info->setup_error = q.sh.fail ? 4 : 5;
      info->polish_status = 0;
      info->iter = 0;
      info->rho = sh.rho;
      info->prim_res = info->dual_res = 0;
    }
    return;
  }
  // warm start (osqp_warm_start: x / D, y / E * c, z = A x) or cold start
  double *X = q.a(W_X), *Z = q.a(W_Z), *Y = q.a(W_Y);
  if (args.x_ws && args.y_ws && (!args.ws_mask || args.ws_mask[b]))
  {
    const double *DI = q.a(W_DI), *EI = q.a(W_EI);
    const bool sc = args.s.scaling > 0;
    QFOR(j, n) X[j] = sc ? args.x_ws[(long long)b * n + j] * DI[j] : args.x_ws[(long long)b * n + j];
    QFOR(r, m) Y[r] = sc ? (args.y_ws[(long long)b * m + r] * EI[r]) * sh.c : args.y_ws[(long long)b * m + r];
    __syncthreads();
    a_mul(q, X, Z);
  }
  else
  {
    QFOR(j, n) X[j] = 0.0;
    QFOR(r, m) Z[r] = Y[r] = 0.0;
  }
  __syncthreads();
  admm_solve(q, args, b, info);
}

__global__ __launch_bounds__(kQB) void qp_csc_kernel(QpArgs args)
{
  extern __shared__ double lv[];
  __shared__ Sh sh;
  if (static_cast<int>(blockIdx.x) >= args.batch)
    return;
  qp_csc_body(args, static_cast<int>(blockIdx.x), lv, sh);
}

// the QPs of several patterns in one launch (thip_qp_launch_staged): workgroup
// blockIdx.x belongs to pattern g with first[g] <= blockIdx.x < first[g + 1]
__global__ __launch_bounds__(kQB) void qp_csc_group_kernel(const QpArgs* list, const int* first, int nlist)
{
  extern __shared__ double lv[];
  __shared__ Sh sh;
  int g = 0;
  for (int k = 1; k < nlist; ++k)
    if (static_cast<int>(blockIdx.x) >= first[k])
      g = k;
  const int b = static_cast<int>(blockIdx.x) - first[g];
  if (b >= list[g].batch)
    return;
  qp_csc_body(list[g], b, lv, sh);
}


// ---------------------------------------------------------------------------
// Resident workspace (update in place): the OSQP 1.0 solver object kept on the
// device between calls, as OsqpEigen::Solver keeps it for trajopt_sqp's
// OSQPEigenSolver (trajopt_optimizers/trajopt_sqp/src/osqp_eigen_solver.cpp:
// 73-320, trust_region_sqp_solver.cpp:202-260).  One launch per API call:
//   OP_SETUP       osqp_setup: data, Ruiz scaling, rho vector, KKT factor, x = z = y = 0
//   OP_UPDATE_VEC  osqp_update_data_vec: q <- c (D q_new); l, u <- E l_new, E u_new, then
//                  the constraint types (rho vector) and a refactorisation only when a
//                  type changed (update_rho_vec)
//   OP_UPDATE_MAT  osqp_update_data_mat: unscale_data, new P / A values (same pattern),
//                  scale_data (q, l, u ride along through unscale and rescale), refactor
//   OP_WARM_START  osqp_warm_start: x / D, z = A x, c y / E
//   OP_SOLVE       osqp_solve: from the kept iterates (warm_starting) or from zero
// The scaled data, scaling, rho vector, iterates and factor stay in the QP's
// HBM workspace; c, 1/c and rho in W_SC.  Only the changed vectors cross the bus.
__device__ void resident_refactor(Qp& q)
{
  kkt_factor(q, false);
}

// OSQP unscale_data: P <- cinv Dinv P Dinv, q <- Dinv (cinv q), A <- Einv A Dinv, l, u <- Einv l, Einv u
__device__ void unscale_data(Qp& q)
{
  const int n = q.n, m = q.m;
  double *PX = q.a(W_PX), *AX = q.a(W_AX), *Q = q.a(W_Q), *L = q.a(W_L), *U = q.a(W_U);
  const double *DI = q.a(W_DI), *EI = q.a(W_EI);
  const double cinv = q.sh.cinv;
  QFOR(j, n)
  for (int e = q.p.Pp[j]; e < q.p.Pp[j + 1]; ++e)
    PX[e] = ((PX[e] * cinv) * DI[q.p.Pi[e]]) * DI[j];
  QFOR(j, n) Q[j] = (Q[j] * cinv) * DI[j];
  QFOR(j, n)
  for (int e = q.p.Ap[j]; e < q.p.Ap[j + 1]; ++e)
    AX[e] = (AX[e] * EI[q.p.Ai[e]]) * DI[j];
  QFOR(r, m)
  {
    L[r] = L[r] * EI[r];
    U[r] = U[r] * EI[r];
  }
  __syncthreads();
}

__device__ void set_unit_scaling(Qp& q)
{
  QFOR(j, q.n) q.a(W_D)[j] = q.a(W_DI)[j] = 1.0;
  QFOR(r, q.m) q.a(W_E)[r] = q.a(W_EI)[r] = 1.0;
  if (threadIdx.x == 0)
    q.sh.c = q.sh.cinv = 1.0;
  __syncthreads();
}

__device__ void report_setup_error(Qp& q, thip_qp_info* info, int code)
{
  if (threadIdx.x == 0)
  {
    info->status = -1;
    info->setup_error = code;
    info->polish_status = 0;
    info->iter = 0;
    info->rho = q.sh.rho;
    info->prim_res = info->dual_res = 0;
  }
}

__global__ __launch_bounds__(kQB) void qp_resident_kernel(QpArgs args, int op)
{
  extern __shared__ double lv[];
  __shared__ Sh sh;
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  const QpPattern& P = args.pat;
  const int n = P.n, m = P.m;
  double* w = args.ws + (long long)b * P.stride;
  Qp q{ P, args.s, w, sh, P.lds_vec ? lv : w + P.off[W_LV], n, m, {}, {}, true };
  fac_views(q, reinterpret_cast<char*>(lv));
  double* SC = q.a(W_SC);
  thip_qp_info* info = args.info + b;
  const bool sc = args.s.scaling > 0;
  if (threadIdx.x == 0)
  {
    sh.c = (op == OP_SETUP) ? 1.0 : SC[SC_C];
    sh.cinv = (op == OP_SETUP) ? 1.0 : SC[SC_CINV];
    sh.rho = (op == OP_SETUP) ? fmin(fmax(args.s.rho, kRhoMin), kRhoMax) : SC[SC_RHO];
    sh.status = UNSOLVED;
    sh.polish = 0;
    sh.iter = 0;
    sh.prim_res = sh.dual_res = 0;
    sh.fail = 0;
    sh.npos = n;
  }
  __syncthreads();
  double *PX = q.a(W_PX), *AX = q.a(W_AX), *Q = q.a(W_Q), *L = q.a(W_L), *U = q.a(W_U);
  double *X = q.a(W_X), *Z = q.a(W_Z), *Y = q.a(W_Y);
  const double *D = q.a(W_D), *E = q.a(W_E);
  bool ok = true;
  int err = 0;
  if (op == OP_SETUP)
  {
    QFOR(e, P.nnz_p) PX[e] = args.Pv[(long long)b * P.nnz_p + e];
    QFOR(e, P.nnz_a) AX[e] = args.Av[(long long)b * P.nnz_a + e];
    QFOR(j, n) Q[j] = args.qv[(long long)b * n + j];
    QFOR(r, m)
    {
      L[r] = args.lv[(long long)b * m + r];
      U[r] = args.uv[(long long)b * m + r];
    }
    __syncthreads();
    if (sc)
      scale_data(q);
    else
      set_unit_scaling(q);
    set_rho_vec(q);
    resident_refactor(q);
    ok = !sh.fail && sh.npos >= n;
    err = sh.fail ? 4 : 5;
    QFOR(j, n) X[j] = 0.0;
    QFOR(r, m) Z[r] = Y[r] = 0.0;
    if (threadIdx.x == 0)
    {
      SC[SC_OK] = ok ? 1.0 : 0.0;
      SC[SC_KKT_DIRTY] = 0.0;
    }
  }
  else if (op == OP_UPDATE_VEC)
  {
    if (args.qv)
      QFOR(j, n) Q[j] = sc ? (D[j] * args.qv[(long long)b * n + j]) * sh.c : args.qv[(long long)b * n + j];
    if (args.lv)
    {
      QFOR(r, m)
      {
        L[r] = sc ? E[r] * args.lv[(long long)b * m + r] : args.lv[(long long)b * m + r];
        U[r] = sc ? E[r] * args.uv[(long long)b * m + r] : args.uv[(long long)b * m + r];
      }
      __syncthreads();
      // update_rho_vec: rows whose constraint type changed get their rho; a
      // refactorisation only if one did
      double *RHO = q.a(W_RHO), *RHOI = q.a(W_RHOI), *CT = q.a(W_CT);
      double changed = 0;
      QFOR(r, m)
      {
        double ct, rv;
        if (L[r] < -kInf * kMinScaling && U[r] > kInf * kMinScaling)
        {
          ct = -1;
          rv = kRhoMin;
        }
        else if (U[r] - L[r] < kRhoTol)
        {
          ct = 1;
          rv = kRhoEq * sh.rho;
        }
        else
        {
          ct = 0;
          rv = sh.rho;
        }
        if (CT[r] != ct)
        {
          CT[r] = ct;
          RHO[r] = rv;
          RHOI[r] = 1.0 / rv;
          changed = 1;
        }
      }
      if (bmax(sh, changed) != 0.0)
      {
        resident_refactor(q);
        ok = !sh.fail && sh.npos >= n;
        err = sh.fail ? 4 : 5;
        if (threadIdx.x == 0)
          SC[SC_KKT_DIRTY] = 0.0;
      }
    }
  }
  else if (op == OP_UPDATE_MAT)
  {
    if (sc)
      unscale_data(q);
    if (args.Pv)
      QFOR(e, P.nnz_p) PX[e] = args.Pv[(long long)b * P.nnz_p + e];
    if (args.Av)
      QFOR(e, P.nnz_a) AX[e] = args.Av[(long long)b * P.nnz_a + e];
    __syncthreads();
    if (sc)
      scale_data(q);
    resident_refactor(q);
    ok = !sh.fail && sh.npos >= n;
    err = sh.fail ? 4 : 5;
    if (threadIdx.x == 0)
      SC[SC_KKT_DIRTY] = 0.0;
  }
  else if (op == OP_WARM_START)
  {
    const double *DI = q.a(W_DI), *EI = q.a(W_EI);
    if (args.x_ws)
    {
      QFOR(j, n) X[j] = sc ? args.x_ws[(long long)b * n + j] * DI[j] : args.x_ws[(long long)b * n + j];
      __syncthreads();
      a_mul(q, X, Z);
    }
    if (args.y_ws)
      QFOR(r, m) Y[r] = sc ? (args.y_ws[(long long)b * m + r] * EI[r]) * sh.c : args.y_ws[(long long)b * m + r];
  }
  else  // OP_SOLVE
  {
    if (SC[SC_OK] == 0.0)
    {
      report_setup_error(q, info, 4);
      return;
    }
    if (SC[SC_KKT_DIRTY] != 0.0)
    {
      resident_refactor(q);  // the same factor OSQP kept
      if (threadIdx.x == 0)
        SC[SC_KKT_DIRTY] = 0.0;
    }
    if (!args.s.warm_starting)
    {
      QFOR(j, n) X[j] = 0.0;
      QFOR(r, m) Z[r] = Y[r] = 0.0;
    }
    __syncthreads();
    admm_solve(q, args, b, info);
    if (threadIdx.x == 0)
    {
      if (sh.polish != 0)
        SC[SC_KKT_DIRTY] = 1.0;  // polish factored its KKT over W_LX / W_DG
      SC[SC_RHO] = sh.rho;
    }
    return;
  }
  __syncthreads();
  if (!ok)
  {
    report_setup_error(q, info, err);
    if (threadIdx.x == 0)
      SC[SC_OK] = 0.0;
  }
  else if (threadIdx.x == 0)
  {
    info->status = 0;
    info->setup_error = 0;
    info->polish_status = 0;
    info->iter = 0;
    info->rho = sh.rho;
    info->prim_res = info->dual_res = 0;
  }
  if (threadIdx.x == 0)
  {
    SC[SC_C] = sh.c;
    SC[SC_CINV] = sh.cinv;
    SC[SC_RHO] = sh.rho;
  }
}

}  // namespace thip_qp_dev

using namespace thip_qp_dev;

struct thip_qp
{
  int device = 0, batch = 0, n = 0, m = 0, nnz_p = 0, nnz_a = 0;
  long long nnz_l = 0;  // entries of the KKT factor L (thip_qp_factor_nnz)
  int max_level = 0;    // nodes of the widest elimination-tree level (thip_qp_shape)
  hipStream_t stream = nullptr;  // thip_qp_submit / thip_qp_collect
  int pending = 0;               // QPs submitted and not yet collected
  bool staged = false;           // thip_qp_stage: inputs on the device, launch deferred
  QpArgs staged_args{};
  hipStream_t done_stream = nullptr;  // the stream the pending launch runs on
  // thip_qp_launch_staged, when this object leads a group: the argument list
  QpArgs* d_list = nullptr;
  int* d_first = nullptr;
  int list_cap = 0;
  std::vector<QpArgs> h_list;
  std::vector<int> h_first;
  std::vector<int> bad;          // per submitted QP: l > u somewhere (osqp_setup's validate_data)
  QpPattern pat{};
  int* d_idx = nullptr;
  double* d_ws = nullptr;
  double *d_in = nullptr, *d_out = nullptr;
  thip_qp_info* d_info = nullptr;
  long long in_doubles = 0;
  size_t lds = 0;
  std::string err;
  // resident workspace (thip_qp_setup ...): the settings of its setup
  thip_osqp_settings rs{};
  bool resident = false;
};

static thread_local std::string g_qp_create_err;

extern "C" {

int thip_qp_create(int device, int n, int m, const int* P_colptr, const int* P_rowind, const int* A_colptr,
                   const int* A_rowind, int batch, thip_qp** out)
{
  if (!out || n <= 0 || m < 0 || batch <= 0 || !P_colptr || !A_colptr)
  {
    g_qp_create_err = "thip_qp_create: bad arguments";
    return THIP_E_INVALID;
  }
  if (n + m > THIP_QP_MAX_KKT)
  {
    g_qp_create_err = "thip_qp_create: n + m = " + std::to_string(n + m) + " exceeds THIP_QP_MAX_KKT (" +
                      std::to_string(THIP_QP_MAX_KKT) + ")";
    return THIP_E_INVALID;
  }
  const int np = P_colptr[n], na = A_colptr[n];
  if (P_colptr[0] != 0 || A_colptr[0] != 0 || np < 0 || na < 0)
  {
    g_qp_create_err = "thip_qp_create: bad column pointers";
    return THIP_E_INVALID;
  }
  for (int j = 0; j < n; ++j)
  {
    if (P_colptr[j + 1] < P_colptr[j] || A_colptr[j + 1] < A_colptr[j])
    {
      g_qp_create_err = "thip_qp_create: column pointers must not decrease";
      return THIP_E_INVALID;
    }
    for (int e = P_colptr[j]; e < P_colptr[j + 1]; ++e)
      if (P_rowind[e] < 0 || P_rowind[e] > j)
      {
        g_qp_create_err = "thip_qp_create: P must be upper triangular CSC";
        return THIP_E_INVALID;
      }
    for (int e = A_colptr[j]; e < A_colptr[j + 1]; ++e)
      if (A_rowind[e] < 0 || A_rowind[e] >= m)
      {
        g_qp_create_err = "thip_qp_create: A row index out of range";
        return THIP_E_INVALID;
      }
  }
  KktSymbolic S;
  const std::string why = kkt_symbolic(n, m, P_colptr, P_rowind, A_colptr, A_rowind, S);
  if (!why.empty())
  {
    g_qp_create_err = "thip_qp_create: " + why;
    return THIP_E_INVALID;
  }
  auto* q = new thip_qp();
  q->device = device;
  q->batch = batch;
  q->n = n;
  q->m = m;
  q->nnz_p = np;
  q->nnz_a = na;
  // rows of P's upper triangle and of A (pattern -> value index maps)
  std::vector<int> prp(n + 1, 0), prj(np), prm(np), arp(m + 1, 0), arj(na), arm(na);
  for (int j = 0; j < n; ++j)
    for (int e = P_colptr[j]; e < P_colptr[j + 1]; ++e)
      prp[P_rowind[e] + 1]++;
  for (int j = 0; j < n; ++j)
    prp[j + 1] += prp[j];
  {
    std::vector<int> nx(prp.begin(), prp.end() - 1);
    for (int j = 0; j < n; ++j)
      for (int e = P_colptr[j]; e < P_colptr[j + 1]; ++e)
      {
        const int k = nx[P_rowind[e]]++;
        prj[k] = j;
        prm[k] = e;
      }
  }
  for (int e = 0; e < na; ++e)
    arp[A_rowind[e] + 1]++;
  for (int r = 0; r < m; ++r)
    arp[r + 1] += arp[r];
  {
    std::vector<int> nx(arp.begin(), arp.end() - 1);
    for (int j = 0; j < n; ++j)
      for (int e = A_colptr[j]; e < A_colptr[j + 1]; ++e)
      {
        const int k = nx[A_rowind[e]]++;
        arj[k] = j;
        arm[k] = e;
      }
  }
  std::vector<int> idx;
  auto push = [&](const int* v, int len) {
    const size_t o = idx.size();
    idx.insert(idx.end(), v, v + len);
    idx.push_back(0);
    return o;
  };
  const size_t oPp = push(P_colptr, n + 1), oPi = push(P_rowind, np), oPrp = push(prp.data(), n + 1),
               oPrj = push(prj.data(), np), oPrm = push(prm.data(), np), oAp = push(A_colptr, n + 1),
               oAi = push(A_rowind, na), oArp = push(arp.data(), m + 1), oArj = push(arj.data(), na),
               oArm = push(arm.data(), na);
  const long long nnzl = static_cast<long long>(S.lrj.size());
  const int nlev = static_cast<int>(S.lvp.size()) - 1;
  const size_t oPerm = push(S.perm.data(), n + m), oLrp = push(S.lrp.data(), n + m + 1),
               oLrj = push(S.lrj.data(), static_cast<int>(nnzl)), oLcp = push(S.lcp.data(), n + m + 1),
               oLci = push(S.lci.data(), static_cast<int>(nnzl)), oLcpos = push(S.lcpos.data(), static_cast<int>(nnzl)),
               oLks = push(S.lksrc.data(), static_cast<int>(nnzl)), oDpd = push(S.dpd.data(), n + m),
               oLvp = push(S.lvp.data(), nlev + 1), oLvn = push(S.lvn.data(), n + m),
               oFip = push(S.fip.data(), nlev + 1), oFik = push(S.fik.data(), static_cast<int>(nnzl)),
               oFic = push(S.fic.data(), static_cast<int>(nnzl));
  const int npass = static_cast<int>(S.fwp.size()) - 1, nseg = S.fwp.back();
  const size_t oFwp = push(S.fwp.data(), npass + 1), oFwk = push(S.fwk.data(), nseg),
               oFwa = push(S.fwa.data(), nseg), oFwb = push(S.fwb.data(), nseg);
  const long long N = n + m;
  // the permuted solve vector in LDS up to 64 KiB
  const bool lds_vec = N <= 8192;
  long long sizes[W_COUNT];
  sizes[W_PX] = std::max(np, 1);
  sizes[W_AX] = std::max(na, 1);
  sizes[W_Q] = sizes[W_D] = sizes[W_DI] = sizes[W_TD] = sizes[W_X] = sizes[W_XP] = sizes[W_DX] = n;
  sizes[W_PXV] = sizes[W_ATY] = sizes[W_RD] = sizes[W_T1] = sizes[W_PXS] = n;
  const long long mm = std::max(m, 1);
  sizes[W_L] = sizes[W_U] = sizes[W_E] = sizes[W_EI] = sizes[W_TE] = sizes[W_RHO] = sizes[W_RHOI] = sizes[W_CT] = mm;
  sizes[W_Z] = sizes[W_ZP] = sizes[W_Y] = sizes[W_DY] = sizes[W_AXV] = sizes[W_RP] = sizes[W_T2] = mm;
  sizes[W_PZS] = sizes[W_PYS] = sizes[W_FLG] = mm;
  sizes[W_XT] = sizes[W_RHS] = sizes[W_RES] = N;
  sizes[W_LX] = std::max(nnzl, 1LL);
  sizes[W_DG] = N;
  sizes[W_LV] = lds_vec ? 1 : N;
  sizes[W_SC] = SC_COUNT;
  long long off = 0;
  for (int k = 0; k < W_COUNT; ++k)
  {
    q->pat.off[k] = off;
    off += (sizes[k] + 31) / 32 * 32;
  }
  q->pat.stride = off;
  q->pat.n = n;
  q->pat.m = m;
  q->pat.nnz_p = np;
  q->pat.nnz_a = na;
  q->pat.N = static_cast<int>(N);
  q->in_doubles = (long long)np + na + n + 2LL * m;
  q->pat.nlev = nlev;
  // diagnostic: THIP_QP_LEVEL_SOLVE=1 runs the forward solve level by level,
  // one thread per node (the A/B baseline; the same sums)
  q->pat.npass = std::getenv("THIP_QP_LEVEL_SOLVE") ? 0 : npass;
  for (int lv = 0; lv < nlev; ++lv)
    q->max_level = std::max(q->max_level, S.lvp[static_cast<size_t>(lv) + 1] - S.lvp[static_cast<size_t>(lv)]);
  q->nnz_l = nnzl;
  q->pat.lds_vec = lds_vec ? 1 : 0;
  q->lds = lds_vec ? static_cast<size_t>(N) * sizeof(double) : 0;
  // the whole factor in LDS when it fits next to the solve vector (16-bit
  // indices: N and the entries of L below 65536)
  {
    const long long nl = std::max(nnzl, 1LL);
    long long o = N * 8;  // the solve vector first
    long long offs[QL_COUNT];
    auto take = [&](int k, long long bytes) {
      offs[k] = o;
      o += (bytes + 15) / 16 * 16;
    };
    take(QL_LX, nl * 8);
    take(QL_DG, N * 8);
    take(QL_LRJ, nl * 2);
    take(QL_LCPOS, nl * 2);
    take(QL_LCI, nl * 2);
    take(QL_LVN, N * 2);
    take(QL_LRP, 2 * (N + 1) * 4);
    take(QL_LVP, (nlev + 1) * 4);
    take(QL_FWK, (long long)nseg * 2);
    take(QL_FWA, (long long)nseg * 2);
    take(QL_FWB, (long long)nseg * 2);
    take(QL_FWP, (long long)(npass + 1) * 4);
    const bool fits = lds_vec && N < 65536 && nnzl < 65536 && o <= kQpLdsBudget;
    q->pat.lds_pat = fits ? 1 : 0;
    if (fits)
    {
      // lds_off[QL_DG] - lds_off[QL_LX] = 8 x entries of L exactly (fac_views)
      offs[QL_DG] = offs[QL_LX] + nl * 8;
      for (int k = 0; k < QL_COUNT; ++k)
        q->pat.lds_off[k] = offs[k];
      q->lds = static_cast<size_t>(o);
    }
  }
  auto fail = [&](const std::string& msg) {
    g_qp_create_err = msg;
    thip_qp_destroy(q);
    return THIP_E_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess)
    return fail(std::string("hipSetDevice: ") + hipGetErrorString(e));
  if ((e = hipMalloc(&q->d_idx, idx.size() * sizeof(int))) != hipSuccess ||
      (e = hipMalloc(&q->d_ws, static_cast<size_t>(q->pat.stride) * batch * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&q->d_in, static_cast<size_t>(q->in_doubles + 2LL * n + m + 2) * batch * sizeof(double))) !=
          hipSuccess ||
      (e = hipMalloc(&q->d_out, static_cast<size_t>(n + m) * batch * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&q->d_info, sizeof(thip_qp_info) * batch)) != hipSuccess)
    return fail(std::string("hipMalloc: ") + hipGetErrorString(e));
  if ((e = hipMemcpy(q->d_idx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(std::string("hipMemcpy: ") + hipGetErrorString(e));
  if ((e = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(std::string("hipStreamCreate: ") + hipGetErrorString(e));
  q->pat.Pp = q->d_idx + oPp;
  q->pat.Pi = q->d_idx + oPi;
  q->pat.Prp = q->d_idx + oPrp;
  q->pat.Prj = q->d_idx + oPrj;
  q->pat.Prmap = q->d_idx + oPrm;
  q->pat.Ap = q->d_idx + oAp;
  q->pat.Ai = q->d_idx + oAi;
  q->pat.Arp = q->d_idx + oArp;
  q->pat.Arj = q->d_idx + oArj;
  q->pat.Armap = q->d_idx + oArm;
  q->pat.perm = q->d_idx + oPerm;
  q->pat.lrp = q->d_idx + oLrp;
  q->pat.lrj = q->d_idx + oLrj;
  q->pat.lcp = q->d_idx + oLcp;
  q->pat.lci = q->d_idx + oLci;
  q->pat.lcpos = q->d_idx + oLcpos;
  q->pat.lksrc = q->d_idx + oLks;
  q->pat.dpd = q->d_idx + oDpd;
  q->pat.lvp = q->d_idx + oLvp;
  q->pat.lvn = q->d_idx + oLvn;
  q->pat.fip = q->d_idx + oFip;
  q->pat.fik = q->d_idx + oFik;
  q->pat.fic = q->d_idx + oFic;
  q->pat.fwp = q->d_idx + oFwp;
  q->pat.fwk = q->d_idx + oFwk;
  q->pat.fwa = q->d_idx + oFwa;
  q->pat.fwb = q->d_idx + oFwb;
  *out = q;
  return THIP_OK;
}

int thip_qp_solve(thip_qp* q, const double* P_values, const double* qvec, const double* A_values, const double* l,
                  const double* u, const thip_osqp_settings* settings, const double* warm_x, const double* warm_y,
                  const double* warm_rho, double* x, double* y, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  return thip_qp_solve_some(q, q->batch, P_values, qvec, A_values, l, u, settings, warm_x, warm_y, nullptr, warm_rho,
                            x, y, info);
}

static int qp_stage(thip_qp* q, int count, const double* P_values, const double* qvec, const double* A_values,
                    const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                    const double* warm_y, const int* warm_mask, const double* warm_rho, bool launch)
{
  if (!q)
    return THIP_E_INVALID;
  if (q->pending || q->staged)
  {
    q->err = "thip_qp_submit: the previous submission is not collected";
    return THIP_E_INVALID;
  }
  if (count < 1 || count > q->batch)
  {
    q->err = "thip_qp_solve_some: count must be in [1, batch]";
    return THIP_E_INVALID;
  }
  const int n = q->n, m = q->m, B = count;
  // (an empty P -- a linear objective -- or an empty A may come with NULL values)
  if ((!P_values && q->nnz_p) || !qvec || (!A_values && q->nnz_a) || (m && (!l || !u)) || !settings)
  {
    q->err = "thip_qp_solve: null argument";
    return THIP_E_INVALID;
  }
  if (settings->max_iter < 1 || settings->check_termination < 0 || settings->scaling < 0 ||
      !(settings->alpha > 0 && settings->alpha < 2) || !(settings->sigma > 0) || !(settings->rho > 0) ||
      !(settings->delta > 0))
  {
    q->err = "thip_qp_solve: bad OSQP settings";
    return THIP_E_INVALID;
  }
  // osqp_setup's validate_data: l <= u (a failing problem is reported, not solved)
  q->bad.assign(static_cast<size_t>(B), 0);
  for (int b = 0; b < B; ++b)
    for (int r = 0; r < m; ++r)
      if (!(l[(long long)b * m + r] <= u[(long long)b * m + r]))
        q->bad[static_cast<size_t>(b)] = 1;
  hipError_t e;
  if ((e = hipSetDevice(q->device)) != hipSuccess)
  {
    q->err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  // inputs packed into one device buffer
  const size_t np = static_cast<size_t>(q->nnz_p) * B, na = static_cast<size_t>(q->nnz_a) * B;
  const size_t nn = static_cast<size_t>(n) * B, mm = static_cast<size_t>(m) * B;
  double* d = q->d_in;
  double *dP = d, *dA = dP + np, *dq = dA + na, *dl = dq + nn, *du = dl + mm, *dxw = du + mm, *dyw = dxw + nn,
         *drw = dyw + mm;
  // (on the QP object's own stream: the submissions of several patterns overlap)
  auto h2d = [&](double* dst, const double* src, size_t cnt) {
    if (cnt && (e = hipMemcpyAsync(dst, src, cnt * sizeof(double), hipMemcpyHostToDevice, q->stream)) != hipSuccess)
      return false;
    return true;
  };
  const bool ws = warm_x && warm_y;
  // the per-QP warm-start flags travel behind the rho values (the buffer holds B + batch doubles there)
  int* dmask = reinterpret_cast<int*>(drw + q->batch);
  if (!h2d(dP, P_values, np) || !h2d(dA, A_values, na) || !h2d(dq, qvec, nn) || !h2d(dl, l, mm) || !h2d(du, u, mm) ||
      (ws && (!h2d(dxw, warm_x, nn) || !h2d(dyw, warm_y, mm))) || (warm_rho && !h2d(drw, warm_rho, B)) ||
      (ws && warm_mask &&
       (e = hipMemcpyAsync(dmask, warm_mask, static_cast<size_t>(B) * sizeof(int), hipMemcpyHostToDevice,
                           q->stream)) != hipSuccess))
  {
    q->err = std::string("hipMemcpy: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  q->resident = false;  // the one-shot solve reuses the workspace
  QpArgs a{};
  a.pat = q->pat;
  a.s = *settings;
  a.Pv = dP;
  a.Av = dA;
  a.qv = dq;
  a.lv = dl;
  a.uv = du;
  a.x_ws = ws ? dxw : nullptr;
  a.y_ws = ws ? dyw : nullptr;
  a.rho_ws = warm_rho ? drw : nullptr;
  a.ws_mask = (ws && warm_mask) ? dmask : nullptr;
  a.x_out = q->d_out;
  a.y_out = q->d_out + nn;
  a.info = q->d_info;
  a.ws = q->d_ws;
  a.batch = B;
  if (q->lds > 65536)
    hipFuncSetAttribute(reinterpret_cast<const void*>(&qp_csc_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        static_cast<int>(q->lds));
  q->done_stream = q->stream;
  if (!launch)
  {
    q->staged_args = a;
    q->staged = true;
    q->pending = B;
    return THIP_OK;
  }
  hipLaunchKernelGGL(qp_csc_kernel, dim3(B), dim3(kQB), q->lds, q->stream, a);
  if ((e = hipGetLastError()) != hipSuccess)
  {
    q->err = std::string("qp_csc_kernel: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  q->pending = B;
  return THIP_OK;
}

int thip_qp_submit(thip_qp* q, int count, const double* P_values, const double* qvec, const double* A_values,
                   const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                   const double* warm_y, const int* warm_mask, const double* warm_rho)
{
  return qp_stage(q, count, P_values, qvec, A_values, l, u, settings, warm_x, warm_y, warm_mask, warm_rho, true);
}

int thip_qp_stage(thip_qp* q, int count, const double* P_values, const double* qvec, const double* A_values,
                  const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                  const double* warm_y, const int* warm_mask, const double* warm_rho)
{
  return qp_stage(q, count, P_values, qvec, A_values, l, u, settings, warm_x, warm_y, warm_mask, warm_rho, false);
}

int thip_qp_launch_staged(thip_qp* const* qps, int n)
{
  if (!qps || n < 1 || !qps[0])
    return THIP_E_INVALID;
  thip_qp* lead = qps[0];
  // any failure: the staged submissions are dropped (staged and pending
  // cleared), so the objects take new submissions instead of refusing every
  // later one as "not collected"
  auto fail = [&](int code, std::string msg) {
    for (int k = 0; k < n; ++k)
      if (qps[k] && qps[k]->staged)
      {
        qps[k]->staged = false;
        qps[k]->pending = 0;
      }
    lead->err = std::move(msg);
    return code;
  };
  for (int k = 0; k < n; ++k)
    if (!qps[k] || !qps[k]->staged || qps[k]->device != lead->device)
      return fail(THIP_E_INVALID, "thip_qp_launch_staged: every object staged, on one device");
  hipError_t e;
  if ((e = hipSetDevice(lead->device)) != hipSuccess)
  {
    return fail(THIP_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  // the staged inputs were copied on each object's stream
  for (int k = 0; k < n; ++k)
    if ((e = hipStreamSynchronize(qps[k]->stream)) != hipSuccess)
    {
      return fail(THIP_E_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
    }
  lead->h_list.resize(static_cast<size_t>(n));
  lead->h_first.resize(static_cast<size_t>(n) + 1);
  size_t lds = 0;
  int total = 0;
  for (int k = 0; k < n; ++k)
  {
    lead->h_list[static_cast<size_t>(k)] = qps[k]->staged_args;
    lead->h_first[static_cast<size_t>(k)] = total;
    total += qps[k]->staged_args.batch;
    lds = std::max(lds, qps[k]->lds);
  }
  lead->h_first[static_cast<size_t>(n)] = total;
  if (lead->list_cap < n)
  {
    hipFree(lead->d_list);
    hipFree(lead->d_first);
    lead->d_list = nullptr;
    lead->d_first = nullptr;
    if ((e = hipMalloc(&lead->d_list, sizeof(QpArgs) * n)) != hipSuccess ||
        (e = hipMalloc(&lead->d_first, sizeof(int) * (n + 1))) != hipSuccess)
    {
      lead->list_cap = 0;
      return fail(THIP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    lead->list_cap = n;
  }
  if ((e = hipMemcpyAsync(lead->d_list, lead->h_list.data(), sizeof(QpArgs) * n, hipMemcpyHostToDevice,
                          lead->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(lead->d_first, lead->h_first.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice,
                          lead->stream)) != hipSuccess)
  {
    return fail(THIP_E_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  if (lds > 65536)
    hipFuncSetAttribute(reinterpret_cast<const void*>(&qp_csc_group_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  hipLaunchKernelGGL(qp_csc_group_kernel, dim3(total), dim3(kQB), lds, lead->stream, lead->d_list, lead->d_first, n);
  if ((e = hipGetLastError()) != hipSuccess)
  {
    return fail(THIP_E_HIP, std::string("qp_csc_group_kernel: ") + hipGetErrorString(e));
  }
  for (int k = 0; k < n; ++k)
  {
    qps[k]->staged = false;
    qps[k]->done_stream = lead->stream;
  }
  return THIP_OK;
}

int thip_qp_collect(thip_qp* q, double* x, double* y, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if (!q->pending || q->staged)
  {
    q->err = q->staged ? "thip_qp_collect: staged and not launched (thip_qp_launch_staged)"
                       : "thip_qp_collect: nothing submitted";
    return THIP_E_INVALID;
  }
  if (!x || !info)
  {
    q->err = "thip_qp_collect: null argument";
    return THIP_E_INVALID;
  }
  const int B = q->pending, n = q->n, m = q->m;
  q->pending = 0;
  const size_t nn = static_cast<size_t>(n) * B, mm = static_cast<size_t>(m) * B;
  hipError_t e;
  if ((e = hipSetDevice(q->device)) != hipSuccess ||
      (e = hipStreamSynchronize(q->done_stream ? q->done_stream : q->stream)) != hipSuccess)
  {
    q->err = std::string("qp_csc_kernel: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  std::vector<thip_qp_info> hinfo(static_cast<size_t>(B));
  if ((e = hipMemcpy(x, q->d_out, nn * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess ||
      (y && m && (e = hipMemcpy(y, q->d_out + nn, mm * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess) ||
      (e = hipMemcpy(hinfo.data(), q->d_info, sizeof(thip_qp_info) * B, hipMemcpyDeviceToHost)) != hipSuccess)
  {
    q->err = std::string("hipMemcpy: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  for (int b = 0; b < B; ++b)
  {
    info[b] = hinfo[static_cast<size_t>(b)];
    if (q->bad[static_cast<size_t>(b)])
    {
      info[b].status = -1;
      info[b].setup_error = 1;  // OSQP_DATA_VALIDATION_ERROR
    }
  }
  return THIP_OK;
}

int thip_qp_solve_some(thip_qp* q, int count, const double* P_values, const double* qvec, const double* A_values,
                       const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                       const double* warm_y, const int* warm_mask, const double* warm_rho, double* x, double* y,
                       thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if (!x || !info)
  {
    q->err = "thip_qp_solve: null argument";
    return THIP_E_INVALID;
  }
  const int rc =
      thip_qp_submit(q, count, P_values, qvec, A_values, l, u, settings, warm_x, warm_y, warm_mask, warm_rho);
  return rc != THIP_OK ? rc : thip_qp_collect(q, x, y, info);
}

// ---- resident workspace (update in place) --------------------------------
static bool qp_settings_ok(thip_qp* q, const thip_osqp_settings* settings)
{
  if (settings->max_iter < 1 || settings->check_termination < 0 || settings->scaling < 0 ||
      !(settings->alpha > 0 && settings->alpha < 2) || !(settings->sigma > 0) || !(settings->rho > 0) ||
      !(settings->delta > 0))
  {
    q->err = "bad OSQP settings";
    return false;
  }
  return true;
}

// one resident operation over the batch: inputs (any may be null) to the
// device, the launch, outputs back
static int qp_resident(thip_qp* q, int op, const double* P_values, const double* qvec, const double* A_values,
                       const double* l, const double* u, const double* x_in, const double* y_in, double* x,
                       double* y, thip_qp_info* info)
{
  const int n = q->n, m = q->m, B = q->batch;
  // the resident calls use d_in / d_ws synchronously on the null stream: an
  // uncollected submission (its own stream) would race them
  if (q->pending || q->staged)
  {
    q->err = "thip_qp resident call: a submission is not collected (thip_qp_collect first)";
    return THIP_E_INVALID;
  }
  hipError_t e;
  if ((e = hipSetDevice(q->device)) != hipSuccess)
  {
    q->err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  const size_t np = static_cast<size_t>(q->nnz_p) * B, na = static_cast<size_t>(q->nnz_a) * B;
  const size_t nn = static_cast<size_t>(n) * B, mm = static_cast<size_t>(m) * B;
  double* d = q->d_in;
  double *dP = d, *dA = dP + np, *dq = dA + na, *dl = dq + nn, *du = dl + mm, *dxw = du + mm, *dyw = dxw + nn;
  auto h2d = [&](double* dst, const double* src, size_t cnt) {
    if (src && cnt && (e = hipMemcpy(dst, src, cnt * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
      return false;
    return true;
  };
  if (!h2d(dP, P_values, np) || !h2d(dA, A_values, na) || !h2d(dq, qvec, nn) || !h2d(dl, l, mm) || !h2d(du, u, mm) ||
      !h2d(dxw, x_in, nn) || !h2d(dyw, y_in, mm))
  {
    q->err = std::string("hipMemcpy: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  QpArgs a{};
  a.pat = q->pat;
  a.s = q->rs;
  a.Pv = P_values ? dP : nullptr;
  a.Av = A_values ? dA : nullptr;
  a.qv = qvec ? dq : nullptr;
  a.lv = l ? dl : nullptr;
  a.uv = u ? du : nullptr;
  a.x_ws = x_in ? dxw : nullptr;
  a.y_ws = y_in ? dyw : nullptr;
  a.rho_ws = nullptr;
  a.x_out = q->d_out;
  a.y_out = q->d_out + nn;
  a.info = q->d_info;
  a.ws = q->d_ws;
  a.batch = B;
  if (q->lds > 65536)
    hipFuncSetAttribute(reinterpret_cast<const void*>(&qp_resident_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(q->lds));
  hipLaunchKernelGGL(qp_resident_kernel, dim3(B), dim3(kQB), q->lds, nullptr, a, op);
  if ((e = hipGetLastError()) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess)
  {
    q->err = std::string("qp_resident_kernel: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  if (op == OP_SOLVE && ((x && (e = hipMemcpy(x, q->d_out, nn * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess) ||
                         (y && m && (e = hipMemcpy(y, q->d_out + nn, mm * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess)))
  {
    q->err = std::string("hipMemcpy: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  if (info && (op != OP_WARM_START) &&
      (e = hipMemcpy(info, q->d_info, sizeof(thip_qp_info) * B, hipMemcpyDeviceToHost)) != hipSuccess)
  {
    q->err = std::string("hipMemcpy: ") + hipGetErrorString(e);
    return THIP_E_HIP;
  }
  return THIP_OK;
}

// osqp_setup's / osqp_update_data_vec's validate: l <= u for every row of every QP
static bool bounds_ok(const thip_qp* q, const double* l, const double* u)
{
  const long long mm = static_cast<long long>(q->m) * q->batch;
  for (long long r = 0; r < mm; ++r)
    if (!(l[r] <= u[r]))
      return false;
  return true;
}

static void fail_info(thip_qp* q, thip_qp_info* info, int code)
{
  for (int b = 0; b < q->batch; ++b)
  {
    info[b] = thip_qp_info{};
    info[b].status = -1;
    info[b].setup_error = code;
  }
}

int thip_qp_setup(thip_qp* q, const double* P_values, const double* qvec, const double* A_values, const double* l,
                  const double* u, const thip_osqp_settings* settings, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if ((!P_values && q->nnz_p) || !qvec || (!A_values && q->nnz_a) || (q->m && (!l || !u)) || !settings || !info)
  {
    q->err = "thip_qp_setup: null argument";
    return THIP_E_INVALID;
  }
  if (!qp_settings_ok(q, settings))
  {
    q->err = "thip_qp_setup: " + q->err;
    return THIP_E_INVALID;
  }
  q->rs = *settings;
  q->resident = true;
  if (q->m && !bounds_ok(q, l, u))
  {
    // OSQP_DATA_VALIDATION_ERROR: no workspace
    q->resident = false;
    fail_info(q, info, 1);
    return THIP_OK;
  }
  const int rc = qp_resident(q, OP_SETUP, P_values, qvec, A_values, l, u, nullptr, nullptr, nullptr, nullptr, info);
  if (rc == THIP_OK)
    for (int b = 0; b < q->batch; ++b)
      if (info[b].status == -1)
        q->resident = false;
  return rc;
}

int thip_qp_update_vec(thip_qp* q, const double* qvec, const double* l, const double* u, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if (!q->resident)
  {
    q->err = "thip_qp_update_vec: no resident workspace (thip_qp_setup first)";
    return THIP_E_STATE;
  }
  if (!info || (!l) != (!u))
  {
    q->err = "thip_qp_update_vec: l and u go together; info is required";
    return THIP_E_INVALID;
  }
  if (l && q->m && !bounds_ok(q, l, u))
  {
    fail_info(q, info, 1);  // rejected, the workspace keeps its data
    return THIP_OK;
  }
  return qp_resident(q, OP_UPDATE_VEC, nullptr, qvec, nullptr, q->m ? l : nullptr, q->m ? u : nullptr, nullptr,
                     nullptr, nullptr, nullptr, info);
}

int thip_qp_update_mat(thip_qp* q, const double* P_values, const double* A_values, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if (!q->resident)
  {
    q->err = "thip_qp_update_mat: no resident workspace (thip_qp_setup first)";
    return THIP_E_STATE;
  }
  if (!info)
  {
    q->err = "thip_qp_update_mat: info is required";
    return THIP_E_INVALID;
  }
  const int rc = qp_resident(q, OP_UPDATE_MAT, q->nnz_p ? P_values : nullptr, nullptr, q->nnz_a ? A_values : nullptr,
                             nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, info);
  if (rc == THIP_OK)
    for (int b = 0; b < q->batch; ++b)
      if (info[b].status == -1)
        q->resident = false;
  return rc;
}

int thip_qp_warm_start(thip_qp* q, const double* x, const double* y)
{
  if (!q)
    return THIP_E_INVALID;
  if (!q->resident)
  {
    q->err = "thip_qp_warm_start: no resident workspace (thip_qp_setup first)";
    return THIP_E_STATE;
  }
  q->rs.warm_starting = 1;  // osqp_warm_start turns warm starting on
  return qp_resident(q, OP_WARM_START, nullptr, nullptr, nullptr, nullptr, nullptr, x, q->m ? y : nullptr, nullptr,
                     nullptr, nullptr);
}

int thip_qp_solve_resident(thip_qp* q, double* x, double* y, thip_qp_info* info)
{
  if (!q)
    return THIP_E_INVALID;
  if (!q->resident)
  {
    q->err = "thip_qp_solve_resident: no resident workspace (thip_qp_setup first)";
    return THIP_E_STATE;
  }
  if (!x || !info)
  {
    q->err = "thip_qp_solve_resident: null argument";
    return THIP_E_INVALID;
  }
  return qp_resident(q, OP_SOLVE, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, x, y, info);
}

void thip_qp_destroy(thip_qp* q)
{
  if (!q)
    return;
  hipSetDevice(q->device);
  // an uncollected group launch runs on another object's stream (done_stream,
  // which may already be destroyed) and may still read this object's buffers:
  // wait for the whole device then
  if (q->pending)
    hipDeviceSynchronize();
  if (q->stream)
  {
    hipStreamSynchronize(q->stream);
    hipStreamDestroy(q->stream);
  }
  hipFree(q->d_list);
  hipFree(q->d_first);
  hipFree(q->d_idx);
  hipFree(q->d_ws);
  hipFree(q->d_in);
  hipFree(q->d_out);
  hipFree(q->d_info);
  delete q;
}

const char* thip_qp_last_error(thip_qp* q) { return q ? q->err.c_str() : g_qp_create_err.c_str(); }

long long thip_qp_factor_nnz(const thip_qp* q) { return q ? q->nnz_l : -1; }

int thip_qp_debug_profile(long long* out, int reset)
{
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qp_prof), sizeof(long long) * 8) != hipSuccess)
    return THIP_E_HIP;
  if (reset)
  {
    const long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_qp_prof), z, sizeof(z)) != hipSuccess)
      return THIP_E_HIP;
  }
  return THIP_OK;
}

int thip_qp_shape(const thip_qp* q, long long* out)
{
  if (!q || !out)
    return THIP_E_INVALID;
  out[0] = q->pat.N;
  out[1] = q->nnz_l;
  out[2] = q->pat.nlev;
  out[3] = q->max_level;
  out[4] = q->pat.lds_pat;
  out[5] = static_cast<long long>(q->lds);
  return THIP_OK;
}

}  // extern "C"
