// Batched BasicTrustRegionSQP on MI355X (gfx950): one 256-thread workgroup per
// problem runs the whole penalty / SQP / trust-region loop of
// trajopt_sco/src/optimizers.cpp:699-991, including
//   * convexification: CartPose error + forward-difference jacobian (one
//     thread per perturbed FK, unperturbed poses staged in LDS) and the
//     constant JointVel quadratic (kinematic_terms.cpp:252-370,
//     trajectory_costs.cpp:257-301, modeling_utils.cpp:168-269)
//   * the QP solve with OSQP 1.0 semantics (osqp_interface.cpp:283-615): Ruiz
//     scaling, vector rho, ADMM with the linear system solved as a
//     waypoint-block-tridiagonal Cholesky after closed-form elimination of the
//     abs/hinge auxiliary variables, termination / infeasibility checks,
//     iteration-based adaptive rho, polishing with iterative refinement and the
//     reference's warm-start policy.
// All arithmetic is fp64. The path is latency / LDS bound, not a dense
// contraction, so there is no MFMA.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <type_traits>

#include "collision_device.hpp"
#include "kin_device.hpp"
#include "layout.hpp"

// THIP_GENERIC_ONLY: the generic-step build (layout.hpp kGenBlock threads, no
// register-resident segment, the fused kernel alone, named sqp_kernel_gen)
#ifndef THIP_GENERIC_ONLY
#define THIP_GENERIC_ONLY 0
#endif
// generic-step build: the d-value / middle-block phase on hoisted layout values
#ifndef THIP_GEN_DV_HOIST
#define THIP_GEN_DV_HOIST 1
#endif
#if THIP_GENERIC_ONLY
#define THIP_SQP_KERNEL sqp_kernel_gen
#else
#define THIP_SQP_KERNEL sqp_kernel
#endif

namespace thip
{
// ------------------------------------------------------------------ constants
constexpr double kInf = 1e30;  // OSQP_INFTY
// lane octets of the block solve: the chain layouts, the register-resident
// ADMM segment and their unrolled per-dof loops take D <= kOct
constexpr int kOct = 8;
// iterations per thread issued together in the generic ADMM step's row and
// column loops (loads of all of them before any store)
constexpr int kGenU = 4;
// ... sized to the loads an iteration issues: a wave tracks at most 63
// outstanding vector-memory operations (vmcnt), beyond which the issue stalls
constexpr int kGenULight = 8;  // a few loads per iteration (streaming vectors, bound rows)
constexpr int kGenUHeavy = 2;  // a CartPose row's coefficients and x (~2 D + 8 loads)
constexpr int kGenUHinge = 2;  // a hinge row's 2 D coefficients and 2 D x values (config E's heavy
                                // problems: ~20 rows per thread, one HBM round trip each at 1)
// Calls f(integral_constant<U'>) with U' the smallest power of two <= U whose
// U' kBlock items cover n (a uniform choice).  A loop over fewer items than
// U kBlock would otherwise issue the clamped loads of U - U' duplicate
// iterations per thread; on the FLAT path those cost issue slots even when
// they hit LDS (config HA: 181 CartPose rows and 210 columns on 256 threads).
// Each item's arithmetic is the same at any U'.  Only the generic-step build
// adapts: in the main build U' = U, and its code is instruction for
// instruction that of the plain loops (the register-resident segment's results
// were seen to depend on how the rest of that kernel compiles).
template <int U, typename F>
__device__ __forceinline__ void unroll_for(int n, F&& f)
{
#if THIP_GENERIC_ONLY
  if constexpr (U > 1)
  {
    if (n <= (U / 2) * kBlock)
    {
      unroll_for<U / 2>(n, f);
      return;
    }
  }
#endif
  f(std::integral_constant<int, U>());
}
// A loop over n items unrolled U per thread: adaptive (unroll_for) in the
// generic-step build, the plain loop with U = UMAX in the main build
#if THIP_GENERIC_ONLY
#define GEN_UNROLL_BEGIN(UMAX, N) unroll_for<(UMAX)>((N), [&](auto uc_) { constexpr int U = decltype(uc_)::value;
#define GEN_UNROLL_END });
#else
#define GEN_UNROLL_BEGIN(UMAX, N) { constexpr int U = (UMAX);
#define GEN_UNROLL_END }
#endif
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoTol = 1e-4, kRhoEq = 1e3;
constexpr double kMinScal = 1e-4, kMaxScal = 1e4;
constexpr double kDivTol = 1.0 / kInf;

enum
{
  ST_SOLVED = 1,
  ST_SOLVED_INACC = 2,
  ST_PINF = 3,
  ST_PINF_INACC = 4,
  ST_DINF = 5,
  ST_DINF_INACC = 6,
  ST_MAXIT = 7,
  ST_NONCVX = 9,
  ST_UNSOLVED = 11
};

// ----------------------------------------------------------- shared control
struct Ctl
{
  // reductions
  double red[kWaves * 16];
  double bc[16];
  // SQP state
  double trust;
  int status;
  int n_sqp, n_qp, n_fev, n_merit;
  int scan_at_x;  // the contact counts / costs of the last scan are those of X (GetContactResultCached)
  long long n_admm;
  // OSQP state
  double c, cinv;
  double rho;       // current rho of the active workspace
  double prev_rho;  // rho of the previous workspace
  int prev_status;  // status of the previous workspace (0 = none)
  int cur;          // double-buffer parity
  int qp_status, polish_status, iter;
  double prim_res, dual_res;
  int flag;
  int can_check;
  int time_up;  // the max_time check of this SQP iteration fired
  // OSQPModel sparsity fingerprint of the last QP setup (pattern_fingerprint)
  unsigned long long fp_hash;
  int fp_n, fp_m;
  long long fp_nnz;
  // diagnostics
  double* trace;
  int trace_cap, trace_n;
  double rho0;
  long long* prof;  // phase cycle counters of this problem (null = off)
  // collision rows of the current QP
  int n_h;
  int n_h_prev;
  int coll_overflow;  // set by the last contact scan
  int flags;          // sticky THIP_FLAG_* of the run
  long long n_contact_rows, n_hinge_admm, n_substates;
  int hcp[THIP_MAX_STEPS + 1];  // first hinge chunk of each step pair (admm_segment)
  int subcnt[THIP_MAX_STEPS];       // contact scan: LVS sub-states of each collision unit
  int suboff[THIP_MAX_STEPS + 1];   // and their prefix (the batched sub-state FK)
  int hboff[THIP_MAX_STEPS + 1];    // first I_HBITS word of each unit (batched scans)
  int hbits_x;                      // the hit bits are those of the last count pass (batched)
};

// The kinematic tree, copied into LDS at kernel entry (stage_chain): every
// FK walk reads its joint origins, axes and types from here.  Read from the
// descriptor in HBM they were FLAT loads with L2 latency at every joint of
// every walk (sub-state FK of the contact scans, the CartPose jacobians).
__shared__ thip_chain g_chain;
#if THIP_GENERIC_ONLY
// contact_test_type FIRST in the fused scan (coll_scan_pairs): per scan wave,
// one bit per sub-state of the unit being scanned -- a contactTest call whose
// first contact has been met in ContactResultMap order
__shared__ unsigned g_first_done[kScanWaves][kSubCap / 32];
#endif

__device__ __forceinline__ void stage_chain(const thip_problem_desc* d)
{
  static_assert(sizeof(thip_chain) % 4 == 0, "word copy");
  const int* src = reinterpret_cast<const int*>(&d->chain);
  int* dst = reinterpret_cast<int*>(&g_chain);
  for (int w = threadIdx.x; w < static_cast<int>(sizeof(thip_chain) / 4); w += blockDim.x)
    dst[w] = src[w];
  __syncthreads();
}

struct Ctx
{
  const Layout& L;
  const Tables& T;
  const thip_problem_desc* d;
  double* w;
  int* iw;
  double* big;
  Ctl* s;
  double* const* ptab;  // LDS table of array base pointers (LDS-resident or HBM), or null
  double** ptab_w = nullptr;  // the same table, writable (dynamic residency plan)
  const double* scene = nullptr;  // this problem's primitives [n_prims][16]
  const double* jpt = nullptr;    // this problem's JointPos targets [n_jpos][D]
  struct CollStage* cs = nullptr; // contact-scan tables staged in static LDS
  int tid, lane, wave;
  __device__ Ctx(const Layout& l, const Tables& t, const thip_problem_desc* dd, double* ww, int* ii, double* bb,
                 Ctl* ss, double* const* pt = nullptr)
    : L(l), T(t), d(dd), w(ww), iw(ii), big(bb), s(ss), ptab(pt)
  {
    tid = threadIdx.x;
    lane = tid & 63;
    wave = tid >> 6;
  }
  __device__ __forceinline__ double* a(int k) const { return ptab ? ptab[k] : w + L.doff[k]; }
  // dynamic QP sizes (base sizes plus the current hinge rows)
  __device__ __forceinline__ int m() const { return L.m_base + 2 * s->n_h; }
  __device__ __forceinline__ int nc() const { return L.nc_base + s->n_h; }
  __device__ __forceinline__ int* ia(int k) const { return iw + L.ioff[k]; }
};

#define FOR(i, n) for (int i = c.tid; i < (n); i += kBlock)
#define BSYNC() __syncthreads()

// Arrays the residency plan always places in LDS (chain matrices, LINV, CV,
// YV: thip_create rejects problems where they would not fit) are accessed
// through LDS-typed pointers so the compiler emits ds_read/ds_write instead of
// flat accesses (flat ops count on vmcnt and lgkmcnt, so every wait would also
// drain outstanding stores).
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ lds_f64* lds(double* p) { return (lds_f64*)p; }
__device__ __forceinline__ const lds_f64* lds(const double* p) { return (const lds_f64*)p; }
// HBM-resident arrays as global-address-space pointers: global_* instead of
// FLAT instructions (a FLAT access also counts against lgkmcnt, so every LDS
// wait would drain it too)
typedef __attribute__((address_space(1))) double gbl_f64;
__device__ __forceinline__ gbl_f64* gbl(double* p) { return (gbl_f64*)p; }
__device__ __forceinline__ const gbl_f64* gbl(const double* p) { return (const gbl_f64*)p; }

// Phase profiling (thip_debug_profile): shader-clock cycles accumulated per
// slot by thread 0.  Slots: 0 admm_step, 1 residuals, 2 termination check,
// 3 factor, 4 polish, 5 linearize, 6 evaluate, 7 build_and_scale,
// 8 solve rhs + block diag (segment: phase A), 9 forward chain, 10 backward
// chain, 11 aux back-substitution (segment: phase E), 12 qp_solve, 13 sqp
// total, 14 sqp total (wall clock, 100 MHz ticks), 15 segment phase B
// (rhs + Linv b), 16 segment phase C2 (Linv^T y + middle block).
struct ProfScope
{
  long long* p;
  int slot;
  long long t0;
  __device__ ProfScope(const Ctx& c, int s) : p(c.tid == 0 ? c.s->prof : nullptr), slot(s), t0(p ? clock64() : 0) {}
  __device__ ~ProfScope()
  {
    if (p)
      p[slot] += clock64() - t0;
  }
};
#define PROF_CAT2(a, b) a##b
#define PROF_CAT(a, b) PROF_CAT2(a, b)
#define PROF(slot) ProfScope PROF_CAT(prof_scope_, __LINE__)(c, slot)

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v);
__device__ __forceinline__ double wave_max(double v);
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v += __shfl_xor(v, o);
  return v;
}

// K simultaneous block max-reductions; results in c.s->bc[0..K)
template <int K>
__device__ void block_max(Ctx& c, double (&v)[K])
{
#pragma unroll
  for (int k = 0; k < K; ++k)
  {
    const double r = wave_max(v[k]);
    if (c.lane == 0)
      c.s->red[c.wave * 16 + k] = r;
  }
  BSYNC();
  if (c.tid < K)
  {
    double r = c.s->red[c.tid];
    for (int wv = 1; wv < kWaves; ++wv)
      r = fmax(r, c.s->red[wv * 16 + c.tid]);
    c.s->bc[c.tid] = r;
  }
  BSYNC();
#pragma unroll
  for (int k = 0; k < K; ++k)
    v[k] = c.s->bc[k];
  BSYNC();
}

// two simultaneous block sums (wave_sum order per value)
__device__ void block_sum2(Ctx& c, double& a, double& b)
{
  const double ra = wave_sum(a), rb = wave_sum(b);
  if (c.lane == 0)
  {
    c.s->red[c.wave * 16] = ra;
    c.s->red[c.wave * 16 + 1] = rb;
  }
  BSYNC();
  double sa = 0, sb = 0;
  for (int wv = 0; wv < kWaves; ++wv)
  {
    sa += c.s->red[wv * 16];
    sb += c.s->red[wv * 16 + 1];
  }
  BSYNC();
  a = sa;
  b = sb;
}

__device__ double block_sum(Ctx& c, double v)
{
  const double r = wave_sum(v);
  if (c.lane == 0)
    c.s->red[c.wave * 16] = r;
  BSYNC();
  double s = 0;
  for (int wv = 0; wv < kWaves; ++wv)
    s += c.s->red[wv * 16];
  BSYNC();
  return s;
}

__device__ __forceinline__ double limit_scaling(double a)
{
  a = a < kMinScal ? 1.0 : a;
  a = a > kMaxScal ? kMaxScal : a;
  return a;
}

// ======================================================================
// Convexification of CartPose terms at trajectory x (nx):
//   A_G [n_abs][D]: weight * cleanupAff(J row), A_GC: weight * (y - J.x),
//   I_MASK: kept-entry bit mask (|J| > 1e-7)
// ======================================================================
__device__ void coll_scan(Ctx& c, const double* x, double* costs, bool rows);

__device__ void linearize(Ctx& c, const double* x, double* raw_jac = nullptr)
{
  PROF(5);
  const Layout& L = c.L;
  const int D = L.D;
  const thip_chain& ch = g_chain;
  double* stage = c.big;  // [n_cart][30]: source pose (12), target^-1 (12), err (6)
  const double* tgt = c.a(A_TGT);
  FOR(k, L.n_cart)
  {
    const int t = c.d->cart_step[k];
    Pose S, So, Tb, To, Tt, Ti;
    chain_fk(ch, x + t * D, c.d->cart_source_link[k], S);
    pose_load(So, c.d->cart_source_offset[k]);
    Pose Ss;
    pose_mul(S, So, Ss);
    pose_load(To, tgt + 12 * k);
    const int tl = c.d->cart_target_link[k];
    if (tl > 0)
      chain_fk(ch, x + t * D, tl, Tb);  // DynamicCartPose: the active target link
    else
      pose_load(Tb, ch.base_pose);
    pose_mul(Tb, To, Tt);
    pose_inv(Tt, Ti);
    double* st = stage + 30 * k;
    for (int i = 0; i < 9; ++i)
    {
      st[i] = Ss.r[i];
      st[12 + i] = Ti.r[i];
    }
    for (int i = 0; i < 3; ++i)
    {
      st[9 + i] = Ss.t[i];
      st[21 + i] = Ti.t[i];
    }
    transform_error(Ti, Ss, st + 24);
    if (c.d->cart_has_tol[k])
      apply_tolerances(st + 24, c.d->cart_lower_tol[k], c.d->cart_upper_tol[k]);
  }
  BSYNC();
  // perturbed FKs: item (k, p)
  const double eps = 1e-5;
  double* G = c.a(A_G);
  FOR(item, L.n_cart * D)
  {
    const int k = item / D, p = item % D;
    const int t = c.d->cart_step[k];
    double q[THIP_MAX_DOF];
    for (int j = 0; j < D; ++j)
      q[j] = x[t * D + j];
    q[p] = q[p] + eps;
    Pose S, So, Sp;
    chain_fk(ch, q, c.d->cart_source_link[k], S);
    pose_load(So, c.d->cart_source_offset[k]);
    pose_mul(S, So, Sp);
    const double* st = stage + 30 * k;
    Pose Ss, Ti;
    for (int i = 0; i < 9; ++i)
    {
      Ss.r[i] = st[i];
      Ti.r[i] = st[12 + i];
    }
    for (int i = 0; i < 3; ++i)
    {
      Ss.t[i] = st[9 + i];
      Ti.t[i] = st[21 + i];
    }
    // calcJacobianTransformErrorDiff(target, source, source_perturbed); DynamicCartPose:
    // (target, target_perturbed, source, source_perturbed), kinematic_terms.cpp:170-177
    Pose pe, ppe;
    pose_mul(Ti, Ss, pe);
    const int tl = c.d->cart_target_link[k];
    if (tl > 0)
    {
      Pose Tq, To, Tp, Tpi;
      chain_fk(ch, q, tl, Tq);
      pose_load(To, c.a(A_TGT) + 12 * k);
      pose_mul(Tq, To, Tp);
      pose_inv(Tp, Tpi);
      pose_mul(Tpi, Sp, ppe);
    }
    else
      pose_mul(Ti, Sp, ppe);
    double diff[6];
    if (c.d->cart_has_tol[k])
      transform_error_diff_tol(pe, ppe, c.d->cart_lower_tol[k], c.d->cart_upper_tol[k], diff);
    else
    {
      double r0[3], r1[3];
      for (int i = 0; i < 3; ++i)
        diff[i] = ppe.t[i] - pe.t[i];
      rot_error(pe.r, r0, true);
      rot_error(ppe.r, r1, true);
      for (int i = 0; i < 3; ++i)
        diff[3 + i] = r1[i] - r0[i];
    }
    const int r0w = c.T.term_row0[k], nr = c.T.term_nrow[k];
    for (int rr = 0; rr < nr; ++rr)
    {
      const int row = r0w + rr;
      G[row * D + p] = diff[c.T.row_comp[row]] / eps;
    }
  }
  BSYNC();
  // affFromValGrad + cleanupAff + exprScale(weight)
  double* GC = c.a(A_GC);
  int* mask = c.ia(I_MASK);
  FOR(row, L.n_abs)
  {
    const int k = c.T.row_term[row];
    if (c.T.row_jpos[row])
    {
      // JointPosEqConstraint row (trajectory_costs.cpp:151-160): exprMult(x_tj - target_j, coeff_j);
      // constant, so identical at every linearisation; the coefficient is kept even when 0 (no cleanupAff)
      const int j = c.T.row_comp[row];
      const double wgt = c.T.row_w[row];
      for (int p = 0; p < D; ++p)
        G[row * D + p] = p == j ? 1.0 * wgt : 0.0;
      if (raw_jac)
        for (int p = 0; p < D; ++p)
          raw_jac[row * D + p] = p == j ? 1.0 : 0.0;
      mask[row] = 1 << j;
      GC[row] = (-c.jpt[k * D + j]) * wgt;
      continue;
    }
    const int t = c.d->cart_step[k];
    const double y = stage[30 * k + 24 + c.T.row_comp[row]];
    double dot = 0;
    for (int j = 0; j < D; ++j)
      dot += G[row * D + j] * x[t * D + j];
    const double wgt = c.T.row_w[row];
    if (raw_jac)
      for (int j = 0; j < D; ++j)
        raw_jac[row * D + j] = G[row * D + j];
    int m = 0;
    for (int j = 0; j < D; ++j)
    {
      const double g = G[row * D + j];
      const bool keep = fabs(g) > 1e-7;
      m |= keep ? (1 << j) : 0;
      G[row * D + j] = keep ? g * wgt : 0.0;
    }
    mask[row] = m;
    GC[row] = (y - dot) * wgt;
  }
  BSYNC();
  if (L.hinge && !raw_jac)
    coll_scan(c, x, nullptr, true);
}

// ======================================================================
// LVS-discrete collision term (config C): contact scan, pair costs, hinge
// rows.  DiscreteCollisionEvaluator::CalcCollisions
// (trajopt/src/collision_terms.cpp:817-898), GetGradient (:195-242),
// CalcDistExpressions* (:463-536), CollisionCost::value (:1287-1306);
// the same arithmetic as oracle/src/collision.cpp.
//
// Each of the first kScanWaves waves takes step pairs t = first + wave, +
// kScanWaves, ...; per pair the
// lanes compute the sphere centers of the LVS sub-states (one sub-state per
// lane, scratch in A_CSCR), then scan the candidates (robot sphere s of link
// group g, primitive p, sub-state i) in the flattened ContactResultMap order
// (link, primitive, then insertion order sub-state, sphere) 64 at a time; a
// ballot gives each contact its rank.  Pass 0 counts contacts and sums the
// pair's cost; pass 1 (rows only) writes the ordered contact list.
// ======================================================================
__device__ __forceinline__ bool coll_fixed_step(const Ctx& c, int t) { return c.T.coll_fixed[t] != 0; }

// Collision units: step pairs (LVS_DISCRETE / LVS_CONTINUOUS), or waypoints
// (DISCRETE, SingleTimestepCollisionEvaluator).  A waypoint unit t files its
// rows in step pair min(t, N - 2), on that pair's half t - pair; the last
// waypoint's rows follow waypoint N - 2's in pair N - 2.
__device__ __forceinline__ int coll_pair_of(const Layout& L, int t) { return L.coll_single ? min(t, L.N - 2) : t; }

// contact rows filed in step pair p
__device__ __forceinline__ int coll_pair_count(const Layout& L, const int* PCNT, int p)
{
  if (!L.coll)
    return 0;
  const bool in = p >= L.coll_first && p < L.coll_last;
  if (!L.coll_single)
    return in ? PCNT[p] : 0;
  int n = (in && p <= L.N - 2) ? PCNT[p] : 0;
  if (p == L.N - 2 && L.N - 1 >= L.coll_first && L.N - 1 < L.coll_last)
    n += PCNT[L.N - 1];
  return n;
}

// first hinge row of unit t (HP: per step pair)
__device__ __forceinline__ int coll_unit_row0(const Layout& L, const int* PCNT, const int* HP, int t)
{
  const int p = coll_pair_of(L, t);
  int r = HP[p];
  if (L.coll_single && t > p && p >= L.coll_first)
    r += PCNT[p];
  return r;
}

// Contact-scan tables and this problem's scene, staged in static LDS once per
// scan (the candidate decode read them from global memory, a chain of
// dependent loads per ballot round).
struct CollStage
{
  double scene[THIP_MAX_PRIMS * 16];
  double rad[THIP_MAX_SPHERES];
  double ctr[THIP_MAX_SPHERES * 3];
  int grp_ns[THIP_MAX_LINKS];
  int grp_s0[THIP_MAX_LINKS];
  int grp_link[THIP_MAX_LINKS];
  int sph_order[THIP_MAX_SPHERES];
  int sph_grp[THIP_MAX_SPHERES];  // inverse of sph_order: group of sphere s
  int sph_e[THIP_MAX_SPHERES];    // and its position in the group
};

__device__ void coll_stage(Ctx& c)
{
  CollStage& S = *c.cs;
  const int P = c.d->n_prims, ns = c.d->n_spheres, ng = c.T.n_groups;
  FOR(e, P * 16) S.scene[e] = c.scene[e];
  FOR(e, ns)
  {
    S.rad[e] = c.d->sphere_radius[e];
    S.sph_order[e] = c.T.sph_order[e];
    for (int r = 0; r < 3; ++r)
      S.ctr[e * 3 + r] = c.d->sphere_center[e][r];
  }
  FOR(e, ng)
  {
    S.grp_ns[e] = c.T.grp_ns[e];
    S.grp_s0[e] = c.T.grp_s0[e];
    S.grp_link[e] = c.T.grp_link[e];
    for (int k = 0; k < c.T.grp_ns[e]; ++k)
    {
      const int s = c.T.sph_order[c.T.grp_s0[e] + k];
      S.sph_grp[s] = e;
      S.sph_e[s] = k;
    }
  }
  BSYNC();
}

// World centers of every robot sphere at joint values q into dst[s * 3]: one
// FK walk over the tree; each sphere group's link pose is the walk's prefix
// (the same operations as chain_fk(.., link, ..)).
__device__ __forceinline__ void sphere_centers_at(const CollStage& S, const thip_chain& ch, int ngr, const double* q,
                                                  double* dst0)
{
  Pose T;
  pose_load(T, ch.base_pose);
  const int last_link = S.grp_link[ngr - 1];
  int g = 0;
  for (int k = 1; k <= last_link; ++k)
  {
    if (ch.parent[k] != k - 1)  // a branch of the tree: restart from the parent link's pose
      chain_fk(ch, q, ch.parent[k], T);
    Pose O, Tn;
    pose_load(O, ch.joint_origin[k]);
    pose_mul(T, O, Tn);
    const int type = ch.joint_type[k];
    if (type == THIP_JOINT_REVOLUTE || type == THIP_JOINT_CONTINUOUS)
    {
      Pose M;
      rot_axis_angle(ch.joint_axis[k], q[ch.joint_dof[k]], M.r);
      M.t[0] = M.t[1] = M.t[2] = 0;
      pose_mul(Tn, M, T);
    }
    else if (type == THIP_JOINT_PRISMATIC)
    {
      Pose M;
      const double v = q[ch.joint_dof[k]];
      M.r[0] = M.r[4] = M.r[8] = 1;
      M.r[1] = M.r[2] = M.r[3] = M.r[5] = M.r[6] = M.r[7] = 0;
      M.t[0] = ch.joint_axis[k][0] * v;
      M.t[1] = ch.joint_axis[k][1] * v;
      M.t[2] = ch.joint_axis[k][2] * v;
      pose_mul(Tn, M, T);
    }
    else
      T = Tn;
    for (; g < ngr && S.grp_link[g] == k; ++g)
      for (int e = 0; e < S.grp_ns[g]; ++e)
      {
        const int s = S.sph_order[S.grp_s0[g] + e];
        const double* cs = S.ctr + s * 3;
        double* dst = dst0 + s * 3;
        for (int r = 0; r < 3; ++r)
          dst[r] = T.r[r * 3 + 0] * cs[0] + T.r[r * 3 + 1] * cs[1] + T.r[r * 3 + 2] * cs[2] + T.t[r];
      }
  }
}

// The LVS sub-states of every collision unit at x, their prefix in
// Ctl::suboff, and -- when they number at most kScanWaves * kSubCap -- the sphere
// centers of all of them computed by the whole workgroup at once into A_CSCR
// (unit t's sub-state i at row suboff[t] + i).  A unit of one wave has ~5
// sub-states, so a per-unit walk keeps ~5 of its 64 lanes busy.  Returns
// whether the centers were computed (else each wave walks its own units).
__device__ bool coll_substates_batched(Ctx& c, const double* x)
{
  const CollStage& S = *c.cs;
  const Layout& L = c.L;
  const int D = L.D, ns = c.d->n_spheres;
  const bool single = L.coll_single != 0;
  FOR(u, L.coll_last - L.coll_first)
  {
    const int t = L.coll_first + u;
    int cnt = 0;
    if (!(single && coll_fixed_step(c, t)))
    {
      const double* q0 = x + t * D;
      cnt = single ? 1 : lvs_count(q0, x + (t + 1) * D, D, c.d->coll_lvs);
      if (cnt > kSubCap)
        cnt = 0;  // the unit's overflow is flagged by its wave
    }
    c.s->subcnt[t] = cnt;
  }
  BSYNC();
  if (c.tid == 0)
  {
    const bool cont = c.d->coll_continuous == 1;
    int acc = 0, wacc = 0;
    for (int t = L.coll_first; t < L.coll_last; ++t)
    {
      c.s->suboff[t] = acc;
      c.s->hboff[t] = wacc;
      const int cnt = c.s->subcnt[t];
      acc += cnt;
      const int nseg = cont ? cnt - 1 : cnt;
      // scene then self candidates, whole 64-bit chunks
      wacc += ((c.d->n_prims * ns + c.T.n_self_sph) * (nseg > 0 ? nseg : 0) + 63) / 64 * 2;
    }
    c.s->suboff[L.coll_last] = acc;
    c.s->hboff[L.coll_last] = wacc;
  }
  BSYNC();
  const int total = c.s->suboff[L.coll_last];
  if (total > kScanWaves * kSubCap)
    return false;
  long long* pf22 = (c.tid == 0) ? c.s->prof : nullptr;
  const long long tfk0 = pf22 ? clock64() : 0;
  double* SCR = c.a(A_CSCR);
  const thip_chain& ch = g_chain;
  FOR(j, total)
  {
    // the unit holding sub-state j (binary search of the prefix)
    int lo = L.coll_first, hi = L.coll_last - 1;
    while (lo < hi)
    {
      const int mid = (lo + hi + 1) >> 1;
      if (c.s->suboff[mid] <= j)
        lo = mid;
      else
        hi = mid - 1;
    }
    const int t = lo, i = j - c.s->suboff[t], cnt = c.s->subcnt[t];
    const double* q0 = x + t * D;
    const double* q1 = single ? q0 : x + (t + 1) * D;
    double q[THIP_MAX_DOF];
    for (int k = 0; k < D; ++k)
      q[k] = linspaced(cnt, q0[k], q1[k], i);
    sphere_centers_at(S, ch, c.T.n_groups, q, SCR + (long long)j * ns * 3);
  }
  BSYNC();
  if (pf22)
    pf22[22] += clock64() - tfk0;
  return true;
}

// Self-collision candidate q of a unit (0 <= q < nseg * n_self_sph, in key
// order: link pair, then sub-state, then sphere pair of the key): its
// sub-state i, spheres (sa, sb), distance, and the cc types of both sides
// (1 Time0, 2 Time1, 3 Between; oracle addSelfContacts).
__device__ __forceinline__ void self_candidate(const Ctx& c, const CollStage& S, const double* SCR, int ns, int nseg,
                                               int last, bool cont, int q, int& i, int& sa, int& sb, double& dist,
                                               int& cta, int& ctb)
{
  int r = q, k = 0;
  for (; k + 1 < c.T.n_self_keys; ++k)
  {
    const int sz = nseg * (c.T.self_kp[k + 1] - c.T.self_kp[k]);
    if (r < sz)
      break;
    r -= sz;
  }
  const int k0 = c.T.self_kp[k], npk = c.T.self_kp[k + 1] - k0;
  i = r / npk;
  const int j = k0 + (r - i * npk);
  sa = c.T.self_sa[j];
  sb = c.T.self_sb[j];
  const double* a0 = SCR + (i * ns + sa) * 3;
  const double* a1 = cont ? SCR + ((i + 1) * ns + sa) * 3 : a0;
  const double* b0 = SCR + (i * ns + sb) * 3;
  const double* b1 = cont ? SCR + ((i + 1) * ns + sb) * 3 : b0;
  double ca0[3], ca1[3], cb0[3], cb1[3];
  for (int e = 0; e < 3; ++e)
  {
    ca0[e] = a0[e];
    ca1[e] = a1[e];
    cb0[e] = b0[e];
    cb1[e] = b1[e];
  }
  double n[3], pa[3], pb[3], ta, tb;
  self_sphere_distance(ca0, ca1, S.rad[sa], cb0, cb1, S.rad[sb], cont, dist, n, pa, pb, ta, tb);
  if (cont)
  {
    cta = (i == 0 && ta == 0.0) ? 1 : ((i + 1 == last && ta == 1.0) ? 2 : 3);
    ctb = (i == 0 && tb == 0.0) ? 1 : ((i + 1 == last && tb == 1.0) ? 2 : 3);
  }
  else
    cta = ctb = (i == 0) ? 1 : ((i == last) ? 2 : 3);
}

// (margin, coeff) of the contact between robot sphere s and scene primitive p
// (p >= 0) or robot sphere -1 - p: the per link-pair tables (pair_data.hpp,
// CollisionMarginData / CollisionCoeffData, collision_terms.cpp:243-386) or
// the term's own dist_pen / coeffs.  A dropped pair (zero coefficient) reads
// margin -inf: no distance is below margin + buffer.
__device__ __forceinline__ double2 pair_mc(const Ctx& c, int s, int p)
{
  if (!c.T.pair_mc)
    return make_double2(c.d->coll_margin, c.d->coll_coeff);
  const int P = c.d->n_prims, W = P + c.d->n_spheres;
  const double* e = c.T.pair_mc + 2 * (s * W + (p >= 0 ? p : P + (-1 - p)));
  return make_double2(e[0], e[1]);
}

// (margin, coeff) of collision hinge row h (its contact's sphere and primitive)
__device__ __forceinline__ double2 row_pair_mc(const Ctx& c, int h)
{
  if (!c.T.pair_mc)
    return make_double2(c.d->coll_margin, c.d->coll_coeff);
  const int* CT = c.ia(I_CONT);
  return pair_mc(c, CT[3 * h + 1], CT[3 * h + 2]);
}

template <int PASS>
__device__ void coll_scan_pairs(Ctx& c, const double* x, int* out_base)
{
  const CollStage& S = *c.cs;
  const Layout& L = c.L;
  const int D = L.D, ns = c.d->n_spheres, P = c.d->n_prims;
  const thip_chain& ch = g_chain;
  // per candidate: the pair's margin and coefficient (pair_mc), contact distance
  // margin + buffer after incrementCollisionMargin(buffer)
  const double buffer = c.d->coll_buffer;
  // the rank pass at the point the count pass just scanned reads the hits it
  // recorded (I_HBITS) instead of recomputing every candidate's distance
  const bool use_bits = (PASS == 1) && c.s->hbits_x;
  const bool batched = use_bits || coll_substates_batched(c, x);
  if (PASS == 0)
  {
    BSYNC();  // every wave past its reads of the previous flag
    if (c.tid == 0)
#if THIP_GENERIC_ONLY
      // (FIRST / CLOSEST select among a call's contacts: the rank pass recomputes them)
      c.s->hbits_x = (batched && c.d->coll_contact_test == THIP_CONTACT_ALL) ? 1 : 0;
#else
      c.s->hbits_x = batched ? 1 : 0;
#endif
  }
  unsigned* const HBITS = reinterpret_cast<unsigned*>(c.ia(I_HBITS));
  double* SCRW = c.a(A_CSCR) + (long long)(c.wave < kScanWaves ? c.wave : 0) * kSubCap * ns * 3;
  int* PCNT = c.ia(I_PCNT);
  double* HCOST = c.a(A_HCOST);
  int* CONT = c.ia(I_CONT);
  int* HT = c.ia(I_HT);
  for (int t = L.coll_first + c.wave; c.wave < kScanWaves && t < L.coll_last; t += kScanWaves)
  {
    const bool single = L.coll_single != 0;
    if (single && coll_fixed_step(c, t))
    {
      // no term at a fixed waypoint
      if (PASS == 0 && c.lane == 0)
      {
        PCNT[t] = 0;
        HCOST[t] = 0.0;
      }
      continue;
    }
    const double* q0 = x + t * D;
    // DISCRETE: one state, q_t (linspaced(1, .., high) = high)
    const double* q1 = single ? q0 : x + (t + 1) * D;
    const int cnt = single ? 1 : lvs_count(q0, q1, D, c.d->coll_lvs);
    if (cnt > kSubCap)
    {
      if (c.lane == 0)
      {
        c.s->coll_overflow = 1;
        if (PASS == 0)
        {
          PCNT[t] = 0;
          HCOST[t] = 0.0;
        }
      }
      continue;
    }
    const bool f0 = !single && coll_fixed_step(c, t), f1 = !single && coll_fixed_step(c, t + 1);
    const int ngr = c.T.n_groups;
    // LVS_CONTINUOUS: candidates are the casts between consecutive sub-states
    const bool cont = c.d->coll_continuous == 1;
    const int nseg = cont ? cnt - 1 : cnt;
    const int last = cnt - 1;
    // sphere centers of the unit's sub-states: computed by the batched walk,
    // or here by this wave (one sub-state per lane)
    const double* SCR = batched ? c.a(A_CSCR) + (long long)c.s->suboff[t] * ns * 3 : SCRW;
    unsigned* const HB = batched ? HBITS + c.s->hboff[t] : nullptr;
    if (PASS == 0 && HB)
    {
      for (int w = c.lane; w < c.s->hboff[t + 1] - c.s->hboff[t]; w += 64)
        HB[w] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (!batched)
    {
      long long* pf22 = (c.tid == 0) ? c.s->prof : nullptr;
      const long long tfk0 = pf22 ? clock64() : 0;
      for (int isub = c.lane; isub < cnt; isub += 64)
      {
        double q[THIP_MAX_DOF];
        for (int j = 0; j < D; ++j)
          q[j] = linspaced(cnt, q0[j], q1[j], isub);
        sphere_centers_at(S, ch, ngr, q, SCRW + (long long)isub * ns * 3);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (pf22)
        pf22[22] += clock64() - tfk0;
    }
#if THIP_GENERIC_ONLY
    if (PASS == 0 && c.d->coll_contact_test == THIP_CONTACT_ALL)
#else
    if (PASS == 0)
#endif
    {
      // counts and cost only: lane = (sub-state, sphere), looping over the
      // primitives, so every distance call of the wave is for one primitive
      // (its type branch is uniform, its record a broadcast LDS read) and a
      // lane loads its sphere centers once; the order of the candidates does
      // not matter for a count and a sum
      double lcost = 0.0, lcount = 0.0;
      const int nsi = ns * nseg;
      for (int idx = c.lane; idx < nsi + 63; idx += 64)
      {
        if (__builtin_amdgcn_readfirstlane(idx - c.lane) >= nsi)
          break;
        const bool act = idx < nsi;
        const int i = act ? idx / ns : 0, s = act ? idx - (idx / ns) * ns : 0;
        const double rad = S.rad[s];
        double cx[3], cy[3];
        {
          const double* cp = SCR + (i * ns + s) * 3;
          const double* cq = SCR + ((cont ? i + 1 : i) * ns + s) * 3;
          for (int r = 0; r < 3; ++r)
          {
            cx[r] = cp[r];
            cy[r] = cq[r];
          }
        }
        for (int p = 0; p < P; ++p)
        {
          double prim[16];
          for (int e = 0; e < 16; ++e)
            prim[e] = S.scene[16 * p + e];
          const double2 mc = pair_mc(c, s, p);
          const double margin = mc.x, coeff = mc.y, threshold = margin + buffer;
          double dist = 0.0;
          bool hit = false;
          int cct = 3;  // CCType of the robot link: 1 Time0, 2 Time1, 3 Between
          if (act)
          {
            double n[3], pr[3];
            if (cont)
            {
              if (swept_lower_bound(cx, cy, rad, prim) < threshold)
              {
                double ts;
                swept_sphere_prim_distance(cx, cy, rad, prim, dist, n, pr, ts);
                hit = dist < threshold;
                cct = (i == 0 && ts == 0.0) ? 1 : ((i + 1 == last && ts == 1.0) ? 2 : 3);
              }
            }
            else
            {
              sphere_prim_distance(cx, rad, prim, dist, n, pr);
              hit = dist < threshold;
              cct = (i == 0) ? 1 : ((i == last) ? 2 : 3);
            }
          }
          hit = hit && !(dist > margin + buffer);
          if (hit && (f0 || f1))
            hit = (f0 && cct != 1) || (f1 && cct != 2);
          lcount += hit ? 1.0 : 0.0;
          lcost += hit ? fmax(margin - dist, 0.0) * coeff : 0.0;
          if (hit && HB)
          {
            // its index in the rank pass's (group, primitive, sub-state, sphere) order
            const int g = S.sph_grp[s], gn = S.grp_ns[g];
            const int cand = P * nseg * S.grp_s0[g] + (p * nseg + i) * gn + S.sph_e[s];
            atomicOr(HB + (cand >> 5), 1u << (cand & 31));
          }
        }
      }
      // self-collision candidates (key order; their hit bits follow the scene's)
      const int nself = c.T.n_self_sph * nseg, scene_total = nsi * P;
      for (int q = c.lane; q < nself + 63; q += 64)
      {
        if (__builtin_amdgcn_readfirstlane(q - c.lane) >= nself)
          break;
        bool hit = false;
        double dist = 0.0, margin = 0.0, coeff = 0.0;
        if (q < nself)
        {
          int i, sa, sb, cta, ctb;
          self_candidate(c, S, SCR, ns, nseg, last, cont, q, i, sa, sb, dist, cta, ctb);
          const double2 mc = pair_mc(c, sa, -1 - sb);
          margin = mc.x;
          coeff = mc.y;
          const double threshold = margin + buffer;
          hit = dist < threshold && !(dist > margin + buffer);
          if (hit && (f0 || f1))
            hit = (f0 && (cta != 1 || ctb != 1)) || (f1 && (cta != 2 || ctb != 2));
        }
        lcount += hit ? 1.0 : 0.0;
        lcost += hit ? fmax(margin - dist, 0.0) * coeff : 0.0;
        if (hit && HB)
        {
          const int cand = scene_total + q;
          atomicOr(HB + (cand >> 5), 1u << (cand & 31));
        }
      }
      const double cost = wave_sum(lcost);
      const int found = static_cast<int>(wave_sum(lcount));
      if (c.lane == 0)
      {
        PCNT[t] = found;
        HCOST[t] = cost;
        atomicAdd(reinterpret_cast<unsigned long long*>(&c.s->n_substates), static_cast<unsigned long long>(cnt));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    int scene_total = 0;
    for (int g = 0; g < ngr; ++g)
      scene_total += P * nseg * S.grp_ns[g];
    const int total = scene_total + c.T.n_self_sph * nseg;
    int running = 0;
    double lcost = 0.0;  // per-lane partial cost, reduced once per pair
    const int base = (PASS == 1) ? coll_unit_row0(L, PCNT, out_base, t) : 0;
    const int pair = coll_pair_of(L, t);
#if THIP_GENERIC_ONLY
    // contact_test_type (trajopt_hip.h THIP_CONTACT_*; oracle applyContactTest):
    // the test selects among each contactTest call's contacts (one call per
    // sub-state) before the evaluator's filter -- CLOSEST the first smallest
    // distance of each (key, sub-state) group, FIRST the call's first contact in
    // ContactResultMap order; the fixed-end rule then applies to the selected one
    const int ctest = c.d->coll_contact_test;
    unsigned* const done = g_first_done[c.wave];
    if (ctest == THIP_CONTACT_FIRST)
    {
      for (int w = c.lane; w < (nseg + 31) / 32; w += 64)
        done[w] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
#endif
    for (int c0 = 0; c0 < total; c0 += 64)
    {
      const int cand = c0 + c.lane;
      bool hit = false;
      double dist = 0.0, margin = 0.0, coeff = 0.0;
      int i = 0, s = 0, p = 0;
#if THIP_GENERIC_ONLY
      bool pre = false, fixed_ok = true;  // a contact of the call; the fixed-end rule keeps it
#endif
      if (cand >= scene_total)
      {
        // a self-collision candidate: (sub-state, sphere a, -1 - sphere b)
        if (cand < total)
        {
          int cta, ctb;
          self_candidate(c, S, SCR, ns, nseg, last, cont, cand - scene_total, i, s, p, dist, cta, ctb);
          p = -1 - p;
          const double2 mc = pair_mc(c, s, p);
          margin = mc.x;
          coeff = mc.y;
          const double threshold = margin + buffer;
          if (use_bits)
            hit = (HB[cand >> 5] >> (cand & 31)) & 1u;
          else
          {
            hit = dist < threshold && !(dist > margin + buffer);
            if (hit && (f0 || f1))
              hit = (f0 && (cta != 1 || ctb != 1)) || (f1 && (cta != 2 || ctb != 2));
          }
#if THIP_GENERIC_ONLY
          if (ctest != THIP_CONTACT_ALL)
          {
            pre = dist < threshold;
            fixed_ok = !(f0 || f1) || (f0 && (cta != 1 || ctb != 1)) || (f1 && (cta != 2 || ctb != 2));
            if (ctest == THIP_CONTACT_CLOSEST && pre)
            {
              // the key of this self candidate and its pair j (self_candidate's decode)
              const int q = cand - scene_total;
              int r = q, k = 0;
              for (; k + 1 < c.T.n_self_keys; ++k)
              {
                const int sz = nseg * (c.T.self_kp[k + 1] - c.T.self_kp[k]);
                if (r < sz)
                  break;
                r -= sz;
              }
              const int npk = c.T.self_kp[k + 1] - c.T.self_kp[k];
              const int j = r - (r / npk) * npk;
              for (int j2 = 0; j2 < npk; ++j2)
              {
                if (j2 == j)
                  continue;
                int i2, sa2, sb2, ca2, cb2;
                double d2;
                self_candidate(c, S, SCR, ns, nseg, last, cont, q - j + j2, i2, sa2, sb2, d2, ca2, cb2);
                const double th2 = pair_mc(c, sa2, -1 - sb2).x + buffer;
                if (d2 < th2 && (d2 < dist || (d2 == dist && j2 < j)))
                  pre = false;  // a closer (or an earlier as close) contact of the key
              }
            }
            hit = pre && fixed_ok;
          }
#endif
        }
      }
      else if (use_bits)
      {
        // the count pass's hits: 64 candidates = two words (each unit's bits
        // start on a 64-bit boundary)
        const unsigned w = HB[(c0 >> 5) + (c.lane >> 5)];
        hit = (cand < total) && ((w >> (c.lane & 31)) & 1u);
        if (hit)
        {
          int rem = cand, g = 0;
          for (int gg = 0; gg + 1 < ngr; ++gg)
          {
            const int sz = P * nseg * S.grp_ns[gg];
            const bool adv = (g == gg) && (rem >= sz);
            rem = adv ? rem - sz : rem;
            g = adv ? g + 1 : g;
          }
          const int gn = S.grp_ns[g];
          p = rem / (nseg * gn);
          const int r2 = rem % (nseg * gn);
          i = r2 / gn;
          s = S.sph_order[S.grp_s0[g] + r2 % gn];
        }
      }
      else if (cand < total)
      {
        // flattened (group, primitive, sub-state, sphere) index; the group
        // walk is uniform, the selects per lane
        int rem = cand, g = 0;
        for (int gg = 0; gg + 1 < ngr; ++gg)
        {
          const int sz = P * nseg * S.grp_ns[gg];
          const bool adv = (g == gg) && (rem >= sz);
          rem = adv ? rem - sz : rem;
          g = adv ? g + 1 : g;
        }
        const int gn = S.grp_ns[g];
        p = rem / (nseg * gn);
        const int r2 = rem % (nseg * gn);
        i = r2 / gn;
        s = S.sph_order[S.grp_s0[g] + r2 % gn];
        double prim[16];
        for (int e = 0; e < 16; ++e)
          prim[e] = S.scene[16 * p + e];
        const double2 mc = pair_mc(c, s, p);
        margin = mc.x;
        coeff = mc.y;
        const double threshold = margin + buffer;
        const double* cp = SCR + (i * ns + s) * 3;
        const double ctr[3] = { cp[0], cp[1], cp[2] };
        double n[3], pr[3];
        int cct;
        if (cont)
        {
          const double* cq = SCR + ((i + 1) * ns + s) * 3;
          const double ctr1[3] = { cq[0], cq[1], cq[2] };
          dist = threshold;  // not a contact unless the cast says so
          cct = 3;
          if (swept_lower_bound(ctr, ctr1, S.rad[s], prim) < threshold)
          {
            double ts;
            swept_sphere_prim_distance(ctr, ctr1, S.rad[s], prim, dist, n, pr, ts);
            cct = (i == 0 && ts == 0.0) ? 1 : ((i + 1 == last && ts == 1.0) ? 2 : 3);
          }
        }
        else
        {
          sphere_prim_distance(ctr, S.rad[s], prim, dist, n, pr);
          cct = (i == 0) ? 1 : ((i == last) ? 2 : 3);
        }
        hit = dist < threshold && !(dist > margin + buffer);
        // removeInvalidContactResults (collision_utils.cpp:73-114): at a
        // fixed end keep only contacts not at that end (cc_type of the
        // robot link: Time0 / Time1 / Between)
        if (hit && (f0 || f1))
          hit = (f0 && cct != 1) || (f1 && cct != 2);
#if THIP_GENERIC_ONLY
        if (ctest != THIP_CONTACT_ALL)
        {
          pre = dist < threshold;
          fixed_ok = !(f0 || f1) || (f0 && cct != 1) || (f1 && cct != 2);
          if (ctest == THIP_CONTACT_CLOSEST && pre)
          {
            // the other spheres of this key (link group g, primitive p) at sub-state i
            const int e = r2 % gn;
            for (int e2 = 0; e2 < gn; ++e2)
            {
              if (e2 == e)
                continue;
              const int s2 = S.sph_order[S.grp_s0[g] + e2];
              const double th2 = pair_mc(c, s2, p).x + buffer;
              const double* cp2 = SCR + (i * ns + s2) * 3;
              const double ctr2[3] = { cp2[0], cp2[1], cp2[2] };
              double d2, n2[3], pr2[3];
              if (cont)
              {
                const double* cq2 = SCR + ((i + 1) * ns + s2) * 3;
                const double ctr21[3] = { cq2[0], cq2[1], cq2[2] };
                d2 = th2;
                if (swept_lower_bound(ctr2, ctr21, S.rad[s2], prim) < th2)
                {
                  double ts2;
                  swept_sphere_prim_distance(ctr2, ctr21, S.rad[s2], prim, d2, n2, pr2, ts2);
                }
              }
              else
                sphere_prim_distance(ctr2, S.rad[s2], prim, d2, n2, pr2);
              if (d2 < th2 && (d2 < dist || (d2 == dist && e2 < e)))
                pre = false;  // a closer (or an earlier as close) contact of the key
            }
          }
          hit = pre && fixed_ok;
        }
#endif
      }
#if THIP_GENERIC_ONLY
      if (ctest == THIP_CONTACT_FIRST)
      {
        // the call's first contact: no earlier lane of this chunk and no earlier
        // chunk of the unit had a contact at sub-state i
        const int iv = pre ? i : -1;
        bool earlier = false;
        for (int l = 0; l < 64; ++l)
        {
          const int il = __shfl(iv, l);
          earlier = earlier || (l < c.lane && iv >= 0 && il == iv);
        }
        const bool was = pre && ((done[i >> 5] >> (i & 31)) & 1u);
        hit = pre && !earlier && !was && fixed_ok;
        __builtin_amdgcn_wave_barrier();
        if (pre)
          atomicOr(done + (i >> 5), 1u << (i & 31));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
#endif
      const unsigned long long mask = __ballot(hit);
      if (PASS == 0)
        lcost += hit ? fmax(margin - dist, 0.0) * coeff : 0.0;
      else if (hit)
      {
        const int rank = __popcll(mask & ((1ull << c.lane) - 1ull));
        const int k = base + running + rank;
        if (k < L.h_cap)
        {
          CONT[3 * k + 0] = single ? t - pair : i;  // DISCRETE: the half of the pair
          CONT[3 * k + 1] = s;
          CONT[3 * k + 2] = p;
          HT[k] = pair;
          c.ia(I_HKIND)[k] = 0;
        }
      }
      running += __popcll(mask);
    }
    const double cost = (PASS == 0) ? wave_sum(lcost) : 0.0;
    if (PASS == 0 && c.lane == 0)
    {
      PCNT[t] = running;
      HCOST[t] = cost;
      atomicAdd(reinterpret_cast<unsigned long long*>(&c.s->n_substates), static_cast<unsigned long long>(cnt));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
}

// Static hinge rows (JointPos / JointVel tolerance forms) into the hinge list:
// row s of the (pair-sorted) static table goes after its pair's contacts.
// The affine expressions are built as the reference's ctors build them
// (trajectory_costs.cpp:66-135, 183-254, 303-374) and stored as is (kind 1):
// row aff(x) - h <= 0.  Constant across SQP iterations.
__device__ void static_hinge_rows(Ctx& c, const int* HP)
{
  const Layout& L = c.L;
  const int D = L.D;
  int *HT = c.ia(I_HT), *HM = c.ia(I_HMASK), *HKD = c.ia(I_HKIND), *HSL = c.ia(I_HSLOT);
  double *HC0 = c.a(A_HC0), *HK = c.a(A_HK);
  FOR(sr, c.T.n_sh)
  {
    const int p = c.T.sh_pair[sr];
    // the pair's static rows close its range [HP[p], HP[p + 1])
    const int h = HP[p + 1] - c.T.sh_ptr[p + 1] + sr;
    const int kind = c.T.sh_kind[sr], k = c.T.sh_owner[sr], j = c.T.sh_joint[sr], t = c.T.sh_step[sr];
    double* a = HC0 + h * 2 * D;
    for (int e = 0; e < 2 * D; ++e)
      a[e] = 0.0;
    double cst;
    int mask;
    if (kind == SH_JP_UP || kind == SH_JP_LO)
    {
      const double cf = c.d->jpos_coeffs[k][j], tg = c.jpt[k * D + j];
      const int e = (t - p) * D + j;
      mask = 1 << e;
      if (kind == SH_JP_UP)
      {
        // expr = pos - upper_tol, scaled: pos = x - targ
        a[e] = 1.0 * cf;
        cst = ((0.0 - tg) - c.d->jpos_upper_tols[k][j]) * cf;
      }
      else
      {
        // expr = lower_tol - pos, scaled
        a[e] = -1.0 * cf;
        cst = (c.d->jpos_lower_tols[k][j] - (0.0 - tg)) * cf;
      }
    }
    else
    {
      // vel = -x_t + x_t+1 - targ; owner n_jpos: the jv_* term, n_jpos + 1 + x: jvx term x
      const int xo = k - L.n_jpos - 1;
      const double cf = (xo >= 0) ? c.d->jvx_coeffs[xo][j] : c.d->jv_coeffs[j];
      const double tg = (xo >= 0) ? c.d->jvx_targets[xo][j] : c.d->jv_targets[j];
      const double up = (xo >= 0) ? c.d->jvx_upper_tols[xo][j] : c.d->jv_upper_tols[j];
      const double lo = (xo >= 0) ? c.d->jvx_lower_tols[xo][j] : c.d->jv_lower_tols[j];
      mask = (1 << j) | (1 << (D + j));
      if (kind == SH_JV_UP)
      {
        // expr = (upper_tol - vel) * -coeff
        a[j] = 1.0 * -cf;
        a[D + j] = -1.0 * -cf;
        cst = (up - (0.0 - tg)) * -cf;
      }
      else
      {
        // expr = (lower_tol - vel) * coeff
        a[j] = 1.0 * cf;
        a[D + j] = -1.0 * cf;
        cst = (lo - (0.0 - tg)) * cf;
      }
    }
    HK[h] = cst;
    HM[h] = mask;
    HT[h] = p;
    HKD[h] = 1;
    HSL[h] = c.T.sh_slot[sr];
  }
}

// Exact values of the static hinge terms at x: JointVelIneqCost::value
// (trajectory_costs.cpp:348-361), JointPosIneqCost::value (:97-110) and
// JointPosIneqConstraint::value + INEQ violation (:216-233, modeling.cpp:151-170).
__device__ void sh_values(Ctx& c, const double* x, double* costs, double* viols)
{
  const Layout& L = c.L;
  const int D = L.D;
  if (L.jv_ineq)
  {
    const int nv = (L.jv_last - L.jv_first) * D;
    double s1 = 0, s2 = 0;
    FOR(i, nv)
    {
      const int t = L.jv_first + i / D, j = i % D;
      const double cf = c.d->jv_coeffs[j];
      const double d0 = (x[(t + 1) * D + j] - x[t * D + j]) - c.d->jv_targets[j];
      s1 += fmax((d0 - c.d->jv_upper_tols[j]) * cf, 0.0);
      s2 += fmax(((d0 * -1) + c.d->jv_lower_tols[j]) * cf, 0.0);
    }
    s1 = block_sum(c, s1);
    s2 = block_sum(c, s2);
    if (c.tid == 0)
      costs[0] = s1 + s2;
  }
  // further JointVel tolerance terms: JointVelIneqCost::value / JointVelIneqConstraint::value
  // (trajectory_costs.cpp:348-361, 472-487; violation = sum of the nonnegative values)
  for (int xo = 0; xo < L.n_jvx; ++xo)
  {
    const int f = c.T.jvx_first[xo], nv = (c.T.jvx_last[xo] - f) * D;
    double s1 = 0, s2 = 0;
    FOR(i, nv)
    {
      const int t = f + i / D, j = i % D;
      const double cf = c.d->jvx_coeffs[xo][j];
      const double d0 = (x[(t + 1) * D + j] - x[t * D + j]) - c.d->jvx_targets[xo][j];
      s1 += fmax((d0 - c.d->jvx_upper_tols[xo][j]) * cf, 0.0);
      s2 += fmax(((d0 * -1) + c.d->jvx_lower_tols[xo][j]) * cf, 0.0);
    }
    s1 = block_sum(c, s1);
    s2 = block_sum(c, s2);
    if (c.tid == 0)
      (c.d->jvx_is_cnt[xo] ? viols : costs)[c.T.jvx_slot[xo]] = s1 + s2;
  }
  for (int k = 0; k < L.n_jpos; ++k)
  {
    if (!c.T.jpos_ineq[k])
      continue;
    const int f = c.T.jpos_first[k], n = (c.T.jpos_last[k] - f + 1) * D;
    double s1 = 0, s2 = 0;
    FOR(i, n)
    {
      const int t = f + i / D, j = i % D;
      const double cf = c.d->jpos_coeffs[k][j];
      const double d0 = x[t * D + j] - c.jpt[k * D + j];
      s1 += fmax((d0 - c.d->jpos_upper_tols[k][j]) * cf, 0.0);
      s2 += fmax(((d0 * -1) + c.d->jpos_lower_tols[k][j]) * cf, 0.0);
    }
    s1 = block_sum(c, s1);
    s2 = block_sum(c, s2);
    if (c.tid == 0)
      (c.d->jpos_is_cnt[k] ? viols : costs)[c.T.jpos_slot[k]] = s1 + s2;
  }
}

// Model values of the static hinge terms at the QP solution SX: costs are
// sum 1 * h (ConvexObjective::value of addHinge(expr, 1)), constraints sum
// pospart(aff(x)) (ConvexConstraints::violation).
__device__ void sh_model_values(Ctx& c, const double* SX, double* mcost, double* mviol)
{
  const Layout& L = c.L;
  const int D = L.D;
  if (c.T.n_sh == 0)
    return;
  const int* HP = c.ia(I_HPTR);
  const int* HMv = c.ia(I_HMASK);
  const double *HC0 = c.a(A_HC0), *HKv = c.a(A_HK);
  for (int o = 0; o <= L.n_jpos + L.n_jvx; ++o)
  {
    // owners: JointPos terms, the jv_* term (n_jpos), the jvx terms (n_jpos + 1 + x)
    const bool jv = (o == L.n_jpos), jx = (o > L.n_jpos);
    const int xo = o - L.n_jpos - 1;
    if (jx ? false : (jv ? !L.jv_ineq : !c.T.jpos_ineq[o]))
      continue;
    const bool cnt = jx ? (c.d->jvx_is_cnt[xo] != 0) : (!jv && c.d->jpos_is_cnt[o]);
    double v = 0;
    FOR(sr, c.T.n_sh)
    {
      if (c.T.sh_owner[sr] != o)
        continue;
      const int p = c.T.sh_pair[sr];
      // (from HP alone: after a rejected step PCNT holds the counts at the
      // candidate point, not at the point these rows were built from)
      const int h = HP[p + 1] - c.T.sh_ptr[p + 1] + sr;
      if (!cnt)
        v += SX[L.nc_base + h];
      else
      {
        double a = HKv[h];
        for (int e = 0; e < 2 * D; ++e)
          if (HMv[h] & (1 << e))
            a += HC0[h * 2 * D + e] * SX[(p + e / D) * D + e % D];
        v += fmax(a, 0.0);
      }
    }
    v = block_sum(c, v);
    if (c.tid == 0)
      (cnt ? mviol : mcost)[jx ? c.T.jvx_slot[xo] : (jv ? 0 : c.T.jpos_slot[o])] = v;
  }
}

// Collision costs at x (Cost::value of each step-pair term); with rows, also
// the linearised hinge rows of the QP (CollisionCost::convex) at x.
__device__ void coll_scan(Ctx& c, const double* x, double* costs, bool rows)
{
  const Layout& L = c.L;
  const int D = L.D;
  int* PCNT = c.ia(I_PCNT);
  if (c.tid == 0)
    c.s->coll_overflow = 0;
  BSYNC();
  if (L.coll)
    coll_stage(c);
  // linearize at an accepted point reuses the counts of evaluate() at that
  // same point (the reference's x-keyed contact cache, collision_terms.cpp:435-461)
  const bool counts_current = rows && c.s->scan_at_x;
  if (L.coll && !counts_current)
  {
    {
      PROF(19);
      coll_scan_pairs<0>(c, x, nullptr);
      BSYNC();
    }
    if (costs)
      FOR(k, L.coll_last - L.coll_first)
      {
        const int slot = c.T.coll_slot[L.coll_first + k];
        if (slot >= 0)
          costs[L.coll_cost0 + slot] = c.a(A_HCOST)[L.coll_first + k];
      }
    if (c.tid == 0 && c.s->coll_overflow)
      c.s->flags |= THIP_FLAG_CONTACT_OVERFLOW;
  }
  if (!rows)
  {
    BSYNC();
    return;
  }
  int* HP = c.ia(I_HPTR);
  if (c.tid == 0)
  {
    // per pair: its contacts, then its static hinge rows
    int acc = 0;
    for (int t = 0; t <= L.N; ++t)
    {
      HP[t] = acc;
      if (t < L.N)
        acc += coll_pair_count(L, PCNT, t);
      if (t < L.N)
        acc += c.T.sh_ptr[t + 1] - c.T.sh_ptr[t];
    }
    if (acc > L.h_cap)
    {
      c.s->coll_overflow = 1;
      acc = 0;
      for (int t = 0; t <= L.N; ++t)
        HP[t] = 0;
    }
    c.s->n_h = acc;
    c.s->n_contact_rows += acc;
  }
  BSYNC();
  if (c.s->coll_overflow)
  {
    if (c.tid == 0)
    {
      c.s->n_h = 0;
      c.s->flags |= THIP_FLAG_CONTACT_OVERFLOW;
    }
    BSYNC();
    return;
  }
  static_hinge_rows(c, HP);
  {
    PROF(20);
    if (L.coll)
      coll_scan_pairs<1>(c, x, HP);
    BSYNC();
  }
  if (!L.coll)
    return;
  PROF(21);
  // rows: distance expression k + a_t.x_t + a_t+1.x_t+1 per contact
  const thip_chain& ch = g_chain;
  const int* CONT = c.ia(I_CONT);
  const int* HT = c.ia(I_HT);
  const int* HKD = c.ia(I_HKIND);
  double *HC0 = c.a(A_HC0), *HK = c.a(A_HK);
  int* HM = c.ia(I_HMASK);
  // scene contacts (robot sphere vs primitive)
  FOR(k, c.s->n_h)
  {
    if (HKD[k] != 0)
      continue;
    const int t = HT[k], i = CONT[3 * k + 0], s = CONT[3 * k + 1], p = CONT[3 * k + 2];
    if (p < 0)
      continue;  // a self contact: below
    const double* q0 = x + t * D;
    const double* q1 = x + (t + 1) * D;
    const bool single = L.coll_single != 0;  // i = the half (waypoint t + i)
    const int cnt = single ? 1 : lvs_count(q0, q1, D, c.d->coll_lvs);
    const int link = c.d->sphere_link[s];
    const bool cont = c.d->coll_continuous == 1;
    double q[THIP_MAX_DOF];
    for (int j = 0; j < D; ++j)
      q[j] = single ? (i ? q1[j] : q0[j]) : linspaced(cnt, q0[j], q1[j], i);
    Pose T, T1;  // link pose at sub-state i (transform) and, for a cast, at i + 1 (cc_transform)
    chain_fk(ch, q, link, T);
    const double* cs = c.d->sphere_center[s];
    double ctr[3];
    for (int r = 0; r < 3; ++r)
      ctr[r] = T.r[r * 3 + 0] * cs[0] + T.r[r * 3 + 1] * cs[1] + T.r[r * 3 + 2] * cs[2] + T.t[r];
    double dist, n[3], pr[3], ts = 0.0;
    if (cont)
    {
      double qn[THIP_MAX_DOF];
      for (int j = 0; j < D; ++j)
        qn[j] = linspaced(cnt, q0[j], q1[j], i + 1);
      chain_fk(ch, qn, link, T1);
      double ctr1[3];
      for (int r = 0; r < 3; ++r)
        ctr1[r] = T1.r[r * 3 + 0] * cs[0] + T1.r[r * 3 + 1] * cs[1] + T1.r[r * 3 + 2] * cs[2] + T1.t[r];
      swept_sphere_prim_distance(ctr, ctr1, c.d->sphere_radius[s], c.scene + 16 * p, dist, n, pr, ts);
    }
    else
    {
      sphere_prim_distance(ctr, c.d->sphere_radius[s], c.scene + 16 * p, dist, n, pr);
      T1 = T;
    }
    // nearest_points_local[0] in the frame of the sub-state (cast start) pose and the
    // reference-point offsets link_transform.linear() * nearest_points_local with
    // link_transform = transform (x_t part) / cc_transform (x_t+1 part), collision_terms.cpp:217-223
    const double w[3] = { pr[0] - T.t[0], pr[1] - T.t[1], pr[2] - T.t[2] };
    double pl[3], rv0[3], rv1[3];
    for (int r = 0; r < 3; ++r)
      pl[r] = T.r[0 * 3 + r] * w[0] + T.r[1 * 3 + r] * w[1] + T.r[2 * 3 + r] * w[2];
    for (int r = 0; r < 3; ++r)
    {
      rv0[r] = T.r[r * 3 + 0] * pl[0] + T.r[r * 3 + 1] * pl[1] + T.r[r * 3 + 2] * pl[2];
      rv1[r] = T1.r[r * 3 + 0] * pl[0] + T1.r[r * 3 + 1] * pl[1] + T1.r[r * 3 + 2] * pl[2];
    }
    // DISCRETE: CCType_None, GetGradient's scale 1 (collision_terms.cpp:214-221): the
    // waypoint's half with scale 1 - 0 (half 0) or 1 (half 1), the other half absent
    const double cc_time =
        single ? double(i) : (cont ? (double(i) + ts) : double(i)) * (1.0 / double(cnt - 1));
    const bool f0 = single ? (i == 1) : coll_fixed_step(c, t), f1 = single ? (i == 0) : coll_fixed_step(c, t + 1);
    double cst = dist;
    int mask = 0;
    double* a = HC0 + k * 2 * D;
    for (int e = 0; e < 2; ++e)
    {
      const bool skip = (e == 0) ? f0 : f1;
      const double* qe = (e == 0) ? q0 : q1;
      if (skip)
      {
        for (int j = 0; j < D; ++j)
          a[e * D + j] = 0.0;
        continue;
      }
      const double scale = (e == 1) ? cc_time : (1 - cc_time);
      const double* rv = (e == 1) ? rv1 : rv0;
      double J[6 * THIP_MAX_DOF];
      chain_jacobian(ch, qe, link, J);
      double gd = 0;
      for (int j = 0; j < D; ++j)
      {
        const double wx = J[3 * D + j], wy = J[4 * D + j], wz = J[5 * D + j];
        const double l0 = J[0 * D + j] + (wy * rv[2] - wz * rv[1]);
        const double l1 = J[1 * D + j] + (wz * rv[0] - wx * rv[2]);
        const double l2 = J[2 * D + j] + (wx * rv[1] - wy * rv[0]);
        const double g = -1.0 * (n[0] * l0 + n[1] * l1 + n[2] * l2);
        const double av = scale * g;
        gd += g * qe[j];
        // cleanupAff (expr_ops.cpp:88-99)
        const bool keep = fabs(av) > 1e-7;
        a[e * D + j] = keep ? av : 0.0;
        mask |= keep ? (1 << (e * D + j)) : 0;
      }
      cst += scale * -gd;
    }
    HK[k] = cst;
    HM[k] = mask;
    c.a(A_HDIST)[k] = dist;
    c.a(A_HCCT)[k] = single ? 0.0 : cc_time;
  }
  // self contacts (robot sphere s vs robot sphere -1 - p, both links moving; GetGradient's two
  // sides).  Kept apart from the scene loop so that loop's code -- and with it the
  // rounding of its contraction choices -- stays as it was.
  FOR(k, c.s->n_h)
  {
    if (HKD[k] != 0)
      continue;
    const int t = HT[k], i = CONT[3 * k + 0], s = CONT[3 * k + 1], p = CONT[3 * k + 2];
    if (p >= 0)
      continue;
    const double* q0 = x + t * D;
    const double* q1 = x + (t + 1) * D;
    const bool single = L.coll_single != 0;  // i = the half (waypoint t + i)
    const int cnt = single ? 1 : lvs_count(q0, q1, D, c.d->coll_lvs);
    const bool cont = c.d->coll_continuous == 1;
    const bool self = p < 0;  // a self contact: the second body is robot sphere -1 - p
    const int nsides = self ? 2 : 1;
    const int sb = self ? -1 - p : 0;
    double q[THIP_MAX_DOF], qn[THIP_MAX_DOF];
    for (int j = 0; j < D; ++j)
    {
      q[j] = single ? (i ? q1[j] : q0[j]) : linspaced(cnt, q0[j], q1[j], i);
      qn[j] = cont ? linspaced(cnt, q0[j], q1[j], i + 1) : q[j];
    }
    // side 0: the robot sphere s; side 1: the scene primitive p, or robot sphere sb.
    // Link poses at sub-state i (transform) and, for a cast, at i + 1 (cc_transform).
    int link[2];
    Pose T[2], T1[2];
    double c0[2][3], c1[2][3];
    for (int sd = 0; sd < nsides; ++sd)
    {
      const int sph = sd ? sb : s;
      link[sd] = c.d->sphere_link[sph];
      chain_fk(ch, q, link[sd], T[sd]);
      if (cont)
        chain_fk(ch, qn, link[sd], T1[sd]);
      else
        T1[sd] = T[sd];
      const double* cs = c.d->sphere_center[sph];
      for (int r = 0; r < 3; ++r)
      {
        c0[sd][r] = T[sd].r[r * 3 + 0] * cs[0] + T[sd].r[r * 3 + 1] * cs[1] + T[sd].r[r * 3 + 2] * cs[2] + T[sd].t[r];
        c1[sd][r] =
            T1[sd].r[r * 3 + 0] * cs[0] + T1[sd].r[r * 3 + 1] * cs[1] + T1[sd].r[r * 3 + 2] * cs[2] + T1[sd].t[r];
      }
    }
    double dist, n[3], pt[2][3], ts[2] = { 0.0, 0.0 };
    if (self)
      self_sphere_distance(c0[0], c1[0], c.d->sphere_radius[s], c0[1], c1[1], c.d->sphere_radius[sb], cont, dist, n,
                           pt[0], pt[1], ts[0], ts[1]);
    else if (cont)
      swept_sphere_prim_distance(c0[0], c1[0], c.d->sphere_radius[s], c.scene + 16 * p, dist, n, pt[0], ts[0]);
    else
      sphere_prim_distance(c0[0], c.d->sphere_radius[s], c.scene + 16 * p, dist, n, pt[0]);
    // per side: nearest_points_local in the frame of the sub-state (cast start) pose and
    // the reference-point offsets link_transform.linear() * nearest_points_local with
    // link_transform = transform (x_t part) / cc_transform (x_t+1 part), collision_terms.cpp:217-223;
    // cc_time: DISCRETE files the waypoint's expression on half i with scale 1 (CCType_None,
    // GetGradient's scale 1, collision_terms.cpp:214-221), the other half absent
    double rv0[2][3], rv1[2][3], cct[2];
    for (int sd = 0; sd < nsides; ++sd)
    {
      const double w[3] = { pt[sd][0] - T[sd].t[0], pt[sd][1] - T[sd].t[1], pt[sd][2] - T[sd].t[2] };
      double pl[3];
      for (int r = 0; r < 3; ++r)
        pl[r] = T[sd].r[0 * 3 + r] * w[0] + T[sd].r[1 * 3 + r] * w[1] + T[sd].r[2 * 3 + r] * w[2];
      for (int r = 0; r < 3; ++r)
      {
        rv0[sd][r] = T[sd].r[r * 3 + 0] * pl[0] + T[sd].r[r * 3 + 1] * pl[1] + T[sd].r[r * 3 + 2] * pl[2];
        rv1[sd][r] = T1[sd].r[r * 3 + 0] * pl[0] + T1[sd].r[r * 3 + 1] * pl[1] + T1[sd].r[r * 3 + 2] * pl[2];
      }
      cct[sd] = single ? double(i) : (cont ? (double(i) + ts[sd]) : double(i)) * (1.0 / double(cnt - 1));
    }
    const bool f0 = single ? (i == 1) : coll_fixed_step(c, t), f1 = single ? (i == 0) : coll_fixed_step(c, t + 1);
    double cst = dist;
    int mask = 0;
    double* a = HC0 + k * 2 * D;
    for (int e = 0; e < 2 * D; ++e)
      a[e] = 0.0;
    for (int e = 0; e < 2; ++e)
    {
      if ((e == 0) ? f0 : f1)
        continue;
      const double* qe = (e == 0) ? q0 : q1;
      // CollisionsToDistanceExpressions: per side varDot(scale g, vars) and scale * -g.q;
      // a variable's side terms summed as the QP builder sums duplicates
      for (int sd = 0; sd < nsides; ++sd)
      {
        const double scale = (e == 1) ? cct[sd] : (1 - cct[sd]);
        const double* rv = (e == 1) ? rv1[sd] : rv0[sd];
        const double sg = sd ? 1.0 : -1.0;  // GetGradient: (i == 0 ? -1 : 1) n^T J (collision_terms.cpp:232)
        double J[6 * THIP_MAX_DOF];
        chain_jacobian(ch, qe, link[sd], J);
        double gd = 0;
        for (int j = 0; j < D; ++j)
        {
          const double wx = J[3 * D + j], wy = J[4 * D + j], wz = J[5 * D + j];
          const double l0 = J[0 * D + j] + (wy * rv[2] - wz * rv[1]);
          const double l1 = J[1 * D + j] + (wz * rv[0] - wx * rv[2]);
          const double l2 = J[2 * D + j] + (wx * rv[1] - wy * rv[0]);
          const double g = sg * (n[0] * l0 + n[1] * l1 + n[2] * l2);
          const double av = scale * g;
          gd += g * qe[j];
          // cleanupAff (expr_ops.cpp:88-99)
          if (fabs(av) > 1e-7)
          {
            const int bit = 1 << (e * D + j);
            a[e * D + j] = (mask & bit) ? a[e * D + j] + av : av;
            mask |= bit;
          }
        }
        cst += scale * -gd;
      }
    }
    HK[k] = cst;
    HM[k] = mask;
    c.a(A_HDIST)[k] = dist;
    c.a(A_HCCT)[k] = single ? 0.0 : cct[0];
  }
  BSYNC();
}

// ======================================================================
// JointPos terms at x: JointPosEqCost::value = sum c_j (x_tj - targ_j)^2
// (trajectory_costs.cpp:54-63); JointPosEqConstraint::value returns
// c_j (x_tj - targ_j)^2 per (t, j) (squared, :162-171) and the violation is
// sum |value| (modeling.cpp:151-170).  Costs and violations by slot.
// ======================================================================
__device__ void jpos_values(Ctx& c, const double* x, double* costs, double* viols)
{
  const Layout& L = c.L;
  const int D = L.D;
  for (int k = 0; k < L.n_jpos; ++k)
  {
    if (c.T.jpos_ineq[k])
      continue;  // sh_values
    const int f = c.T.jpos_first[k], n = (c.T.jpos_last[k] - f + 1) * D;
    const bool cnt = c.d->jpos_is_cnt[k] != 0;
    double v = 0;
    FOR(i, n)
    {
      const int t = f + i / D, j = i % D;
      const double dd = x[t * D + j] - c.jpt[k * D + j];
      const double e = (dd * dd) * c.d->jpos_coeffs[k][j];
      v += cnt ? fabs(e) : e;
    }
    v = block_sum(c, v);
    if (c.tid == 0)
      (cnt ? viols : costs)[c.T.jpos_slot[k]] = v;
  }
}

// JointAccEqCost::value (trajectory_costs.cpp:533-542) of jdt term k at x:
// sum over (i, j) of c_j (diffAxis0(diffAxis0(traj))_{i,j} - targ_j)^2, the
// repeated difference (x_i+2 - x_i+1) - (x_i+1 - x_i) as diffAxis0 forms it.
// Also its model value (the quadratic is exact).  All threads; block sum.
__device__ double jacc_value(Ctx& c, const double* x, int k)
{
  const int D = c.L.D, f = c.d->jdt_first_step[k], n = (c.d->jdt_last_step[k] - 2 - f + 1) * D;
  double v = 0;
  FOR(e, n)
  {
    const int i = f + e / D, j = e % D;
    const double x0 = x[i * D + j], x1 = x[(i + 1) * D + j], x2 = x[(i + 2) * D + j];
    const double dd = ((x2 - x1) - (x1 - x0)) - c.d->jdt_targets[k][j];
    v += (dd * dd) * c.d->jdt_coeffs[k][j];
  }
  return block_sum(c, v);
}

// ======================================================================
// Exact cost values / constraint violations at x (Cost::value,
// Constraint::violation).  costs[n_costs], viols[n_cnts]
// ======================================================================
__device__ void evaluate(Ctx& c, const double* x, double* costs, double* viols)
{
  PROF(6);
  const Layout& L = c.L;
  const int D = L.D;
  const thip_chain& ch = g_chain;
  // JointVel: sum_{t,j} c_j (x_{t+1,j} - x_{t,j} - targ_j)^2
  double jv = 0;
  if (c.d->jv_enabled && !L.jv_ineq)
  {
    const int nv = (L.jv_last - L.jv_first) * D;
    FOR(i, nv)
    {
      const int t = L.jv_first + i / D, j = i % D;
      const double dd = (x[(t + 1) * D + j] - x[t * D + j]) - c.d->jv_targets[j];
      jv += (dd * dd) * c.d->jv_coeffs[j];
    }
  }
  jv = block_sum(c, jv);
  if (c.tid == 0 && c.d->jv_enabled && !L.jv_ineq)
    costs[0] = jv;
  for (int k = 0; k < L.n_jacc; ++k)
  {
    const double v = jacc_value(c, x, k);
    if (c.tid == 0)
      costs[L.jacc_slot[k]] = v;
  }
  const double* tgt = c.a(A_TGT);
  FOR(k, L.n_cart)
  {
    const int t = c.d->cart_step[k];
    Pose S, So, Ss, Tb, To, Tt, Ti;
    chain_fk(ch, x + t * D, c.d->cart_source_link[k], S);
    pose_load(So, c.d->cart_source_offset[k]);
    pose_mul(S, So, Ss);
    pose_load(To, tgt + 12 * k);
    if (c.d->cart_target_link[k] > 0)
      chain_fk(ch, x + t * D, c.d->cart_target_link[k], Tb);  // DynamicCartPose
    else
      pose_load(Tb, ch.base_pose);
    pose_mul(Tb, To, Tt);
    pose_inv(Tt, Ti);
    double err[6];
    transform_error(Ti, Ss, err);
    if (c.d->cart_has_tol[k])
      apply_tolerances(err, c.d->cart_lower_tol[k], c.d->cart_upper_tol[k]);
    const int r0 = c.T.term_row0[k], nr = c.T.term_nrow[k];
    double v = 0;
    if (c.d->cart_is_cnt[k])
    {
      for (int rr = 0; rr < nr; ++rr)
        v += fabs(err[c.T.row_comp[r0 + rr]] * c.T.row_w[r0 + rr]);
      viols[c.T.term_slot[k]] = v;
    }
    else
    {
      for (int rr = 0; rr < nr; ++rr)
        v += fabs(err[c.T.row_comp[r0 + rr]]) * c.T.row_w[r0 + rr];
      costs[c.T.term_slot[k]] = v;
    }
  }
  BSYNC();
  jpos_values(c, x, costs, viols);
  sh_values(c, x, costs, viols);
  if (L.coll)
    coll_scan(c, x, L.coll_cnt ? viols : costs, false);
}

// ======================================================================
// QP assembly + Ruiz scaling (osqp scale_data) on the structured QP.
// Rows: [fixed rows | abs rows | bound rows(n_cols)].
// ======================================================================
__device__ __forceinline__ int bound_row(const Layout& L, int col)
{
  return col < L.nc_base ? L.n_rows + col : L.m_base + 2 * (col - L.nc_base) + 1;
}
// row kinds: fixed-timestep, CartPose (abs), bound of a column, hinge
enum RowKind : int
{
  RK_FIXED = 0,
  RK_ABS,
  RK_BOUND,
  RK_HINGE
};
__device__ __forceinline__ int row_kind(const Layout& L, int r, int& idx)
{
  if (r < L.n_fixed_rows)
  {
    idx = r;
    return RK_FIXED;
  }
  if (r < L.n_rows)
  {
    idx = r - L.n_fixed_rows;
    return RK_ABS;
  }
  if (r < L.m_base)
  {
    idx = r - L.n_rows;
    return RK_BOUND;
  }
  const int h2 = r - L.m_base;
  if (h2 & 1)
  {
    idx = L.nc_base + (h2 >> 1);
    return RK_BOUND;
  }
  idx = h2 >> 1;
  return RK_HINGE;
}

__device__ void build_and_scale(Ctx& c)
{
  PROF(7);
  const Layout& L = c.L;
  const int D = L.D, nx = L.nx;
  const thip_osqp_settings& os = c.d->osqp;
  double *PD = c.a(A_PD), *PO = c.a(A_PO), *Q = c.a(A_Q), *DS = c.a(A_DS), *BS = c.a(A_BS);
  double *GS = c.a(A_GS), *WS = c.a(A_WS), *FS = c.a(A_FS), *E = c.a(A_E);
  const double *G = c.a(A_G), *MU = c.a(A_MU);
  // ---- unscaled data
  double* PO2 = (L.grp > 1) ? c.a(A_PO2) : nullptr;
  FOR(col, nx)
  {
    const int t = col / D, j = col % D;
    double pd = 0, po = 0, po2 = 0, q = 0;
    // JointAccEqCost (trajectory_costs.cpp:502-531): coeff * exprSquare(x_i - 2 x_i+1
    // + x_i+2 - targ) per (i, j), i = first .. last - 2: squares a_p^2 c on the
    // diagonal (P_tt = 2 sum), cross terms (2 a_p a_r) c on (t, t+1) and (t, t+2),
    // linear (2 (-targ) a_p) c (expr_ops.cpp exprSquare; zero coefficients skipped)
    double jsq = 0, jq = 0;
    for (int k = 0; k < L.n_jacc; ++k)
    {
      const double ck = c.d->jdt_coeffs[k][j], tk = c.d->jdt_targets[k][j];
      const int f = c.d->jdt_first_step[k], l = c.d->jdt_last_step[k] - 2;
      constexpr double st[3] = { 1.0, -2.0, 1.0 };
      for (int p = 0; p < 3; ++p)
        if (t - p >= f && t - p <= l)
        {
          jsq += (st[p] * st[p]) * ck;
          const double v = (2 * (-tk) * st[p]) * ck;
          if (v != 0.)
            jq += v;
        }
      if (t >= f && t <= l)
      {
        po += (2 * st[0] * st[1]) * ck;  // term i = t: positions 0, 1
        po2 += (2 * st[0] * st[2]) * ck;
      }
      if (t - 1 >= f && t - 1 <= l)
        po += (2 * st[1] * st[2]) * ck;  // term i = t - 1: positions 1, 2
    }
    if (c.d->jv_enabled && !L.jv_ineq)
    {
      const double cj = c.d->jv_coeffs[j], tg = c.d->jv_targets[j];
      const bool prev = (t - 1 >= L.jv_first) && (t - 1 <= L.jv_last - 1);
      const bool here = (t >= L.jv_first) && (t <= L.jv_last - 1);
      double dsum = 0;
      if (prev)
        dsum += cj;
      if (here)
        dsum += cj;
      dsum += jsq;
      pd = dsum + dsum;
      po = (here ? cj * -2.0 : 0.0) + po;
      // q: term t-1 contributes (2*(-tg)*1)*c, term t (2*(-tg)*(-1))*c; zero coefficients skipped
      double qa = 0;
      if (prev)
      {
        const double v = (2 * (-tg) * 1.0) * cj;
        if (v != 0.)
          qa += v;
      }
      if (here)
      {
        const double v = (2 * (-tg) * -1.0) * cj;
        if (v != 0.)
          qa += v;
      }
      q = qa + jq;
    }
    else
    {
      pd = jsq + jsq;
      q = jq;
    }
    // JointPosEqCost: exprSquare(x - targ) * c -> P diagonal 2c, q -2 targ c (trajectory_costs.cpp:40-51)
    for (int k = 0; k < L.n_jpos; ++k)
      if (!c.d->jpos_is_cnt[k] && !c.T.jpos_ineq[k] && t >= c.T.jpos_first[k] && t <= c.T.jpos_last[k])
      {
        const double cj = c.d->jpos_coeffs[k][j];
        pd += cj + cj;
        const double v = (2 * (-c.jpt[k * D + j]) * 1.0) * cj;
        if (v != 0.)
          q += v;
      }
    PD[col] = pd;
    PO[col] = po;
    if (PO2)
      PO2[col] = po2;
    Q[col] = q;
    DS[col] = 1.0;
    BS[col] = 1.0;
  }
  FOR(r, L.n_abs)
  {
    const int ca = nx + 2 * r;
    const int sl = c.T.row_slot[r];
    const double qv = sl >= 0 ? MU[sl] : 1.0;
    Q[ca] = qv;
    Q[ca + 1] = qv;
    DS[ca] = DS[ca + 1] = 1.0;
    BS[ca] = BS[ca + 1] = 1.0;
    WS[2 * r] = 1.0;
    WS[2 * r + 1] = -1.0;
    for (int j = 0; j < D; ++j)
      GS[r * D + j] = G[r * D + j];
  }
  FOR(f, L.n_fixed_rows) FS[f] = 1.0;
  // hinge rows (CollisionCost::convex -> addHinge): viol - h <= 0 with
  // viol = margin - (k + a.x): row coefficients -a (x_t, x_t+1) and -1 (h),
  // objective coeff * h (modeling.cpp:19-27)
  const int nh = c.s->n_h;
  {
    const double* HC0 = c.a(A_HC0);
    double *HC = c.a(A_HC), *HW = c.a(A_HW);
    // constraint form (CollisionConstraint::convex + cntsToCosts): row exprMult(margin - dist, coeff) - h <= 0,
    // objective mu_pair * h (collision_terms.cpp:1347-1364, optimizers.cpp:59-81)
    // static rows (kind 1) are stored as the affine expression itself: addHinge(aff, 1) for
    // costs, cntsToCosts' addHinge(aff, mu) for constraints
    const int *HTq = c.ia(I_HT), *HKDq = c.ia(I_HKIND), *HSLq = c.ia(I_HSLOT);
    FOR(e, nh * 2 * D)
    {
      const int h = e / (2 * D);
      HC[e] = HKDq[h] ? HC0[e] : (L.coll_cnt ? (-HC0[e]) * row_pair_mc(c, h).y : -HC0[e]);
    }
    FOR(h, nh)
    {
      HW[h] = -1.0;
      const int col = L.nc_base + h;
      if (HKDq[h])
        Q[col] = HSLq[h] >= 0 ? MU[HSLq[h]] : 1.0;
      else
        Q[col] = L.coll_cnt ? MU[L.coll_cost0 + c.T.coll_slot[HTq[h] + (L.coll_single ? c.ia(I_CONT)[3 * h] : 0)]]
                            : row_pair_mc(c, h).y;
      DS[col] = 1.0;
      BS[col] = 1.0;
    }
  }
  FOR(r, c.m()) E[r] = 1.0;
  if (c.tid == 0)
    c.s->c = 1.0;
  BSYNC();
  double* Dt = c.a(A_DG);
  double* Et = c.a(A_PRV);
  for (int it = 0; it < os.scaling; ++it)
  {
    // column norms of [P; A]
    FOR(col, c.nc())
    {
      double v;
      if (col < nx)
      {
        const int t = col / D, j = col % D;
        v = fabs(PD[col]);
        if (t < L.N - 1)
          v = fmax(v, fabs(PO[col]));
        if (t > 0)
          v = fmax(v, fabs(PO[col - D]));
        if (PO2)
        {
          if (t < L.N - 2)
            v = fmax(v, fabs(PO2[col]));
          if (t > 1)
            v = fmax(v, fabs(PO2[col - 2 * D]));
        }
        const int f = c.T.fixed_of_step[t];
        if (f >= 0)
          v = fmax(v, fabs(FS[f * D + j]));
        for (int p = c.T.step_ptr[t]; p < c.T.step_ptr[t + 1]; ++p)
          v = fmax(v, fabs(GS[c.T.step_rows[p] * D + j]));
        if (nh > 0)
        {
          const double* HC = c.a(A_HC);
          const int* HP = c.ia(I_HPTR);
          for (int h = HP[t]; h < HP[t + 1]; ++h)
            v = fmax(v, fabs(HC[h * 2 * D + j]));
          if (t > 0)
            for (int h = HP[t - 1]; h < HP[t]; ++h)
              v = fmax(v, fabs(HC[h * 2 * D + D + j]));
        }
        v = fmax(v, fabs(BS[col]));
      }
      else if (col < L.nc_base)
      {
        const int r = (col - nx) >> 1, sd = (col - nx) & 1;
        v = fmax(fabs(WS[2 * r + sd]), fabs(BS[col]));
      }
      else
        v = fmax(fabs(c.a(A_HW)[col - L.nc_base]), fabs(BS[col]));
      Dt[col] = 1.0 / sqrt(limit_scaling(v));
    }
    FOR(r, c.m())
    {
      double v;
      int idx;
      const int kind = row_kind(L, r, idx);
      if (kind == RK_FIXED)
        v = fabs(FS[r]);
      else if (kind == RK_ABS)
      {
        const int a = idx;
        v = 0;
        for (int j = 0; j < D; ++j)
          v = fmax(v, fabs(GS[a * D + j]));
        v = fmax(v, fabs(WS[2 * a]));
        v = fmax(v, fabs(WS[2 * a + 1]));
      }
      else if (kind == RK_BOUND)
        v = fabs(BS[idx]);
      else
      {
        const double* HC = c.a(A_HC);
        v = 0;
        for (int k = 0; k < 2 * D; ++k)
          v = fmax(v, fabs(HC[idx * 2 * D + k]));
        v = fmax(v, fabs(c.a(A_HW)[idx]));
      }
      Et[r] = 1.0 / sqrt(limit_scaling(v));
    }
    BSYNC();
    FOR(col, c.nc())
    {
      if (col < nx)
      {
        const int t = col / D;
        PD[col] = (PD[col] * Dt[col]) * Dt[col];
        if (t < L.N - 1)
          PO[col] = (PO[col] * Dt[col]) * Dt[col + D];
        if (PO2 && t < L.N - 2)
          PO2[col] = (PO2[col] * Dt[col]) * Dt[col + 2 * D];
      }
      BS[col] = (BS[col] * Et[bound_row(L, col)]) * Dt[col];
      Q[col] *= Dt[col];
      DS[col] *= Dt[col];
    }
    FOR(r, L.n_abs)
    {
      const int t = c.T.row_step[r];
      const int er = L.n_fixed_rows + r;
      for (int j = 0; j < D; ++j)
        GS[r * D + j] = (GS[r * D + j] * Et[er]) * Dt[t * D + j];
      WS[2 * r] = (WS[2 * r] * Et[er]) * Dt[nx + 2 * r];
      WS[2 * r + 1] = (WS[2 * r + 1] * Et[er]) * Dt[nx + 2 * r + 1];
    }
    FOR(f, L.n_fixed_rows)
    {
      const int slot = f / D, j = f % D;
      const int col = c.d->fixed_steps[slot] * D + j;
      FS[f] = (FS[f] * Et[f]) * Dt[col];
    }
    if (nh > 0)
    {
      double *HC = c.a(A_HC), *HW = c.a(A_HW);
      const int* HT = c.ia(I_HT);
      FOR(e, nh * 2 * D)
      {
        const int h = e / (2 * D), k = e % (2 * D);
        const int col = (HT[h] + (k >= D ? 1 : 0)) * D + (k % D);
        HC[e] = (HC[e] * Et[L.m_base + 2 * h]) * Dt[col];
      }
      FOR(h, nh) HW[h] = (HW[h] * Et[L.m_base + 2 * h]) * Dt[L.nc_base + h];
    }
    FOR(r, c.m()) E[r] *= Et[r];
    BSYNC();
    // cost normalisation
    double colsum = 0, qn = 0;
    FOR(col, c.nc())
    {
      if (col < nx)
      {
        const int t = col / D;
        double v = fabs(PD[col]);
        if (t < L.N - 1)
          v = fmax(v, fabs(PO[col]));
        if (t > 0)
          v = fmax(v, fabs(PO[col - D]));
        if (PO2)
        {
          if (t < L.N - 2)
            v = fmax(v, fabs(PO2[col]));
          if (t > 1)
            v = fmax(v, fabs(PO2[col - 2 * D]));
        }
        colsum += v;
      }
      qn = fmax(qn, fabs(Q[col]));
    }
    colsum = block_sum(c, colsum);
    double qq[1] = { qn };
    block_max<1>(c, qq);
    double ct = colsum / (double)c.nc();
    const double iq = limit_scaling(qq[0]);
    ct = fmax(ct, iq);
    ct = limit_scaling(ct);
    ct = 1.0 / ct;
    FOR(col, c.nc())
    {
      if (col < nx)
      {
        PD[col] *= ct;
        PO[col] *= ct;
        if (PO2)
          PO2[col] *= ct;
      }
      Q[col] *= ct;
    }
    if (c.tid == 0)
      c.s->c *= ct;
    BSYNC();
  }
  if (c.tid == 0)
    c.s->cinv = 1.0 / c.s->c;
  BSYNC();
}

// ======================================================================
// Linear system: K = P + sig I + A' diag(rK) A, aux variables eliminated,
// block tridiagonal Cholesky over waypoints.  rK per row in A_RHO (ADMM) or
// given by the polish active set.
// ======================================================================
struct Solver
{
  double* M;   // LDS [N][D][D] forward chain matrices
  double* Nb;  // LDS [N][D][D] backward chain matrices
};

// row rho for the factor: ADMM uses A_RHO, polish 1/delta on active rows
__device__ __forceinline__ double rho_k(const Ctx& c, int r, bool polish, double delta)
{
  if (!polish)
    return c.a(A_RHO)[r];
  return c.ia(I_ACT)[r] != 0 ? 1.0 / delta : 0.0;
}

__device__ __forceinline__ void wave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// In-place lower Cholesky of the D x D block S (one wave; lane i owns row i),
// then Li = L^-1 (lane j solves column j).  Flags `bad` if S is not positive
// definite.  S and Li are in LDS (factor()'s scratch and A_LINV, which the
// residency plan always places in LDS).  The column solve runs over DM >= D
// rows with compile-time indices, so its column stays in registers (indexed
// with a runtime bound it was a private array in scratch memory: a scratch
// round trip per term).
template <int DM>
__device__ __forceinline__ void chol_inv_block_t(double* Sp, double* Lip, int D, int lane, int& bad)
{
  lds_f64* S = lds(Sp);
  lds_f64* Li = lds(Lip);
  for (int j = 0; j < D; ++j)
  {
    if (lane == j)
    {
      double v = S[j * D + j];
      for (int k = 0; k < j; ++k)
        v -= S[j * D + k] * S[j * D + k];
      if (!(v > 0))
      {
        bad = 1;
        v = 1.0;
      }
      S[j * D + j] = sqrt(v);
    }
    wave_sync();
    if (lane > j && lane < D)
    {
      const int i = lane;
      double v = S[i * D + j];
      for (int k = 0; k < j; ++k)
        v -= S[i * D + k] * S[j * D + k];
      S[i * D + j] = v / S[j * D + j];
    }
    wave_sync();
  }
  if (lane < D)
  {
    const int j = lane;
    double xcol[DM];
#pragma unroll
    for (int i = 0; i < DM; ++i)
    {
      if (i < D)
      {
        double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < i; ++k)
          v -= S[i * D + k] * xcol[k];
        xcol[i] = (i < j) ? 0.0 : v / S[i * D + i];
      }
      else
        xcol[i] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < DM; ++i)
      if (i < D)
        Li[i * D + j] = xcol[i];
  }
  wave_sync();
}

__device__ __forceinline__ void chol_inv_block(double* S, double* Li, int D, int lane, int& bad)
{
  if (D > kOct)
    chol_inv_block_t<THIP_MAX_DOF>(S, Li, D, lane, bad);
  else
    chol_inv_block_t<kOct>(S, Li, D, lane, bad);
}

// v + sum_{h in [h0, h1)} W[h] * (HC[h][a] * HC[h][b]), in order, 8 rows per
// chunk with every load of the chunk issued first (masked rows add 0)
__device__ __forceinline__ double hinge_outer_sum(const double* HC, const double* W, int stride, int a, int b, int h0,
                                                  int h1, double v)
{
  for (int q = h0; q < h1; q += 8)
  {
    double w[8], p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
    {
      const int h = min(q + u, h1 - 1);
      w[u] = W[h];
      p[u] = (HC[h * stride + a] * HC[h * stride + b]) * ((q + u < h1) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v += w[u] * p[u];
  }
  return v;
}

// One half of the twisted block Cholesky (see factor()): wave 0 eliminates
// waypoints 0..m-1, wave 1 waypoints N-1..m+1.  The block scratch S, the
// coupling Ls and LI are LDS (typed: ds_read instead of FLAT); the inner
// products run over DM >= D terms with clamped loads and masked terms, in the
// order of the plain loops.
template <int DM>
__device__ __noinline__ void twisted_factor_half(Ctx& c, Solver& sv, const double* KB, double* LIp, const double* PO,
                                                 double* Sp, double* Lsp, int& bad)
{
  const Layout& L = c.L;
  // the solve layout's blocks (Layout::nbr): wave 2b runs branch b's top half,
  // wave 2b + 1 its bottom half
  // (N: the solve blocks of a branch, Layout::sNb)
  const int D = L.sD, N = L.sNb, DD = D * D, m = L.tw_mid, half = c.wave & 1, base = (c.wave >> 1) * N;
  const int len = (half == 0) ? m : (N - 1 - m);
  const bool use_cpl = L.hinge || L.nbr > 1 || L.grp > 1;
  lds_f64* S = lds(Sp);
  lds_f64* Ls = lds(Lsp);
  for (int k = 0; k < len; ++k)
  {
    const int t = base + ((half == 0) ? k : (N - 1 - k));
    const int cpl = (half == 0) ? t : t - 1;  // coupling block to the next block of the half
    // the half's first block has no coupling (and Ls holds stale or
    // uninitialised LDS then: never read, not even under a zero mask)
    for (int e = c.lane; e < DD; e += 64)
    {
      const int i = e / D, j = e % D;
      double v = KB[t * DD + e];
      if (k > 0)
      {
        double a[DM], b[DM];
#pragma unroll
        for (int q = 0; q < DM; ++q)
        {
          const int qc = min(q, D - 1);
          a[q] = Ls[i * D + qc];
          b[q] = Ls[j * D + qc] * ((q < D) ? 1.0 : 0.0);
        }
#pragma unroll
        for (int q = 0; q < DM; ++q)
          v -= a[q] * b[q];
      }
      S[e] = v;
    }
    wave_sync();
    chol_inv_block(Sp, LIp + t * DD, D, c.lane, bad);
    const lds_f64* Li = lds(LIp) + t * DD;
    for (int e = c.lane; e < DD; e += 64)
    {
      const int i = e / D, j = e % D;
      double v = 0;  // zero for the half's first block (the segment's chain reads it)
      if (k > 0)
      {
        double a[DM], b[DM];
#pragma unroll
        for (int q = 0; q < DM; ++q)
        {
          const int qc = min(q, D - 1);
          a[q] = Li[i * D + qc];
          b[q] = Ls[qc * D + j] * ((q <= i) ? 1.0 : 0.0);
        }
#pragma unroll
        for (int q = 0; q < DM; ++q)
          v += a[q] * b[q];
      }
      sv.M[t * DD + e] = v;
    }
    wave_sync();
    if (!use_cpl)
      for (int e = c.lane; e < DD; e += 64)
      {
        const int i = e / D, q = e % D;
        Ls[e] = PO[cpl * D + i] * Li[q * D + i];
      }
    else
    {
      // Lsub[i][q] = sum_j K[i][j] LI_t[q][j] with K = K_{t+1,t} (top)
      // or K_{t-1,t} = K_{t,t-1}^T (bottom)
      const double* Kc = c.a(A_CPL) + cpl * DD;
      for (int e = c.lane; e < DD; e += 64)
      {
        const int i = e / D, q = e % D;
        double a[DM], b[DM];
#pragma unroll
        for (int j = 0; j < DM; ++j)
        {
          const int jc = min(j, D - 1);
          a[j] = (half == 0) ? Kc[i * D + jc] : Kc[jc * D + i];
          b[j] = Li[q * D + jc] * ((j <= q) ? 1.0 : 0.0);
        }
        double v = 0;
#pragma unroll
        for (int j = 0; j < DM; ++j)
          v += a[j] * b[j];
        Ls[e] = v;
      }
    }
    wave_sync();
    for (int e = c.lane; e < DD; e += 64)
    {
      const int i = e / D, j = e % D;
      double a[DM], b[DM];
#pragma unroll
      for (int q = 0; q < DM; ++q)
      {
        const int qc = min(q, D - 1);
        a[q] = Li[qc * D + i];
        b[q] = Ls[j * D + qc] * ((q >= i && q < D) ? 1.0 : 0.0);
      }
      double v = 0;
#pragma unroll
      for (int q = 0; q < DM; ++q)
        v += a[q] * b[q];
      sv.Nb[t * DD + e] = v;
    }
    wave_sync();
  }
}

__device__ int build_hinge_chunks(Ctx& c);
__device__ __forceinline__ bool lds_resident(const Ctx& c, const double* p);

// the QP's ADMM iterations run the register-resident segment (qp_solve); it
// addresses MR, the hinge chunk table and chunk sums as LDS
__device__ __forceinline__ bool seg_path(const Ctx& c)
{
  return c.L.seg_ok && lds_resident(c, c.a(A_MR)) && lds_resident(c, c.a(A_CPK)) &&
         (c.s->n_h == 0 || (lds_resident(c, c.a(A_HCHK)) && lds_resident(c, c.a(A_HPART))));
}

// returns false if the reduced matrix is not positive definite
__device__ bool factor(Ctx& c, Solver& sv, double sigK, bool polish, double delta)
{
  PROF(3);
  long long* pf = (c.tid == 0) ? c.s->prof : nullptr;
  long long tq = pf ? clock64() : 0;
  const Layout& L = c.L;
  const int D = L.D, nx = L.nx, N = L.N;
  const double *PD = c.a(A_PD), *PO = c.a(A_PO), *BS = c.a(A_BS), *GS = c.a(A_GS), *WS = c.a(A_WS),
               *FS = c.a(A_FS);
  double *DG = c.a(A_DG), *RE = c.a(A_RE), *KB = c.a(A_KB), *LI = c.a(A_LINV);
  FOR(col, c.nc())
  {
    const double rb = rho_k(c, bound_row(L, col), polish, delta);
    DG[col] = sigK + rb * (BS[col] * BS[col]);
  }
  BSYNC();
  FOR(r, L.n_abs)
  {
    const int ca = nx + 2 * r;
    const double rr = rho_k(c, L.n_fixed_rows + r, polish, delta);
    // rho_eff = rho dn dp / det(K_aa), det = dn dp + rho (dn wp^2 + dp wn^2):
    // every term positive, no cancellation even when dn or dp ~ delta
    const double dn = DG[ca], dp = DG[ca + 1], wn = WS[2 * r], wp = WS[2 * r + 1];
    const double det = dn * dp + rr * (dn * wp * wp + dp * wn * wn);
    RE[r] = rr * dn * dp / det;
  }
  // hinge rows: one hinge variable, rho_eff = rho d / (d + rho w^2)
  const int nh = c.s->n_h;
  FOR(h, nh)
  {
    const int col = L.nc_base + h;
    const double rr = rho_k(c, L.m_base + 2 * h, polish, delta);
    const double dn = DG[col], w = c.a(A_HW)[h];
    c.a(A_HRE)[h] = rr * dn / (dn + rr * w * w);
  }
  BSYNC();
  // the hinge chunk table for reduced_solve's row-parallel column sums (the
  // QP's hinge rows are fixed from here to its last solve), and the field-major
  // copy of the hinge coefficients its back-substitution reads (A_HCT, odd
  // stride; the ADMM segment builds the same): one coalesced load per
  // coefficient and wave instead of 2 D loads that each touch 64 cache lines
  build_hinge_chunks(c);
  if (nh > 0 && !seg_path(c))  // (the segment builds its own copy)
  {
    const int nhs = nh | 1;
    const double* HC = c.a(A_HC);
    double* HCT = c.a(A_HCT);
    FOR(e, nh * 2 * D)
    {
      const int h = e / (2 * D), k = e - h * 2 * D;
      HCT[k * nhs + h] = HC[e];
    }
    BSYNC();
  }
  // waypoint t's diagonal block entry (i, j): P, sigma + bound rows, the fixed
  // rows, its CartPose rows and the hinge rows of pairs t and t - 1 (the row
  // sums in chunks of 8 rows, all loads of a chunk first; masked terms add
  // fma(w, 0, v) = v: a loop of dependent loads otherwise)
  const int nh_ = nh;
  auto wblock = [&](int t, int i, int j) {
    double v = 0;
    if (i == j)
    {
      v = PD[t * D + i] + DG[t * D + i];
      const int f = c.T.fixed_of_step[t];
      if (f >= 0)
      {
        const int fr = f * D + i;
        v += rho_k(c, fr, polish, delta) * (FS[fr] * FS[fr]);
      }
    }
    {
      const int p0 = c.T.step_ptr[t], p1 = c.T.step_ptr[t + 1];
      for (int p = p0; p < p1; p += 8)
      {
        int rr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          rr[u] = c.T.step_rows[min(p + u, p1 - 1)];
        double w[8], a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
        {
          w[u] = RE[rr[u]];
          a[u] = (GS[rr[u] * D + i] * GS[rr[u] * D + j]) * ((p + u < p1) ? 1.0 : 0.0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v += w[u] * a[u];
      }
    }
    if (nh_ > 0)
    {
      const double *HC = c.a(A_HC), *HRE = c.a(A_HRE);
      const int* HP = c.ia(I_HPTR);
      v = hinge_outer_sum(HC, HRE, 2 * D, i, j, HP[t], HP[t + 1], v);
      if (t > 0)
        v = hinge_outer_sum(HC, HRE, 2 * D, D + i, D + j, HP[t - 1], HP[t], v);
    }
    return v;
  };
  // the coupling K_{t+1,t}[i][j] = diag(PO_t) + sum_h rho_eff a_t+1 a_t^T over
  // the hinge rows of pair t (t < N - 1)
  auto wcoup = [&](int t, int i, int j) {
    double v = (i == j) ? PO[t * D + i] : 0.0;
    if (nh_ > 0)
      v = hinge_outer_sum(c.a(A_HC), c.a(A_HRE), 2 * D, D + i, j, c.ia(I_HPTR)[t], c.ia(I_HPTR)[t + 1], v);
    return v;
  };
  const int sD = L.sD, sDD = sD * sD, sNb = L.sNb;
  if (L.grp == 1)
  {
    // diagonal blocks, in the solve layout (Layout::nbr): block T = b N + t holds
    // waypoint t's dofs [b sD, (b + 1) sD); the other branches' entries of the
    // waypoint block are exact zeros (no term touches two branches)
    FOR(e, L.sN * sDD)
    {
      const int T = e / sDD, bi = T / N, t = T - bi * N;
      const int i = bi * sD + (e / sD) % sD, j = bi * sD + e % sD;  // dofs of the waypoint block
      KB[e] = wblock(t, i, j);
    }
    if (L.hinge || L.nbr > 1)
    {
      // dense couplings K_{t+1,t}, per solve block (T, T + 1) of one branch
      // (block N - 1 of a branch couples to nothing; its entry is unused)
      double* CPL = c.a(A_CPL);
      FOR(e, (L.sN - 1) * sDD)
      {
        const int T = e / sDD, bi = T / N, t = T - bi * N;
        const int il = (e / sD) % sD, jl = e % sD, i = bi * sD + il, j = bi * sD + jl;
        CPL[e] = (t < N - 1) ? wcoup(t, i, j) : 0.0;
      }
    }
  }
  else
  {
    // waypoint pairs (Layout::grp = 2, JointAccEqCost): solve block T holds
    // waypoints 2T (rows / columns [0, D)) and 2T + 1 ([D, 2D)); P couples
    // t and t + 2 (A_PO2, diagonal), so the couplings between blocks T and
    // T + 1 are K_{2T+2,2T} = diag(PO2_2T), K_{2T+2,2T+1} (the waypoint
    // coupling of pair 2T + 1), K_{2T+3,2T+1} = diag(PO2_2T+1), K_{2T+3,2T} = 0
    const double* PO2 = c.a(A_PO2);
    FOR(e, L.sN * sDD)
    {
      const int T = e / sDD, il = (e / sD) % sD, jl = e % sD;
      const int wi = il / D, wj = jl / D, i = il - wi * D, j = jl - wj * D;
      double v;
      if (wi == wj)
        v = wblock(2 * T + wi, i, j);
      else if (wi == 1)
        v = wcoup(2 * T, i, j);  // K_{2T+1,2T}
      else
        v = wcoup(2 * T, j, i);  // K_{2T,2T+1} = K_{2T+1,2T}^T
      KB[e] = v;
    }
    double* CPL = c.a(A_CPL);
    FOR(e, (L.sN - 1) * sDD)
    {
      const int T = e / sDD, il = (e / sD) % sD, jl = e % sD;
      const int wi = il / D, wj = jl / D, i = il - wi * D, j = jl - wj * D;
      double v = 0.0;
      if (wi == 0 && wj == 1)
        v = wcoup(2 * T + 1, i, j);  // K_{2T+2,2T+1}
      else if (wi == wj && i == j)
        v = PO2[(2 * T + wi) * D + i];  // K_{2T+2,2T}, K_{2T+3,2T+1}
      CPL[e] = v;
    }
  }
  BSYNC();
  if (pf)
  {
    const long long tn = clock64();
    pf[32] += tn - tq;
    tq = tn;
  }
  // Twisted ("burn at both ends") block Cholesky.  Wave 0 eliminates the
  // waypoints 0..m-1 from the top, wave 1 eliminates N-1..m+1 from the bottom
  // (the same recurrence on the reversed block order; the JointVel couplings
  // K_{t+1,t} = diag(PO_t) are symmetric), concurrently; the middle block m
  // takes both Schur complements.  Per eliminated block t:
  //   S_t = KB_t - Lsub Lsub^T, L_t = chol(S_t), LI_t = L_t^-1,
  //   M_t = LI_t Lsub (coupling from the previous block of its half),
  //   Lsub <- O LI_t^T (coupling into the next block), N_t = LI_t^T Lsub^T.
  // Bottom-half matrices are stored at their own waypoint index; the middle
  // stores M_m (top coupling) in M[m] and M'_m (bottom coupling) in Nb[m].
  // per-half block and coupling scratch in the dynamic LDS after the chain
  // scratch (Layout::fac_off, 4 D x D blocks)
  // per-wave block and coupling scratch in the dynamic LDS after the chain
  // scratch (Layout::fac_off, 4 D x D >= 4 nbr sD x sD doubles): wave w's block
  // Sblk(w), its coupling Lsub(w)
  auto Sblk = [&](int w) { return c.big + L.fac_off + w * sDD; };
  auto Lsub = [&](int w) { return c.big + L.fac_off + (2 * L.nbr + w) * sDD; };
  __shared__ int bad;
  const int m = L.tw_mid;
  if (c.tid == 0)
    bad = 0;
  BSYNC();
  if (c.wave < 2 * L.nbr)
  {
    if (sD > kOct)
      twisted_factor_half<THIP_MAX_DOF>(c, sv, KB, LI, PO, Sblk(c.wave), Lsub(c.wave), bad);
    else
      twisted_factor_half<kOct>(c, sv, KB, LI, PO, Sblk(c.wave), Lsub(c.wave), bad);
  }
  BSYNC();
  if ((c.wave & 1) == 0 && c.wave < 2 * L.nbr)
  {
    // the middle block of branch b: both halves' Schur complements
    const int bi = c.wave >> 1, mb = bi * sNb + m;
    const bool top = m > 0, bot = (sNb - 1 - m) > 0;
    double* S = Sblk(c.wave);
    const double *Lt = Lsub(c.wave), *Lb = Lsub(c.wave + 1);
    for (int e = c.lane; e < sDD; e += 64)
    {
      const int i = e / sD, j = e % sD;
      double v = KB[mb * sDD + e];
      if (top)
        for (int q = 0; q < sD; ++q)
          v -= Lt[i * sD + q] * Lt[j * sD + q];
      if (bot)
        for (int q = 0; q < sD; ++q)
          v -= Lb[i * sD + q] * Lb[j * sD + q];
      S[e] = v;
    }
    wave_sync();
    chol_inv_block(S, LI + mb * sDD, sD, c.lane, bad);
    const double* Li = LI + mb * sDD;
    for (int e = c.lane; e < sDD; e += 64)
    {
      const int i = e / sD, j = e % sD;
      double vt = 0, vb = 0;
      for (int q = 0; q <= i; ++q)
      {
        vt += Li[i * sD + q] * Lt[q * sD + j];
        vb += Li[i * sD + q] * Lb[q * sD + j];
      }
      if (top)
        sv.M[mb * sDD + e] = vt;
      if (bot)
        sv.Nb[mb * sDD + e] = vb;
#if THIP_GENERIC_ONLY
      // the wide middle's couplings also in the scratch (blocks 0, 1: consumed
      // above) for twisted_middle_wide's reads, the rest of the factorisation
      if (L.wide)
      {
        Sblk(0)[e] = vt;
        Sblk(1)[e] = vb;
      }
#endif
    }
  }
  BSYNC();
  if (pf)
    pf[33] += clock64() - tq;
  if (c.tid == 0 && c.s->prof)
    c.s->prof[29] += 1;  // factor calls (diagnostic count)
  const bool ok = (bad == 0);
  BSYNC();
  return ok;
}

// is p (a generic pointer from the residency plan) inside this workgroup's
// dynamic LDS?
__device__ __forceinline__ bool lds_resident(const Ctx& c, const double* p)
{
  return p >= c.big && p < c.big + c.L.lds_budget;
}

// ---- wave-level chain of the block solve ---------------------------------
// 64-bit DPP move (two 32-bit halves)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// sum over the 8 lanes of a lane octet (lane & 7): xor 1, xor 2 (quad_perm),
// then the mirrored octet half (row_half_mirror)
__device__ __forceinline__ double octet_sum(double v)
{
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  return v;
}
// sum over the 8 octets (lane >> 3) at fixed lane & 7: xor 8 (row_ror:8),
// xor 16 (v_permlane16_swap), xor 32 (v_permlane32_swap) -- gfx950
__device__ __forceinline__ double cross_octet_sum(double v)
{
  v += dpp_f64<0x128>(v);  // row_ror:8 within each 16-lane row
  {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  return v;
}

// max over the wave: DPP / permlane exchanges in registers (the octet and
// cross-octet patterns of the chain) instead of six ds_bpermute round trips;
// max is exact, so the order is immaterial
__device__ __forceinline__ double wave_max(double v)
{
  v = fmax(v, dpp_f64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmax(v, dpp_f64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmax(v, dpp_f64<0x141>(v));  // row_half_mirror
  v = fmax(v, dpp_f64<0x128>(v));  // row_ror:8
  {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = fmax(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
  }
  {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = fmax(__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1]));
  }
  return v;
}

// sum_{k in [k0, k1)} a[k * sa] * b[k * sb], in order, for k1 <= KMAX:
// all loads issued first (clamped indices, finite operands), masked
// accumulation
template <int KMAX, typename AP, typename BP>
__device__ __forceinline__ double masked_dot(AP a, int sa, BP b, int sb, int k0, int k1)
{
  double av[KMAX], bv[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
  {
    const int kk = min(k, k1 - 1);
    av[k] = a[kk * sa];
    bv[k] = b[kk * sb];
  }
  // masked terms add fma(a, 0, v) = v: the same sum, and no branch the
  // compiler could sink the loads into (a guarded add compiled to one branch,
  // one load and one full vmcnt wait per term)
  double v = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    v = fma(av[k], bv[k] * ((k >= k0 && k < k1) ? 1.0 : 0.0), v);
  return v;
}

// Block-bidiagonal recurrence v_t = c_t - G_t v_{t-1} (FWD, t = 1..N-1) or
// v_t = c_t - G_t v_{t+1} (backward, t = N-2..0), run by one wave.  Lane
// (i, k) = (lane >> 3, lane & 7) multiplies one element of the D x D block.
// The vector alternates between "column" layout (value indexed by k) and
// "row" layout (indexed by i): odd steps reduce over k inside an octet, even
// steps use the transposed block and reduce over i across octets, so no
// lane permutation (ds_bpermute) sits on the serial path.  Blocks and c
// values are loaded kChainChunk steps at a time into registers (one LDS wait
// per chunk); inside a chunk the steps are unrolled with static parity.
constexpr int kChainChunk = 8;

// v_t = c_t - G_t v_{t-dir} for t = t0 + dir, ..., t0 + dir * nsteps, from
// v_{t0} = c_{t0} (written to out[t0] if store_first).
template <typename GP>
__device__ __forceinline__ void block_chain(GP G, const double* cvp, double* outp, int t0, int nsteps, int dir,
                                            bool store_first, int D, int lane)
{
  const lds_f64* cv = lds(cvp);
  lds_f64* out = lds(outp);
  const int i = lane >> 3, k = lane & 7;
  const bool act = (i < D) && (k < D);
  const int DD = D * D;
  double v = (k < D) ? cv[t0 * D + k] : 0.0;  // column layout
  if (store_first && i == 0 && k < D)
    out[t0 * D + k] = v;
  // offsets of this lane's element in the normal / transposed block
  const int off_n = i * D + k, off_t = k * D + i;
  for (int s0 = 1; s0 <= nsteps; s0 += kChainChunk)
  {
    double g[kChainChunk], cc[kChainChunk];
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const int s = s0 + u;
      const bool ok = s <= nsteps;
      const int t = ok ? t0 + dir * s : t0;  // clamped: every lane loads a valid address
      // s0 is odd, so even u are odd steps (normal block, c by row i)
      const double gv = G[t * DD + (((u & 1) == 0) ? off_n : off_t)];
      const double cvv = cv[t * D + (((u & 1) == 0) ? (i < D ? i : 0) : (k < D ? k : 0))];
      g[u] = (ok && act) ? -gv : 0.0;
      // c_t enters the reduction on one lane of each output (k == 0 for the
      // octet sum, i == 0 for the cross-octet sum): v_t = sum(c_t - G v),
      // one fma per lane and no subtraction after the reduction
      const bool lead = ((u & 1) == 0) ? (k == 0) : (i == 0);
      cc[u] = (ok && lead && (((u & 1) == 0) ? (i < D) : (k < D))) ? cvv : 0.0;
    }
    // serial part: no loads, stores or branches (steps past nsteps compute zeros)
    double vs[kChainChunk];
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const double p = fma(g[u], v, cc[u]);
      if ((u & 1) == 0)
        v = octet_sum(p);  // row layout: v = v_t[i]
      else
        v = cross_octet_sum(p);  // column layout: v = v_t[k]
      vs[u] = v;
    }
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const int s = s0 + u;
      const int t = t0 + dir * s;
      if ((u & 1) == 0)
      {
        if (s <= nsteps && k == 0 && i < D)
          out[t * D + i] = vs[u];
      }
      else if (s <= nsteps && i == 0 && k < D)
        out[t * D + k] = vs[u];
    }
  }
}

// The same recurrence for blocks wider than a lane octet (D > kOct, e.g.
// the 14-DoF dual arm), with the chain matrices in HBM (Layout::wide).  Lane
// (i, q) = (lane >> 2, lane & 3) owns columns 4q..4q+3 of row i: a step is
// four fmas against the previous vector (read back from LDS) and a two-level
// quad reduction.  The blocks of kWideChunk steps are loaded into registers
// before the chunk's serial steps, so the HBM latency is paid once per chunk
// instead of once per step.
constexpr int kWideChunk = 8;
__device__ __noinline__ void block_chain_wide(const double* Gp, const double* cvp, double* outp, int t0, int nsteps,
                                              int dir, bool store_first, int D, int lane)
{
  const gbl_f64* G = gbl(Gp);  // HBM (Layout::wide)
  const lds_f64* cv = lds(cvp);
  lds_f64* out = lds(outp);
  const int DD = D * D;
  const int i = lane >> 2, q = lane & 3;
  const bool row_ok = i < D;
  const int ic = row_ok ? i : D - 1;
  // masks as multipliers on loaded values (finite), never as conditions: a
  // guarded load compiled to a branch and a full vmcnt wait per load
  int kk[4];
  double kmask[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
  {
    const bool kok = 4 * q + e < D;
    kk[e] = kok ? 4 * q + e : D - 1;  // clamped: every lane reads a valid address
    kmask[e] = kok ? 1.0 : 0.0;
  }
  const double qmask = (q == 0) ? 1.0 : 0.0;
  if (store_first && q == 0 && row_ok)
    out[t0 * D + i] = cv[t0 * D + i];
  wave_sync();
  for (int s0 = 1; s0 <= nsteps; s0 += kWideChunk)
  {
    double g[kWideChunk][4], cc[kWideChunk];
#pragma unroll
    for (int u = 0; u < kWideChunk; ++u)
    {
      // steps past nsteps are never computed; rows i >= D are never stored
      const int s = s0 + u;
      const int t = (s <= nsteps) ? t0 + dir * s : t0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        g[u][e] = G[t * DD + ic * D + kk[e]];
      // c_t enters the reduction on lane q == 0 of its row (out may alias cv
      // in the backward pass: every c of the chunk is read before its step
      // writes)
      cc[u] = cv[t * D + ic] * qmask;
    }
#pragma unroll
    for (int u = 0; u < kWideChunk; ++u)
    {
      const int s = s0 + u;
      if (s > nsteps)
        break;
      const int t = t0 + dir * s, tp = t - dir;
      double p = cc[u];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        p = fma(-g[u][e], out[tp * D + kk[e]] * kmask[e], p);
      p += dpp_f64<0xB1>(p);  // quad_perm [1,0,3,2]
      p += dpp_f64<0x4E>(p);  // quad_perm [2,3,0,1]
      if (q == 0 && row_ok)
        out[t * D + i] = p;
      wave_sync();
    }
  }
}

// the chain matrices in LDS, or in HBM (Layout::wide, Layout::chm_hbm)
__device__ __forceinline__ void chain_any(const double* G, const double* cv, double* out, int t0, int nsteps, int dir,
                                          bool store_first, int D, int lane, bool wide, bool chm_hbm)
{
  if (wide)
    block_chain_wide(G, cv, out, t0, nsteps, dir, store_first, D, lane);
  else if (chm_hbm)
    block_chain(gbl(G), cv, out, t0, nsteps, dir, store_first, D, lane);
  else
    block_chain(lds(G), cv, out, t0, nsteps, dir, store_first, D, lane);
}

// Forward solve of the twisted factor: y = L^-1 b given c_t = LI_t b_t in
// CV.  Wave 0 runs the top chain (t = 1..m-1), wave 1 the bottom chain
// (t = N-2..m+1); the middle block is finished by twisted_middle().
__device__ __forceinline__ void twisted_forward(const Ctx& c, const Solver& sv, double* CV, double* YV)
{
  // solve layout (Layout::nbr): branch b's blocks b N .. b N + N - 1, its top
  // half on wave 2b, its bottom half on wave 2b + 1
  const Layout& L = c.L;
  const int N = L.sNb, m = L.tw_mid, half = c.wave & 1, base = (c.wave >> 1) * N;  // (N: blocks per branch)
  if (c.wave >= 2 * L.nbr)
    return;
  if (half == 0)
    chain_any(sv.M, CV, YV, base, m - 1, +1, true, L.sD, c.lane, L.wide, L.chm_hbm);
  else if (N - 1 - m > 0)
    chain_any(sv.M, CV, YV, base + N - 1, N - 2 - m, -1, true, L.sD, c.lane, L.wide, L.chm_hbm);
}

// Backward solve of the twisted factor, in place in CV (holding d_t =
// LI_t^T y_t and x_m at the middle): top chain x_t = d_t - N_t x_{t+1} on
// wave 0, bottom chain x_t = d_t - N'_t x_{t-1} on wave 1 (per branch: 2b, 2b + 1).
__device__ __forceinline__ void twisted_backward(const Ctx& c, const Solver& sv, double* CV)
{
  const Layout& L = c.L;
  const int N = L.sNb, m = L.tw_mid, half = c.wave & 1, base = (c.wave >> 1) * N;  // (N: blocks per branch)
  if (c.wave >= 2 * L.nbr)
    return;
  if (half == 0)
    chain_any(sv.Nb, CV, CV, base + m, m, -1, false, L.sD, c.lane, L.wide, L.chm_hbm);
  else
    chain_any(sv.Nb, CV, CV, base + m, N - 1 - m, +1, false, L.sD, c.lane, L.wide, L.chm_hbm);
}

// d_t[i] = (LI_t^T y_t)[i] for column (t, i), t != middle.
__device__ __forceinline__ double twisted_dvalue(const Ctx& c, const double* LIp, const double* YVp, int t, int i)
{
  const int D = c.L.sD, DD = D * D;  // solve block t (Layout::nbr)
  const lds_f64* LI = lds(LIp);
  const lds_f64* YV = lds(YVp);
  if (c.L.wide)
    return masked_dot<THIP_MAX_DOF>(LI + t * DD + i, D, YV + t * D, 1, i, D);
  // unconditional loads from clamped indices, two accumulators (even / odd k):
  // no branch per term and half the dependent adds
  double v0 = 0, v1 = 0;
#pragma unroll
  for (int k = 0; k < kOct; ++k)
  {
    const int kk = (k < D) ? k : D - 1;
    // masked by a 0/1 multiplier, not a select (see masked_dot)
    const double a = LI[t * DD + kk * D + i] * (YV[t * D + kk] * (((k >= i) && (k < D)) ? 1.0 : 0.0));
    if (k & 1)
      v1 += a;
    else
      v0 += a;
  }
  return v0 + v1;
}

// The middle block of the twisted solve, by one whole wave in the chain's
// octet layout: y_m = c_m - M_m y_{m-1} - M'_m y_{m+1} (octet reduction),
// x_m = LI_m^T y_m (cross-octet reduction), written over c_m in CV.
__device__ __noinline__ void twisted_middle_wide(const Ctx& c, const Solver& sv, const double* LIp, double* CVp,
                                                double* YVp)
{
  // solve blocks (Layout::grp: a waypoint pair), one branch
  const int D = c.L.sD, DD = D * D, m = c.L.tw_mid, N = c.L.sNb, i = c.lane;
  const lds_f64* LI = lds(LIp);
#if THIP_GENERIC_ONLY
  // M_m and M'_m as factor() left them in its LDS scratch (the HBM copies'
  // values: one LDS round trip instead of one HBM round trip per solve)
  const lds_f64* Mm = lds(static_cast<const double*>(c.big + c.L.fac_off));
  const lds_f64* Mbm = Mm + DD;
#else
  const gbl_f64* M = gbl(sv.M);  // HBM (Layout::wide)
  const gbl_f64* Mb = gbl(sv.Nb);
#endif
  lds_f64* CV = lds(CVp);
  lds_f64* YV = lds(YVp);
  if (i < D)
  {
    // all loads first (clamped), then the sum in the original order
    const bool top = m > 0, bot = N - 1 - m > 0;
    double mt[THIP_MAX_DOF], yt[THIP_MAX_DOF], mb[THIP_MAX_DOF], yb[THIP_MAX_DOF];
#pragma unroll
    for (int k = 0; k < THIP_MAX_DOF; ++k)
    {
      const int kk = min(k, D - 1);
#if THIP_GENERIC_ONLY
      mt[k] = Mm[i * D + kk];
      yt[k] = YV[max(m - 1, 0) * D + kk];
      mb[k] = Mbm[i * D + kk];
#else
      mt[k] = M[m * DD + i * D + kk];
      yt[k] = YV[max(m - 1, 0) * D + kk];
      mb[k] = Mb[m * DD + i * D + kk];
#endif
      yb[k] = YV[min(m + 1, N - 1) * D + kk];
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < THIP_MAX_DOF; ++k)
      if (k < D)
      {
        if (top)
          s += mt[k] * yt[k];
        if (bot)
          s += mb[k] * yb[k];
      }
    YV[m * D + i] = CV[m * D + i] - s;  // y_m (YV's middle row is not a chain output)
  }
  wave_sync();
  if (i < D)
    CV[m * D + i] = masked_dot<THIP_MAX_DOF>(LI + m * DD + i, D, YV + m * D, 1, i, D);
  wave_sync();
}

#if THIP_GENERIC_ONLY && THIP_GEN_DV_HOIST
// twisted_dvalue on layout values the caller holds (the same sum)
__device__ __forceinline__ double twisted_dvalue_l(const double* LIp, const double* YVp, int t, int i, int D, bool wide)
{
  const int DD = D * D;
  const lds_f64* LI = lds(LIp);
  const lds_f64* YV = lds(YVp);
  if (wide)
    return masked_dot<THIP_MAX_DOF>(LI + t * DD + i, D, YV + t * D, 1, i, D);
  double v0 = 0, v1 = 0;
#pragma unroll
  for (int k = 0; k < kOct; ++k)
  {
    const int kk = (k < D) ? k : D - 1;
    const double a = LI[t * DD + kk * D + i] * (YV[t * D + kk] * (((k >= i) && (k < D)) ? 1.0 : 0.0));
    if (k & 1)
      v1 += a;
    else
      v0 += a;
  }
  return v0 + v1;
}

// twisted_middle_wide on layout values the caller holds: M_m, M'_m from
// factor()'s LDS scratch (Mm), middle block m of N, D dofs (the same sums)
__device__ __forceinline__ void twisted_middle_wide_l(const lds_f64* Mm, const double* LIp, double* CVp, double* YVp,
                                                     int D, int m, int N, int i)
{
  const int DD = D * D;
  const lds_f64* LI = lds(LIp);
  const lds_f64* Mbm = Mm + DD;
  lds_f64* CV = lds(CVp);
  lds_f64* YV = lds(YVp);
  if (i < D)
  {
    const bool top = m > 0, bot = N - 1 - m > 0;
    double mt[THIP_MAX_DOF], yt[THIP_MAX_DOF], mb[THIP_MAX_DOF], yb[THIP_MAX_DOF];
#pragma unroll
    for (int k = 0; k < THIP_MAX_DOF; ++k)
    {
      const int kk = min(k, D - 1);
      mt[k] = Mm[i * D + kk];
      yt[k] = YV[max(m - 1, 0) * D + kk];
      mb[k] = Mbm[i * D + kk];
      yb[k] = YV[min(m + 1, N - 1) * D + kk];
    }
    // branch-free: a masked term is fma(0, y, s) = s (the coupling itself is
    // selected away: an absent half's scratch block is not initialised), the
    // same sum in the same order as the guarded adds, which compiled to one
    // branch and one LDS wait per term
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < THIP_MAX_DOF; ++k)
    {
      s = fma((top && k < D) ? mt[k] : 0.0, yt[k], s);
      s = fma((bot && k < D) ? mb[k] : 0.0, yb[k], s);
    }
    YV[m * D + i] = CV[m * D + i] - s;
  }
  wave_sync();
  if (i < D)
    CV[m * D + i] = masked_dot<THIP_MAX_DOF>(LI + m * DD + i, D, YV + m * D, 1, i, D);
  wave_sync();
}
#endif

template <typename MP>
__device__ __forceinline__ void twisted_middle_narrow(const Ctx& c, MP M, MP Mb, const double* LIp, double* CVp,
                                                      const double* YVp, int branch)
{
  const int D = c.L.sD, DD = D * D, N = c.L.sNb, mloc = c.L.tw_mid, m = branch * N + mloc;
  const int i = c.lane >> 3, k = c.lane & 7;
  const bool act = (i < D) && (k < D);
  const lds_f64* LI = lds(LIp);
  const lds_f64* YV = lds(YVp);
  lds_f64* CV = lds(CVp);
  double p = 0.0;
  if (act)
  {
    if (mloc > 0)
      p = M[m * DD + i * D + k] * YV[(m - 1) * D + k];
    if (N - 1 - mloc > 0)
      p += Mb[m * DD + i * D + k] * YV[(m + 1) * D + k];
  }
  const double s = octet_sum(p);
  const double ym = (i < D) ? CV[m * D + i] - s : 0.0;  // row layout
  const double q = act ? LI[m * DD + i * D + k] * ym : 0.0;
  const double xm = cross_octet_sum(q);                  // column layout
  wave_sync();
  if (i == 0 && k < D)
    CV[m * D + k] = xm;
}

// the middle block of branch `branch` (wide blocks: one branch)
__device__ __forceinline__ void twisted_middle(const Ctx& c, const Solver& sv, const double* LIp, double* CVp,
                                               const double* YVp, int branch)
{
  if (c.L.wide)
    twisted_middle_wide(c, sv, LIp, CVp, const_cast<double*>(YVp));
  else if (c.L.chm_hbm)
    twisted_middle_narrow(c, gbl(static_cast<const double*>(sv.M)), gbl(static_cast<const double*>(sv.Nb)), LIp, CVp,
                          YVp, branch);
  else
    twisted_middle_narrow(c, lds(static_cast<const double*>(sv.M)), lds(static_cast<const double*>(sv.Nb)), LIp, CVp,
                          YVp, branch);
}

// b + sum over the CSR entries p in [p0, p1) of GS[rows[p]][j] * MR[rows[p]],
// in order; the row indices and values of four entries are loaded before
// their products are summed (a serial chain of dependent loads otherwise)
__device__ __forceinline__ double csr_row_gather(const int* rows, int p0, int p1, const double* GS, const double* MR,
                                                 int D, int j, double b)
{
  for (int p = p0; p < p1; p += 4)
  {
    int rr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      rr[u] = rows[min(p + u, p1 - 1)];
    double g[4], mv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
    {
      g[u] = GS[rr[u] * D + j];
      mv[u] = MR[rr[u]];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      b = fma(g[u], mv[u] * ((p + u < p1) ? 1.0 : 0.0), b);  // masked: b unchanged
  }
  return b;
}


// csr_row_gather for contiguous rows (Layout::rows_contig): the rows [p0, p1)
// themselves, at most R, every load issued before the sum (in the same order)
template <int R>
__device__ __forceinline__ double contig_row_gather(int p0, int p1, const double* GS, const double* MR, int D, int j,
                                                    double b)
{
  double g[R], mv[R];
#pragma unroll
  for (int u = 0; u < R; ++u)
  {
    const int r = max(min(p0 + u, p1 - 1), 0);  // clamped: every load valid (an empty range reads row 0)
    g[u] = GS[r * D + j];
    mv[u] = MR[r];
  }
#pragma unroll
  for (int u = 0; u < R; ++u)
    b = fma(g[u], mv[u] * ((p0 + u < p1) ? 1.0 : 0.0), b);  // masked: b unchanged
  return b;
}

// a hinge row's distance-expression value a_t.x_t + a_t+1.x_t+1 (two
// independent partial sums, one per waypoint); x points at x_t
template <typename XP>
__device__ __forceinline__ double hinge_dot(const double* hc, XP x, int D)
{
  // masked fixed-length sums (all loads in flight together), original order
  if (D > kOct)
    return masked_dot<THIP_MAX_DOF>(hc, 1, x, 1, 0, D) + masked_dot<THIP_MAX_DOF>(hc + D, 1, x + D, 1, 0, D);
  return masked_dot<kOct>(hc, 1, x, 1, 0, D) + masked_dot<kOct>(hc + D, 1, x + D, 1, 0, D);
}

// b + PART[q][k] for q in [q0, q1), added in order; eight loads issued before
// their adds (one HBM round trip per chunk otherwise: ~26 per column on the
// heavy problems, where the chunk sums do not fit in LDS).  Masked terms add
// an exact zero.
__device__ __forceinline__ double chunk_sum_add(const double* PART, int pw, int q0, int q1, int k, double b)
{
  for (int q = q0; q < q1; q += 8)
  {
    double p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      p[i] = PART[min(q + i, q1 - 1) * pw + k];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      b += p[i] * ((q + i < q1) ? 1.0 : 0.0);
  }
  return b;
}

// Solve K [x; aux] = r + A' eta, with r (n_cols) in A_BXW (overwritten) and
// eta over all m rows; K = P + diag(sigK) + A' diag(rho) A as in factor().
// The 2x2 aux block of each CartPose row is eliminated with its explicit
// inverse, expanded so that the rho^2 and eta_r terms cancel analytically:
// with polish rho = 1/delta the textbook Sherman-Morrison form subtracts
// O(1/delta^2) quantities and loses ~12 digits.  The hinge rows' share of each
// column is summed per chunk of kHChunk rows of one step pair (even and odd
// rows apart) and the chunk sums added in order: the association of
// admm_segment's row-parallel gather, so that both paths give identical iterates.
__device__ void reduced_solve(Ctx& c, Solver& sv, bool polish, double delta, const double* eta, double* out)
{
  long long* pf = (c.tid == 0) ? c.s->prof : nullptr;
  long long tq = pf ? clock64() : 0;
#define PROF_LAP(slot)          \
  if (pf)                       \
  {                             \
    const long long tn = clock64(); \
    pf[slot] += tn - tq;        \
    tq = tn;                    \
  }
  // the Ctx / Layout / Tables values the loops use, in registers (the Ctx
  // lives in private memory and would be re-read with dependent FLAT loads
  // after every store the compiler cannot prove does not alias it)
  const int tid = c.tid;
  const Layout& L = c.L;
  const int D = L.D, nx = L.nx, nfr = L.n_fixed_rows, n_abs = L.n_abs, n_rows = L.n_rows;
  const int nc_base = L.nc_base, m_base = L.m_base;
  const bool wide = L.wide;
  const double *GS = c.a(A_GS), *WS = c.a(A_WS), *DG = c.a(A_DG), *LI = c.a(A_LINV), *BS = c.a(A_BS),
               *FS = c.a(A_FS);
  double *BX = c.a(A_BXW), *BA = c.a(A_BA), *MR = c.a(A_MR), *CV = c.a(A_CV), *YV = c.a(A_YV);
  const double *RHO = c.a(A_RHO), *HW = c.a(A_HW), *HC = c.a(A_HC);
  const int *ACT = c.ia(I_ACT), *HT = c.ia(I_HT);
  const int *fixed_of_step = c.T.fixed_of_step, *step_ptr = c.T.step_ptr, *step_rows = c.T.step_rows,
            *row_step = c.T.row_step;
  // rho_k() and bound_row() on the hoisted values (same expressions)
  auto rho_l = [&](int r) { return !polish ? RHO[r] : (ACT[r] != 0 ? 1.0 / delta : 0.0); };
  auto brow = [&](int col) { return col < nc_base ? n_rows + col : m_base + 2 * (col - nc_base) + 1; };
  // kGenU rows per thread at once, every load before any store (see admm_step)
  GEN_UNROLL_BEGIN(kGenU, n_abs)
  for (int r0 = tid; r0 < n_abs; r0 += U * kBlock)
  {
    double mr[U], rnv[U], rpv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int r = min(r0 + u * kBlock, n_abs - 1);
      const int ca = nx + 2 * r;
      const double rr = rho_l(nfr + r);
      const double dn = DG[ca], dp = DG[ca + 1], wn = WS[2 * r], wp = WS[2 * r + 1];
      const double rn = BX[ca] + BS[ca] * eta[brow(ca)];
      const double rp = BX[ca + 1] + BS[ca + 1] * eta[brow(ca + 1)];
      const double det = dn * dp + rr * (dn * wp * wp + dp * wn * wn);
      mr[u] = (eta[nfr + r] * dn * dp - rr * (wn * dp * rn + wp * dn * rp)) / det;
      rnv[u] = rn;
      rpv[u] = rp;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int r = r0 + u * kBlock;
      if (r >= n_abs)
        break;
      MR[r] = mr[u];
      BA[nx + 2 * r] = rnv[u];
      BA[nx + 2 * r + 1] = rpv[u];
    }
  }
  GEN_UNROLL_END
  const int nh = c.s->n_h;
  GEN_UNROLL_BEGIN(kGenU, nh)
  for (int h0 = tid; h0 < nh; h0 += U * kBlock)
  {
    double mr[U], rnv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int h = min(h0 + u * kBlock, nh - 1);
      const int col = nc_base + h;
      const double rr = rho_l(m_base + 2 * h);
      const double dn = DG[col], w = HW[h];
      const double rn = BX[col] + BS[col] * eta[brow(col)];
      mr[u] = (eta[m_base + 2 * h] * dn - rr * w * rn) / (dn + rr * w * w);
      rnv[u] = rn;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int h = h0 + u * kBlock;
      if (h >= nh)
        break;
      MR[n_rows + h] = mr[u];
      BA[nc_base + h] = rnv[u];
    }
  }
  GEN_UNROLL_END
  BSYNC();
  PROF_LAP(23);
  // the hinge share of the column sums, row-parallel: chunk q's partial sum of
  // coefficient k over its rows (build_hinge_chunks, at the factorisation),
  // each in the association described above; the columns below add their step
  // pairs' chunk sums in order, so b is bitwise what gathering every row of
  // the column serially gave (one thread per column walked up to ~100 rows
  // per pair in HBM on config E's heavy problems)
  const int* const HCP = c.s->hcp;
  const int pw = L.part_w;
  double* const PART = c.a(A_HPART);
  if (nh > 0)
  {
    const int* CHK = reinterpret_cast<const int*>(c.a(A_HCHK));
    const int nchk = HCP[L.N], k = tid % pw, cstep = kBlock / pw;
    constexpr int kChU = 4;  // chunks per thread at once: 4 x 8 coefficient loads in flight
    if (k < 2 * D)
      for (int q0 = tid / pw; q0 < nchk; q0 += kChU * cstep)
      {
        double hc[kChU][kHChunk], mv[kChU][kHChunk];
        int h0v[kChU], h1v[kChU];
#pragma unroll
        for (int u = 0; u < kChU; ++u)
        {
          const int q = min(q0 + u * cstep, nchk - 1);  // clamped: every load valid
          const int h0 = CHK[2 * q], h1 = CHK[2 * q + 1];
          h0v[u] = h0;
          h1v[u] = h1;
#pragma unroll
          for (int i = 0; i < kHChunk; ++i)
          {
            const int h = min(h0 + i, h1 - 1);
            hc[u][i] = HC[h * 2 * D + k];
            mv[u][i] = MR[n_rows + h];
          }
        }
#pragma unroll
        for (int u = 0; u < kChU; ++u)
        {
          const int q = q0 + u * cstep, h0 = h0v[u], h1 = h1v[u];
          if (q >= nchk)
            break;
          double s0 = 0, s1 = 0;
#pragma unroll
          for (int i = 0; i < kHChunk; i += 2)
          {
            s0 = fma(hc[u][i], mv[u][i] * ((h0 + i < h1) ? 1.0 : 0.0), s0);  // masked: unchanged
            s1 = fma(hc[u][i + 1], mv[u][i + 1] * ((h0 + i + 1 < h1) ? 1.0 : 0.0), s1);
          }
          PART[q * pw + k] = s0 + s1;
        }
      }
    BSYNC();
  }
  // the waypoint right-hand sides, kRhsU columns per thread at once (their
  // loads overlap; each column's sums in the order of one column alone)
  constexpr int kRhsU = 3;
#if THIP_GENERIC_ONLY
  // (the main build keeps the 16-row gather, see unroll_for)
  const bool rows8 = L.max_step_rows <= 8, rows16 = L.rows_contig && L.max_step_rows <= 16;
#endif
  GEN_UNROLL_BEGIN(kRhsU, nx)
  for (int c0 = tid; c0 < nx; c0 += U * kBlock)
  {
    double bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int col = min(c0 + u * kBlock, nx - 1);  // clamped: every load valid
      const int t = col / D, j = col % D;
      double b = BX[col] + BS[col] * eta[brow(col)];
      const int f = fixed_of_step[t];
      if (f >= 0)
        b += FS[f * D + j] * eta[f * D + j];
#if THIP_GENERIC_ONLY
      if (rows16 && rows8)
        b = contig_row_gather<8>(step_ptr[t], step_ptr[t + 1], GS, MR, D, j, b);
      else if (rows16)
        b = contig_row_gather<16>(step_ptr[t], step_ptr[t + 1], GS, MR, D, j, b);
      else
#else
      if (L.rows_contig && L.max_step_rows <= 16)
        b = contig_row_gather<16>(step_ptr[t], step_ptr[t + 1], GS, MR, D, j, b);
      else
#endif
        b = csr_row_gather(step_rows, step_ptr[t], step_ptr[t + 1], GS, MR, D, j, b);
      if (nh > 0)
      {
        b = chunk_sum_add(PART, pw, HCP[t], HCP[t + 1], j, b);  // pair t, coefficient j
        if (t > 0)
          b = chunk_sum_add(PART, pw, HCP[t - 1], HCP[t], D + j, b);  // pair t - 1, coefficient D + j
      }
      bv[u] = b;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c0 + u * kBlock < nx)
        BX[c0 + u * kBlock] = bv[u];
  }
  GEN_UNROLL_END
  BSYNC();
  PROF_LAP(24);
  // c = LI b per solve block (Layout::nbr): solve index v is row i of block T,
  // branch bi's part of waypoint t
  const int sD = L.sD, sDD = sD * sD, N = L.sNb, nbr = L.nbr;
  for (int v = tid; v < nx; v += kBlock)
  {
    const int T = v / sD, i = v - T * sD, bi = T / N, t = T - bi * N;
    // the block's first column: waypoint t's branch bi part, or (waypoint
    // pairs, Layout::grp) columns T sD onwards
    const double* bt = (L.grp > 1) ? BX + T * sD : BX + t * D + bi * sD;
    const double cv = wide ? masked_dot<THIP_MAX_DOF>(lds(LI) + T * sDD + i * sD, 1, bt, 1, 0, i + 1)
                           : masked_dot<kOct>(lds(LI) + T * sDD + i * sD, 1, bt, 1, 0, i + 1);
    lds(CV)[v] = cv;
  }
  BSYNC();
  PROF_LAP(25);
  // forward chains (twisted factor): y = L^-1 b
  twisted_forward(c, sv, CV, YV);
  BSYNC();
  PROF_LAP(9);
  {
    // d = LI^T y off the middle block (all columns read before any write),
    // x_m at the middle block by the last wave
    constexpr int kCols = (THIP_MAX_STEPS * THIP_MAX_DOF + kBlock - 1) / kBlock;
    const int m = L.tw_mid;
    double dv[kCols];
    auto off_middle = [&](int cu) { return cu < nx && (cu / sD) % N != m; };
#if THIP_GENERIC_ONLY && THIP_GEN_DV_HOIST
    // the same sums on the hoisted layout values (twisted_dvalue / twisted_middle
    // re-read them from the Ctx, which lives in private memory: dependent FLAT
    // round trips ahead of every block's loads)
#pragma unroll
    for (int u = 0; u < kCols; ++u)
    {
      const int cu = tid + kBlock * u;
      dv[u] = off_middle(cu) ? twisted_dvalue_l(LI, YV, cu / sD, cu % sD, sD, wide) : 0.0;
    }
    PROF_LAP(35);
    if (c.wave >= kWaves - nbr)  // the last nbr waves: one middle block each
    {
      if (wide)
        twisted_middle_wide_l(lds(static_cast<const double*>(c.big + L.fac_off)), LI, CV, YV, sD, m, N, c.lane);
      else
        twisted_middle(c, sv, LI, CV, YV, c.wave - (kWaves - nbr));
    }
    BSYNC();
    PROF_LAP(36);
#else
#pragma unroll
    for (int u = 0; u < kCols; ++u)
    {
      const int cu = tid + kBlock * u;
      dv[u] = off_middle(cu) ? twisted_dvalue(c, LI, YV, cu / sD, cu % sD) : 0.0;
    }
#if THIP_GENERIC_ONLY
    PROF_LAP(35);
#endif
    if (c.wave >= kWaves - nbr)  // the last nbr waves: one middle block each
      twisted_middle(c, sv, LI, CV, YV, c.wave - (kWaves - nbr));
    BSYNC();
#if THIP_GENERIC_ONLY
    PROF_LAP(36);
#endif
#endif
#pragma unroll
    for (int u = 0; u < kCols; ++u)
    {
      const int cu = tid + kBlock * u;
      if (off_middle(cu))
        lds(CV)[cu] = dv[u];
    }
  }
  BSYNC();
  PROF_LAP(26);
  // backward chains, in place: x lands in CV (solve layout)
  twisted_backward(c, sv, CV);
  BSYNC();
  PROF_LAP(10);
  // x in column order: in CV itself, or (branches) gathered into YV for the
  // row products below
  const double* XC = CV;
  if (nbr > 1)
  {
    for (int col = tid; col < nx; col += kBlock)
    {
      const double xv = lds(CV)[solve_index(L, col)];
      out[col] = xv;
      lds(YV)[col] = xv;
    }
    BSYNC();
    XC = YV;
  }
  else
    for (int col = tid; col < nx; col += kBlock)
      out[col] = CV[col];
  // aux back-substitution
  GEN_UNROLL_BEGIN(kGenUHeavy, n_abs)
  for (int r0 = tid; r0 < n_abs; r0 += U * kBlock)
  {
    double on[U], op[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int r = min(r0 + u * kBlock, n_abs - 1);
      const int t = row_step[r];
      const int ca = nx + 2 * r;
      const int o = (nbr > 1) ? c.T.row_off[r] : 0;  // the row's branch (exact zeros elsewhere)
      const double g = (nbr > 1)  ? masked_dot<kOct>(GS + r * D + o, 1, lds(XC) + t * D + o, 1, 0, sD)
                       : (D > kOct) ? masked_dot<THIP_MAX_DOF>(GS + r * D, 1, lds(XC) + t * D, 1, 0, D)
                                    : masked_dot<kOct>(GS + r * D, 1, lds(XC) + t * D, 1, 0, D);
      const double rr = rho_l(nfr + r);
      const double dn = DG[ca], dp = DG[ca + 1], wn = WS[2 * r], wp = WS[2 * r + 1];
      const double rn = BA[ca], rp = BA[ca + 1];
      const double det = dn * dp + rr * (dn * wp * wp + dp * wn * wn);
      const double cross = wp * rn - wn * rp;
      const double h = eta[nfr + r] - rr * g;
      on[u] = (dp * rn + rr * wp * cross + wn * dp * h) / det;
      op[u] = (dn * rp - rr * wn * cross + wp * dn * h) / det;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int r = r0 + u * kBlock;
      if (r >= n_abs)
        break;
      out[nx + 2 * r] = on[u];
      out[nx + 2 * r + 1] = op[u];
    }
  }
  GEN_UNROLL_END
  const double* const HCT = c.a(A_HCT);
  const int nhs = nh | 1;
  GEN_UNROLL_BEGIN(kGenUHinge, nh)
  for (int h0 = tid; h0 < nh; h0 += U * kBlock)
  {
    double ov[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int h = min(h0 + u * kBlock, nh - 1);
      const int t = HT[h];
      // hinge_dot(HC + h 2D, x_t) on the field-major copy (same terms, same order)
      const double g = (D > kOct) ? masked_dot<THIP_MAX_DOF>(HCT + h, nhs, lds(XC) + t * D, 1, 0, D) +
                                        masked_dot<THIP_MAX_DOF>(HCT + D * nhs + h, nhs, lds(XC) + (t + 1) * D, 1, 0, D)
                                  : masked_dot<kOct>(HCT + h, nhs, lds(XC) + t * D, 1, 0, D) +
                                        masked_dot<kOct>(HCT + D * nhs + h, nhs, lds(XC) + (t + 1) * D, 1, 0, D);
      const int col = nc_base + h;
      const double rr = rho_l(m_base + 2 * h);
      const double dn = DG[col], w = HW[h];
      ov[u] = (BA[col] + w * (eta[m_base + 2 * h] - rr * g)) / (dn + rr * w * w);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int h = h0 + u * kBlock;
      if (h >= nh)
        break;
      out[nc_base + h] = ov[u];
    }
  }
  GEN_UNROLL_END
  BSYNC();
  PROF_LAP(11);
#undef PROF_LAP
}

// A x for one row (scaled); x over n_cols
__device__ __forceinline__ double row_ax(const Ctx& c, int r, const double* x)
{
  const Layout& L = c.L;
  const int D = L.D;
  if (r < L.n_fixed_rows)
  {
    const int slot = r / D, j = r % D;
    return c.a(A_FS)[r] * x[c.d->fixed_steps[slot] * D + j];
  }
  if (r < L.n_rows)
  {
    const int a = r - L.n_fixed_rows;
    const int t = c.T.row_step[a];
    const double* GS = c.a(A_GS);
    // fixed-length masked product: every load in flight at once, the terms
    // summed in the plain loop's order
    double v;
    if (L.nbr > 1)  // only the row's branch has nonzero coefficients (exact zeros elsewhere)
    {
      const int o = c.T.row_off[a];
      v = masked_dot<kOct>(GS + a * D + o, 1, x + t * D + o, 1, 0, L.sD);
    }
    else
      v = (D > kOct) ? masked_dot<THIP_MAX_DOF>(GS + a * D, 1, x + t * D, 1, 0, D)
                     : masked_dot<kOct>(GS + a * D, 1, x + t * D, 1, 0, D);
    const int ca = L.nx + 2 * a;
    v += c.a(A_WS)[2 * a] * x[ca] + c.a(A_WS)[2 * a + 1] * x[ca + 1];
    return v;
  }
  if (r < L.m_base)
  {
    const int col = r - L.n_rows;
    return c.a(A_BS)[col] * x[col];
  }
  const int h2 = r - L.m_base, h = h2 >> 1;
  if (h2 & 1)
  {
    const int col = L.nc_base + h;
    return c.a(A_BS)[col] * x[col];
  }
  // hinge row: a_t.x_t + a_t+1.x_t+1 + w h
  const int t = c.ia(I_HT)[h];
  double v = hinge_dot(c.a(A_HC) + h * 2 * D, x + t * D, D);
  v += c.a(A_HW)[h] * x[L.nc_base + h];
  return v;
}

// Hinge chunk table: chunks of kHChunk rows inside each step pair
// (c.s->hcp: first chunk of each pair; A_HCHK: (first row, end row)).
// Returns the chunk count.  Also used by the ADMM segment.
__device__ int build_hinge_chunks(Ctx& c)
{
  const int N = c.L.N, nh = c.s->n_h;
  const int* HP = c.ia(I_HPTR);
  int* CHK = reinterpret_cast<int*>(c.a(A_HCHK));
  if (nh == 0)
    return 0;
  if (c.tid == 0)
  {
    int acc = 0;
    for (int t = 0; t < N; ++t)
    {
      c.s->hcp[t] = acc;
      acc += (HP[t + 1] - HP[t] + kHChunk - 1) / kHChunk;
    }
    c.s->hcp[N] = acc;
  }
  BSYNC();
  for (int t = c.tid; t < N; t += kBlock)
  {
    const int h1 = HP[t + 1];
    int q = c.s->hcp[t];
    for (int h = HP[t]; h < h1; h += kHChunk, ++q)
    {
      CHK[2 * q] = h;
      CHK[2 * q + 1] = min(h + kHChunk, h1);
    }
  }
  BSYNC();
  return c.s->hcp[N];
}

// Row-parallel hinge share of A'v: A_HPART[q][k] = sum over chunk q of
// HC[h][k] * v[hinge row h] (Layout::part_w lanes per chunk, lane k = coefficient k).
// col_aty then adds the chunk sums of its two step pairs instead of looping
// over every hinge row of them (a serial chain of loads per column).
__device__ void hinge_chunk_sums(Ctx& c, const double* v, int nchk)
{
  const int D = c.L.D, mb = c.L.m_base;
  const double* HC = c.a(A_HC);
  const int* CHK = reinterpret_cast<const int*>(c.a(A_HCHK));
  double* PART = c.a(A_HPART);
  const int pw = c.L.part_w, k = c.tid % pw;  // lanes per chunk: 2 D coefficients
  if (k < 2 * D)
    for (int q = c.tid / pw; q < nchk; q += kBlock / pw)
    {
      const int h0 = CHK[2 * q], h1 = CHK[2 * q + 1];
      double s0 = 0, s1 = 0;
#pragma unroll
      for (int i = 0; i < kHChunk; i += 2)
      {
        const int ha = min(h0 + i, h1 - 1), hb = min(h0 + i + 1, h1 - 1);
        // masked by 0/1 multipliers, not selects (see masked_dot)
        const double aa = HC[ha * 2 * D + k] * (v[mb + 2 * ha] * ((h0 + i < h1) ? 1.0 : 0.0));
        const double ab = HC[hb * 2 * D + k] * (v[mb + 2 * hb] * ((h0 + i + 1 < h1) ? 1.0 : 0.0));
        s0 += aa;
        s1 += ab;
      }
      PART[q * pw + k] = s0 + s1;
    }
  BSYNC();
}

// (P x)_col and (A' y)_col (scaled)
__device__ __forceinline__ double col_px(const Ctx& c, int col, const double* x)
{
  const Layout& L = c.L;
  if (col >= L.nx)
    return 0.0;
  const int D = L.D, t = col / D;
  const double *PD = c.a(A_PD), *PO = c.a(A_PO);
  double v = PD[col] * x[col];
  if (t < L.N - 1)
    v += PO[col] * x[col + D];
  if (t > 0)
    v += PO[col - D] * x[col - D];
  if (L.grp > 1)  // JointAccEqCost's (t, t+2) coupling
  {
    const double* PO2 = c.a(A_PO2);
    if (t < L.N - 2)
      v += PO2[col] * x[col + 2 * D];
    if (t > 1)
      v += PO2[col - 2 * D] * x[col - 2 * D];
  }
  return v;
}
__device__ __forceinline__ double col_aty(const Ctx& c, int col, const double* y, bool chunked = false)
{
  const Layout& L = c.L;
  const int D = L.D;
  double v = c.a(A_BS)[col] * y[bound_row(L, col)];
  if (col < L.nx)
  {
    const int t = col / D, j = col % D;
    const int f = c.T.fixed_of_step[t];
    if (f >= 0)
      v += c.a(A_FS)[f * D + j] * y[f * D + j];
    const double* GS = c.a(A_GS);
    for (int p = c.T.step_ptr[t]; p < c.T.step_ptr[t + 1]; ++p)
    {
      const int a = c.T.step_rows[p];
      v += GS[a * D + j] * y[L.n_fixed_rows + a];
    }
    if (c.s->n_h > 0 && chunked)
    {
      const double* PART = c.a(A_HPART);
      for (int q = c.s->hcp[t]; q < c.s->hcp[t + 1]; ++q)
        v += PART[q * c.L.part_w + j];
      if (t > 0)
        for (int q = c.s->hcp[t - 1]; q < c.s->hcp[t]; ++q)
          v += PART[q * c.L.part_w + D + j];
    }
    else if (c.s->n_h > 0)
    {
      const double* HC = c.a(A_HC);
      const int* HP = c.ia(I_HPTR);
      for (int h = HP[t]; h < HP[t + 1]; ++h)
        v += HC[h * 2 * D + j] * y[L.m_base + 2 * h];
      if (t > 0)
        for (int h = HP[t - 1]; h < HP[t]; ++h)
          v += HC[h * 2 * D + D + j] * y[L.m_base + 2 * h];
    }
  }
  else if (col < L.nc_base)
  {
    const int a = (col - L.nx) >> 1, sd = (col - L.nx) & 1;
    v += c.a(A_WS)[2 * a + sd] * y[L.n_fixed_rows + a];
  }
  else
  {
    const int h = col - L.nc_base;
    v += c.a(A_HW)[h] * y[L.m_base + 2 * h];
  }
  return v;
}

// Loops of the generic (non-segment) code: U iterations per thread at once,
// the loads of all of them (ld) before any store (st), see kGenU.
template <int U, typename LD, typename ST>
__device__ __forceinline__ void gen_loop(const Ctx& c, int b, int e, LD ld, ST st)
{
  for (int i0 = b + c.tid; i0 < e; i0 += U * kBlock)
  {
    decltype(ld(0)) v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ld(min(i0 + u * kBlock, e - 1));  // clamped: every load valid
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int i = i0 + u * kBlock;
      if (i >= e)
        break;
      st(i, v[u]);
    }
  }
}

// (A x)_r for every row, one straight-line loop per row kind (as the ADMM
// update): ld(r, ax) gathers the row's other operands, st(r, value) stores
template <typename LD, typename ST>
__device__ __forceinline__ void gen_rows_ax(const Ctx& c, const double* x, LD ld, ST st)
{
  const Layout& L = c.L;
  const int m = c.m(), D = L.D;
  const double* BS = c.a(A_BS);
  gen_loop<kGenUHeavy>(c, 0, L.n_rows, [&](int r) { return ld(r, row_ax(c, r, x)); }, st);
  gen_loop<kGenULight>(c, L.n_rows, L.m_base, [&](int r) { return ld(r, BS[r - L.n_rows] * x[r - L.n_rows]); }, st);
  if (m > L.m_base)
  {
    const double *HC = c.a(A_HC), *HW = c.a(A_HW);
    const int* HT = c.ia(I_HT);
    gen_loop<kGenUHinge>(c, L.m_base, m,
                         [&](int r) {
                           const int h2 = r - L.m_base, h = h2 >> 1, col = L.nc_base + h;
                           const double ax = (h2 & 1) ? BS[col] * x[col]
                                                      : hinge_dot(HC + h * 2 * D, x + HT[h] * D, D) + HW[h] * x[col];
                           return ld(r, ax);
                         },
                         st);
  }
}

struct RowV
{
  double ax, a, b, d, e;
  int act;
};

// ======================================================================
// OSQP solve on the structured QP (one workgroup)
// ======================================================================
__device__ void set_rho_vec(Ctx& c)
{
  const double *Lo = c.a(A_L), *Up = c.a(A_U);
  double* RH = c.a(A_RHO);
  int* TY = c.ia(I_TYPE);
  const double rho = c.s->rho;
  FOR(r, c.m())
  {
    int ty;
    double rv;
    if (Lo[r] < -kInf * kMinScal && Up[r] > kInf * kMinScal)
    {
      ty = -1;
      rv = kRhoMin;
    }
    else if (Up[r] - Lo[r] < kRhoTol)
    {
      ty = 1;
      rv = kRhoEq * rho;
    }
    else
    {
      ty = 0;
      rv = rho;
    }
    TY[r] = ty;
    RH[r] = rv;
  }
  BSYNC();
}

// residuals at (x, z, y); stores prim/dual residuals and the tolerance /
// rho-estimate norms in bc[]: returns via c.s
struct Norms
{
  double prim_res, dual_res;
  double zE, axE, qD, atyD, pxD;  // scaled-for-termination norms
  double pr, dr, z, ax, q, aty, px;  // raw (scaled-space) norms for rho estimate
  // the infeasibility certificates' first tests (is_primal_infeasible /
  // is_dual_infeasible), precomputed by the ADMM segment when inf_ready:
  // max |E dy|, sum u (dy)+ + l (dy)- over the clipped delta y, max |D dx|, q'dx
  int inf_ready;
  double ndy, lhs, ndx, qdx;
};

__device__ void compute_residuals(Ctx& c, const double* x, const double* z, const double* y, Norms& nm)
{
  PROF(1);
  const double *E = c.a(A_E), *DS = c.a(A_DS), *Q = c.a(A_Q);
  double v[12] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };
  // (no stores in these loops: the next rows' loads are not ordered behind them)
#pragma unroll 2
  FOR(r, c.m())
  {
    const double ax = row_ax(c, r, x);
    const double pr = ax - z[r];
    const double einv = 1.0 / E[r];
    v[0] = fmax(v[0], fabs(einv * pr));
    v[1] = fmax(v[1], fabs(einv * z[r]));
    v[2] = fmax(v[2], fabs(einv * ax));
    v[3] = fmax(v[3], fabs(pr));
    v[4] = fmax(v[4], fabs(z[r]));
    v[5] = fmax(v[5], fabs(ax));
  }
  // hinge share of A'y from row-parallel chunk sums (many contacts: the
  // per-column loop over a step pair's hinge rows was a serial load chain)
  const bool chunked = c.s->n_h > 0;
  if (chunked)
    hinge_chunk_sums(c, y, build_hinge_chunks(c));
#pragma unroll 2
  FOR(col, c.nc())
  {
    const double px = col_px(c, col, x);
    const double aty = col_aty(c, col, y, chunked);
    const double dr = Q[col] + px + aty;
    const double dinv = 1.0 / DS[col];
    v[6] = fmax(v[6], fabs(dinv * dr));
    v[7] = fmax(v[7], fabs(dinv * Q[col]));
    v[8] = fmax(v[8], fabs(dinv * aty));
    v[9] = fmax(v[9], fabs(dinv * px));
    v[10] = fmax(v[10], fabs(dr));
    v[11] = fmax(v[11], fmax(fabs(Q[col]), fmax(fabs(aty), fabs(px))));
  }
  block_max<12>(c, v);
  nm.inf_ready = 0;
  nm.prim_res = (c.m() > 0) ? v[0] : 0.0;
  nm.zE = v[1];
  nm.axE = v[2];
  nm.pr = v[3];
  nm.z = v[4];
  nm.ax = v[5];
  nm.dual_res = c.s->cinv * v[6];
  nm.qD = v[7];
  nm.atyD = v[8];
  nm.pxD = v[9];
  nm.dr = v[10];
  nm.q = v[11];  // max(|q|,|A'y|,|Px|) combined (used only inside max())
}

__device__ bool is_primal_infeasible(Ctx& c, double eps)
{
  if (c.tid == 0 && c.s->prof)
    c.s->prof[27] += 1;  // calls (diagnostic count)
  double* DY = c.a(A_DY);
  const double *Lo = c.a(A_L), *Up = c.a(A_U), *E = c.a(A_E), *DS = c.a(A_DS);
  const int m = c.m();
  double nv[1] = { 0 };
  double lhs = 0;  // this thread's rows in FOR order, as the plain loop
  gen_loop<kGenULight>(
      c, 0, m, [&](int r) { return RowV{ 0.0, DY[r], Up[r], Lo[r], E[r], 0 }; },
      [&](int r, const RowV& v) {
        double dy = v.a;
        if (v.b > kInf * kMinScal)
          dy = (v.d < -kInf * kMinScal) ? 0.0 : fmin(dy, 0.0);
        else if (v.d < -kInf * kMinScal)
          dy = fmax(dy, 0.0);
        DY[r] = dy;
        nv[0] = fmax(nv[0], fabs(v.e * dy));
        lhs += v.b * fmax(dy, 0.0) + v.d * fmin(dy, 0.0);
      });
  block_max<1>(c, nv);
  const double ndy = nv[0];
  if (!(ndy > kDivTol))
    return false;
  lhs = block_sum(c, lhs);
  if (!(lhs < eps * ndy))
    return false;
  double av[1] = { 0 };
  const bool chunked = c.s->n_h > 0;
  if (chunked)
  {
    BSYNC();  // DY rewritten above
    hinge_chunk_sums(c, DY, build_hinge_chunks(c));
  }
  gen_loop<kGenUHeavy>(
      c, 0, c.nc(), [&](int col) { return (1.0 / DS[col]) * col_aty(c, col, DY, chunked); },
      [&](int, double v) { av[0] = fmax(av[0], fabs(v)); });
  block_max<1>(c, av);
  return av[0] < eps * ndy;
}

__device__ bool is_dual_infeasible(Ctx& c, double eps)
{
  if (c.tid == 0 && c.s->prof)
    c.s->prof[28] += 1;  // calls (diagnostic count)
  const double *DX = c.a(A_DX), *DS = c.a(A_DS), *Q = c.a(A_Q), *E = c.a(A_E), *Lo = c.a(A_L), *Up = c.a(A_U);
  double nv[1] = { 0 };
  double qdx = 0;  // this thread's columns in FOR order, as the plain loop
  gen_loop<kGenULight>(
      c, 0, c.nc(), [&](int col) { return RowV{ 0.0, DS[col], DX[col], Q[col], 0.0, 0 }; },
      [&](int, const RowV& v) {
        nv[0] = fmax(nv[0], fabs(v.a * v.b));
        qdx += v.d * v.b;
      });
  block_max<1>(c, nv);
  const double ndx = nv[0];
  const double cs = c.s->c;
  if (!(ndx > kDivTol))
    return false;
  qdx = block_sum(c, qdx);
  if (!(qdx < cs * eps * ndx))
    return false;
  double pv[1] = { 0 };
  gen_loop<kGenULight>(
      c, 0, c.nc(), [&](int col) { return (1.0 / DS[col]) * col_px(c, col, DX); },
      [&](int, double v) { pv[0] = fmax(pv[0], fabs(v)); });
  block_max<1>(c, pv);
  if (!(pv[0] < cs * eps * ndx))
    return false;
  double bad[1] = { 0 };
  gen_rows_ax(
      c, DX, [&](int r, double ax) { return RowV{ ax, E[r], Up[r], Lo[r], 0.0, 0 }; },
      [&](int, const RowV& v) {
        const double adx = (1.0 / v.a) * v.ax;
        if (((v.b < kInf * kMinScal) && (adx > eps * ndx)) || ((v.d > -kInf * kMinScal) && (adx < -eps * ndx)))
          bad[0] = 1.0;
      });
  block_max<1>(c, bad);
  return bad[0] == 0.0;
}

// check_termination; sets c.s->qp_status when it fires
__device__ bool check_termination(Ctx& c, const Norms& nm, bool approx)
{
  PROF(2);
  const thip_osqp_settings& os = c.d->osqp;
  double ea = os.eps_abs, er = os.eps_rel, epi = os.eps_prim_inf, edi = os.eps_dual_inf;
  if (approx)
  {
    ea *= 10;
    er *= 10;
    epi *= 10;
    edi *= 10;
  }
  bool prim_ok = false, dual_ok = false, pinf = false, dinf = false;
  if (c.m() == 0)
    prim_ok = true;
  else
  {
    const double eps_prim = ea + er * fmax(nm.zE, nm.axE);
    if (nm.prim_res < eps_prim)
      prim_ok = true;
    else if (nm.inf_ready && (!(nm.ndy > kDivTol) || !(nm.lhs < epi * nm.ndy)))
      pinf = false;  // is_primal_infeasible's first two tests, from the segment
    else
      pinf = is_primal_infeasible(c, epi);
  }
  const double eps_dual = ea + er * (c.s->cinv * fmax(fmax(nm.qD, nm.atyD), nm.pxD));
  if (nm.dual_res < eps_dual)
    dual_ok = true;
  else if (nm.inf_ready && (!(nm.ndx > kDivTol) || !(nm.qdx < c.s->c * edi * nm.ndx)))
    dinf = false;  // is_dual_infeasible's first two tests, from the segment
  else
    dinf = is_dual_infeasible(c, edi);
  int st = 0;
  if (prim_ok && dual_ok)
    st = approx ? ST_SOLVED_INACC : ST_SOLVED;
  else if (pinf)
    st = approx ? ST_PINF_INACC : ST_PINF;
  else if (dinf)
    st = approx ? ST_DINF_INACC : ST_DINF;
  if (c.tid == 0 && st != 0)
    c.s->qp_status = st;
  BSYNC();
  return st != 0;
}

// pre_ready: ETA and BX already hold this step's rho zp - y and sigma xp - q
// (the previous admm_step computed them from its new iterate, with rho
// unchanged since); every step leaves them ready for the next one
__device__ void admm_step(Ctx& c, Solver& sv, bool pre_ready)
{
  PROF(0);
  const int tid = c.tid;  // (the Ctx values the loops use, in registers: see reduced_solve)
  const thip_osqp_settings& os = c.d->osqp;
  const double sig = os.sigma, al = os.alpha;
  // swap buffers
  const int cur = c.s->cur ^ 1;
  BSYNC();
  if (tid == 0)
    c.s->cur = cur;
  double* x = c.a(cur ? A_XA1 : A_XA0);
  const double* xp = c.a(cur ? A_XA0 : A_XA1);
  double* z = c.a(cur ? A_Z1 : A_Z0);
  const double* zp = c.a(cur ? A_Z0 : A_Z1);
  double *Y = c.a(A_Y), *XT = c.a(A_XT), *DX = c.a(A_DX), *DY = c.a(A_DY);
  double* BX = c.a(A_BXW);
  const double *Q = c.a(A_Q), *RH = c.a(A_RHO), *Lo = c.a(A_L), *Up = c.a(A_U);
  double* ETA = c.a(A_PZ);  // eta = rho zp - y over all rows (scratch)
  long long* pf = (tid == 0) ? c.s->prof : nullptr;
  long long tq = pf ? clock64() : 0;
  // the generic step's loops run kGenU iterations per thread at once, all
  // loads before any store: the arrays are generic pointers (LDS or HBM per
  // the residency plan), so the compiler cannot hoist the next iteration's
  // loads above this one's stores and each iteration paid a full memory
  // round trip (config E: 14-DoF x 50 waypoints, ~4,300 rows)
  const int m = c.m(), nc = c.nc();
  GEN_UNROLL_BEGIN(kGenULight, m)
  for (int r0 = tid; r0 < (pre_ready ? 0 : m); r0 += U * kBlock)
  {
    double e[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int r = min(r0 + u * kBlock, m - 1);
      e[u] = RH[r] * zp[r] - Y[r];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r0 + u * kBlock < m)
        ETA[r0 + u * kBlock] = e[u];
  }
  GEN_UNROLL_END
  GEN_UNROLL_BEGIN(kGenULight, nc)
  for (int c0 = tid; c0 < (pre_ready ? 0 : nc); c0 += U * kBlock)
  {
    double e[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int col = min(c0 + u * kBlock, nc - 1);
      e[u] = sig * xp[col] - Q[col];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c0 + u * kBlock < nc)
        BX[c0 + u * kBlock] = e[u];
  }
  GEN_UNROLL_END
  BSYNC();
  if (pf)
    pf[30] += clock64() - tq;
  reduced_solve(c, sv, false, 0.0, ETA, XT);
  if (pf)
    tq = clock64();
  // z tilde = A x tilde; updates.  One loop per row kind (CartPose / fixed
  // rows, the columns' bound rows, hinge rows with their hinge variable's
  // bound row), each straight-line: a loop over all rows diverged into every
  // kind's branch in every wave and serialised their loads
  auto update_rows = [&](int rb, int re, auto zt_of, auto unroll) {
    constexpr int U = decltype(unroll)::value;  // rows per thread at once (see kGenU)
    for (int r0 = rb + tid; r0 < re; r0 += U * kBlock)
    {
      double zt[U], rh[U], yv[U], zv[U], lo[U], up[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        const int r = min(r0 + u * kBlock, re - 1);  // clamped: every load valid
        zt[u] = zt_of(r);
        rh[u] = RH[r];
        yv[u] = Y[r];
        zv[u] = zp[r];
        lo[u] = Lo[r];
        up[u] = Up[r];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        const int r = r0 + u * kBlock;
        if (r >= re)
          break;
        const double rho = rh[u];
        double zr = (1.0 / rho) * yv[u];
        zr = zr + al * zt[u];
        zr = zr + (1.0 - al) * zv[u];
        zr = fmin(fmax(zr, lo[u]), up[u]);
        z[r] = zr;
        const double dy = rho * (al * zt[u] + (1.0 - al) * zv[u] - zr);
        DY[r] = dy;
        const double yn = yv[u] + dy;
        Y[r] = yn;
        ETA[r] = rho * zr - yn;  // the next step's rho zp - y (same expression)
      }
    }
  };
  const Layout& L = c.L;
  const int D = L.D, nx = L.nx, nfr = L.n_fixed_rows, n_rows = L.n_rows, m_base = L.m_base, nc_base = L.nc_base;
  const double *FS = c.a(A_FS), *GS = c.a(A_GS), *WS = c.a(A_WS), *BS = c.a(A_BS);
  const int *row_step = c.T.row_step, *fixed_steps = c.d->fixed_steps, *row_off = c.T.row_off;
  const int nbr = L.nbr, sD = L.sD;
  // row_ax() for the fixed and CartPose rows, on the hoisted values (same expressions)
  auto row_ax_l = [&](int r) {
    if (r < nfr)
    {
      const int slot = r / D, j = r % D;
      return FS[r] * XT[fixed_steps[slot] * D + j];
    }
    const int a = r - nfr;
    const int t = row_step[a];
    double v;
    if (nbr > 1)  // the row's branch only (exact zeros elsewhere)
    {
      const int o = row_off[a];
      v = masked_dot<kOct>(GS + a * D + o, 1, XT + t * D + o, 1, 0, sD);
    }
    else
      v = (D > kOct) ? masked_dot<THIP_MAX_DOF>(GS + a * D, 1, XT + t * D, 1, 0, D)
                     : masked_dot<kOct>(GS + a * D, 1, XT + t * D, 1, 0, D);
    const int ca = nx + 2 * a;
    v += WS[2 * a] * XT[ca] + WS[2 * a + 1] * XT[ca + 1];
    return v;
  };
  GEN_UNROLL_BEGIN(kGenUHeavy, n_rows) update_rows(0, n_rows, row_ax_l, std::integral_constant<int, U>()); GEN_UNROLL_END
  {
    GEN_UNROLL_BEGIN(kGenULight, m_base - n_rows)
    update_rows(n_rows, m_base, [&](int r) { return BS[r - n_rows] * XT[r - n_rows]; },
                std::integral_constant<int, U>());
    GEN_UNROLL_END
    if (m > m_base)
    {
      // hinge row m_base + 2h: a_t.x_t + a_t+1.x_t+1 + w h; m_base + 2h + 1:
      // the bound row of h.  One thread per hinge variable updates both rows
      // (a loop over the rows alternated the two kinds lane by lane)
      const double *HC = c.a(A_HC), *HW = c.a(A_HW);
      const int* HT = c.ia(I_HT);
      const int nh = (m - m_base) >> 1;
      for (int h = tid; h < nh; h += kBlock)
      {
        const int col = nc_base + h, r0 = m_base + 2 * h;
        const double xh = XT[col];
        // (reusing the back-substitution's a.x here -- the same x columns --
        // broke torso_arm_8dof_C problem 2 deterministically: cause not found)
        const double zt2[2] = { hinge_dot(HC + h * 2 * D, XT + HT[h] * D, D) + HW[h] * xh, BS[col] * xh };
        double rh[2], yv[2], zv[2], lo[2], up[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
        {
          rh[u] = RH[r0 + u];
          yv[u] = Y[r0 + u];
          zv[u] = zp[r0 + u];
          lo[u] = Lo[r0 + u];
          up[u] = Up[r0 + u];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
        {
          const int r = r0 + u;
          const double rho = rh[u];
          double zr = (1.0 / rho) * yv[u];
          zr = zr + al * zt2[u];
          zr = zr + (1.0 - al) * zv[u];
          zr = fmin(fmax(zr, lo[u]), up[u]);
          z[r] = zr;
          const double dy = rho * (al * zt2[u] + (1.0 - al) * zv[u] - zr);
          DY[r] = dy;
          const double yn = yv[u] + dy;
          Y[r] = yn;
          ETA[r] = rho * zr - yn;
        }
      }
    }
  }
  GEN_UNROLL_BEGIN(kGenULight, nc)
  for (int c0 = tid; c0 < nc; c0 += U * kBlock)
  {
    double xt[U], xo[U], qv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int col = min(c0 + u * kBlock, nc - 1);
      xt[u] = XT[col];
      xo[u] = xp[col];
      qv[u] = Q[col];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const int col = c0 + u * kBlock;
      if (col >= nc)
        break;
      const double xv = al * xt[u] + (1.0 - al) * xo[u];
      x[col] = xv;
      DX[col] = xv - xo[u];
      BX[col] = sig * xv - qv[u];  // the next step's sigma xp - q (same expression)
    }
  }
  GEN_UNROLL_END
  BSYNC();
  if (pf)
    pf[31] += clock64() - tq;
}

#if !THIP_GENERIC_ONLY
// ======================================================================
// Register-resident ADMM segment (the hot loop)
// ======================================================================
// Runs n_iter ADMM iterations with the per-QP constants and the x/z/y state
// of every owned row/column in registers; only the coupling values travel
// through LDS.  Ownership (static for the whole segment):
//   column slot q = tid + kBlock*u  -> waypoint t = q / 8, dof i = q % 8:
//       x column (t, i), its bound row and its fixed-timestep row;
//   abs slot    a = tid + kBlock*u  -> CartPose row a, its two aux columns
//       and their bound rows.
// Per iteration: A (abs rows: row multipliers MR), B (columns: waypoint rhs
// and Linv_t b_t, gathered inside each lane octet), forward chain, Linv_t^T,
// backward chain, E (aux back-substitution, z~ = A x~, relaxed z/y/x
// updates).  The arithmetic (operation order and expression shapes) is that
// of admm_step() + reduced_solve(), so both paths give identical iterates.
// State is written back to A_XA0/A_Z0/A_Y/A_DX/A_DY at the end of the segment
// for the residual / termination / rho-update / polish code.
// ---- fused twisted solve of the ADMM segment ------------------------------
// K x = b with the twisted block factor (factor()), one pass per half on the
// two chain waves, the factor's blocks in registers for the whole segment:
//   forward   y_t = LI_t b_t - M_t y_{t-1}     (top half; bottom: y_{t+1})
//   middle    y_m = LI_m b_m - M_m y_{m-1} - M'_m y_{m+1},  x_m = LI_m^T y_m
//   backward  x_t = LI_t^T y_t - N_t x_{t+1}   (top half; bottom: x_{t-1})
// Each step is one lane-level fma and one 3-level reduction: lane (i, k) =
// (lane >> 3, lane & 7) holds one block element, the LI_t b_t and LI_t^T y_t
// terms enter the same reduction as the chain term (computed off the serial
// path), and the vector alternates between ROW layout (v[i] in octet i, from
// octet_sum) and COL layout (v[k] at lane & 7 = k, from cross_octet_sum), so
// no lane permutation sits on the serial path.  Steps of a half are indexed by
// r = distance from the middle (t = m - 1 - r on wave 0, m + 1 + r on wave
// 1): forward outputs are COL at even r, ROW at odd r; backward outputs the
// opposite, which is the layout the forward pass left y_t in; the middle
// reads y_{m-1}, y_{m+1}, b_m in COL layout, so both waves compute it
// identically.  This replaces reduced_solve's four barrier-separated passes
// (LI b, forward chain, LI^T y + middle, backward chain) by two.
static_assert(kCpkSteps * 2 * 8 >= kBlock, "segment halves cover N <= 32");

// The middle block's elements in the lane's layout (ROW output), fixed for a
// segment, and the half's length.
struct SegChain
{
  double mli, mm, mnb;  // LI_m, M_m, M'_m elements
  int R;                // steps in this wave's half (0 off the chain waves)
  int D, m, lane, wave;
  lds_f64* P;           // the chain pack (A_CPK)
  lds_f64* XV;          // x out (A_CV)
};

// Fill the chain pack (layout.hpp kCpk*) from the factor's blocks: step r of
// half h is waypoint t = m - 1 - r (h = 0) or m + 1 + r (h = 1); lane (i, k)
// of a COL-output step (even r) holds element (k, i) of LI_t and M_t, of a
// ROW-output step (odd r) element (i, k); the backward block N'_t the other
// way round.  Entries past the half's length, outside the D x D block, and the
// right-hand-side slots are zero.  All threads; ends with a barrier.
__device__ void seg_chain_pack(const Ctx& c, const Solver& sv, SegChain& ch)
{
  const int D = c.L.D, DD = D * D, N = c.L.N, m = c.L.tw_mid;
  lds_f64* P = lds(c.a(A_CPK));
  const lds_f64* LI = lds(c.a(A_LINV));
  const double* M = sv.M;  // LDS or HBM (Layout::chm_hbm): generic loads, once per segment
  const double* Nb = sv.Nb;
  const int Rh[2] = { m, N - 1 - m };
  for (int e = c.tid; e < 2 * kCpkSteps * 64; e += kBlock)
  {
    const int h = e / (kCpkSteps * 64), r = (e / 64) % kCpkSteps, lane = e & 63;
    const int i = lane >> 3, k = lane & 7;
    double li = 0.0, mf = 0.0, nb = 0.0;
    if (r < Rh[h] && i < D && k < D)
    {
      const int t = (h == 0) ? m - 1 - r : m + 1 + r;
      const int offN = t * DD + i * D + k, offT = t * DD + k * D + i;
      li = LI[(r & 1) ? offN : offT];
      mf = M[(r & 1) ? offN : offT];
      nb = Nb[(r & 1) ? offT : offN];
    }
    P[kCpkLM + 2 * e] = li;
    P[kCpkLM + 2 * e + 1] = mf;
    P[kCpkNB + e] = nb;
  }
  for (int e = c.tid; e < kCpk - kCpkB; e += kBlock)
    P[kCpkB + e] = 0.0;
  {
    const int i = c.lane >> 3, k = c.lane & 7;
    const bool act = (i < D) && (k < D);
    const int offN = i * D + k;
    ch.R = (c.wave < 2) ? Rh[c.wave] : 0;
    ch.D = D;
    ch.m = m;
    ch.lane = c.lane;
    ch.wave = c.wave;
    ch.P = P;
    ch.XV = lds(c.a(A_CV));
    const bool top = m > 0, bot = N - 1 - m > 0;
    ch.mli = act ? LI[m * DD + offN] : 0.0;
    ch.mm = (act && top) ? M[m * DD + offN] : 0.0;
    ch.mnb = (act && bot) ? Nb[m * DD + offN] : 0.0;
  }
  BSYNC();
}

// the pack slot of column (t, i)'s right-hand side (phase B writes it there)
__device__ __forceinline__ int seg_b_slot(int t, int i, int m)
{
  if (t < m)
    return kCpkB + (m - 1 - t) * 8 + i;
  if (t > m)
    return kCpkB + kCpkSteps * 8 + (t - m - 1) * 8 + i;
  return kCpkBM + i;
}

// x = K^-1 b: b in the pack (phase B), x into XV.  Ends with every wave past a
// workgroup barrier.  Both halves run kCpkSteps steps with no branches: the
// steps r >= R of a shorter half read zero blocks and a zero right-hand side
// and produce exact zeros, so y enters the first real step as 0 (the
// recurrence's start) and the real steps' arithmetic is unchanged.  Every load
// is one LDS instruction from a per-lane base with an immediate offset (the
// pack's lane order), and the forward pass loads the (LI, M) pair of a step
// as one 16-byte read; the next group of kSegGroup steps is loaded while the
// current group runs, and the backward pass's blocks are loaded before the
// barrier between the passes (their latency overlaps the wait for the other
// half).
constexpr int kSegGroup = 4;
static_assert(kCpkSteps % kSegGroup == 0, "chain groups");
typedef __attribute__((ext_vector_type(2))) double dbl2;
typedef __attribute__((address_space(3))) dbl2 lds_dbl2;

__device__ __forceinline__ void seg_chain_solve(const SegChain& ch, long long& lap_fwd, long long& lap_bwd,
                                                long long* pf, long long& tq, long long& own_fwd, long long& own_bwd)
{
  const int D = ch.D, m = ch.m, lane = ch.lane, wave = ch.wave;
  const int i = lane >> 3, k = lane & 7;
  const int ic = (i < D) ? i : D - 1, kc = (k < D) ? k : D - 1;
  lds_f64* P = ch.P;
  lds_f64* XV = ch.XV;
  const int R = __builtin_amdgcn_readfirstlane(ch.R);  // wave-uniform
  const int h = (wave == 1) ? 1 : 0;
  const int tdir = (wave == 0) ? -1 : 1;               // t = m + tdir * (1 + r)
  double q[kCpkSteps];
  double nb[kCpkSteps];  // the backward blocks, loaded before the barrier (their latency hides in its wait)
  double y = 0.0;
  if (wave < 2)
  {
    const lds_dbl2* LMp = (const lds_dbl2*)(P + kCpkLM + h * kCpkSteps * 128) + lane;  // + r * 64
    const lds_f64* Be = P + kCpkB + h * kCpkSteps * 8 + ic;                              // + r * 8, even r
    const lds_f64* Bo = P + kCpkB + h * kCpkSteps * 8 + kc;                              // odd r
    dbl2 lm[kCpkSteps];
    double lb[kCpkSteps];
    auto load = [&](int r) {
      lm[r] = LMp[r * 64];
      lb[r] = (r & 1) ? Bo[r * 8] : Be[r * 8];
    };
#pragma unroll
    for (int u = 0; u < kSegGroup; ++u)
      load(kCpkSteps - 1 - u);
#pragma unroll
    for (int g = 0; g < kCpkSteps / kSegGroup; ++g)
    {
      if (g + 1 < kCpkSteps / kSegGroup)
      {
#pragma unroll
        for (int u = 0; u < kSegGroup; ++u)
          load(kCpkSteps - 1 - kSegGroup * (g + 1) - u);
      }
      // the LI_t b_t products of the group, off the serial path
      double lib[kSegGroup];
#pragma unroll
      for (int u = 0; u < kSegGroup; ++u)
      {
        const int r = kCpkSteps - 1 - kSegGroup * g - u;
        lib[u] = lm[r].x * lb[r];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < kSegGroup; ++u)
      {
        const int r = kCpkSteps - 1 - kSegGroup * g - u;
        const double p = fma(-lm[r].y, y, lib[u]);
        y = (r & 1) ? octet_sum(p) : cross_octet_sum(p);
        q[r] = lm[r].x * y;  // the backward step's LI^T y term
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // y_{m -+ 1} (COL layout) to the middle
    if (i == 0 && k < D)
      P[kCpkYM + h * 8 + k] = y;
    const lds_f64* NBp = P + kCpkNB + h * kCpkSteps * 64 + lane;  // + r * 64
#pragma unroll
    for (int r = 0; r < kCpkSteps; ++r)
      nb[r] = NBp[r * 64];
  }
  if (pf)
    own_fwd += clock64() - tq;  // wave 0's own forward half, without the barrier
  BSYNC();
  if (pf)
  {
    const long long tn = clock64();
    lap_fwd += tn - tq;
    tq = tn;
  }
  if (wave < 2)
  {
    // the middle's operands first: the LDS returns in order (a missing half
    // has a zero hand-off slot and a zero M_m / M'_m)
    const double ym1 = P[kCpkYM + kc];
    const double yp1 = P[kCpkYM + 8 + kc];
    const double bm = P[kCpkBM + kc];
    __builtin_amdgcn_sched_barrier(0);
    const double p = fma(-ch.mnb, yp1, fma(-ch.mm, ym1, ch.mli * bm));
    const double ym = octet_sum(p);           // ROW
    double x = cross_octet_sum(ch.mli * ym);  // x_m, COL
    if (wave == 0 && i == 0 && k < D)
      XV[m * D + k] = x;
    __builtin_amdgcn_sched_barrier(0);
    double xs[kCpkSteps];
#pragma unroll
    for (int r = 0; r < kCpkSteps; ++r)
    {
      const double p2 = fma(-nb[r], x, q[r]);
      x = (r & 1) ? cross_octet_sum(p2) : octet_sum(p2);
      xs[r] = x;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < kCpkSteps; ++r)
      if (r < R)
      {
        const int t = m + tdir * (1 + r);
        if (r & 1)
        {
          if (i == 0 && k < D)
            XV[t * D + k] = xs[r];
        }
        else if (k == 0 && i < D)
          XV[t * D + i] = xs[r];
      }
  }
  if (pf)
    own_bwd += clock64() - tq;
  BSYNC();
  if (pf)
  {
    const long long tn = clock64();
    lap_bwd += tn - tq;
    tq = tn;
  }
}

// rinv = 1 / rho, precomputed per segment (OSQP keeps rho_inv_vec)
__device__ __forceinline__ void admm_row_update(double& z, double& y, double& dy, double zt, double rho, double rinv,
                                                double lo, double up, double al)
{
  double zr = rinv * y;
  zr = zr + al * zt;
  zr = zr + (1.0 - al) * z;
  zr = fmin(fmax(zr, lo), up);
  dy = rho * (al * zt + (1.0 - al) * z - zr);
  y += dy;
  z = zr;
}

template <int CS, int AS>
__device__ void admm_segment(Ctx& c, Solver& sv, int n_iter, Norms* res)
{
  PROF(0);
  // the Ctx fields the iterations use, in registers: the Ctx itself lives in
  // private memory and is re-read with dependent FLAT loads after every store
  // the compiler cannot prove does not alias it
  const int tid = c.tid;
  const Layout& L = c.L;
  const int D = L.D, N = L.N, nx = L.nx, nfr = L.n_fixed_rows, nr = L.n_rows;
  const thip_osqp_settings& os = c.d->osqp;
  const double sig = os.sigma, al = os.alpha;
  double *XA = c.a(A_XA0), *Z = c.a(A_Z0), *Y = c.a(A_Y), *DX = c.a(A_DX), *DY = c.a(A_DY);
  const double *Q = c.a(A_Q), *BS = c.a(A_BS), *RH = c.a(A_RHO), *Lo = c.a(A_L), *Up = c.a(A_U);
  const double *FS = c.a(A_FS), *GS = c.a(A_GS), *WS = c.a(A_WS), *DG = c.a(A_DG);
  double *MR = c.a(A_MR), *CV = c.a(A_CV), *YV = c.a(A_YV);
  // hinge rows (collision, config C): owned by h = tid + kBlock*j, state kept
  // in the planned arrays (LDS-resident under plan_lds_dynamic)
  const int nh = c.s->n_h;
  const int mb = L.m_base, ncb = L.nc_base;
  const double *HC = c.a(A_HC), *HW = c.a(A_HW);
  const int* HT = c.ia(I_HT);
  double* HPK = c.a(A_HPK);
#define HP_(f) HPK[(f) * nh + h]
  // pack fields: 0 z, 1 z_bound, 2 y, 3 y_bound, 4 x (hinge variable), 5 u,
  // 6 DG, 7 w, 8 bound-row coefficient, 9 q, 10 rn, 11 eta (A -> E scratch),
  // 12 first x column, 13 1 / (DG + rho w^2).  Both rows of a hinge are
  // inequalities (u finite, l = -inf; bound row l = 0, u = +inf), so their
  // rho is the scalar rho (set_rho_vec) and only the finite bounds are kept.
  const double rho_s = c.s->rho, rho_si = 1.0 / rho_s;
  for (int h = tid; h < nh; h += kBlock)
  {
    const int rh = mb + 2 * h, rb = rh + 1, col = ncb + h;
    HP_(0) = Z[rh];
    HP_(1) = Z[rb];
    HP_(2) = Y[rh];
    HP_(3) = Y[rb];
    HP_(4) = XA[col];
    HP_(5) = Up[rh];
    HP_(6) = DG[col];
    HP_(7) = HW[h];
    HP_(8) = BS[col];
    HP_(9) = Q[col];
    HP_(12) = static_cast<double>(HT[h] * D);
    HP_(13) = 1.0 / (DG[col] + rho_s * HW[h] * HW[h]);
  }
  // field-major copy of the hinge coefficients (odd stride)
  const int nhs = nh | 1;
  double* HCT = c.a(A_HCT);
  FOR(e, nh * 2 * D)
  {
    const int h = e / (2 * D), k = e - h * 2 * D;
    HCT[k * nhs + h] = HC[e];
  }
  // hinge chunk table: chunks of kHChunk rows inside each step pair
  int* CHK = reinterpret_cast<int*>(c.a(A_HCHK));
  double* PART = c.a(A_HPART);
  const int nchk = build_hinge_chunks(c);
  if (tid == 0)
    c.s->cur = 0;
  // MR, the chunk table and the chunk sums are LDS-resident (qp_solve checks
  // it): ds_* instructions.  The pack and HCT are LDS-resident when the QP's
  // plan has room for them, else in HBM: each hinge phase is instantiated
  // for both pointer kinds (a generic pointer would make every access a FLAT
  // instruction, which pays the vector-memory latency even on LDS).
  lds_f64* const MRl = lds(MR);
  const lds_f64* const PARTl = lds(static_cast<const double*>(PART));
  lds_f64* const PARTlw = lds(PART);
  const int* const CHKc = CHK;
  const __attribute__((address_space(3))) int* const CHKl = (const __attribute__((address_space(3))) int*)CHKc;
  const bool pk_l = lds_resident(c, HPK), hct_l = lds_resident(c, HCT);
  // phase A, hinge rows: multipliers MR_h; rn, eta kept in the pack
  auto hinge_a = [&](auto PKP) {
    for (int h = tid; h < nh; h += kBlock)
    {
      const double zh = PKP[h], zb = PKP[nh + h], yh = PKP[2 * nh + h], yb = PKP[3 * nh + h];
      const double xa = PKP[4 * nh + h], dn = PKP[6 * nh + h], w = PKP[7 * nh + h], bs = PKP[8 * nh + h];
      const double q = PKP[9 * nh + h], deni = PKP[13 * nh + h];
      const double eta = rho_s * zh - yh;
      const double rn = (sig * xa - q) + bs * (rho_s * zb - yb);
      MRl[nr + h] = (eta * dn - rho_s * w * rn) * deni;
      PKP[10 * nh + h] = rn;
      PKP[11 * nh + h] = eta;
    }
  };
  // phase B': hinge-row share of the waypoint rhs, row-parallel: 16 lanes
  // per chunk, lane k sums HC[h][k] * MR_h over the chunk's rows
  auto hinge_gather_seg = [&](auto HTP) {
    const int k = tid & 15;
    if (k < 2 * D)
#pragma unroll 2
      for (int q = tid >> 4; q < nchk; q += kBlock / 16)
      {
        const int h0 = CHKl[2 * q], h1 = CHKl[2 * q + 1];
        double s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < kHChunk; i += 2)
        {
          const int ha = min(h0 + i, h1 - 1), hb = min(h0 + i + 1, h1 - 1);  // in bounds
          const double aa = HTP[k * nhs + ha], ma = MRl[nr + ha];
          const double ab = HTP[k * nhs + hb], mb2 = MRl[nr + hb];
          // masked by 0/1 multipliers, not selects (see masked_dot)
          s0 += aa * (ma * ((h0 + i < h1) ? 1.0 : 0.0));
          s1 += ab * (mb2 * ((h0 + i + 1 < h1) ? 1.0 : 0.0));
        }
        PARTlw[q * 16 + k] = s0 + s1;
      }
  };
  // phase E, hinge rows: hinge variable, z~ = A x~, relaxed z/y/x updates
  // (admm_row_update with the infinite bound dropped)
  auto hinge_e = [&](auto PKP, auto HTP, bool last) {
    for (int h = tid; h < nh; h += kBlock)
    {
      // every pack field is read before any store (the stores could alias
      // them as far as the compiler knows)
      const int t0 = static_cast<int>(PKP[12 * nh + h]);
      const double zh = PKP[h], zb = PKP[nh + h], yh = PKP[2 * nh + h], yb = PKP[3 * nh + h];
      const double xo = PKP[4 * nh + h], uh = PKP[5 * nh + h], w = PKP[7 * nh + h], bs = PKP[8 * nh + h];
      const double rn = PKP[10 * nh + h], eta = PKP[11 * nh + h], deni = PKP[13 * nh + h];
      double g0 = 0, g1 = 0;
      // clamped indices (always in bounds), masked accumulation: the loads
      // of all terms are in flight together
#pragma unroll
      for (int k = 0; k < kOct; ++k)
      {
        const int kk = (k < D) ? k : D - 1;
        const double a0 = HTP[kk * nhs + h], a1 = HTP[(D + kk) * nhs + h];
        const double x0 = lds(CV)[t0 + kk], x1 = lds(CV)[t0 + D + kk];
        const double mk = (k < D) ? 1.0 : 0.0;  // a 0/1 multiplier, not a select (see masked_dot)
        g0 += a0 * (x0 * mk);
        g1 += a1 * (x1 * mk);
      }
      const double g = g0 + g1;
      const double av = (rn + w * (eta - rho_s * g)) * deni;
      const double zth = g + w * av;
      double zr = rho_si * yh;
      zr = zr + al * zth;
      zr = zr + (1.0 - al) * zh;
      zr = fmin(zr, uh);
      const double dyh = rho_s * (al * zth + (1.0 - al) * zh - zr);
      const double ztb = bs * av;
      double zs = rho_si * yb;
      zs = zs + al * ztb;
      zs = zs + (1.0 - al) * zb;
      zs = fmax(zs, 0.0);
      const double dyb = rho_s * (al * ztb + (1.0 - al) * zb - zs);
      const double xv = al * av + (1.0 - al) * xo;
      PKP[h] = zr;
      PKP[nh + h] = zs;
      PKP[2 * nh + h] = yh + dyh;
      PKP[3 * nh + h] = yb + dyb;
      PKP[4 * nh + h] = xv;
      if (last)
      {
        const int rh = mb + 2 * h;
        DY[rh] = dyh;
        DY[rh + 1] = dyb;
        DX[ncb + h] = xv - xo;
      }
    }
  };

  // ---- column owners: constants + state
  bool cact[CS];
  int ccol[CS], cfr[CS], cnrow[CS], crow[CS][kMaxStepRows];
  int chp0[CS], chp1[CS], chp2[CS];  // hinge chunks of pair t-1: [chp0, chp1), of pair t: [chp1, chp2)
  double cq[CS], cbs[CS], clb[CS], cub[CS], crb[CS], cfs[CS], clf[CS], cuf[CS], crf[CS];
  double cx[CS], czb[CS], cyb[CS], czf[CS], cyf[CS], cdx[CS], cdyb[CS], cdyf[CS], crbi[CS], crfi[CS];
  double cgs[CS][kMaxStepRows];
#pragma unroll
  for (int u = 0; u < CS; ++u)
  {
    const int q = tid + kBlock * u;
    const int t = q >> 3, i = q & 7;
    cact[u] = (t < N) && (i < D);
    cfr[u] = -1;
    cnrow[u] = 0;
    chp0[u] = chp1[u] = chp2[u] = 0;
    if (cact[u] && nh > 0)
    {
      chp1[u] = c.s->hcp[t];
      chp2[u] = c.s->hcp[t + 1];
      chp0[u] = (t > 0) ? c.s->hcp[t - 1] : chp1[u];
    }
    if (cact[u])
    {
      const int col = t * D + i, br = nr + col;
      ccol[u] = col;
      cq[u] = Q[col];
      cbs[u] = BS[col];
      clb[u] = Lo[br];
      cub[u] = Up[br];
      crb[u] = RH[br];
      crbi[u] = 1.0 / crb[u];
      cx[u] = XA[col];
      czb[u] = Z[br];
      cyb[u] = Y[br];
      const int f = c.T.fixed_of_step[t];
      if (f >= 0)
      {
        const int fr = f * D + i;
        cfr[u] = fr;
        cfs[u] = FS[fr];
        clf[u] = Lo[fr];
        cuf[u] = Up[fr];
        crf[u] = RH[fr];
        crfi[u] = 1.0 / crf[u];
        czf[u] = Z[fr];
        cyf[u] = Y[fr];
      }
      const int p0 = c.T.step_ptr[t], p1 = c.T.step_ptr[t + 1];
      cnrow[u] = p1 - p0;
#pragma unroll
      for (int p = 0; p < kMaxStepRows; ++p)
        if (p < p1 - p0)
        {
          const int r = c.T.step_rows[p0 + p];
          crow[u][p] = r;
          cgs[u][p] = GS[r * D + i];
        }
    }
    cdx[u] = cdyb[u] = cdyf[u] = 0.0;
  }
  // ---- abs-row owners
  bool aact[AS];
  int at[AS];
  double arr[AS], alr[AS], aur[AS], awn[AS], awp[AS], adn[AS], adp[AS], adet[AS], ags[AS][kOct];
  double aqn[AS], aqp[AS], absn[AS], absp[AS], albn[AS], aubn[AS], arbn[AS], albp[AS], aubp[AS], arbp[AS];
  double axn[AS], axp[AS], azr[AS], ayr[AS], azbn[AS], aybn[AS], azbp[AS], aybp[AS];
  double adxn[AS], adxp[AS], adyr[AS], adybn[AS], adybp[AS];
  double arn[AS], arp[AS], aeta[AS], arri[AS], arbni[AS], arbpi[AS], adeti[AS];
#pragma unroll
  for (int u = 0; u < AS; ++u)
  {
    const int a = tid + kBlock * u;
    aact[u] = a < L.n_abs;
    if (aact[u])
    {
      const int r = nfr + a, ca = nx + 2 * a, brn = nr + ca, brp = brn + 1;
      at[u] = c.T.row_step[a];
      arr[u] = RH[r];
      alr[u] = Lo[r];
      aur[u] = Up[r];
      awn[u] = WS[2 * a];
      awp[u] = WS[2 * a + 1];
      adn[u] = DG[ca];
      adp[u] = DG[ca + 1];
      adet[u] = adn[u] * adp[u] + arr[u] * (adn[u] * awp[u] * awp[u] + adp[u] * awn[u] * awn[u]);
      adeti[u] = 1.0 / adet[u];
      arri[u] = 1.0 / arr[u];
#pragma unroll
      for (int j = 0; j < kOct; ++j)
        ags[u][j] = (j < D) ? GS[a * D + j] : 0.0;
      aqn[u] = Q[ca];
      aqp[u] = Q[ca + 1];
      absn[u] = BS[ca];
      absp[u] = BS[ca + 1];
      albn[u] = Lo[brn];
      aubn[u] = Up[brn];
      arbn[u] = RH[brn];
      albp[u] = Lo[brp];
      aubp[u] = Up[brp];
      arbp[u] = RH[brp];
      arbni[u] = 1.0 / arbn[u];
      arbpi[u] = 1.0 / arbp[u];
      axn[u] = XA[ca];
      axp[u] = XA[ca + 1];
      azr[u] = Z[r];
      ayr[u] = Y[r];
      azbn[u] = Z[brn];
      aybn[u] = Y[brn];
      azbp[u] = Z[brp];
      aybp[u] = Y[brp];
    }
    adxn[u] = adxp[u] = adyr[u] = adybn[u] = adybp[u] = 0.0;
  }
  // the chain pack of this factorisation (ends with a barrier)
  SegChain ch;
  seg_chain_pack(c, sv, ch);
  int cbslot[CS];  // pack slot of each owned column's right-hand side
#pragma unroll
  for (int u = 0; u < CS; ++u)
  {
    const int q = tid + kBlock * u;
    cbslot[u] = seg_b_slot(q >> 3, q & 7, L.tw_mid);
  }
  lds_f64* const CPKl = lds(c.a(A_CPK));

  // phase laps accumulate in registers and are flushed once per segment
  // (a global read-modify-write per lap would stall wave 0 inside the loop)
  long long* pf = (tid == 0) ? c.s->prof : nullptr;
  long long tq = pf ? clock64() : 0;
  long long lap8 = 0, lap9 = 0, lap10 = 0, lap11 = 0, lap15 = 0, lap16 = 0, lap17 = 0, lap18 = 0, lap34 = 0;
#define SEG_LAP(acc)                  \
  if (pf)                             \
  {                                   \
    const long long tn = clock64();   \
    acc += tn - tq;                   \
    tq = tn;                          \
  }
  for (int iter = 0; iter < n_iter; ++iter)
  {
    // A: CartPose rows -> MR (aux block eliminated, see reduced_solve)
#pragma unroll
    for (int u = 0; u < AS; ++u)
      if (aact[u])
      {
        const double bxn = sig * axn[u] - aqn[u];
        const double bxp = sig * axp[u] - aqp[u];
        const double ebn = arbn[u] * azbn[u] - aybn[u];
        const double ebp = arbp[u] * azbp[u] - aybp[u];
        aeta[u] = arr[u] * azr[u] - ayr[u];
        arn[u] = bxn + absn[u] * ebn;
        arp[u] = bxp + absp[u] * ebp;
        const double dn = adn[u], dp = adp[u], wn = awn[u], wp = awp[u], rr = arr[u];
        MRl[tid + kBlock * u] = (aeta[u] * dn * dp - rr * (wn * dp * arn[u] + wp * dn * arp[u])) * adeti[u];
      }
    if (nh > 0)
    {
      if (pk_l)
        hinge_a(lds(HPK));
      else
        hinge_a(gbl(HPK));
    }
    BSYNC();
    SEG_LAP(lap8);
    if (nh > 0)
    {
      if (hct_l)
        hinge_gather_seg(lds(static_cast<const double*>(HCT)));
      else
        hinge_gather_seg(gbl(static_cast<const double*>(HCT)));
      BSYNC();
    }
    SEG_LAP(lap17);
    // B: waypoint right-hand sides b -> YV
#pragma unroll
    for (int u = 0; u < CS; ++u)
    {
      if (cact[u])
      {
        const double bx = sig * cx[u] - cq[u];
        const double eb = crb[u] * czb[u] - cyb[u];
        double b = bx + cbs[u] * eb;
        if (cfr[u] >= 0)
        {
          const double ef = crf[u] * czf[u] - cyf[u];
          b += cfs[u] * ef;
        }
#pragma unroll
        for (int p = 0; p < kMaxStepRows; ++p)
          if (p < cnrow[u])
            b += cgs[u][p] * MRl[crow[u][p]];
        if (nh > 0)
        {
          const int j = (tid + kBlock * u) & 7;
          for (int q = chp1[u]; q < chp2[u]; ++q)
            b += PARTl[q * 16 + j];
          for (int q = chp0[u]; q < chp1[u]; ++q)
            b += PARTl[q * 16 + D + j];
        }
        CPKl[cbslot[u]] = b;
      }
    }
    BSYNC();
    SEG_LAP(lap15);
    // x~ = K^-1 b into CV: forward halves, middle + backward halves
    seg_chain_solve(ch, lap9, lap10, pf, tq, lap16, lap34);
    // E: back-substitution, z~ = A x~, relaxed updates
    const bool last = (iter == n_iter - 1);
#pragma unroll
    for (int u = 0; u < CS; ++u)
      if (cact[u])
      {
        const double xt = lds(CV)[ccol[u]];
        admm_row_update(czb[u], cyb[u], cdyb[u], cbs[u] * xt, crb[u], crbi[u], clb[u], cub[u], al);
        if (cfr[u] >= 0)
          admm_row_update(czf[u], cyf[u], cdyf[u], cfs[u] * xt, crf[u], crfi[u], clf[u], cuf[u], al);
        const double xv = al * xt + (1.0 - al) * cx[u];
        cdx[u] = xv - cx[u];
        cx[u] = xv;
      }
#pragma unroll
    for (int u = 0; u < AS; ++u)
      if (aact[u])
      {
        const int t = at[u];
        double g0 = 0, g1 = 0;
#pragma unroll
        for (int j = 0; j < kOct; ++j)
        {
          const double xv = lds(CV)[t * D + ((j < D) ? j : D - 1)];
          const double xm = xv * ((j < D) ? 1.0 : 0.0);  // a 0/1 multiplier, not a select
          if (j & 1)
            g1 += ags[u][j] * xm;
          else
            g0 += ags[u][j] * xm;
        }
        const double g = g0 + g1;
        const double dn = adn[u], dp = adp[u], wn = awn[u], wp = awp[u], rr = arr[u];
        const double rn = arn[u], rp = arp[u];
        const double deti = adeti[u];
        const double cross = wp * rn - wn * rp;
        const double h = aeta[u] - rr * g;
        const double an = (dp * rn + rr * wp * cross + wn * dp * h) * deti;
        const double ap = (dn * rp - rr * wn * cross + wp * dn * h) * deti;
        double zt = g;
        zt += wn * an + wp * ap;
        admm_row_update(azr[u], ayr[u], adyr[u], zt, rr, arri[u], alr[u], aur[u], al);
        admm_row_update(azbn[u], aybn[u], adybn[u], absn[u] * an, arbn[u], arbni[u], albn[u], aubn[u], al);
        admm_row_update(azbp[u], aybp[u], adybp[u], absp[u] * ap, arbp[u], arbpi[u], albp[u], aubp[u], al);
        const double xvn = al * an + (1.0 - al) * axn[u];
        const double xvp = al * ap + (1.0 - al) * axp[u];
        adxn[u] = xvn - axn[u];
        adxp[u] = xvp - axp[u];
        axn[u] = xvn;
        axp[u] = xvp;
      }
    SEG_LAP(lap11);
    if (nh > 0)
    {
      if (pk_l && hct_l)
        hinge_e(lds(HPK), lds(static_cast<const double*>(HCT)), last);
      else if (pk_l)
        hinge_e(lds(HPK), gbl(static_cast<const double*>(HCT)), last);
      else if (hct_l)
        hinge_e(gbl(HPK), lds(static_cast<const double*>(HCT)), last);
      else
        hinge_e(gbl(HPK), gbl(static_cast<const double*>(HCT)), last);
    }
    SEG_LAP(lap18);
  }
#undef SEG_LAP
  if (pf)
  {
    pf[8] += lap8;
    pf[9] += lap9;
    pf[10] += lap10;
    pf[11] += lap11;
    pf[15] += lap15;
    pf[16] += lap16;
    pf[34] += lap34;
    pf[17] += lap17;
    pf[18] += lap18;
  }
  // residuals at the segment's last iterate (compute_residuals' quantities,
  // with its arithmetic order), from the state in registers: x of the
  // waypoint columns into YV and y of the CartPose / hinge rows into MR, one
  // barrier, the hinge share of A'y as chunk sums (phase B's gather on y),
  // then every owner's rows (A x - z) and columns (q + P x + A'y)
  if (res)
  {
    PROF(1);
#pragma unroll
    for (int u = 0; u < CS; ++u)
      if (cact[u])
        lds(YV)[ccol[u]] = cx[u];
#pragma unroll
    for (int u = 0; u < AS; ++u)
      if (aact[u])
        MRl[tid + kBlock * u] = ayr[u];
    for (int h = tid; h < nh; h += kBlock)
      MRl[nr + h] = HPK[2 * nh + h];
    BSYNC();
    if (nh > 0)
    {
      if (hct_l)
        hinge_gather_seg(lds(static_cast<const double*>(HCT)));
      else
        hinge_gather_seg(gbl(static_cast<const double*>(HCT)));
      BSYNC();
    }
    const double *E = c.a(A_E), *DS = c.a(A_DS), *PD = c.a(A_PD), *PO = c.a(A_PO);
    // v[12] = max |E dy| and v[13] = max |D dx| over the clipped delta y / delta x
    // of the last iteration (is_primal_infeasible / is_dual_infeasible)
    double v[14] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };
    double lhs = 0.0, qdx = 0.0;
    auto inf_row = [&](double dy, double lo, double up, double e) {
      if (up > kInf * kMinScal)
        dy = (lo < -kInf * kMinScal) ? 0.0 : fmin(dy, 0.0);
      else if (lo < -kInf * kMinScal)
        dy = fmax(dy, 0.0);
      v[12] = fmax(v[12], fabs(e * dy));
      lhs += up * fmax(dy, 0.0) + lo * fmin(dy, 0.0);
    };
    auto inf_col = [&](double dx, double q, double ds) {
      v[13] = fmax(v[13], fabs(ds * dx));
      qdx += q * dx;
    };
    auto row_terms = [&](double ax, double z, double e) {
      const double pr = ax - z;
      const double einv = 1.0 / e;
      v[0] = fmax(v[0], fabs(einv * pr));
      v[1] = fmax(v[1], fabs(einv * z));
      v[2] = fmax(v[2], fabs(einv * ax));
      v[3] = fmax(v[3], fabs(pr));
      v[4] = fmax(v[4], fabs(z));
      v[5] = fmax(v[5], fabs(ax));
    };
    auto col_terms = [&](double q, double px, double aty, double ds) {
      const double dr = q + px + aty;
      const double dinv = 1.0 / ds;
      v[6] = fmax(v[6], fabs(dinv * dr));
      v[7] = fmax(v[7], fabs(dinv * q));
      v[8] = fmax(v[8], fabs(dinv * aty));
      v[9] = fmax(v[9], fabs(dinv * px));
      v[10] = fmax(v[10], fabs(dr));
      v[11] = fmax(v[11], fmax(fabs(q), fmax(fabs(aty), fabs(px))));
    };
#pragma unroll
    for (int u = 0; u < CS; ++u)
      if (cact[u])
      {
        const int col = ccol[u], br = nr + col, t = col / D;
        const double eb = E[br], ds = DS[col];
        row_terms(cbs[u] * cx[u], czb[u], eb);
        inf_row(cdyb[u], clb[u], cub[u], eb);
        inf_col(cdx[u], cq[u], ds);
        if (cfr[u] >= 0)
        {
          const double ef = E[cfr[u]];
          row_terms(cfs[u] * cx[u], czf[u], ef);
          inf_row(cdyf[u], clf[u], cuf[u], ef);
        }
        // col_px
        double px = PD[col] * cx[u];
        if (t < N - 1)
          px += PO[col] * lds(YV)[col + D];
        if (t > 0)
          px += PO[col - D] * lds(YV)[col - D];
        // col_aty (chunked)
        double aty = cbs[u] * cyb[u];
        if (cfr[u] >= 0)
          aty += cfs[u] * cyf[u];
#pragma unroll
        for (int p = 0; p < kMaxStepRows; ++p)
          if (p < cnrow[u])
            aty += cgs[u][p] * MRl[crow[u][p]];
        if (nh > 0)
        {
          const int j = (tid + kBlock * u) & 7;
          for (int q = chp1[u]; q < chp2[u]; ++q)
            aty += PARTl[q * 16 + j];
          for (int q = chp0[u]; q < chp1[u]; ++q)
            aty += PARTl[q * 16 + D + j];
        }
        col_terms(cq[u], px, aty, ds);
      }
#pragma unroll
    for (int u = 0; u < AS; ++u)
      if (aact[u])
      {
        const int a = tid + kBlock * u;
        const int r = nfr + a, ca = nx + 2 * a, brn = nr + ca, brp = brn + 1;
        const int t = at[u];
        double ax = 0;
#pragma unroll
        for (int j = 0; j < kOct; ++j)  // 0/1 multiplier, not a guard (see masked_dot)
          ax += ags[u][j] * (lds(YV)[t * D + min(j, D - 1)] * ((j < D) ? 1.0 : 0.0));
        ax += awn[u] * axn[u] + awp[u] * axp[u];
        const double er = E[r], en = E[brn], ep = E[brp], dn = DS[ca], dp = DS[ca + 1];
        row_terms(ax, azr[u], er);
        row_terms(absn[u] * axn[u], azbn[u], en);
        row_terms(absp[u] * axp[u], azbp[u], ep);
        col_terms(aqn[u], 0.0, absn[u] * aybn[u] + awn[u] * ayr[u], dn);
        col_terms(aqp[u], 0.0, absp[u] * aybp[u] + awp[u] * ayr[u], dp);
        inf_row(adyr[u], alr[u], aur[u], er);
        inf_row(adybn[u], albn[u], aubn[u], en);
        inf_row(adybp[u], albp[u], aubp[u], ep);
        inf_col(adxn[u], aqn[u], dn);
        inf_col(adxp[u], aqp[u], dp);
      }
    for (int h = tid; h < nh; h += kBlock)
    {
      const int rh = mb + 2 * h, col = ncb + h, t0 = static_cast<int>(HPK[12 * nh + h]);
      const double xh = HPK[4 * nh + h], wh = HPK[7 * nh + h], bsh = HPK[8 * nh + h];
      double ax = 0, ax1 = 0;
      for (int k = 0; k < D; ++k)
      {
        ax += HC[h * 2 * D + k] * lds(YV)[t0 + k];
        ax1 += HC[h * 2 * D + D + k] * lds(YV)[t0 + D + k];
      }
      ax = ax + ax1 + wh * xh;  // row_ax: hinge_dot + w h
      const double e0 = E[rh], e1 = E[rh + 1], ds = DS[col];
      row_terms(ax, HPK[h], e0);
      row_terms(bsh * xh, HPK[nh + h], e1);
      col_terms(HPK[9 * nh + h], 0.0, bsh * HPK[3 * nh + h] + wh * HPK[2 * nh + h], ds);
      // (DY / DX of the last iteration, written by hinge_e)
      inf_row(DY[rh], Lo[rh], Up[rh], e0);
      inf_row(DY[rh + 1], Lo[rh + 1], Up[rh + 1], e1);
      inf_col(DX[col], HPK[9 * nh + h], ds);
    }
    block_max<14>(c, v);
    block_sum2(c, lhs, qdx);
    res->inf_ready = 1;
    res->ndy = v[12];
    res->lhs = lhs;
    res->ndx = v[13];
    res->qdx = qdx;
    res->prim_res = (c.m() > 0) ? v[0] : 0.0;
    res->zE = v[1];
    res->axE = v[2];
    res->pr = v[3];
    res->z = v[4];
    res->ax = v[5];
    res->dual_res = c.s->cinv * v[6];
    res->qD = v[7];
    res->atyD = v[8];
    res->pxD = v[9];
    res->dr = v[10];
    res->q = v[11];
  }
  // write back
#pragma unroll
  for (int u = 0; u < CS; ++u)
    if (cact[u])
    {
      const int col = ccol[u], br = nr + col;
      XA[col] = cx[u];
      DX[col] = cdx[u];
      Z[br] = czb[u];
      Y[br] = cyb[u];
      DY[br] = cdyb[u];
      if (cfr[u] >= 0)
      {
        Z[cfr[u]] = czf[u];
        Y[cfr[u]] = cyf[u];
        DY[cfr[u]] = cdyf[u];
      }
    }
#pragma unroll
  for (int u = 0; u < AS; ++u)
    if (aact[u])
    {
      const int a = tid + kBlock * u;
      const int r = nfr + a, ca = nx + 2 * a, brn = nr + ca, brp = brn + 1;
      XA[ca] = axn[u];
      XA[ca + 1] = axp[u];
      DX[ca] = adxn[u];
      DX[ca + 1] = adxp[u];
      Z[r] = azr[u];
      Y[r] = ayr[u];
      DY[r] = adyr[u];
      Z[brn] = azbn[u];
      Y[brn] = aybn[u];
      DY[brn] = adybn[u];
      Z[brp] = azbp[u];
      Y[brp] = aybp[u];
      DY[brp] = adybp[u];
    }
  for (int h = tid; h < nh; h += kBlock)
  {
    const int rh = mb + 2 * h;
    Z[rh] = HP_(0);
    Z[rh + 1] = HP_(1);
    Y[rh] = HP_(2);
    Y[rh + 1] = HP_(3);
    XA[ncb + h] = HP_(4);
  }
#undef HP_
  BSYNC();
}

__device__ void admm_iterations(Ctx& c, Solver& sv, int n_iter, Norms* res)
{
  admm_segment<1, 1>(c, sv, n_iter, res);
}

#endif  // !THIP_GENERIC_ONLY

__device__ double rho_estimate(Ctx& c, const Norms& nm)
{
  double pr = nm.pr, dr = nm.dr;
  const double prn = fmax(nm.z, nm.ax);
  pr /= (prn + kDivTol);
  const double drn = nm.q;
  dr /= (drn + kDivTol);
  double est = c.s->rho * sqrt(pr / (dr + kDivTol));
  return fmin(fmax(est, kRhoMin), kRhoMax);
}

// polish: returns nothing; updates x/z/y buffers on success
__device__ void polish(Ctx& c, Solver& sv, Norms& nm)
{
  PROF(4);
  const thip_osqp_settings& os = c.d->osqp;
  const double delta = os.delta;
  const int cur = c.s->cur;
  double* x = c.a(cur ? A_XA1 : A_XA0);
  double* z = c.a(cur ? A_Z1 : A_Z0);
  double* Y = c.a(A_Y);
  const double *Lo = c.a(A_L), *Up = c.a(A_U), *Q = c.a(A_Q);
  int* ACT = c.ia(I_ACT);
  const int m = c.m();
  // (the loops below are the plain per-row / per-column loops of OSQP's
  // polish, in the loads-first form of gen_loop / gen_rows_ax)
  gen_loop<kGenULight>(
      c, 0, m, [&](int r) { return RowV{ 0.0, z[r], Lo[r], Up[r], Y[r], 0 }; },
      [&](int r, const RowV& v) {
        int f = 0;
        if (v.a - v.b < -v.e)
          f = -1;
        else if (v.d - v.a < v.e)
          f = 1;
        ACT[r] = f;
      });
  BSYNC();
  if (!factor(c, sv, delta, true, delta))
  {
    if (c.tid == 0)
      c.s->polish_status = -1;
    BSYNC();
    return;
  }
  // PB = [b_x (n_cols); b_y (m)], PS = solution [x; y], PR = residual
  double *PB = c.a(A_PB), *PS = c.a(A_PS), *PR = c.a(A_PR), *PZ = c.a(A_PZ);
  double *BX = c.a(A_BXW), *XT = c.a(A_XT);
  const int nc = c.nc();
  gen_loop<kGenULight>(c, 0, nc, [&](int col) { return Q[col]; },
                       [&](int col, double q) {
                         PB[col] = -q;
                         PR[col] = -q;
                         PS[col] = 0.0;
                       });
  gen_loop<kGenULight>(
      c, 0, m, [&](int r) { return RowV{ 0.0, Lo[r], Up[r], 0.0, 0.0, ACT[r] }; },
      [&](int r, const RowV& v) {
        const double b = (v.act < 0) ? v.a : ((v.act > 0) ? v.b : 0.0);
        PB[nc + r] = b;
        PR[nc + r] = b;
        PS[nc + r] = 0.0;
      });
  BSYNC();
  // OSQP 1.0 polish: one solve with the delta-regularised KKT, then exactly
  // polish_refine_iter iterative-refinement steps on the unregularised KKT.
  // In exact arithmetic the refinement iterates depend only on K_delta^-1,
  // not on how it is applied (OSQP: LDL of the quasi-definite KKT; here the
  // waypoint-block normal equations), so the same step count reproduces
  // OSQP's polished point, including when 3 steps leave it inexact.
  const int max_refine = os.polish_refine_iter;
  const int nchk = (c.s->n_h > 0) ? build_hinge_chunks(c) : 0;
  for (int it = 0; it <= max_refine; ++it)
  {
    // solve K_delta d = PR  (rhs_x + A_act' r_y / delta), d_y = (A_act d_x - r_y) / delta
    double* eta = PZ;  // r_y / delta on active rows
    gen_loop<kGenULight>(
        c, 0, m, [&](int r) { return RowV{ 0.0, PR[nc + r], 0.0, 0.0, 0.0, ACT[r] }; },
        [&](int r, const RowV& v) { eta[r] = (v.act != 0) ? v.a / delta : 0.0; });
    gen_loop<kGenULight>(c, 0, nc, [&](int col) { return PR[col]; }, [&](int col, double v) { BX[col] = v; });
    BSYNC();
    reduced_solve(c, sv, true, delta, eta, XT);
    gen_loop<kGenULight>(
        c, 0, nc, [&](int col) { return RowV{ 0.0, PS[col], XT[col], 0.0, 0.0, 0 }; },
        [&](int col, const RowV& v) { PS[col] = v.a + v.b; });
    gen_rows_ax(
        c, XT, [&](int r, double ax) { return RowV{ ax, PR[nc + r], PS[nc + r], 0.0, 0.0, ACT[r] }; },
        [&](int r, const RowV& v) {
          if (v.act != 0)
            PS[nc + r] = v.b + (v.ax - v.a) / delta;
        });
    BSYNC();
    if (it == max_refine)
      break;
    // residual of the unregularised KKT: PR = PB - K [x; y] (the hinge share of
    // A'y from row-parallel chunk sums, as compute_residuals)
    if (nchk > 0)
      hinge_chunk_sums(c, PS + nc, nchk);
    gen_loop<kGenUHeavy>(
        c, 0, nc, [&](int col) { return PB[col] - col_px(c, col, PS) - col_aty(c, col, PS + nc, nchk > 0); },
        [&](int col, double v) { PR[col] = v; });
    gen_rows_ax(
        c, PS, [&](int r, double ax) { return RowV{ ax, PB[nc + r], 0.0, 0.0, 0.0, ACT[r] }; },
        [&](int r, const RowV& v) { PR[nc + r] = (v.act != 0) ? v.a - v.ax : 0.0; });
    BSYNC();
  }
  // polished point: x, z = A x, y (active) -> normal cone projection
  double* pz = PZ;
  double* py = PR + nc;  // reuse
  gen_rows_ax(
      c, PS, [&](int r, double ax) { return RowV{ ax, PS[nc + r], Lo[r], Up[r], 0.0, ACT[r] }; },
      [&](int r, const RowV& v) {
        const double yr = (v.act != 0) ? v.a : 0.0;
        const double tv = v.ax + yr;
        const double zc = fmin(fmax(tv, v.b), v.d);
        pz[r] = zc;
        py[r] = tv - zc;
      });
  BSYNC();
  Norms pn;
  compute_residuals(c, PS, pz, py, pn);
  const bool ok = (pn.prim_res < nm.prim_res && pn.dual_res < nm.dual_res) ||
                  (pn.prim_res < nm.prim_res && nm.dual_res < 1e-10) ||
                  (pn.dual_res < nm.dual_res && nm.prim_res < 1e-10);
  if (ok)
  {
    gen_loop<kGenULight>(c, 0, nc, [&](int col) { return PS[col]; }, [&](int col, double v) { x[col] = v; });
    gen_loop<kGenULight>(
        c, 0, m, [&](int r) { return RowV{ 0.0, pz[r], py[r], 0.0, 0.0, 0 }; },
        [&](int r, const RowV& v) {
          z[r] = v.a;
          Y[r] = v.b;
        });
    nm.prim_res = pn.prim_res;
    nm.dual_res = pn.dual_res;
  }
  if (c.tid == 0)
    c.s->polish_status = ok ? 1 : -1;
  BSYNC();
}

// One OSQPModel::optimize(): setup (bounds, rho, warm start, factor) + solve.
// Scaled P/A/q must be current (build_and_scale).  Trust-box bounds from X.
// Returns the CvxOptStatus.
__device__ int qp_solve(Ctx& c, Solver& sv, bool pattern_equal)
{
  PROF(12);
  const Layout& L = c.L;
  const int nx = L.nx, D = L.D;
  const thip_osqp_settings& os = c.d->osqp;
  const thip_chain& ch = g_chain;
  const double* X = c.a(A_X);
  double *Lo = c.a(A_L), *Up = c.a(A_U);
  const double *E = c.a(A_E), *GC = c.a(A_GC), *INIT = c.a(A_INIT), *DS = c.a(A_DS);
  // bounds (unscaled -> scaled by E)
  const double tb = c.s->trust;
  FOR(r, c.m())
  {
    double lo, up;
    int idx;
    const int kind = row_kind(L, r, idx);
    if (kind == RK_FIXED)
    {
      const int slot = r / D, j = r % D;
      lo = up = INIT[c.d->fixed_steps[slot] * D + j];
    }
    else if (kind == RK_ABS)
    {
      lo = up = -GC[idx];
    }
    else if (kind == RK_HINGE)
    {
      // ineq row viol - h <= 0: l = -inf, u = -(margin - k) (osqp_interface.cpp:213-281)
      lo = -kInf;
      if (c.ia(I_HKIND)[idx])
        up = -c.a(A_HK)[idx];  // affine row aff - h <= 0
      else
      {
        const double2 mc = row_pair_mc(c, idx);
        up = L.coll_cnt ? -((mc.x - c.a(A_HK)[idx]) * mc.y) : -(mc.x - c.a(A_HK)[idx]);
      }
    }
    else
    {
      const int col = idx;
      if (col < nx)
      {
        const int j = col % D;
        const double lb = ch.lower[j], ub = ch.upper[j];
        const double xi = fmin(fmax(X[col], lb), ub);  // std::clamp
        lo = fmax(xi - tb, lb);
        up = fmin(xi + tb, ub);
        lo = fmax(lo, -kInf);
        up = fmin(up, kInf);
      }
      else
      {
        lo = 0.0;
        up = kInf;
      }
    }
    Lo[r] = lo * E[r];
    Up[r] = up * E[r];
  }
  // warm start policy (osqp_interface.cpp:283-370)
  const bool warm = (c.s->prev_status == ST_SOLVED || c.s->prev_status == ST_SOLVED_INACC) && os.warm_starting &&
                    pattern_equal;
  if (c.tid == 0)
  {
    c.s->rho = fmin(fmax(warm ? c.s->prev_rho : os.rho, kRhoMin), kRhoMax);
    c.s->rho0 = c.s->rho;
    c.s->cur = 0;
    c.s->qp_status = ST_UNSOLVED;
    c.s->polish_status = 0;
  }
  BSYNC();
  set_rho_vec(c);
  double* x = c.a(A_XA0);
  double* z = c.a(A_Z0);
  double* Y = c.a(A_Y);
  const double *SX = c.a(A_SOLX), *SY = c.a(A_SOLY);
  if (warm)
  {
    FOR(col, c.nc()) x[col] = SX[col] * (1.0 / DS[col]);
    FOR(r, c.m()) Y[r] = (SY[r] * (1.0 / E[r])) * c.s->c;
    BSYNC();
    FOR(r, c.m()) z[r] = row_ax(c, r, x);
  }
  else
  {
    FOR(col, c.nc()) x[col] = 0.0;
    FOR(r, c.m())
    {
      z[r] = 0.0;
      Y[r] = 0.0;
    }
  }
  BSYNC();
  if (!factor(c, sv, os.sigma, false, 0.0))
  {
    // setup failure: CVX_FAILED, no workspace for the next warm start
    if (c.tid == 0)
    {
      c.s->prev_status = 0;
      if (c.s->trace && c.s->trace_n < c.s->trace_cap)
      {
        double* rec = c.s->trace + THIP_TRACE_W * c.s->trace_n++;
        for (int i = 0; i < THIP_TRACE_W; ++i)
          rec[i] = 0;
        rec[3] = -1;
        rec[9] = c.s->trust;
      }
    }
    BSYNC();
    return THIP_CVX_FAILED;
  }
  const int interval = (os.adaptive_rho == 1 && os.adaptive_rho_interval == 0) ?
                           (os.check_termination ? 4 * os.check_termination : 100) :
                           os.adaptive_rho_interval;
  Norms nm{};
  bool can_check = false, have_res = false;
  int it;
  bool fail = false;
  const int ct = os.check_termination;
  // the segment addresses MR, the hinge chunk table and chunk sums as LDS
#if THIP_GENERIC_ONLY
  const bool seg = false;  // (this build has no segment: its QPs run the generic step)
#else
  const bool seg = seg_path(c);
#endif
  bool pre_ready = false;  // admm_step's ETA / BX (cleared when rho changes)
  for (it = 1; it <= os.max_iter; ++it)
  {
    if (seg)
    {
      // register-resident segment up to the next iteration that checks
      // termination or adapts rho (same iterates as admm_step)
      int stop = os.max_iter;
      if (ct)
        stop = min(stop, (it + ct - 1) / ct * ct);
      if (os.adaptive_rho && interval)
        stop = min(stop, (it + interval - 1) / interval * interval);
      // the segment computes the residuals of its last iterate when they are needed
      const bool want = (ct && stop % ct == 0) || (os.adaptive_rho && interval && stop % interval == 0);
#if !THIP_GENERIC_ONLY
      admm_iterations(c, sv, stop - it + 1, want ? &nm : nullptr);
#endif
      have_res = want;
      it = stop;
    }
    else
    {
      admm_step(c, sv, pre_ready);
      pre_ready = true;
      have_res = false;
    }
    can_check = ct && (it % ct == 0);
    const int cur = c.s->cur;
    const double* xc = c.a(cur ? A_XA1 : A_XA0);
    const double* zc = c.a(cur ? A_Z1 : A_Z0);
    if (can_check)
    {
      if (!have_res)
        compute_residuals(c, xc, zc, Y, nm);
      if (check_termination(c, nm, false))
        break;
    }
    if (os.adaptive_rho && interval && (it % interval == 0))
    {
      if (!can_check && !have_res)
        compute_residuals(c, xc, zc, Y, nm);
      const double rn = rho_estimate(c, nm);
      const double rho = c.s->rho;
      if (rn > rho * os.adaptive_rho_tolerance || rn < rho / os.adaptive_rho_tolerance)
      {
        BSYNC();
        if (c.tid == 0)
          c.s->rho = fmin(fmax(rn, kRhoMin), kRhoMax);
        BSYNC();
        const double nr = c.s->rho;
        double* RH = c.a(A_RHO);
        const int* TY = c.ia(I_TYPE);
        FOR(r, c.m())
        {
          if (TY[r] == 0)
            RH[r] = nr;
          else if (TY[r] == 1)
            RH[r] = kRhoEq * nr;
        }
        BSYNC();
        pre_ready = false;  // ETA = rho zp - y changes with rho
        if (!factor(c, sv, os.sigma, false, 0.0))
        {
          fail = true;
          break;
        }
      }
    }
  }
  if (fail)
  {
    if (c.tid == 0)
    {
      c.s->qp_status = ST_NONCVX;
      c.s->prev_status = ST_NONCVX;
      c.s->iter = it;
    }
    BSYNC();
    return THIP_CVX_FAILED;
  }
  const int cur = c.s->cur;
  double* xc = c.a(cur ? A_XA1 : A_XA0);
  double* zc = c.a(cur ? A_Z1 : A_Z0);
  int iters = it;
  if (!can_check)
  {
    iters = it - 1;
    compute_residuals(c, xc, zc, Y, nm);
    check_termination(c, nm, false);
  }
  if (c.s->qp_status == ST_UNSOLVED)
  {
    if (!check_termination(c, nm, true))
    {
      if (c.tid == 0)
        c.s->qp_status = ST_MAXIT;
      BSYNC();
    }
  }
  if (os.polishing && c.s->qp_status == ST_SOLVED)
    polish(c, sv, nm);
  // store_solution (unscaled) -> warm-start memory
  const int st = c.s->qp_status;
  const bool inf = (st == ST_PINF || st == ST_PINF_INACC || st == ST_DINF || st == ST_DINF_INACC);
  double *SXw = c.a(A_SOLX), *SYw = c.a(A_SOLY);
  FOR(col, c.nc()) SXw[col] = inf ? NAN : DS[col] * xc[col];
  FOR(r, c.m()) SYw[r] = inf ? NAN : c.s->cinv * (E[r] * Y[r]);
  BSYNC();
  if (c.tid == 0)
  {
    c.s->prev_status = st;
    c.s->prev_rho = c.s->rho;
    c.s->iter = iters;
    c.s->n_admm += iters;
    c.s->n_hinge_admm += static_cast<long long>(c.s->n_h) * iters;
  }
  BSYNC();
  if (c.s->trace)
  {
    double xs = 0;
    FOR(col, c.nc()) xs += fabs(SXw[col]);
    xs = block_sum(c, xs);
    if (c.tid == 0 && c.s->trace_n < c.s->trace_cap)
    {
      double* rec = c.s->trace + THIP_TRACE_W * c.s->trace_n;
      for (int i = 10; i < THIP_TRACE_W; ++i)
        rec[i] = 0;
      rec[0] = warm ? 1.0 : 0.0;
      rec[1] = c.s->rho0;
      rec[2] = iters;
      rec[3] = st;
      rec[4] = c.s->polish_status;
      rec[5] = c.s->rho;
      rec[6] = nm.prim_res;
      rec[7] = nm.dual_res;
      rec[8] = xs;
      rec[9] = c.s->trust;
      c.s->trace_n++;
    }
    BSYNC();
  }
  if (st == ST_SOLVED || st == ST_SOLVED_INACC)
    return THIP_CVX_SOLVED;
  if (inf)
    return THIP_CVX_INFEASIBLE;
  return THIP_CVX_FAILED;
}

// ======================================================================
// Dynamic LDS residency plan (collision problems): the QP size changes with
// the contact count, so after every linearisation the QP-internal arrays are
// re-placed greedily (same priority order as the host plan, plus the hinge
// arrays) for the actual sizes.  Only arrays recomputed within the SQP
// iteration after this point are planned.
// ======================================================================
__device__ void plan_lds_dynamic(Ctx& c)
{
  if (!c.ptab_w)
    return;
  if (c.tid == 0)
  {
    const Layout& L = c.L;
    const long long nx = L.nx, nc = c.nc(), m = c.m(), nh = c.s->n_h, D = L.D;
    const long long NDD = (long long)L.sN * L.sD * L.sD, nab = L.n_abs > 0 ? L.n_abs : 1;
    // the ADMM segment's working set first (chains, rhs, multipliers, the
    // hinge-row pack and coefficients), then the rest as in the host plan
    const int order[] = { A_LINV, A_CV, A_YV, A_CPK, A_MR, A_HPART, A_HCHK, A_HCT, A_HPK, A_HC, A_BXW, A_BA, A_HW, A_HRE, A_DG, A_GS, A_WS,
                          A_FS,   A_BS, A_XA0, A_XA1, A_Z0, A_Z1, A_Y, A_XT, A_PZ, A_RHO, A_L,  A_U,  A_Q,
                          A_DX,   A_DY, A_PD,  A_PO,  A_PO2, A_E,  A_DS, A_RE, A_CPL, A_PB, A_PS, A_PR };
    long long used = L.lds_scratch;
    for (int k : order)
    {
      long long n;
      switch (k)
      {
        case A_LINV: case A_CPL: n = NDD; break;
        case A_CPK: n = (L.loff[A_CPK] >= 0) ? kCpk : 0; break;  // the host plan's offset
        case A_CV: case A_YV: case A_PD: case A_PO: n = nx; break;
        case A_PO2: n = (L.grp > 1) ? nx : 0; break;
        case A_MR: n = L.n_rows + nh; break;
        case A_RE: n = L.n_rows; break;
        case A_HC: n = nh * 2 * D; break;
        case A_HW: case A_HRE: n = nh; break;
        case A_HPK: n = nh * kHPack; break;
        case A_HCT: n = (nh | 1) * 2 * D; break;
        case A_HCHK: n = nh / kHChunk + L.N + 1; break;
        case A_HPART: n = (nh / kHChunk + L.N + 1) * L.part_w; break;
        case A_GS: n = nab * D; break;
        case A_WS: n = nab * 2; break;
        case A_FS: n = L.n_fixed_rows; break;
        case A_Z0: case A_Z1: case A_Y: case A_PZ: case A_RHO: case A_L: case A_U: case A_DY: case A_E: n = m; break;
        case A_PB: case A_PS: case A_PR: n = nc + m; break;
        default: n = nc; break;
      }
      n = (n + 7) / 8 * 8;
      if (n > 0 && used + n <= L.lds_budget)
      {
        c.ptab_w[k] = c.big + used;
        used += n;
      }
      else
        c.ptab_w[k] = c.w + L.doff[k];
    }
  }
  BSYNC();
}

// ======================================================================
// The SQP driver kernel: BasicTrustRegionSQP::optimize per workgroup
// ======================================================================
// OSQPModel's sparsity test (osqp_interface.cpp:199-201, 268-271, quirk Q2):
// the constraint matrix A counts as unchanged when n, m and nnz are equal and
// the first n + 1 BYTES of its 64-bit column pointers and the first nnz BYTES
// of its 64-bit row indices are equal -- a byte count used as an element
// count, so only a prefix of the pattern (about the first n / 8 column pointers
// and nnz / 8 row indices: the early waypoints) is ever compared.  This walks
// A in OSQPModel's CSC order (x columns waypoint-major, then the aux columns
// of the abs rows, then the hinge columns; rows fixed < abs < hinge < the
// identity block) and hashes exactly the compared prefix, byte-masked where a
// count ends inside a 64-bit element.  Thread 0 of the workgroup; the result is
// (n, m, nnz, hash) in the control block's fp_* fields.
__device__ __forceinline__ unsigned long long fp_mix(unsigned long long h, unsigned long long v)
{
  h ^= v + 0x9E3779B97F4A7C15ULL + (h << 6) + (h >> 2);
  return h * 0xBF58476D1CE4E5B9ULL;
}

__device__ void pattern_fingerprint(Ctx& c, unsigned long long& hash, int& n_out, int& m_out, long long& nnz_out)
{
  const Layout& L = c.L;
  const int D = L.D, nx = L.nx, nh = c.s->n_h, n = c.nc();
  const int *mask = c.ia(I_MASK), *HP = c.ia(I_HPTR), *HM = c.ia(I_HMASK);
  const int* fos = c.T.fixed_of_step;
  long long nnz = (long long)L.n_fixed_rows + 2LL * L.n_abs + nh + n;
  for (int r = 0; r < L.n_abs; ++r)
    nnz += __popc(mask[r]);
  for (int h = 0; h < nh; ++h)
    nnz += __popc(HM[h]);
  const long long row_hinge0 = L.n_rows, row_ident0 = (long long)L.n_rows + nh;
  // byte prefixes: p[0..(n+1)/8) whole + (n+1)%8 low bytes of the next; same for i with nnz
  const long long kp = (n + 1) / 8, kpr = (n + 1) % 8, ki = nnz / 8, kir = nnz % 8;
  auto low = [](unsigned long long v, long long bytes) {
    return bytes >= 8 ? v : (v & ((1ULL << (8 * bytes)) - 1ULL));
  };
  unsigned long long h = 0x6A09E667F3BCC908ULL;
  long long ptr = 0, e = 0;  // column pointer value, entry counter
  auto entry = [&](long long row) {
    if (e < ki)
      h = fp_mix(h, (unsigned long long)row);
    else if (e == ki && kir)
      h = fp_mix(h, low((unsigned long long)row, kir) ^ 0x5555ULL);
    ++e;
  };
  for (int col = 0; col <= n; ++col)
  {
    if (col < kp)
      h = fp_mix(h, (unsigned long long)ptr);
    else if (col == kp && kpr)
      h = fp_mix(h, low((unsigned long long)ptr, kpr) ^ 0xAAAAULL);
    if (col == n || (col >= kp && e > ki))
      break;
    const long long e0 = e;
    if (col < nx)
    {
      const int t = col / D, j = col % D;
      if (fos[t] >= 0)
        entry((long long)fos[t] * D + j);
      for (int q = c.T.step_ptr[t]; q < c.T.step_ptr[t + 1]; ++q)
      {
        const int r = c.T.step_rows[q];
        if ((mask[r] >> j) & 1)
          entry(L.n_fixed_rows + r);
      }
      if (L.hinge)
      {
        // hinge rows of step pair t - 1 (waypoint t is its second half) then of pair t
        if (t > 0)
          for (int hh = HP[t - 1]; hh < HP[t]; ++hh)
            if ((HM[hh] >> (D + j)) & 1)
              entry(row_hinge0 + hh);
        if (t < L.N - 1)
          for (int hh = HP[t]; hh < HP[t + 1]; ++hh)
            if ((HM[hh] >> j) & 1)
              entry(row_hinge0 + hh);
      }
    }
    else if (col < L.nc_base)
      entry(L.n_fixed_rows + (col - nx) / 2);  // neg / pos of abs row (col - nx) / 2
    else
      entry(row_hinge0 + (col - L.nc_base));   // the hinge variable of hinge row col - nc_base
    entry(row_ident0 + col);                    // identity block (variable bounds)
    ptr += e - e0;
  }
  hash = h;
  n_out = n;
  m_out = c.m();
  nnz_out = nnz;
}

__device__ void sqp_optimize(Ctx& c, Solver& sv)
{
  PROF(13);
  const Layout& L = c.L;
  const int nx = L.nx, D = L.D;
  const thip_sqp_params& P = c.d->sqp;
  double *X = c.a(A_X), *XN = c.a(A_XN);
  double *COST = c.a(A_COST), *VIOL = c.a(A_VIOL), *NCOST = c.a(A_NCOST), *NVIOL = c.a(A_NVIOL), *MU = c.a(A_MU);
  const thip_chain& ch = g_chain;
  // getClosestFeasiblePoint(x, 1e-3)
  FOR(col, nx)
  {
    const int j = col % D;
    const double lb = ch.lower[j], ub = ch.upper[j];
    const double inset = fmin(1e-3, (ub - lb) / 2);
    X[col] = fmin(fmax(X[col], lb + inset), ub - inset);
  }
  FOR(i, L.n_cnts) MU[i] = P.initial_merit_error_coeff;
  if (c.tid == 0)
  {
    c.s->trust = P.trust_box_size;
    c.s->status = THIP_OPT_INVALID;
    c.s->n_sqp = c.s->n_qp = c.s->n_fev = c.s->n_merit = 0;
    c.s->n_admm = 0;
    c.s->prev_status = 0;
    c.s->prev_rho = c.d->osqp.rho;
    c.s->n_h = 0;
    c.s->n_h_prev = -1;
    c.s->scan_at_x = 0;
    c.s->flags = 0;
    c.s->coll_overflow = 0;
    c.s->n_contact_rows = c.s->n_hinge_admm = c.s->n_substates = 0;
  }
  BSYNC();
  int* mask = c.ia(I_MASK);
  int* pmask = c.ia(I_PMASK);
  bool have_prev_setup = false;
  bool first_eval = true;
  int retval = THIP_OPT_INVALID;
  // cost / violation values before the first evaluation: an empty OptResults
  // (a time limit can end the run before it, optimizers.cpp:739-753)
  FOR(i, L.n_costs) COST[i] = 0.0;
  FOR(i, L.n_cnts) VIOL[i] = 0.0;
  const long long t_start = wall_clock64();
  for (int mi = 0; mi < P.max_merit_coeff_increases; ++mi)
  {
    bool goto_penalty = false, goto_cleanup = false;
    for (int iter = 1;; ++iter)
    {
      // time limit (optimizers.cpp:739-753), before the iteration body: the
      // problem's own clock since sqp_optimize began
      if (L.max_ticks != LLONG_MAX)
      {
        if (c.tid == 0)
          c.s->time_up = (wall_clock64() - t_start) > L.max_ticks ? 1 : 0;
        BSYNC();
        if (c.s->time_up)
        {
          retval = THIP_OPT_TIME_LIMIT;
          double vm = -INFINITY;
          for (int i = 0; i < L.n_cnts; ++i)
            vm = fmax(vm, VIOL[i]);
          if (first_eval || L.n_cnts == 0 || vm < P.cnt_tolerance)
            retval = THIP_OPT_CONVERGED;
          goto_cleanup = true;
          break;
        }
      }
      if (c.tid == 0)
        c.s->n_sqp++;
      if (first_eval)
      {
        evaluate(c, X, COST, VIOL);
        if (c.tid == 0)
          c.s->scan_at_x = 1;
        if (c.tid == 0)
          c.s->n_fev++;
        first_eval = false;
      }
      // convexify
      linearize(c, X);
      if (L.hinge)
        plan_lds_dynamic(c);
      build_and_scale(c);
      // pattern of A vs the previous QP setup, as OSQPModel tests it (quirk Q2)
      BSYNC();
      if (c.tid == 0)
      {
        unsigned long long fh;
        int fn, fm;
        long long fz;
        pattern_fingerprint(c, fh, fn, fm, fz);
        c.s->flag = (fn == c.s->fp_n && fm == c.s->fp_m && fz == c.s->fp_nnz && fh == c.s->fp_hash) ? 1 : 0;
        c.s->fp_n = fn;
        c.s->fp_m = fm;
        c.s->fp_nnz = fz;
        c.s->fp_hash = fh;
      }
      BSYNC();
      bool pattern_equal = have_prev_setup && c.s->flag == 1;
      BSYNC();
      FOR(r, L.n_abs) pmask[r] = mask[r];
      if (L.hinge)
      {
        const int *HT = c.ia(I_HT), *HM = c.ia(I_HMASK);
        int *PHT = c.ia(I_PHT), *PHM = c.ia(I_PHMASK);
        FOR(h, c.s->n_h)
        {
          PHT[h] = HT[h];
          PHM[h] = HM[h];
        }
        BSYNC();
        if (c.tid == 0)
          c.s->n_h_prev = c.s->n_h;
      }
      have_prev_setup = true;
      BSYNC();
      int qp_failures = 0;
      bool converged_inner = false, failed = false;
      while (c.s->trust >= P.min_trust_box_size)
      {
        const int st = qp_solve(c, sv, pattern_equal);
        pattern_equal = true;  // same P/A within this SQP iteration
        if (c.tid == 0)
          c.s->n_qp++;
        BSYNC();
        if (st != THIP_CVX_SOLVED)
        {
          if (qp_failures < P.max_qp_solver_failures - 1)
          {
            if (c.tid == 0)
              c.s->trust *= P.trust_shrink_ratio;
            BSYNC();
            ++qp_failures;
            continue;
          }
          if (qp_failures == P.max_qp_solver_failures - 1)
          {
            if (c.tid == 0)
              c.s->trust = P.min_trust_box_size;
            BSYNC();
            ++qp_failures;
            continue;
          }
          failed = true;
          break;
        }
        // model values at the QP solution (unscaled solution in A_SOLX)
        const double* SX = c.a(A_SOLX);
        FOR(col, nx) XN[col] = SX[col];
        BSYNC();
        // JointVel model value (quadratic, exact), CartPose model values
        double jvm = 0;
        if (c.d->jv_enabled && !L.jv_ineq)
        {
          const int nv = (L.jv_last - L.jv_first) * D;
          FOR(i, nv)
          {
            const int t = L.jv_first + i / D, j = i % D;
            const double dd = (XN[(t + 1) * D + j] - XN[t * D + j]) - c.d->jv_targets[j];
            jvm += (dd * dd) * c.d->jv_coeffs[j];
          }
        }
        jvm = block_sum(c, jvm);
        double* mcost = c.big;                 // [n_costs]
        double* mviol = c.big + L.n_costs;     // [n_cnts]
        if (c.tid == 0 && c.d->jv_enabled && !L.jv_ineq)
          mcost[0] = jvm;
        for (int k = 0; k < L.n_jacc; ++k)  // JointAccEqCost: quadratic, model = exact
        {
          const double v = jacc_value(c, XN, k);
          if (c.tid == 0)
            mcost[L.jacc_slot[k]] = v;
        }
        const double *G = c.a(A_G), *GC = c.a(A_GC);
        // JointPos: costs are quadratic (model = exact value), constraint
        // rows are abs rows like CartPose constraint rows (below)
        sh_model_values(c, SX, mcost, mviol);
        for (int k = 0; k < L.n_jpos; ++k)
        {
          if (c.d->jpos_is_cnt[k] || c.T.jpos_ineq[k])
            continue;
          const int f = c.T.jpos_first[k], n = (c.T.jpos_last[k] - f + 1) * D;
          double v = 0;
          FOR(i, n)
          {
            const int t = f + i / D, j = i % D;
            const double dd = XN[t * D + j] - c.jpt[k * D + j];
            v += (dd * dd) * c.d->jpos_coeffs[k][j];
          }
          v = block_sum(c, v);
          if (c.tid == 0)
            mcost[c.T.jpos_slot[k]] = v;
        }
        FOR(k, L.n_cart + L.n_jpos)
        {
          const bool jp = k >= L.n_cart;
          const int kk = jp ? k - L.n_cart : k;
          if (jp && (!c.d->jpos_is_cnt[kk] || c.T.jpos_ineq[kk]))
            continue;
          const int r0 = jp ? c.T.jpos_row0[kk] : c.T.term_row0[k], nr = jp ? c.T.jpos_nrow[kk] : c.T.term_nrow[k];
          double v = 0;
          if (jp || c.d->cart_is_cnt[k])
          {
            for (int rr = 0; rr < nr; ++rr)
            {
              const int row = r0 + rr;
              const int t = c.T.row_step[row];
              double a = GC[row];
              for (int j = 0; j < D; ++j)
                if (mask[row] & (1 << j))
                  a += G[row * D + j] * XN[t * D + j];
              v += fabs(a);
            }
            mviol[jp ? c.T.jpos_slot[kk] : c.T.term_slot[k]] = v;
          }
          else
          {
            for (int rr = 0; rr < nr; ++rr)
            {
              const int ca = nx + 2 * (r0 + rr);
              v += SX[ca];
              v += SX[ca + 1];
            }
            mcost[c.T.term_slot[k]] = v;
          }
        }
        if (L.coll)
        {
          // ConvexObjective::value of each step-pair term: sum coeff * h
          const int* HP = c.ia(I_HPTR);
          const int* HTv = c.ia(I_HT);
          const int* CONTv = c.ia(I_CONT);
          FOR(k, L.coll_last - L.coll_first)
          {
            const int u = L.coll_first + k, slot = c.T.coll_slot[u];
            if (slot < 0)
              continue;
            // rows of unit u: the contact rows of step pair t (DISCRETE: those on u's half).
            // From HP and the rows alone: after a rejected step PCNT holds the counts at
            // the candidate point, not at the point these rows were built from.
            const int t = coll_pair_of(L, u);
            const int h0 = HP[t], h1 = HP[t + 1];
            auto other = [&](int h) { return L.coll_single && HTv[h] + CONTv[3 * h] != u; };
            double v = 0;
            if (L.coll_cnt)
            {
              // ConvexConstraints::violation: sum pospart(aff(x)), aff = exprMult(margin - dist, coeff)
              const double *HC0 = c.a(A_HC0), *HKv = c.a(A_HK);
              const int* HMv = c.ia(I_HMASK);
              const int* HKD = c.ia(I_HKIND);
              for (int h = h0; h < h1; ++h)
              {
                if (HKD[h] || other(h))
                  continue;
                const double2 mc = row_pair_mc(c, h);
                const double cf = mc.y;
                double a = (mc.x - HKv[h]) * cf;
                for (int e = 0; e < 2 * D; ++e)
                  if (HMv[h] & (1 << e))
                    a += ((-HC0[h * 2 * D + e]) * cf) * SX[(t + e / D) * D + e % D];
                v += fmax(a, 0.0);
              }
              mviol[L.coll_cost0 + slot] = v;
            }
            else
            {
              const int* HKD = c.ia(I_HKIND);
              for (int h = h0; h < h1; ++h)
                if (!HKD[h] && !other(h))
                  v += row_pair_mc(c, h).y * SX[L.nc_base + h];
              mcost[L.coll_cost0 + slot] = v;
            }
          }
        }
        BSYNC();
        evaluate(c, XN, NCOST, NVIOL);
        if (c.tid == 0)
          c.s->scan_at_x = 0;
        int decision = 0;  // 1 converged, 2 shrink, 3 accept
        if (c.tid == 0)
        {
          double oc = 0, mc = 0, nc = 0, ov = 0, mv = 0, nvv = 0;
          for (int i = 0; i < L.n_costs; ++i)
          {
            oc += COST[i];
            mc += mcost[i];
            nc += NCOST[i];
          }
          for (int i = 0; i < L.n_cnts; ++i)
          {
            ov += VIOL[i] * MU[i];
            mv += mviol[i] * MU[i];
            nvv += NVIOL[i] * MU[i];
          }
          const double old_merit = oc + ov, model_merit = mc + mv, new_merit = nc + nvv;
          const double approx = old_merit - model_merit;
          const double exact = old_merit - new_merit;
          const double ratio = exact / approx;
          c.s->n_fev++;
          if (approx < P.min_approx_improve)
            decision = 1;
          else if (approx / old_merit < P.min_approx_improve_frac)
            decision = 1;
          else if (exact < 0 || ratio < P.improve_ratio_threshold)
          {
            decision = 2;
            c.s->trust *= P.trust_shrink_ratio;
          }
          else
          {
            decision = 3;
            c.s->trust *= P.trust_expand_ratio;
          }
          c.s->flag = decision;
          if (c.s->trace && c.s->trace_n > 0 && c.s->trace_n == c.s->n_qp)  // (not after a full trace)
          {
            // the record of the QP this step solved (writeSolver's fields)
            double* rec = c.s->trace + THIP_TRACE_W * (c.s->trace_n - 1);
            rec[10] = old_merit;
            rec[11] = new_merit;
            rec[12] = approx;
            rec[13] = exact;
            rec[14] = ratio;
            rec[15] = decision;
          }
        }
        BSYNC();
        decision = c.s->flag;
        BSYNC();
        if (decision == 1)
        {
          converged_inner = true;
          break;
        }
        if (decision == 3)
        {
          if (c.tid == 0)
            c.s->scan_at_x = 1;  // X := XN, the point just scanned
          FOR(col, nx) X[col] = XN[col];
          FOR(i, L.n_costs) COST[i] = NCOST[i];
          FOR(i, L.n_cnts) VIOL[i] = NVIOL[i];
          BSYNC();
          break;
        }
      }
      if (failed)
      {
        retval = THIP_OPT_FAILED;
        goto_cleanup = true;
        break;
      }
      if (converged_inner)
      {
        retval = THIP_OPT_CONVERGED;
        goto_penalty = true;
        break;
      }
      if (c.s->trust < P.min_trust_box_size)
      {
        retval = THIP_OPT_CONVERGED;
        goto_penalty = true;
        break;
      }
      else if (iter >= P.max_iter)
      {
        retval = THIP_OPT_SCO_ITERATION_LIMIT;
        double vm = -INFINITY;
        for (int i = 0; i < L.n_cnts; ++i)
          vm = fmax(vm, VIOL[i]);
        if (L.n_cnts == 0 || vm < P.cnt_tolerance)
          retval = THIP_OPT_CONVERGED;
        goto_cleanup = true;
        break;
      }
    }
    if (goto_cleanup)
      break;
    // penalty adjustment
    (void)goto_penalty;
    double vm = -INFINITY;
    for (int i = 0; i < L.n_cnts; ++i)
      vm = fmax(vm, VIOL[i]);
    if (L.n_cnts == 0 || vm < P.cnt_tolerance)
      goto done;
    BSYNC();
    if (c.tid == 0)
    {
      for (int i = 0; i < L.n_cnts; ++i)
        if (!P.inflate_constraints_individually || VIOL[i] > P.cnt_tolerance)
          MU[i] *= P.merit_coeff_increase_ratio;
      c.s->trust = fmax(c.s->trust, P.min_trust_box_size / P.trust_shrink_ratio * 1.5);
      c.s->n_merit++;
    }
    BSYNC();
    if (mi + 1 >= P.max_merit_coeff_increases)
    {
      retval = THIP_OPT_PENALTY_ITERATION_LIMIT;
      goto done;
    }
  }
done:
  if (c.tid == 0)
    c.s->status = retval;
  BSYNC();
}

__device__ __forceinline__ void solve_problem(const KernelArgs& args, int b, double* dyn, Ctl& ctl,
                                              double** ptab, CollStage& cstage);

__global__ __launch_bounds__(kBlock) void THIP_SQP_KERNEL(KernelArgs args)
{
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ Ctl ctl;
  __shared__ int next_problem;
  // LDS residency plan (Layout::loff): hot QP arrays live in LDS for the
  // whole launch, the rest in this problem's HBM workspace
  __shared__ double* ptab[A_COUNT];
  __shared__ CollStage cstage;
  if (!args.work && static_cast<int>(blockIdx.x) >= args.batch)
    return;
  stage_chain(args.desc);
  // One problem per workgroup (args.work null), or a persistent workgroup per
  // resident slot taking problems in order from the launch's counter: the
  // grid is dealt round-robin over the XCDs, so with a static mapping each
  // die solves a fixed eighth of the batch and the die with the heaviest
  // eighth ends the launch; with the counter, a die that finishes its
  // problems early takes more.  Every problem is still solved by one
  // workgroup from its own inputs, so results do not depend on the mapping.
  for (int b = blockIdx.x;;)
  {
    if (args.work)
    {
      __syncthreads();  // the previous problem is done with next_problem
      if (threadIdx.x == 0)
        next_problem = atomicAdd(&args.work[0], 1);
      __syncthreads();
      b = __builtin_amdgcn_readfirstlane(next_problem);
      if (b >= args.batch)
        break;
    }
    solve_problem(args, b, dyn, ctl, ptab, cstage);
    if (!args.work)
      return;
  }
  // the last workgroup out resets the counters for the stream's next launch
  if (threadIdx.x == 0 && atomicAdd(&args.work[1], 1) == static_cast<int>(gridDim.x) - 1)
  {
    atomicExch(&args.work[0], 0);
    atomicExch(&args.work[1], 0);
  }
}

__device__ __forceinline__ void solve_problem(const KernelArgs& args, int b, double* dyn, Ctl& ctl,
                                              double** ptab, CollStage& cstage)
{
  const Layout& L = args.L;
  double* wsb = args.ws + (long long)b * L.dstride;
  for (int k = threadIdx.x; k < A_COUNT; k += kBlock)
    ptab[k] = L.loff[k] >= 0 ? dyn + L.loff[k] : wsb + L.doff[k];
  Ctx c(L, args.T, args.desc, wsb, args.iws + (long long)b * L.istride, dyn, &ctl, ptab);
  c.ptab_w = L.hinge ? ptab : nullptr;
  c.cs = &cstage;
  c.scene = args.scene ? args.scene + (long long)b * (args.desc->n_prims > 0 ? args.desc->n_prims : 1) * 16 : nullptr;
  c.jpt = args.jpt + (long long)b * (L.n_jpos > 0 ? L.n_jpos : 1) * L.D;
  Solver sv;
  // chain matrices: the LDS scratch, or HBM for wide blocks (Layout::wide)
  sv.M = (L.wide || L.chm_hbm) ? wsb + L.doff[A_CHM] : dyn;
  sv.Nb = sv.M + L.sN * L.sD * L.sD;
  if (threadIdx.x == 0)
  {
    ctl.trace = args.trace ? args.trace + (long long)b * args.trace_cap * THIP_TRACE_W : nullptr;
    ctl.trace_cap = args.trace_cap;
    ctl.trace_n = 0;
    ctl.prof = args.prof ? args.prof + (long long)b * kProfSlots : nullptr;
  }
  if (args.stage_init)
  {
    // the uploaded inputs into this problem's (HBM-resident) INIT, X and TGT
    for (int i = threadIdx.x; i < L.nx; i += kBlock)
    {
      const double v = args.stage_init[(long long)b * L.nx + i];
      wsb[L.doff[A_INIT] + i] = v;
      wsb[L.doff[A_X] + i] = v;
    }
    for (int i = threadIdx.x; i < L.n_cart * 12; i += kBlock)
      wsb[L.doff[A_TGT] + i] = args.stage_tgt[(long long)b * L.n_cart * 12 + i];
  }
  __syncthreads();
  const long long w0 = wall_clock64();
  sqp_optimize(c, sv);
  if (args.xout)
  {
    __syncthreads();
    for (int i = threadIdx.x; i < L.nx; i += kBlock)
      args.xout[(long long)b * L.nx + i] = wsb[L.doff[A_X] + i];
  }
  if (threadIdx.x == 0 && ctl.prof)
    ctl.prof[14] += wall_clock64() - w0;
  if (threadIdx.x == 0 && args.trace_n)
    args.trace_n[b] = ctl.trace_n;
  if (c.tid == 0)
  {
    thip_result r{};
    r.status = ctl.status;
    r.n_sqp_iters = ctl.n_sqp;
    r.n_qp_solves = ctl.n_qp;
    r.n_func_evals = ctl.n_fev;
    r.n_admm_iters = ctl.n_admm;
    r.n_merit_increases = ctl.n_merit;
    double tc = 0;
    const double* COST = c.a(A_COST);
    for (int i = 0; i < L.n_costs; ++i)
      tc += COST[i];
    r.total_cost = tc;
    double vm = 0;
    const double* VIOL = c.a(A_VIOL);
    for (int i = 0; i < L.n_cnts; ++i)
      vm = (i == 0) ? VIOL[i] : fmax(vm, VIOL[i]);
    r.max_cnt_viol = vm;
    r.final_trust_box = ctl.trust;
    r.n_costs = L.n_costs;
    r.n_cnts = L.n_cnts;
    r.flags = ctl.flags;
    r.n_contact_rows = ctl.n_contact_rows;
    r.n_hinge_admm = ctl.n_hinge_admm;
    r.n_substates = ctl.n_substates;
    if (ctl.flags & THIP_FLAG_CONTACT_OVERFLOW)
      r.status = THIP_OPT_FAILED;
    args.res[b] = r;
  }
}

// standalone convexification (thip_linearize): writes rows into err/jac layout
#if !THIP_GENERIC_ONLY
__global__ __launch_bounds__(kBlock) void linearize_kernel(KernelArgs args, const double* xin, double* err,
                                                           double* jac)
{
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ Ctl ctl;
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  stage_chain(args.desc);
  const Layout& L = args.L;
  Ctx c(L, args.T, args.desc, args.ws + (long long)b * L.dstride, args.iws + (long long)b * L.istride, dyn, &ctl);
  c.scene = args.scene + (long long)b * (args.desc->n_prims > 0 ? args.desc->n_prims : 1) * 16;
  c.jpt = args.jpt + (long long)b * (L.n_jpos > 0 ? L.n_jpos : 1) * L.D;
  if (threadIdx.x == 0)
  {
    ctl.n_h = 0;
    ctl.flags = 0;
    ctl.coll_overflow = 0;
    ctl.scan_at_x = 0;
    ctl.prof = nullptr;
    ctl.n_contact_rows = ctl.n_hinge_admm = ctl.n_substates = 0;
  }
  const int D = L.D;
  double* X = c.a(A_XN);
  FOR(i, L.nx) X[i] = xin[(long long)b * L.nx + i];
  BSYNC();
  double* raw = c.a(A_PB);  // scratch (n_cols + m >= n_abs * D)
  linearize(c, X, raw);
  FOR(k, L.n_cart)
  {
    const int r0 = c.T.term_row0[k], nr = c.T.term_nrow[k];
    double* eo = err + ((long long)b * L.n_cart + k) * 6;
    double* jo = jac + ((long long)b * L.n_cart + k) * 6 * D;
    for (int i = 0; i < 6; ++i)
    {
      eo[i] = 0;
      for (int j = 0; j < D; ++j)
        jo[i * D + j] = 0;
    }
    for (int rr = 0; rr < nr; ++rr)
    {
      const int row = r0 + rr;
      eo[rr] = c.big[30 * k + 24 + c.T.row_comp[row]];
      for (int j = 0; j < D; ++j)
        jo[rr * D + j] = raw[row * D + j];
    }
  }
}

__global__ __launch_bounds__(kBlock) void fwd_kin_kernel(KernelArgs args, const double* xin, double* poses)
{
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  stage_chain(args.desc);
  const Layout& L = args.L;
  const thip_chain& ch = g_chain;
  for (int i = threadIdx.x; i < L.N * L.n_links; i += kBlock)
  {
    const int t = i / L.n_links, l = i % L.n_links;
    Pose P;
    chain_fk(ch, xin + ((long long)b * L.N + t) * L.D, l, P);
    double* o = poses + (((long long)b * L.N + t) * L.n_links + l) * 12;
    for (int r = 0; r < 3; ++r)
    {
      for (int k = 0; k < 3; ++k)
        o[r * 4 + k] = P.r[r * 3 + k];
      o[r * 4 + 3] = P.t[r];
    }
  }
}


#endif  // !THIP_GENERIC_ONLY

// (in both builds: the generic-step build's, coll_rows_kernel_gen, scans with
// its contact_test_type selection)
#if THIP_GENERIC_ONLY
#define THIP_COLL_ROWS_KERNEL coll_rows_kernel_gen
#else
#define THIP_COLL_ROWS_KERNEL coll_rows_kernel
#endif
// Linearised collision rows at a given trajectory (parity/debug entry
// thip_collision_rows): records [t, link, prim, sphere, substate, distance,
// cc_time, n_kept, a_t[D], a_t+1[D], constant] in the hinge-row order.
__global__ __launch_bounds__(kBlock) void THIP_COLL_ROWS_KERNEL(KernelArgs args, const double* xin, double* out, int cap,
                                                          int* counts)
{
  __shared__ Ctl ctl;
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  stage_chain(args.desc);
  const Layout& L = args.L;
  Ctx c(L, args.T, args.desc, args.ws + (long long)b * L.dstride, args.iws + (long long)b * L.istride, nullptr,
        &ctl);
  c.scene = args.scene + (long long)b * (args.desc->n_prims > 0 ? args.desc->n_prims : 1) * 16;
  c.jpt = args.jpt + (long long)b * (L.n_jpos > 0 ? L.n_jpos : 1) * L.D;
  __shared__ CollStage cstage;
  c.cs = &cstage;
  if (threadIdx.x == 0)
  {
    ctl.n_h = 0;
    ctl.flags = 0;
    ctl.coll_overflow = 0;
    ctl.scan_at_x = 0;
    ctl.prof = nullptr;
    ctl.n_contact_rows = ctl.n_hinge_admm = ctl.n_substates = 0;
  }
  double* XN = c.a(A_XN);
  FOR(i, L.nx) XN[i] = xin[(long long)b * L.nx + i];
  BSYNC();
  coll_scan(c, XN, nullptr, true);
  const int D = L.D, W = 8 + 2 * D + 1;
  const int* CONT = c.ia(I_CONT);
  const int* HT = c.ia(I_HT);
  const int* HM = c.ia(I_HMASK);
  const double *HC0 = c.a(A_HC0), *HK = c.a(A_HK), *HD = c.a(A_HDIST);
  double* ob = out + (long long)b * cap * W;
  const int* HKD = c.ia(I_HKIND);
  FOR(k, ctl.n_h)
  {
    if (HKD[k] != 0)
      continue;  // static hinge rows follow each pair's contacts
    const int t = HT[k], i = CONT[3 * k];
    const int o = k - c.T.sh_ptr[t];
    if (o >= cap)
      continue;
    const int cnt = lvs_count(XN + t * D, XN + (t + 1) * D, D, args.desc->coll_lvs);
    double* r = ob + (long long)o * W;
    const bool single = L.coll_single != 0;  // DISCRETE: i is the half; record = waypoint t + i
    r[0] = single ? t + i : t;
    r[1] = args.desc->sphere_link[CONT[3 * k + 1]];
    r[2] = CONT[3 * k + 2];
    r[3] = CONT[3 * k + 1];
    r[4] = single ? 0 : i;
    r[5] = HD[k];
    r[6] = c.a(A_HCCT)[k];
    (void)cnt;
    r[7] = __popc(HM[k]);
    for (int j = 0; j < 2 * D; ++j)
      r[8 + j] = single ? (j < D ? HC0[k * 2 * D + i * D + j] : 0.0) : HC0[k * 2 * D + j];
    r[8 + 2 * D] = HK[k];
  }
  if (threadIdx.x == 0)
    counts[b] = (ctl.flags & THIP_FLAG_CONTACT_OVERFLOW) ? -1 : ctl.n_h - c.T.n_sh;
}
}  // namespace thip

