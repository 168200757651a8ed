// C-ABI of the batched SQP (include/trajopt_hip.h): lowering of the shared
// problem structure into device tables, per-problem workspace allocation,
// launches on one HIP stream, event timing.  No torch types, no exceptions
// across the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <cstdlib>
#include <functional>

#include "layout.hpp"
#include "pair_data.hpp"
#include "self_pairs.hpp"

namespace thip
{
__global__ void sqp_kernel(KernelArgs args);
__global__ void sqp_kernel_gen(KernelArgs args);  // the generic-step build (kGenBlock threads)
__global__ void linearize_kernel(KernelArgs args, const double* xin, double* err, double* jac);
__global__ void fwd_kin_kernel(KernelArgs args, const double* xin, double* poses);
__global__ void stage_inputs_kernel(KernelArgs args, const double* init, const double* tgt);
__global__ void gather_x_kernel(KernelArgs args, double* xout);
__global__ void coll_rows_kernel(KernelArgs args, const double* xin, double* out, int cap, int* counts);
__global__ void coll_rows_kernel_gen(KernelArgs args, const double* xin, double* out, int cap, int* counts);
}  // namespace thip

using namespace thip;

struct thip_ctx
{
  int device = 0;
  int batch = 0;
  thip_problem_desc desc{};
  Layout L{};
  // device buffers
  thip_problem_desc* d_desc = nullptr;
  int* d_tables = nullptr;
  double* d_tables_f = nullptr;
  double* d_pair = nullptr;  // per link-pair collision margins / coefficients (pair_data.hpp), or null
  Tables T{};
  double* d_ws = nullptr;
  int* d_iws = nullptr;
  thip_result* d_res = nullptr;
  double* d_init = nullptr;
  double* d_tgt = nullptr;
  double* d_scene = nullptr;
  double* d_jpt = nullptr;   // JointPos targets [batch][max(n_jpos,1)][D]
  double* d_x = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double* d_trace = nullptr;
  int* d_trace_n = nullptr;
  int trace_cap = 0;
  long long* d_prof = nullptr;
  bool uploaded = false;
  bool ran = false;
  size_t lds_bytes = 0;      // sqp_kernel: scratch + LDS-resident arrays
  size_t lds_lin_bytes = 0;  // linearize_kernel: scratch only
  int* d_work = nullptr;     // sqp_kernel's problem counter (KernelArgs::work); null: static mapping
  int grid = 0;              // sqp_kernel workgroups (resident slots, or the batch)
  bool gen = false;          // the QPs never take the segment: launch the generic-step build
                             // (sqp_kernel_gen, kGenBlock threads) instead of sqp_kernel
  std::string err;
};

static thread_local std::string g_create_err;

#define HIPCHK(ctx, call)                                                            \
  do                                                                                 \
  {                                                                                  \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess)                                                            \
    {                                                                                \
      (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                \
      return THIP_E_HIP;                                                             \
    }                                                                                \
  } while (0)

extern "C" {

const char* thip_build_info(void) { return "trajopt-1_amd thip 0.1 gfx950 fp64 (one workgroup per problem)"; }

int thip_sizeof_desc(void) { return static_cast<int>(sizeof(thip_problem_desc)); }
int thip_sizeof_result(void) { return static_cast<int>(sizeof(thip_result)); }

void thip_default_sqp_params(thip_sqp_params* p)
{
  p->improve_ratio_threshold = 0.25;
  p->min_trust_box_size = 1e-4;
  p->min_approx_improve = 1e-4;
  p->min_approx_improve_frac = -1.7976931348623157e308;
  p->max_iter = 50;
  p->trust_shrink_ratio = 0.1;
  p->trust_expand_ratio = 1.5;
  p->cnt_tolerance = 1e-4;
  p->max_merit_coeff_increases = 5;
  p->max_qp_solver_failures = 3;
  p->merit_coeff_increase_ratio = 10;
  p->initial_merit_error_coeff = 10;
  p->inflate_constraints_individually = 1;
  p->trust_box_size = 1e-1;
  p->max_time = DBL_MAX;  // optimizers.hpp:117
}

void thip_default_osqp_settings(thip_osqp_settings* s)
{
  s->rho = 0.1;
  s->sigma = 1e-6;
  s->alpha = 1.6;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 0;
  s->adaptive_rho_tolerance = 5;
  s->max_iter = 8192;
  s->eps_abs = 1e-4;
  s->eps_rel = 1e-6;
  s->eps_prim_inf = 1e-4;
  s->eps_dual_inf = 1e-4;
  s->check_termination = 25;
  s->warm_starting = 1;
  s->polishing = 1;
  s->delta = 1e-6;
  s->polish_refine_iter = 3;
}

// thip_debug_set_path: diagnostic solve-path overrides for contexts created afterwards
static int g_debug_path = 0;

int thip_debug_solve_layout(const thip_ctx* ctx, int* out, int n)
{
  if (!ctx || !out || n < 0)
    return THIP_E_INVALID;
  const int v[THIP_LAYOUT_INFO_N] = {ctx->L.nbr, ctx->L.sD, ctx->L.wide, ctx->L.seg_ok, ctx->gen ? 1 : 0,
                                     ctx->gen ? kGenBlock : kBlock, ctx->L.grp, ctx->L.sNb};
  for (int k = 0; k < n && k < THIP_LAYOUT_INFO_N; ++k)
    out[k] = v[k];
  return THIP_OK;
}

int thip_debug_set_path(int flags)
{
  if (flags & ~(THIP_DEBUG_NO_SEGMENT | THIP_DEBUG_FORCE_WIDE | THIP_DEBUG_NO_BRANCH | THIP_DEBUG_STATIC_DISPATCH |
                THIP_DEBUG_GEN_BUILD | THIP_DEBUG_MAIN_BUILD))
    return THIP_E_INVALID;
  g_debug_path = flags;
  return THIP_OK;
}

extern "C" int thip_jdt_fused(const thip_problem_desc* d)
{
  int k, j;
  if (d->n_jdt == 0)
    return 1;
  if (d->n_jdt < 0 || d->n_jdt > THIP_MAX_JDT || d->n_steps % 2 != 0 || 2 * d->chain.n_dof > THIP_MAX_DOF ||
      d->use_time)
    return 0;
  for (k = 0; k < d->n_jdt; ++k)
  {
    if (d->jdt_order[k] != 2 || d->jdt_is_cnt[k])
      return 0;
    for (j = 0; j < d->chain.n_dof; ++j)
      if (d->jdt_upper_tols[k][j] >= 1e-5 || d->jdt_upper_tols[k][j] <= -1e-5 || d->jdt_lower_tols[k][j] >= 1e-5 ||
          d->jdt_lower_tols[k][j] <= -1e-5)
        return 0;
  }
  return 1;
}

static int validate(const thip_problem_desc* d, std::string& why)
{
  if (d->abi_version != THIP_ABI_VERSION)
    return why = "descriptor abi_version " + std::to_string(d->abi_version) + " != THIP_ABI_VERSION " +
                 std::to_string(THIP_ABI_VERSION) + " (caller built against another trajopt_hip.h)",
           THIP_E_INVALID;
  const thip_chain& ch = d->chain;
  if (ch.n_dof <= 0 || ch.n_dof > THIP_MAX_DOF)
    return why = "n_dof out of range", THIP_E_INVALID;
  if (ch.n_links < 1 || ch.n_links > THIP_MAX_LINKS)
    return why = "n_links out of range", THIP_E_INVALID;
  if (d->n_steps < 2 || d->n_steps > THIP_MAX_STEPS)
    return why = "n_steps must be in [2, " + std::to_string(THIP_MAX_STEPS) +
                 "] for the batched kernel (single-waypoint problems run sco::BasicTrustRegionSQP's generic path)",
           THIP_E_INVALID;
  for (int k = 1; k < ch.n_links; ++k)
  {
    const int ty = ch.joint_type[k];
    if (ty < 0 || ty > 3)
      return why = "bad joint type", THIP_E_INVALID;
    if (ty != THIP_JOINT_FIXED && (ch.joint_dof[k] < 0 || ch.joint_dof[k] >= ch.n_dof))
      return why = "bad joint dof index", THIP_E_INVALID;
    if (ch.is_tree && (ch.parent[k] < 0 || ch.parent[k] >= k))
      return why = "bad parent link (links must be in tree order, 0 <= parent[k] < k)", THIP_E_INVALID;
  }
  if (d->n_fixed < 0 || d->n_fixed > THIP_MAX_STEPS)
    return why = "n_fixed out of range", THIP_E_INVALID;
  std::vector<int> seen(static_cast<size_t>(d->n_steps), 0);
  for (int f = 0; f < d->n_fixed; ++f)
  {
    const int t = d->fixed_steps[f];
    if (t < 0 || t >= d->n_steps)
      return why = "Fixed timestep index is outside the bounds of the initial trajectory.", THIP_E_INVALID;
    if (seen[static_cast<size_t>(t)]++)
      return why = "duplicate fixed timestep", THIP_E_INVALID;
  }
  if (d->n_cart < 0 || d->n_cart > THIP_MAX_CART)
    return why = "n_cart out of range", THIP_E_INVALID;
  for (int k = 0; k < d->n_cart; ++k)
  {
    if (d->cart_step[k] < 0 || d->cart_step[k] >= d->n_steps)
      return why = "CartPose timestep out of range", THIP_E_INVALID;
    if (d->cart_source_link[k] <= 0 || d->cart_source_link[k] >= ch.n_links)
      return why = "CartPose source frame must be an active chain link", THIP_E_INVALID;
    if (d->cart_target_link[k] < 0 || d->cart_target_link[k] >= ch.n_links)
      return why = "CartPose target link out of range (0: the static chain root)", THIP_E_INVALID;
  }
  if (d->n_jvx < 0 || d->n_jvx > THIP_MAX_JVX)
    return why = "n_jvx out of range", THIP_E_INVALID;
  for (int x = 0; x < d->n_jvx; ++x)
  {
    bool tol = false;
    for (int j = 0; j < d->chain.n_dof; ++j)
      tol = tol || std::fabs(d->jvx_upper_tols[x][j]) >= 1e-5 || std::fabs(d->jvx_lower_tols[x][j]) >= 1e-5;
    if (!tol)
      return why = "jvx terms are the tolerance forms (JointVelIneqCost / JointVelIneqConstraint): "
                   "a term with zero tolerances goes in jv_*",
             THIP_E_INVALID;
  }
  if (!thip_jdt_fused(d))
    return why = "JointAcc / JointJerk terms other than JointAccEqCost on an even number of waypoints with "
                 "2 n_dof <= THIP_MAX_DOF, and JointVel equality constraints, are not lowered into the batched "
                 "kernel: solve such a problem with sco::BasicTrustRegionSQP (the generic path, GpuModel)",
           THIP_E_INVALID;
  if (d->use_time != 0 || d->n_jvt != 0 || d->n_ttt != 0 || d->n_fixed_dofs != 0)
    return why = "time-parameterised problems (use_time, JointVel terms with use_time, TotalTime) and fixed dofs are not "
                 "lowered into the batched kernel: solve such a problem with sco::BasicTrustRegionSQP (the generic "
                 "path, GpuModel)",
           THIP_E_INVALID;
  if (d->coll_enabled && d->coll_contact_test != THIP_CONTACT_ALL && d->coll_contact_test != THIP_CONTACT_FIRST &&
      d->coll_contact_test != THIP_CONTACT_CLOSEST)
    return why = "coll_contact_test is not a THIP_CONTACT_* value", THIP_E_INVALID;
  if (d->n_coll_extra != 0)
    return why = "more than one collision term is not lowered into the batched kernel: solve such a problem with "
                 "sco::BasicTrustRegionSQP (the generic path, device-evaluated terms and GpuModel)",
           THIP_E_INVALID;
  if (d->n_jpos < 0 || d->n_jpos > THIP_MAX_JPOS)
    return why = "n_jpos out of range", THIP_E_INVALID;
  for (int k = 0; k < d->n_jpos; ++k)
    for (int j = 0; j < ch.n_dof; ++j)
    {
      if (!std::isfinite(d->jpos_coeffs[k][j]) || !std::isfinite(d->jpos_targets[k][j]) ||
          !std::isfinite(d->jpos_upper_tols[k][j]) || !std::isfinite(d->jpos_lower_tols[k][j]))
        return why = "JointPos coeffs / targets / tolerances must be finite", THIP_E_INVALID;
    }
  if (d->coll_enabled)
  {
    if (d->n_spheres < 1 || d->n_spheres > THIP_MAX_SPHERES)
      return why = "collision: n_spheres out of range", THIP_E_INVALID;
    for (int s = 0; s < d->n_spheres; ++s)
      if (d->sphere_link[s] < 1 || d->sphere_link[s] >= ch.n_links || !(d->sphere_radius[s] >= 0))
        return why = "collision: bad robot sphere", THIP_E_INVALID;
    if (d->n_prims < 0 || d->n_prims > THIP_MAX_PRIMS)
      return why = "collision: n_prims out of range", THIP_E_INVALID;
    const int last = d->coll_last_step < 0 ? d->n_steps - 1 : d->coll_last_step;
    if (d->coll_first_step < 0 || d->coll_first_step >= d->n_steps || last < d->coll_first_step ||
        last >= d->n_steps)
      return why = "collision: bad first/last step", THIP_E_INVALID;
    if (d->coll_continuous < 0 || d->coll_continuous > 2)
      return why = "collision: coll_continuous must be 0 (LVS_DISCRETE), 1 (LVS_CONTINUOUS) or 2 (DISCRETE)",
             THIP_E_INVALID;
    const bool single = d->coll_continuous == 2;
    if (single && d->n_steps < 2)
      return why = "collision: DISCRETE needs at least 2 waypoints", THIP_E_INVALID;
    if ((!single && !(d->coll_lvs > 0)) || !(d->coll_buffer >= 0))
      return why = "collision: bad longest_valid_segment_length / buffer", THIP_E_INVALID;
    // (single-timestep terms skip fixed waypoints; only the step-pair evaluators reject
    // adjacent fixed steps, problem_description.cpp:1765-1767 vs :1785-1795)
    for (int t = d->coll_first_step; !single && t < last; ++t)
    {
      bool a = false, b = false;
      for (int k = 0; k < d->coll_n_fixed; ++k)
      {
        a |= d->coll_fixed_steps[k] == t;
        b |= d->coll_fixed_steps[k] == t + 1;
      }
      if (a && b)
        return why = "Currently two adjacent fixed steps are not supported in collision term.", THIP_E_INVALID;
    }
  }
  for (int k = 0; k < d->n_cart; ++k)
    if (d->cart_has_tol[k])
      for (int i = 0; i < 6; ++i)
        if (!(d->cart_lower_tol[k][i] <= d->cart_upper_tol[k][i]))
          return why = "CartPoseErrCalculator: Inverted tolerance band - lower > upper at one or more indices",
                 THIP_E_INVALID;
  if (d->coll_enabled && (d->coll_max_contacts < 0 || d->coll_max_contacts > THIP_MAX_CONTACTS))
    return why = "collision: coll_max_contacts out of range", THIP_E_INVALID;
  if (d->coll_enabled)
  {
    std::vector<int> sa, sb, kp;
    const std::string w = self_sphere_pairs(*d, sa, sb, kp);
    if (!w.empty())
      return why = w, THIP_E_INVALID;
  }
  {
    const std::string w = validate_coll_pairs(*d);
    if (!w.empty())
      return why = w, THIP_E_INVALID;
  }
  if (!(d->sqp.max_time >= 0))
    return why = "sqp.max_time must be >= 0 (DBL_MAX: no limit)", THIP_E_INVALID;
  if (!(d->sqp.trust_shrink_ratio > 0 && d->sqp.trust_shrink_ratio < 1) || !(d->sqp.min_trust_box_size > 0) ||
      !(d->sqp.trust_box_size > 0))
    return why = "sqp: need 0 < trust_shrink_ratio < 1, min_trust_box_size > 0 and trust_box_size > 0",
           THIP_E_INVALID;
  if (d->osqp.check_termination < 0 || d->osqp.max_iter < 1 || d->osqp.scaling < 0)
    return why = "bad OSQP settings", THIP_E_INVALID;
  return THIP_OK;
}

int thip_create(int device, const thip_problem_desc* desc, int batch, thip_ctx** out)
{
  if (!desc || !out || batch <= 0)
  {
    g_create_err = "thip_create: null argument or batch <= 0";
    return THIP_E_INVALID;
  }
  std::string why;
  if (validate(desc, why) != THIP_OK)
  {
    g_create_err = "thip_create: " + why;
    return THIP_E_INVALID;
  }
  auto* ctx = new thip_ctx();
  ctx->device = device;
  ctx->batch = batch;
  ctx->desc = *desc;
  if (!ctx->desc.chain.is_tree)  // serial chain: parent[] is not read from the caller
    for (int k = 0; k < THIP_MAX_LINKS; ++k)
      ctx->desc.chain.parent[k] = k > 0 ? k - 1 : 0;
  const thip_problem_desc& d = ctx->desc;
  Layout& L = ctx->L;
  L.N = d.n_steps;
  L.D = d.chain.n_dof;
  L.nx = L.N * L.D;
  L.n_links = d.chain.n_links;
  L.n_fixed = d.n_fixed;
  L.n_fixed_rows = d.n_fixed * L.D;
  L.n_cart = d.n_cart;
  // JointVelTermInfo::hatch step clamping (problem_description.cpp:1228-1245)
  auto jv_clamp = [&](int first, int last, int& f_out, int& l_out) {
    if (last <= -1)
      last = L.N - 1;
    if ((L.N - 2) <= first)
      first = L.N - 2;
    if ((L.N - 1) <= last)
      last = L.N - 1;
    if (last == first)
      last += 1;
    if (last < first)
      std::swap(first, last);
    f_out = first;
    l_out = last;
  };
  jv_clamp(d.jv_first_step, d.jv_last_step, L.jv_first, L.jv_last);
  std::vector<int> jvx_first(THIP_MAX_JVX, 0), jvx_last(THIP_MAX_JVX, 0), jvx_slot(THIP_MAX_JVX, 0);
  for (int x = 0; x < d.n_jvx; ++x)
    jv_clamp(d.jvx_first_step[x], d.jvx_last_step[x], jvx_first[static_cast<size_t>(x)],
             jvx_last[static_cast<size_t>(x)]);
  L.n_jvx = d.n_jvx;
  // zero tolerances: trajopt_common::doubleEquals(tol, 0.) (problem_description.cpp:1135-1138,1249-1252)
  auto zero_tol = [](double v) { return std::fabs(v) < 1e-5; };
  L.jv_ineq = 0;
  if (d.jv_enabled)
    for (int j = 0; j < L.D; ++j)
      if (!zero_tol(d.jv_upper_tols[j]) || !zero_tol(d.jv_lower_tols[j]))
        L.jv_ineq = 1;
  std::vector<int> jpos_ineq(THIP_MAX_JPOS, 0);
  for (int k = 0; k < d.n_jpos; ++k)
    for (int j = 0; j < L.D; ++j)
      if (!zero_tol(d.jpos_upper_tols[k][j]) || !zero_tol(d.jpos_lower_tols[k][j]))
        jpos_ineq[static_cast<size_t>(k)] = 1;
  // CartPose rows: cost terms first (convexifyCosts order), then constraint terms (cntsToCosts)
  std::vector<int> row_term, row_comp, row_step, term_row0(THIP_MAX_CART, 0), term_nrow(THIP_MAX_CART, 0),
      term_slot(THIP_MAX_CART, 0);
  std::vector<double> row_w;
  int n_costs = d.jv_enabled ? 1 : 0, n_cnts = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int k = 0; k < d.n_cart; ++k)
    {
      if ((pass == 0) != (d.cart_is_cnt[k] == 0))
        continue;
      term_row0[k] = static_cast<int>(row_term.size());
      for (int i = 0; i < 6; ++i)
      {
        const double cf = (i < 3) ? d.cart_pos_coeffs[k][i] : d.cart_rot_coeffs[k][i - 3];
        if (std::fabs(cf) > 1e-5)
        {
          row_term.push_back(k);
          row_comp.push_back(i);
          row_step.push_back(d.cart_step[k]);
          row_w.push_back(cf);
        }
      }
      term_nrow[k] = static_cast<int>(row_term.size()) - term_row0[k];
      term_slot[k] = (pass == 0) ? n_costs++ : n_cnts++;
    }
  std::vector<int> row_slot, row_jpos(row_term.size(), 0);
  for (size_t r = 0; r < row_term.size(); ++r)
    row_slot.push_back(d.cart_is_cnt[row_term[r]] ? term_slot[static_cast<size_t>(row_term[r])] : -1);
  // JointPosTermInfo::hatch (problem_description.cpp:1097-1196): step clamping; costs are
  // quadratic (no rows), constraints add one EQ row per (step, joint) after the CartPose
  // constraint rows (cnt_infos order, JointPosEqConstraint ctor order: step-major)
  std::vector<int> jpos_first(THIP_MAX_JPOS, 0), jpos_last(THIP_MAX_JPOS, 0), jpos_slot(THIP_MAX_JPOS, 0),
      jpos_row0(THIP_MAX_JPOS, 0), jpos_nrow(THIP_MAX_JPOS, 0);
  L.n_jpos = d.n_jpos;
  for (int k = 0; k < d.n_jpos; ++k)
  {
    int f = d.jpos_first_step[k], l = d.jpos_last_step[k];
    if (l <= -1)
      l = L.N - 1;
    if ((L.N - 1) <= f)
      f = L.N - 1;
    if ((L.N - 1) <= l)
      l = L.N - 1;
    if (l < f)
      std::swap(f, l);
    f = std::max(f, 0);
    jpos_first[static_cast<size_t>(k)] = f;
    jpos_last[static_cast<size_t>(k)] = l;
    if (!d.jpos_is_cnt[k])
      jpos_slot[static_cast<size_t>(k)] = n_costs++;
  }
  for (int x = 0; x < d.n_jvx; ++x)
    if (!d.jvx_is_cnt[x])
      jvx_slot[static_cast<size_t>(x)] = n_costs++;
  // JointAccEqCost terms (thip_jdt_fused): cost slots after the JointVel
  // tolerance costs (the oracle's / ConstructProblem's cost order)
  L.n_jacc = d.n_jdt;
  for (int k = 0; k < THIP_MAX_JDT; ++k)
    L.jacc_slot[k] = (k < d.n_jdt) ? n_costs++ : -1;
  for (int k = 0; k < d.n_jpos; ++k)
  {
    if (!d.jpos_is_cnt[k])
      continue;
    jpos_slot[static_cast<size_t>(k)] = n_cnts++;
    if (jpos_ineq[static_cast<size_t>(k)])
      continue;  // hinge rows (static hinge table below), no abs rows
    jpos_row0[static_cast<size_t>(k)] = static_cast<int>(row_term.size());
    for (int t = jpos_first[static_cast<size_t>(k)]; t <= jpos_last[static_cast<size_t>(k)]; ++t)
      for (int j = 0; j < L.D; ++j)
      {
        row_term.push_back(k);
        row_comp.push_back(j);
        row_step.push_back(t);
        row_w.push_back(d.jpos_coeffs[k][j]);
        row_slot.push_back(jpos_slot[static_cast<size_t>(k)]);
        row_jpos.push_back(1);
      }
    jpos_nrow[static_cast<size_t>(k)] = static_cast<int>(row_term.size()) - jpos_row0[static_cast<size_t>(k)];
  }
  for (int x = 0; x < d.n_jvx; ++x)
    if (d.jvx_is_cnt[x])
      jvx_slot[static_cast<size_t>(x)] = n_cnts++;
  L.n_abs = static_cast<int>(row_term.size());
  L.n_abs_cost = 0;
  for (int r = 0; r < L.n_abs; ++r)
    if (row_slot[static_cast<size_t>(r)] < 0)
      L.n_abs_cost++;
  // static hinge rows: JointVelIneqCost (owner n_jpos, cost slot 0) and the
  // JointPos tolerance terms; a row on waypoint t alone is filed under pair
  // min(t, N-2) (second half when t = N-1), a velocity row under pair t
  std::vector<int> sh_kind, sh_owner, sh_joint, sh_step, sh_pair, sh_slot;
  auto add_sh = [&](int kind, int owner, int j, int t, int pair, int slot) {
    sh_kind.push_back(kind);
    sh_owner.push_back(owner);
    sh_joint.push_back(j);
    sh_step.push_back(t);
    sh_pair.push_back(pair);
    sh_slot.push_back(slot);
  };
  if (L.jv_ineq)
    for (int t = L.jv_first; t <= L.jv_last - 1; ++t)
      for (int j = 0; j < L.D; ++j)
      {
        add_sh(SH_JV_UP, d.n_jpos, j, t, t, -1);
        add_sh(SH_JV_LO, d.n_jpos, j, t, t, -1);
      }
  // further JointVel tolerance terms: owner n_jpos + 1 + x
  for (int x = 0; x < d.n_jvx; ++x)
  {
    const int slot = d.jvx_is_cnt[x] ? jvx_slot[static_cast<size_t>(x)] : -1;
    for (int t = jvx_first[static_cast<size_t>(x)]; t <= jvx_last[static_cast<size_t>(x)] - 1; ++t)
      for (int j = 0; j < L.D; ++j)
      {
        add_sh(SH_JV_UP, d.n_jpos + 1 + x, j, t, t, slot);
        add_sh(SH_JV_LO, d.n_jpos + 1 + x, j, t, t, slot);
      }
  }
  for (int k = 0; k < d.n_jpos; ++k)
  {
    if (!jpos_ineq[static_cast<size_t>(k)])
      continue;
    const int slot = d.jpos_is_cnt[k] ? jpos_slot[static_cast<size_t>(k)] : -1;
    for (int t = jpos_first[static_cast<size_t>(k)]; t <= jpos_last[static_cast<size_t>(k)]; ++t)
      for (int j = 0; j < L.D; ++j)
      {
        add_sh(SH_JP_UP, k, j, t, std::min(t, L.N - 2), slot);
        add_sh(SH_JP_LO, k, j, t, std::min(t, L.N - 2), slot);
      }
  }
  const int n_sh = static_cast<int>(sh_kind.size());
  std::vector<int> sh_ptr(static_cast<size_t>(L.N + 1), 0), sh_order(static_cast<size_t>(n_sh));
  for (int s2 = 0; s2 < n_sh; ++s2)
    sh_ptr[static_cast<size_t>(sh_pair[static_cast<size_t>(s2)] + 1)]++;
  for (int t = 0; t < L.N; ++t)
    sh_ptr[static_cast<size_t>(t + 1)] += sh_ptr[static_cast<size_t>(t)];
  {
    std::vector<int> nxt(sh_ptr.begin(), sh_ptr.end() - 1);
    for (int s2 = 0; s2 < n_sh; ++s2)
      sh_order[static_cast<size_t>(nxt[static_cast<size_t>(sh_pair[static_cast<size_t>(s2)])]++)] = s2;
  }
  auto permute = [&](std::vector<int>& v) {
    std::vector<int> o(v.size());
    for (size_t i = 0; i < v.size(); ++i)
      o[i] = v[static_cast<size_t>(sh_order[i])];
    v.swap(o);
  };
  permute(sh_kind);
  permute(sh_owner);
  permute(sh_joint);
  permute(sh_step);
  permute(sh_pair);
  permute(sh_slot);
  // collision: one cost term per step pair after the CartPose costs
  // (cost_infos order; CollisionTermInfo::hatch, problem_description.cpp:1747)
  L.coll = d.coll_enabled ? 1 : 0;
  L.coll_first = d.coll_first_step;
  L.coll_last = (d.coll_last_step < 0) ? L.N - 1 : d.coll_last_step;
  // DISCRETE: one SingleTimestepCollisionEvaluator term per waypoint of [first, last] that is
  // not a fixed step (problem_description.cpp:1782-1796)
  L.coll_single = (L.coll && d.coll_continuous == 2) ? 1 : 0;
  if (L.coll_single)
    L.coll_last += 1;
  std::vector<int> coll_slot(static_cast<size_t>(L.N), -1);
  int n_units = 0;
  for (int t = L.coll_first; L.coll && t < L.coll_last; ++t)
  {
    bool fx = false;
    for (int k = 0; k < d.coll_n_fixed; ++k)
      fx |= d.coll_fixed_steps[k] == t;
    if (!(L.coll_single && fx))
      coll_slot[static_cast<size_t>(t)] = n_units++;
  }
  // (constraint form: one ineq constraint term per step pair after the other
  // constraints, problem_description.cpp:1797-1840 / OptProb eq-then-ineq order)
  L.coll_cnt = (L.coll && d.coll_is_cnt) ? 1 : 0;
  L.coll_cost0 = L.coll_cnt ? n_cnts : n_costs;
  if (L.coll)
    (L.coll_cnt ? n_cnts : n_costs) += n_units;
  if (L.coll)
  {
    // every (sphere, primitive, sub-state) and (self sphere pair, sub-state) candidate of
    // every unit is at most one contact
    std::vector<int> ssa, ssb, skp;
    self_sphere_pairs(d, ssa, ssb, skp);
    const long long bound = static_cast<long long>(n_units) * (L.coll_single ? 1 : 64) *
                            (static_cast<long long>(d.n_spheres) * std::max(d.n_prims, 1) +
                             static_cast<long long>(ssa.size()));
    // automatic: the bound, within THIP_MAX_CONTACTS and a 16 GB share of HBM for the
    // hinge-row arrays of the whole batch (~800 B per row and problem), at least 2048
    const long long by_mem = std::max<long long>(2048, (16LL << 30) / (800LL * batch));
    L.h_cap = d.coll_max_contacts > 0
                  ? d.coll_max_contacts
                  : static_cast<int>(std::min<long long>({ bound, (long long)THIP_MAX_CONTACTS, by_mem }));
  }
  else
    L.h_cap = 0;
  L.h_cap += n_sh;
  L.hinge = (L.h_cap > 0) ? 1 : 0;
  L.n_costs = n_costs;
  L.n_cnts = n_cnts;
  L.nc_base = L.nx + 2 * L.n_abs;
  L.n_rows = L.n_fixed_rows + L.n_abs;
  L.m_base = L.n_rows + L.nc_base;
  L.n_cols = L.nc_base + L.h_cap;
  L.m = L.m_base + 2 * L.h_cap;
  // step -> rows CSR
  std::vector<int> step_ptr(static_cast<size_t>(L.N + 1), 0), step_rows(static_cast<size_t>(std::max(L.n_abs, 1)));
  for (int r = 0; r < L.n_abs; ++r)
    step_ptr[static_cast<size_t>(row_step[static_cast<size_t>(r)] + 1)]++;
  for (int t = 0; t < L.N; ++t)
    step_ptr[static_cast<size_t>(t + 1)] += step_ptr[static_cast<size_t>(t)];
  {
    std::vector<int> nxt(step_ptr.begin(), step_ptr.end() - 1);
    for (int r = 0; r < L.n_abs; ++r)
      step_rows[static_cast<size_t>(nxt[static_cast<size_t>(row_step[static_cast<size_t>(r)])]++)] = r;
  }
  std::vector<int> fixed_of_step(static_cast<size_t>(L.N), -1);
  for (int f = 0; f < d.n_fixed; ++f)
    fixed_of_step[static_cast<size_t>(d.fixed_steps[f])] = f;

  // workspace layout (doubles)
  const long long nx = L.nx, nc = L.n_cols, m = L.m;
  const long long nab = std::max(L.n_abs, 1), D = L.D, hc = std::max(L.h_cap, 1);
  long long sizes[A_COUNT];
  for (int k = 0; k < A_COUNT; ++k)
    sizes[k] = -1;
  sizes[A_X] = sizes[A_XN] = sizes[A_INIT] = nx;
  sizes[A_TGT] = (long long)std::max(L.n_cart, 1) * 12;
  sizes[A_G] = sizes[A_GS] = nab * D;
  sizes[A_GC] = nab;
  sizes[A_COST] = sizes[A_NCOST] = std::max(L.n_costs, 1);
  sizes[A_VIOL] = sizes[A_NVIOL] = sizes[A_MU] = std::max(L.n_cnts, 1);
  sizes[A_PD] = sizes[A_PO] = sizes[A_CV] = sizes[A_YV] = nx;
  sizes[A_PO2] = (d.n_jdt > 0) ? nx : 1;
  sizes[A_Q] = sizes[A_DS] = sizes[A_BS] = sizes[A_XA0] = sizes[A_XA1] = sizes[A_XT] = sizes[A_DX] = nc;
  sizes[A_BA] = sizes[A_PX] = sizes[A_ATY] = sizes[A_DRV] = sizes[A_DG] = sizes[A_SOLX] = sizes[A_BXW] = nc;
  sizes[A_WS] = nab * 2;
  sizes[A_FS] = std::max(L.n_fixed_rows, 1);
  sizes[A_E] = sizes[A_L] = sizes[A_U] = sizes[A_RHO] = sizes[A_Z0] = sizes[A_Z1] = sizes[A_Y] = m;
  sizes[A_ZT] = sizes[A_DY] = sizes[A_AX] = sizes[A_PRV] = sizes[A_SOLY] = sizes[A_PZ] = m;
  sizes[A_MR] = std::max(L.n_rows, 1) + L.h_cap;
  sizes[A_RE] = std::max(L.n_rows, 1);
  // branches of the block solve (Layout::nbr): the dofs split into groups no
  // term couples -- every CartPose term joins the dofs on the root paths of its
  // source (and dynamic target) link, every collision sphere those of its link,
  // every self-collision link pair those of both links (config E's inter-arm
  // pairs join the arms: it runs the 14-dof wide path); joint-space terms touch
  // single dofs.  Two contiguous groups of <= 8 dofs
  // each (the dual arm) solve as two independent narrow block chains.
  L.nbr = 1;
  L.sD = L.D;
  std::vector<int> row_off(static_cast<size_t>(std::max(L.n_abs, 1)), 0);
  if (L.D > 8 && d.chain.is_tree && !(g_debug_path & (THIP_DEBUG_NO_BRANCH | THIP_DEBUG_FORCE_WIDE)))
  {
    std::vector<int> uf(static_cast<size_t>(L.D));
    for (int k = 0; k < L.D; ++k)
      uf[static_cast<size_t>(k)] = k;
    std::function<int(int)> root = [&](int a) {
      return uf[static_cast<size_t>(a)] == a ? a : (uf[static_cast<size_t>(a)] = root(uf[static_cast<size_t>(a)]));
    };
    auto join_path = [&](int link, int& first) {
      for (int k = link; k > 0 && k < d.chain.n_links; k = d.chain.parent[k])
      {
        const int dof = d.chain.joint_dof[k];
        if (dof < 0)
          continue;
        if (first < 0)
          first = dof;
        else
          uf[static_cast<size_t>(root(dof))] = root(first);
      }
    };
    for (int c = 0; c < d.n_cart; ++c)
    {
      int first = -1;
      join_path(d.cart_source_link[c], first);
      if (d.cart_target_link[c] > 0)
        join_path(d.cart_target_link[c], first);
    }
    if (d.coll_enabled)
    {
      for (int s2 = 0; s2 < d.n_spheres; ++s2)
      {
        int first = -1;
        join_path(d.sphere_link[s2], first);
      }
      // a self-collision pair's contacts move both links: their paths join
      for (int k = 0; k < d.n_self_pairs; ++k)
      {
        int first = -1;
        join_path(d.self_pair[k][0], first);
        join_path(d.self_pair[k][1], first);
      }
    }
    const int half = L.D / 2;
    bool split = (L.D % 2 == 0) && half <= 8 && root(0) != root(half);
    for (int k = 0; k < L.D && split; ++k)
      split = root(k) == root(k < half ? 0 : half);
    if (split)
    {
      L.nbr = 2;
      L.sD = half;
      // the branch of every CartPose / JointPos constraint row: its coefficients
      // outside the branch's dofs are exact zeros
      for (int r = 0; r < L.n_abs; ++r)
      {
        int dof = -1;
        if (row_jpos[static_cast<size_t>(r)])
          dof = row_comp[static_cast<size_t>(r)];
        else
        {
          int first = -1;
          std::vector<int> keep(uf);
          join_path(d.cart_source_link[row_term[static_cast<size_t>(r)]], first);
          uf = keep;
          dof = first;
        }
        row_off[static_cast<size_t>(r)] = (dof >= half) ? half : 0;
      }
    }
  }
  L.sN = L.nbr * L.N;
  // JointAccEqCost couples waypoints t and t + 2: solve over waypoint pairs
  // (Layout::grp; thip_jdt_fused guarantees N even and 2 D <= THIP_MAX_DOF, and
  // D <= 8 never takes the branch split above)
  L.grp = (d.n_jdt > 0) ? 2 : 1;
  if (L.grp == 2)
  {
    L.nbr = 1;
    L.sD = 2 * L.D;
    L.sN = L.N / 2;
  }
  L.sNb = L.sN / L.nbr;
  const long long sNDD = (long long)L.sN * L.sD * L.sD;
  sizes[A_LINV] = sizes[A_KB] = sNDD;
  L.wide = (L.sD > 8) ? 1 : 0;
  if (g_debug_path & THIP_DEBUG_FORCE_WIDE)  // diagnostic: the wide-block solve for any D
    L.wide = 1;
  // chain matrices M, N in HBM: for collision problems on the segment (its chain
  // runs from the pack, the LDS goes to hinge-row data) and for branched solves
  // (2 sN sD^2 doubles, 78 KB for the dual arm: the LDS keeps LINV, the solve
  // vectors and the rows' working set instead)
  L.chm_hbm = (!L.wide && ((L.hinge && L.N * 8 <= kBlock && L.N <= 2 * kCpkSteps) || L.nbr > 1)) ? 1 : 0;
  sizes[A_CHM] = (L.wide || L.chm_hbm) ? 2 * sNDD : 1;
  sizes[A_PB] = std::max(nc + m, nab * D);
  sizes[A_PS] = sizes[A_PR] = nc + m;
  sizes[A_HC0] = sizes[A_HC] = hc * 2 * D;
  sizes[A_HK] = sizes[A_HW] = sizes[A_HRE] = sizes[A_HDIST] = sizes[A_HCCT] = hc;
  sizes[A_CPL] = (L.hinge || L.nbr > 1 || L.grp > 1) ? sNDD : 1;  // dense couplings (factor())
  sizes[A_CSCR] = L.coll ? (long long)kScanWaves * kSubCap * d.n_spheres * 3 : 1;
  sizes[A_HCOST] = L.N;
  sizes[A_HPK] = L.hinge ? hc * kHPack : 1;
  const long long nchk_cap = hc / kHChunk + L.N + 1;
  sizes[A_HCHK] = L.hinge ? nchk_cap : 1;
  L.part_w = (2 * L.D <= 16) ? 16 : 32;
  sizes[A_HPART] = L.hinge ? nchk_cap * L.part_w : 1;
  sizes[A_HCT] = L.hinge ? 2 * D * (hc + 1) : 1;
  // the segment's chain pack: narrow blocks and N <= 32 only (the segment's domain)
  const bool cpk = !L.wide && L.N * 8 <= kBlock && L.N <= 2 * kCpkSteps;
  sizes[A_CPK] = cpk ? kCpk : 1;
  for (int k = 0; k < A_COUNT; ++k)
    if (sizes[k] < 0)
    {
      g_create_err = "internal: workspace size table incomplete";
      delete ctx;
      return THIP_E_INVALID;
    }
  long long off = 0;
  for (int k = 0; k < A_COUNT; ++k)
  {
    L.doff[k] = off;
    off += (sizes[k] + 7) / 8 * 8;
  }
  L.dstride = off;
  long long isizes[I_COUNT];
  isizes[I_MASK] = isizes[I_PMASK] = nab;
  isizes[I_TYPE] = isizes[I_ACT] = m;
  isizes[I_HT] = isizes[I_HMASK] = isizes[I_PHMASK] = isizes[I_PHT] = hc;
  isizes[I_HPTR] = L.N + 1;
  isizes[I_CONT] = 3 * hc;
  isizes[I_PCNT] = L.N;
  isizes[I_HKIND] = isizes[I_HSLOT] = hc;
  // one bit per (primitive, sub-state, sphere) and (self sphere pair, sub-state)
  // candidate of every unit while the sub-states number at most kScanWaves * kSubCap
  // (the batched scan), each unit's bits padded to 64
  std::vector<int> hb_sa, hb_sb, hb_kp;
  if (L.coll)
    self_sphere_pairs(d, hb_sa, hb_sb, hb_kp);
  isizes[I_HBITS] = L.coll ? (((long long)std::max(d.n_prims, 1) * d.n_spheres + (long long)hb_sa.size()) *
                                  kScanWaves * kSubCap +
                              31) / 32 +
                                 2LL * (L.N + 1)
                           : 1;
  long long ioff = 0;
  for (int k = 0; k < I_COUNT; ++k)
  {
    L.ioff[k] = ioff;
    ioff += (isizes[k] + 15) / 16 * 16;
  }
  L.istride = ioff;
  const size_t lds_d = std::max<size_t>({ (size_t)((L.wide || L.chm_hbm) ? 0 : 2 * sNDD), (size_t)(30 * std::max(L.n_cart, 1)),
                                          (size_t)(L.n_costs + L.n_cnts + 2) });
  ctx->lds_lin_bytes = lds_d * sizeof(double);
  // LDS residency plan: the per-ADMM-iteration working set, hottest first,
  // until the budget of one workgroup per CU is used; the rest stays in HBM.
  {
    const int order[] = { A_LINV, A_CV,  A_YV, A_CPK, A_BXW, A_BA, A_MR, A_DG, A_GS, A_WS, A_FS, A_BS, A_XA0, A_XA1,
                          A_Z0,   A_Z1,  A_Y,  A_XT,  A_PZ, A_RHO, A_L, A_U,  A_Q,  A_DX, A_DY, A_PD,  A_PO,  A_PO2,
                          A_E,    A_DS,  A_RE, A_PB,  A_PS, A_PR };
    int max_step_rows = 0;
    for (int t = 0; t < L.N; ++t)
      max_step_rows = std::max(max_step_rows, step_ptr[static_cast<size_t>(t) + 1] - step_ptr[static_cast<size_t>(t)]);
    // QPs outside the register-resident segment's domain (below) run the
    // generic ADMM step for the whole solve: the generic-step build of the fused
    // kernel (kGenBlock threads, no segment code) takes them; its larger static
    // LDS (reductions over 16 waves) leaves a smaller dynamic budget
    const bool seg_cand = max_step_rows <= kMaxStepRows && !L.wide && L.N * 8 <= kBlock && L.n_abs <= kBlock && cpk;
    // (contact_test_type FIRST / CLOSEST: only the generic-step build's contact scan selects among a call's contacts)
    const bool ctest = d.coll_enabled && d.coll_contact_test != THIP_CONTACT_ALL;
    ctx->gen = ctest || (!seg_cand && !(g_debug_path & THIP_DEBUG_MAIN_BUILD)) ||
               ((g_debug_path & THIP_DEBUG_NO_SEGMENT) && (g_debug_path & THIP_DEBUG_GEN_BUILD));
    const long long budget =
        (ctx->gen ? kLdsBudgetGenBytes : kLdsBudgetBytes) / static_cast<long long>(sizeof(double));
    long long used = static_cast<long long>(lds_d);
    used = (used + 7) / 8 * 8;
    L.fac_off = static_cast<int>(used);  // factor()'s 4 D x D blocks (4 nbr sD x sD; pairs: 4 of 2D x 2D)
    used += (4LL * std::max<long long>((long long)L.D * L.D, (long long)L.nbr * L.sD * L.sD) + 7) / 8 * 8;
    L.lds_scratch = static_cast<int>(used);
    for (int k = 0; k < A_COUNT; ++k)
      L.loff[k] = -1;
    for (int k : order)
    {
      const long long n = (sizes[k] + 7) / 8 * 8;
      if (used + n > budget)
        continue;
      L.loff[k] = static_cast<int>(used);
      used += n;
    }
    L.lds_doubles = static_cast<int>(used);
    L.max_step_rows = max_step_rows;
    L.rows_contig = 1;
    for (int r = 0; r < L.n_abs; ++r)
      if (step_rows[static_cast<size_t>(r)] != r)
        L.rows_contig = 0;
    // one column slot (t, i) and one CartPose row per thread: N <= 32 and
    // n_abs <= 256; larger problems run the generic admm_step()
    // (collision problems: hinge rows are loop-owned inside the segment)
    L.seg_ok = (seg_cand && L.loff[A_CPK] >= 0) ? 1 : 0;
    if ((g_debug_path & THIP_DEBUG_NO_SEGMENT) || ctx->gen)  // diagnostic: the generic ADMM step
      L.seg_ok = 0;
    L.seg_slots = 1;
    L.tw_mid = L.sNb / 2;
    if (L.loff[A_LINV] < 0 || L.loff[A_CV] < 0 || L.loff[A_YV] < 0)
    {
      g_create_err = "thip_create: problem too large, the block-solve factor does not fit in LDS";
      delete ctx;
      return THIP_E_INVALID;
    }
    ctx->lds_bytes = static_cast<size_t>(used) * sizeof(double);
    if (L.hinge)
    {
      // collision: the kernel re-plans residency for every QP with the
      // actual contact count (plan_lds_dynamic, same priority order, so
      // LINV/CV/YV keep their offsets); the launch provides the whole budget
      for (int k = 0; k < A_COUNT; ++k)
        if (k != A_LINV && k != A_CV && k != A_YV && k != A_CPK)
          L.loff[k] = -1;
      ctx->lds_bytes = static_cast<size_t>(budget) * sizeof(double);
      L.lds_doubles = static_cast<int>(budget);
    }
    L.lds_budget = static_cast<int>(ctx->lds_bytes / sizeof(double));
    if (std::getenv("THIP_DEBUG_PLAN"))  // diagnostic: the residency plan (doubles), on stderr
    {
      std::fprintf(stderr, "thip plan: gen %d wide %d hinge %d N %d D %d sN %d sD %d nx %d m %d nc %d budget %lld "
                           "fac_off %d lds_scratch %d lds_doubles %d; HBM:",
                   ctx->gen ? 1 : 0, L.wide, L.hinge, L.N, L.D, L.sN, L.sD, L.nx, L.m, L.n_cols, budget, L.fac_off,
                   L.lds_scratch, L.lds_doubles);
      for (int k : order)
        if (L.loff[k] < 0)
          std::fprintf(stderr, " %d(%lld)", k, sizes[k]);
      std::fprintf(stderr, "\n");
    }
  }

  auto fail = [&](const std::string& msg) {
    g_create_err = msg;
    thip_destroy(ctx);
    return THIP_E_HIP;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess)
    return fail(std::string("hipSetDevice: ") + hipGetErrorString(e));
  {
    // BasicTrustRegionSQPParameters::max_time (seconds) in wall_clock64() ticks
    int rate_khz = 0;
    if ((e = hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device)) != hipSuccess || rate_khz <= 0)
      return fail("hipDeviceGetAttribute(WallClockRate) failed");
    const double ticks = d.sqp.max_time * 1e3 * static_cast<double>(rate_khz);
    L.max_ticks = (ticks >= 9.0e18) ? LLONG_MAX : (ticks <= 0 ? 0LL : static_cast<long long>(ticks));
  }
  if (ctx->lds_lin_bytes > 60 * 1024)
    return fail("problem too large for the LDS-resident block solve");
  // tables
  std::vector<int> itab;
  auto push = [&](const std::vector<int>& v, size_t n) {
    const size_t o = itab.size();
    itab.insert(itab.end(), v.begin(), v.begin() + static_cast<long>(n));
    itab.resize(itab.size() + 1);  // pad so empty tables get a valid pointer
    return o;
  };
  const size_t na = static_cast<size_t>(L.n_abs);
  const size_t o_rt = push(row_term, na), o_rc = push(row_comp, na), o_rs = push(row_step, na);
  const size_t o_sp = push(step_ptr, static_cast<size_t>(L.N + 1));
  const size_t o_sr = push(step_rows, na);
  const size_t o_t0 = push(term_row0, THIP_MAX_CART), o_tn = push(term_nrow, THIP_MAX_CART),
               o_ts = push(term_slot, THIP_MAX_CART);
  const size_t o_fs = push(fixed_of_step, static_cast<size_t>(L.N));
  const size_t o_rsl = push(row_slot, na), o_rjp = push(row_jpos, na), o_rof = push(row_off, na);
  const size_t o_jq = push(jpos_ineq, THIP_MAX_JPOS);
  const size_t nsh = static_cast<size_t>(n_sh);
  const size_t o_shk = push(sh_kind, nsh), o_sho = push(sh_owner, nsh), o_shj = push(sh_joint, nsh),
               o_shs = push(sh_step, nsh), o_shp = push(sh_pair, nsh), o_shl = push(sh_slot, nsh),
               o_shq = push(sh_ptr, static_cast<size_t>(L.N + 1));
  const size_t o_jf = push(jpos_first, THIP_MAX_JPOS), o_jl = push(jpos_last, THIP_MAX_JPOS),
               o_js = push(jpos_slot, THIP_MAX_JPOS), o_j0 = push(jpos_row0, THIP_MAX_JPOS),
               o_jn = push(jpos_nrow, THIP_MAX_JPOS);
  const size_t o_xf = push(jvx_first, THIP_MAX_JVX), o_xl = push(jvx_last, THIP_MAX_JVX),
               o_xs = push(jvx_slot, THIP_MAX_JVX);
  // collision model tables: spheres grouped by link, ascending (scan order)
  std::vector<int> grp_link, grp_s0, grp_ns, sph_order, coll_fixed(static_cast<size_t>(L.N), 0);
  if (L.coll)
  {
    for (int s2 = 0; s2 < d.n_spheres; ++s2)
      sph_order.push_back(s2);
    std::stable_sort(sph_order.begin(), sph_order.end(),
                     [&](int a, int b) { return d.sphere_link[a] < d.sphere_link[b]; });
    for (size_t k = 0; k < sph_order.size(); ++k)
    {
      const int link = d.sphere_link[sph_order[k]];
      if (grp_link.empty() || grp_link.back() != link)
      {
        grp_link.push_back(link);
        grp_s0.push_back(static_cast<int>(k));
        grp_ns.push_back(0);
      }
      grp_ns.back()++;
    }
    for (int k = 0; k < d.coll_n_fixed; ++k)
      if (d.coll_fixed_steps[k] >= 0 && d.coll_fixed_steps[k] < L.N)
        coll_fixed[static_cast<size_t>(d.coll_fixed_steps[k])] = 1;
  }
  std::vector<int> self_sa, self_sb, self_kp(1, 0);
  if (L.coll)
    self_sphere_pairs(d, self_sa, self_sb, self_kp);
  const size_t o_gl = push(grp_link, grp_link.size()), o_g0 = push(grp_s0, grp_s0.size()),
               o_gn = push(grp_ns, grp_ns.size()), o_so = push(sph_order, sph_order.size()),
               o_cf = push(coll_fixed, coll_fixed.size()), o_cs = push(coll_slot, coll_slot.size()),
               o_ssa = push(self_sa, self_sa.size()), o_ssb = push(self_sb, self_sb.size()),
               o_skp = push(self_kp, self_kp.size());
  row_w.resize(std::max<size_t>(na, 1));
  if ((e = hipMalloc(&ctx->d_tables, itab.size() * sizeof(int))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_tables_f, row_w.size() * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_desc, sizeof(thip_problem_desc))) != hipSuccess)
    return fail(std::string("hipMalloc: ") + hipGetErrorString(e));
  hipMemcpy(ctx->d_tables, itab.data(), itab.size() * sizeof(int), hipMemcpyHostToDevice);
  hipMemcpy(ctx->d_tables_f, row_w.data(), row_w.size() * sizeof(double), hipMemcpyHostToDevice);
  hipMemcpy(ctx->d_desc, &ctx->desc, sizeof(thip_problem_desc), hipMemcpyHostToDevice);
  Tables& T = ctx->T;
  T.row_term = ctx->d_tables + o_rt;
  T.row_comp = ctx->d_tables + o_rc;
  T.row_step = ctx->d_tables + o_rs;
  T.step_ptr = ctx->d_tables + o_sp;
  T.step_rows = ctx->d_tables + o_sr;
  T.term_row0 = ctx->d_tables + o_t0;
  T.term_nrow = ctx->d_tables + o_tn;
  T.term_slot = ctx->d_tables + o_ts;
  T.fixed_of_step = ctx->d_tables + o_fs;
  T.row_slot = ctx->d_tables + o_rsl;
  T.row_jpos = ctx->d_tables + o_rjp;
  T.row_off = ctx->d_tables + o_rof;
  T.jpos_first = ctx->d_tables + o_jf;
  T.jpos_last = ctx->d_tables + o_jl;
  T.jpos_slot = ctx->d_tables + o_js;
  T.jpos_row0 = ctx->d_tables + o_j0;
  T.jpos_nrow = ctx->d_tables + o_jn;
  T.jpos_ineq = ctx->d_tables + o_jq;
  T.jvx_first = ctx->d_tables + o_xf;
  T.jvx_last = ctx->d_tables + o_xl;
  T.jvx_slot = ctx->d_tables + o_xs;
  T.n_sh = n_sh;
  T.sh_kind = ctx->d_tables + o_shk;
  T.sh_owner = ctx->d_tables + o_sho;
  T.sh_joint = ctx->d_tables + o_shj;
  T.sh_step = ctx->d_tables + o_shs;
  T.sh_pair = ctx->d_tables + o_shp;
  T.sh_slot = ctx->d_tables + o_shl;
  T.sh_ptr = ctx->d_tables + o_shq;
  T.n_groups = static_cast<int>(grp_link.size());
  T.grp_link = ctx->d_tables + o_gl;
  T.grp_s0 = ctx->d_tables + o_g0;
  T.grp_ns = ctx->d_tables + o_gn;
  T.sph_order = ctx->d_tables + o_so;
  T.coll_fixed = ctx->d_tables + o_cf;
  T.coll_slot = ctx->d_tables + o_cs;
  T.n_self_keys = static_cast<int>(self_kp.size()) - 1;
  T.n_self_sph = static_cast<int>(self_sa.size());
  T.self_sa = ctx->d_tables + o_ssa;
  T.self_sb = ctx->d_tables + o_ssb;
  T.self_kp = ctx->d_tables + o_skp;
  T.row_w = ctx->d_tables_f;
  T.pair_mc = nullptr;
  {
    std::vector<double> ptab;
    if (L.coll && coll_pair_table(d, 0, ptab))
    {
      if ((e = hipMalloc(&ctx->d_pair, ptab.size() * sizeof(double))) != hipSuccess ||
          (e = hipMemcpy(ctx->d_pair, ptab.data(), ptab.size() * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(std::string("hipMalloc(pair table): ") + hipGetErrorString(e));
      T.pair_mc = ctx->d_pair;
    }
  }
  const size_t B = static_cast<size_t>(batch);
  if ((e = hipMalloc(&ctx->d_ws, B * static_cast<size_t>(L.dstride) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_iws, B * static_cast<size_t>(L.istride) * sizeof(int))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_res, B * sizeof(thip_result))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_init, B * static_cast<size_t>(nx) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_tgt, B * static_cast<size_t>(std::max(L.n_cart, 1)) * 12 * sizeof(double))) !=
          hipSuccess ||
      (e = hipMalloc(&ctx->d_x, B * static_cast<size_t>(nx) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_jpt, B * static_cast<size_t>(std::max(L.n_jpos, 1) * L.D) * sizeof(double))) !=
          hipSuccess)
    return fail(std::string("hipMalloc(workspace): ") + hipGetErrorString(e));
  {
    // every problem starts with the descriptor's JointPos targets
    const size_t per = static_cast<size_t>(std::max(L.n_jpos, 1) * L.D);
    std::vector<double> jpt(B * per, 0.0);
    for (size_t b = 0; b < B; ++b)
      for (int k = 0; k < L.n_jpos; ++k)
        for (int j = 0; j < L.D; ++j)
          jpt[b * per + static_cast<size_t>(k * L.D + j)] = d.jpos_targets[k][j];
    if ((e = hipMemcpy(ctx->d_jpt, jpt.data(), jpt.size() * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(std::string("hipMemcpy(jpos targets): ") + hipGetErrorString(e));
  }
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(std::string("hipStreamCreate: ") + hipGetErrorString(e));
  ctx->own_stream = true;
  // zeroed on the context's own (non-blocking) stream and waited for here: a
  // non-blocking stream does not order against the null stream, and the
  // caller may swap in its own stream (thip_set_stream) before the first run
  if ((e = hipMemsetAsync(ctx->d_iws, 0, B * static_cast<size_t>(L.istride) * sizeof(int), ctx->stream)) !=
          hipSuccess ||
      (e = hipMemsetAsync(ctx->d_res, 0, B * sizeof(thip_result), ctx->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
    return fail(std::string("hipMemsetAsync(workspace): ") + hipGetErrorString(e));
  if ((e = hipEventCreate(&ctx->ev0)) != hipSuccess || (e = hipEventCreate(&ctx->ev1)) != hipSuccess)
    return fail(std::string("hipEventCreate: ") + hipGetErrorString(e));
  const void* fused = ctx->gen ? reinterpret_cast<const void*>(&sqp_kernel_gen) : reinterpret_cast<const void*>(&sqp_kernel);
  const int fused_block = ctx->gen ? kGenBlock : kBlock;
  if ((e = hipFuncSetAttribute(fused, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ctx->lds_bytes))) !=
          hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(&linearize_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ctx->lds_lin_bytes))) !=
          hipSuccess)
    return fail(std::string("hipFuncSetAttribute(dynamic LDS): ") + hipGetErrorString(e));
  // dynamic problem assignment: one persistent workgroup per resident slot
  // (KernelArgs::work), unless THIP_DEBUG_STATIC_DISPATCH is set (one workgroup per problem)
  ctx->grid = batch;
  if (!(g_debug_path & THIP_DEBUG_STATIC_DISPATCH))
  {
    int per_cu = 0, n_cu = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fused, fused_block, ctx->lds_bytes)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
      return fail(std::string("occupancy query: ") + hipGetErrorString(e));
    const long long slots = static_cast<long long>(std::max(per_cu, 1)) * std::max(n_cu, 1);
    if (slots < batch)
    {
      if ((e = hipMalloc(&ctx->d_work, 2 * sizeof(int))) != hipSuccess ||
          (e = hipMemsetAsync(ctx->d_work, 0, 2 * sizeof(int), ctx->stream)) != hipSuccess ||
          (e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
        return fail(std::string("work counter: ") + hipGetErrorString(e));
      ctx->grid = static_cast<int>(slots);
    }
  }
  *out = ctx;
  return THIP_OK;
}

int thip_set_stream(thip_ctx* ctx, void* stream)
{
  if (!ctx)
    return THIP_E_INVALID;
  if (stream == nullptr)
    return THIP_OK;
  if (ctx->own_stream && ctx->stream)
    hipStreamDestroy(ctx->stream);
  ctx->stream = static_cast<hipStream_t>(stream);
  ctx->own_stream = false;
  return THIP_OK;
}

static KernelArgs make_args(thip_ctx* ctx)
{
  KernelArgs a;
  a.L = ctx->L;
  a.T = ctx->T;
  a.desc = ctx->d_desc;
  a.ws = ctx->d_ws;
  a.iws = ctx->d_iws;
  a.res = ctx->d_res;
  a.batch = ctx->batch;
  a.scene = ctx->d_scene;
  a.jpt = ctx->d_jpt;
  a.trace = ctx->d_trace;
  a.trace_n = ctx->d_trace_n;
  a.trace_cap = ctx->trace_cap;
  a.prof = ctx->d_prof;
  a.stage_init = nullptr;
  a.stage_tgt = nullptr;
  a.xout = nullptr;
  a.work = nullptr;
  return a;
}

static int upload_common(thip_ctx* ctx, const double* init, const double* tgt, hipMemcpyKind kind)
{
  const size_t B = static_cast<size_t>(ctx->batch);
  const size_t nx = static_cast<size_t>(ctx->L.nx);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (!init)
    return ctx->err = "thip_upload: init_traj is required", THIP_E_INVALID;
  HIPCHK(ctx, hipMemcpyAsync(ctx->d_init, init, B * nx * sizeof(double), kind, ctx->stream));
  if (ctx->L.n_cart > 0)
  {
    if (!tgt)
      return ctx->err = "thip_upload: cart_targets required when n_cart > 0", THIP_E_INVALID;
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_tgt, tgt, B * static_cast<size_t>(ctx->L.n_cart) * 12 * sizeof(double), kind,
                               ctx->stream));
  }
  KernelArgs a = make_args(ctx);
  hipLaunchKernelGGL(stage_inputs_kernel, dim3(ctx->batch), dim3(kBlock), 0, ctx->stream, a, ctx->d_init, ctx->d_tgt);
  HIPCHK(ctx, hipGetLastError());
  ctx->uploaded = true;
  return THIP_OK;
}

static int upload_scene(thip_ctx* ctx, const double* scene, hipMemcpyKind kind)
{
  if (!ctx->L.coll)
    return THIP_OK;
  if (!scene && ctx->desc.n_prims > 0)
    return ctx->err = "thip_upload: scene required when collision is enabled", THIP_E_INVALID;
  const size_t bytes = static_cast<size_t>(ctx->batch) * std::max(ctx->desc.n_prims, 1) * 16 * sizeof(double);
  if (!ctx->d_scene)
    HIPCHK(ctx, hipMalloc(&ctx->d_scene, bytes));
  if (ctx->desc.n_prims > 0)
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_scene, scene, bytes, kind, ctx->stream));
  return THIP_OK;
}

int thip_upload(thip_ctx* ctx, const double* init_traj, const double* cart_targets, const double* scene)
{
  if (!ctx)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (const int rs = upload_scene(ctx, scene, hipMemcpyHostToDevice); rs != THIP_OK)
    return rs;
  const int rc = upload_common(ctx, init_traj, cart_targets, hipMemcpyHostToDevice);
  if (rc == THIP_OK)
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return rc;
}

int thip_upload_joint_targets(thip_ctx* ctx, const double* jpos_targets)
{
  if (!ctx)
    return THIP_E_INVALID;
  if (ctx->L.n_jpos == 0)
    return THIP_OK;
  if (!jpos_targets)
    return ctx->err = "thip_upload_joint_targets: null targets", THIP_E_INVALID;
  const size_t n = static_cast<size_t>(ctx->batch) * ctx->L.n_jpos * ctx->L.D;
  for (size_t i = 0; i < n; ++i)
    if (!std::isfinite(jpos_targets[i]))
      return ctx->err = "thip_upload_joint_targets: non-finite target", THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemcpyAsync(ctx->d_jpt, jpos_targets, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return THIP_OK;
}

int thip_upload_device(thip_ctx* ctx, const double* d_init_traj, const double* d_cart_targets, const double* d_scene)
{
  if (!ctx)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (const int rs = upload_scene(ctx, d_scene, hipMemcpyDeviceToDevice); rs != THIP_OK)
    return rs;
  return upload_common(ctx, d_init_traj, d_cart_targets, hipMemcpyDeviceToDevice);
}

int thip_sqp_run(thip_ctx* ctx)
{
  if (!ctx)
    return THIP_E_INVALID;
  if (!ctx->uploaded)
    return ctx->err = "thip_sqp_run: call thip_upload first", THIP_E_STATE;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  KernelArgs a = make_args(ctx);
  // one launch: each workgroup re-stages its problem's uploaded inputs (a run always
  // starts from the uploaded initial trajectory) and gathers its final trajectory, so
  // no small kernels queue behind another batch's workgroups when batches overlap
  a.stage_init = ctx->d_init;
  a.stage_tgt = ctx->d_tgt;
  a.xout = ctx->d_x;
  a.work = ctx->d_work;
  HIPCHK(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  if (ctx->gen)
    hipLaunchKernelGGL(sqp_kernel_gen, dim3(ctx->d_work ? ctx->grid : ctx->batch), dim3(kGenBlock), ctx->lds_bytes,
                       ctx->stream, a);
  else
    hipLaunchKernelGGL(sqp_kernel, dim3(ctx->d_work ? ctx->grid : ctx->batch), dim3(kBlock), ctx->lds_bytes,
                       ctx->stream, a);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  ctx->ran = true;
  return THIP_OK;
}

int thip_synchronize(thip_ctx* ctx)
{
  if (!ctx)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

double thip_last_kernel_ms(thip_ctx* ctx)
{
  if (!ctx || !ctx->ran)
    return -1.0;
  float ms = 0;
  if (hipEventSynchronize(ctx->ev1) != hipSuccess)
    return -1.0;
  if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess)
    return -1.0;
  return static_cast<double>(ms);
}

int thip_download(thip_ctx* ctx, double* x, thip_result* results)
{
  if (!ctx)
    return THIP_E_INVALID;
  if (!ctx->ran)
    return ctx->err = "thip_download: nothing has run", THIP_E_STATE;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t B = static_cast<size_t>(ctx->batch);
  if (x)
    HIPCHK(ctx, hipMemcpyAsync(x, ctx->d_x, B * static_cast<size_t>(ctx->L.nx) * sizeof(double),
                               hipMemcpyDeviceToHost, ctx->stream));
  if (results)
    HIPCHK(ctx, hipMemcpyAsync(results, ctx->d_res, B * sizeof(thip_result), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return THIP_OK;
}

const double* thip_device_x(thip_ctx* ctx) { return ctx ? ctx->d_x : nullptr; }

int thip_linearize(thip_ctx* ctx, const double* x, double* err, double* jac)
{
  if (!ctx || !x || !err || !jac)
    return THIP_E_INVALID;
  if (!ctx->uploaded)
    return ctx->err = "thip_linearize: call thip_upload first (targets)", THIP_E_STATE;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t B = static_cast<size_t>(ctx->batch);
  const Layout& L = ctx->L;
  double *dx = nullptr, *de = nullptr, *dj = nullptr;
  const size_t ne = B * static_cast<size_t>(L.n_cart) * 6, nj = ne * static_cast<size_t>(L.D);
  HIPCHK(ctx, hipMalloc(&dx, B * static_cast<size_t>(L.nx) * sizeof(double)));
  HIPCHK(ctx, hipMalloc(&de, std::max<size_t>(ne, 1) * sizeof(double)));
  HIPCHK(ctx, hipMalloc(&dj, std::max<size_t>(nj, 1) * sizeof(double)));
  hipMemcpyAsync(dx, x, B * static_cast<size_t>(L.nx) * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  KernelArgs a = make_args(ctx);
  hipLaunchKernelGGL(linearize_kernel, dim3(ctx->batch), dim3(kBlock), ctx->lds_lin_bytes, ctx->stream, a, dx, de, dj);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
  {
    hipMemcpyAsync(err, de, ne * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    hipMemcpyAsync(jac, dj, nj * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    e = hipStreamSynchronize(ctx->stream);
  }
  hipFree(dx);
  hipFree(de);
  hipFree(dj);
  if (e != hipSuccess)
    return ctx->err = std::string("thip_linearize: ") + hipGetErrorString(e), THIP_E_HIP;
  return THIP_OK;
}

int thip_fwd_kin(thip_ctx* ctx, const double* x, double* poses)
{
  if (!ctx || !x || !poses)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t B = static_cast<size_t>(ctx->batch);
  const Layout& L = ctx->L;
  const size_t np = B * static_cast<size_t>(L.N) * static_cast<size_t>(L.n_links) * 12;
  double *dx = nullptr, *dp = nullptr;
  HIPCHK(ctx, hipMalloc(&dx, B * static_cast<size_t>(L.nx) * sizeof(double)));
  HIPCHK(ctx, hipMalloc(&dp, np * sizeof(double)));
  hipMemcpyAsync(dx, x, B * static_cast<size_t>(L.nx) * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  KernelArgs a = make_args(ctx);
  hipLaunchKernelGGL(fwd_kin_kernel, dim3(ctx->batch), dim3(kBlock), 0, ctx->stream, a, dx, dp);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
  {
    hipMemcpyAsync(poses, dp, np * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    e = hipStreamSynchronize(ctx->stream);
  }
  hipFree(dx);
  hipFree(dp);
  if (e != hipSuccess)
    return ctx->err = std::string("thip_fwd_kin: ") + hipGetErrorString(e), THIP_E_HIP;
  return THIP_OK;
}

int thip_debug_trace(thip_ctx* ctx, int capacity)
{
  if (!ctx || capacity < 0)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ctx->d_trace)
    hipFree(ctx->d_trace);
  if (ctx->d_trace_n)
    hipFree(ctx->d_trace_n);
  ctx->d_trace = nullptr;
  ctx->d_trace_n = nullptr;
  ctx->trace_cap = capacity;
  if (capacity == 0)
    return THIP_OK;
  const size_t B = static_cast<size_t>(ctx->batch);
  HIPCHK(ctx, hipMalloc(&ctx->d_trace, B * static_cast<size_t>(capacity) * THIP_TRACE_W * sizeof(double)));
  HIPCHK(ctx, hipMalloc(&ctx->d_trace_n, B * sizeof(int)));
  // ordered with the runs on the context's stream (non-blocking: the null
  // stream would not order against it)
  HIPCHK(ctx, hipMemsetAsync(ctx->d_trace_n, 0, B * sizeof(int), ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return THIP_OK;
}

int thip_debug_layout(thip_ctx* ctx, long long* doff, long long* ioff, long long* dims)
{
  if (!ctx)
    return THIP_E_INVALID;
  const Layout& L = ctx->L;
  for (int k = 0; k < A_COUNT; ++k)
    doff[k] = L.doff[k];
  for (int k = 0; k < I_COUNT; ++k)
    ioff[k] = L.ioff[k];
  const long long d[] = { L.N, L.D, L.nx, L.n_fixed_rows, L.n_abs, L.n_cols, L.n_rows, L.m, L.dstride, L.istride,
                          A_COUNT, I_COUNT };
  for (int k = 0; k < 12; ++k)
    dims[k] = d[k];
  return THIP_OK;
}

int thip_debug_workspace(thip_ctx* ctx, double* dws, int* iws)
{
  if (!ctx)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  const size_t B = static_cast<size_t>(ctx->batch);
  HIPCHK(ctx, hipMemcpy(dws, ctx->d_ws, B * static_cast<size_t>(ctx->L.dstride) * sizeof(double),
                        hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemcpy(iws, ctx->d_iws, B * static_cast<size_t>(ctx->L.istride) * sizeof(int),
                        hipMemcpyDeviceToHost));
  return THIP_OK;
}

int thip_collision_rows(thip_ctx* ctx, const double* x, double* records, int cap, int* counts)
{
  if (!ctx || !x || !records || !counts || cap <= 0)
    return THIP_E_INVALID;
  if (!ctx->L.coll)
    return ctx->err = "thip_collision_rows: collision is not enabled", THIP_E_STATE;
  if (!ctx->uploaded || !ctx->d_scene)
    return ctx->err = "thip_collision_rows: call thip_upload first (scene)", THIP_E_STATE;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t B = static_cast<size_t>(ctx->batch);
  const Layout& L = ctx->L;
  const size_t W = 8 + 2 * static_cast<size_t>(L.D) + 1;
  double *dx = nullptr, *dout = nullptr;
  int* dcnt = nullptr;
  hipError_t e;
  if ((e = hipMalloc(&dx, B * L.nx * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&dout, B * static_cast<size_t>(cap) * W * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&dcnt, B * sizeof(int))) != hipSuccess)
  {
    hipFree(dx);
    hipFree(dout);
    hipFree(dcnt);
    return ctx->err = std::string("thip_collision_rows: hipMalloc: ") + hipGetErrorString(e), THIP_E_NOMEM;
  }
  hipMemcpyAsync(dx, x, B * L.nx * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  hipMemsetAsync(dout, 0, B * static_cast<size_t>(cap) * W * sizeof(double), ctx->stream);
  KernelArgs a = make_args(ctx);
  // the contact scan of the build the context's SQP runs
  if (ctx->gen)
    hipLaunchKernelGGL(coll_rows_kernel_gen, dim3(ctx->batch), dim3(kGenBlock), 0, ctx->stream, a, dx, dout, cap, dcnt);
  else
    hipLaunchKernelGGL(coll_rows_kernel, dim3(ctx->batch), dim3(kBlock), 0, ctx->stream, a, dx, dout, cap, dcnt);
  e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(records, dout, B * static_cast<size_t>(cap) * W * sizeof(double), hipMemcpyDeviceToHost,
                       ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(counts, dcnt, B * sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess)
    e = hipStreamSynchronize(ctx->stream);
  hipFree(dx);
  hipFree(dout);
  hipFree(dcnt);
  if (e != hipSuccess)
    return ctx->err = std::string("thip_collision_rows: ") + hipGetErrorString(e), THIP_E_HIP;
  return THIP_OK;
}

int thip_debug_profile(thip_ctx* ctx, int enable)
{
  if (!ctx)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ctx->d_prof)
    hipFree(ctx->d_prof);
  ctx->d_prof = nullptr;
  if (!enable)
    return THIP_OK;
  const size_t n = static_cast<size_t>(ctx->batch) * kProfSlots;
  HIPCHK(ctx, hipMalloc(&ctx->d_prof, n * sizeof(long long)));
  HIPCHK(ctx, hipMemsetAsync(ctx->d_prof, 0, n * sizeof(long long), ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return THIP_OK;
}

int thip_debug_get_profile(thip_ctx* ctx, long long* counters)
{
  if (!ctx || !ctx->d_prof || !counters)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipMemcpy(counters, ctx->d_prof, static_cast<size_t>(ctx->batch) * kProfSlots * sizeof(long long),
                        hipMemcpyDeviceToHost));
  return THIP_OK;
}

int thip_debug_get_trace(thip_ctx* ctx, double* records, int* counts)
{
  if (!ctx || !ctx->d_trace || !records || !counts)
    return THIP_E_INVALID;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  const size_t B = static_cast<size_t>(ctx->batch);
  HIPCHK(ctx, hipMemcpy(records, ctx->d_trace, B * static_cast<size_t>(ctx->trace_cap) * THIP_TRACE_W * sizeof(double),
                        hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemcpy(counts, ctx->d_trace_n, B * sizeof(int), hipMemcpyDeviceToHost));
  return THIP_OK;
}

void thip_destroy(thip_ctx* ctx)
{
  if (!ctx)
    return;
  hipSetDevice(ctx->device);
  if (ctx->stream)
    hipStreamSynchronize(ctx->stream);
  hipFree(ctx->d_desc);
  hipFree(ctx->d_tables);
  hipFree(ctx->d_tables_f);
  hipFree(ctx->d_pair);
  hipFree(ctx->d_ws);
  hipFree(ctx->d_iws);
  hipFree(ctx->d_res);
  hipFree(ctx->d_work);
  hipFree(ctx->d_init);
  hipFree(ctx->d_tgt);
  hipFree(ctx->d_scene);
  hipFree(ctx->d_jpt);
  hipFree(ctx->d_x);
  hipFree(ctx->d_trace);
  hipFree(ctx->d_trace_n);
  if (ctx->ev0)
    hipEventDestroy(ctx->ev0);
  if (ctx->ev1)
    hipEventDestroy(ctx->ev1);
  if (ctx->own_stream && ctx->stream)
    hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* thip_last_error(thip_ctx* ctx)
{
  if (!ctx)
    return g_create_err.c_str();
  return ctx->err.c_str();
}

}  // extern "C"

// small kernels: stage per-problem inputs into the workspace, gather results
namespace thip
{
__global__ void stage_inputs_kernel(KernelArgs args, const double* init, const double* tgt)
{
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  const Layout& L = args.L;
  double* w = args.ws + (long long)b * L.dstride;
  for (int i = threadIdx.x; i < L.nx; i += blockDim.x)
  {
    const double v = init[(long long)b * L.nx + i];
    w[L.doff[A_INIT] + i] = v;
    w[L.doff[A_X] + i] = v;
  }
  for (int i = threadIdx.x; i < L.n_cart * 12; i += blockDim.x)
    w[L.doff[A_TGT] + i] = tgt[(long long)b * L.n_cart * 12 + i];
}

__global__ void gather_x_kernel(KernelArgs args, double* xout)
{
  const int b = blockIdx.x;
  if (b >= args.batch)
    return;
  const Layout& L = args.L;
  const double* w = args.ws + (long long)b * L.dstride;
  for (int i = threadIdx.x; i < L.nx; i += blockDim.x)
    xout[(long long)b * L.nx + i] = w[L.doff[A_X] + i];
}
}  // namespace thip
