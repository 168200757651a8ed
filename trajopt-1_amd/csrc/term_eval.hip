// Device evaluation of the kinematic terms for the host SQP loop (the generic
// path): CartPose error + forward-difference jacobian and the collision
// contacts of one collision term with their linearised distance expressions,
// for problems the fused sqp_kernel does not lower (single-waypoint problems,
// several collision terms, CartPose / collision next to JointAcc / JointJerk /
// time terms or a user sco::Cost).  include/trajopt_hip.h thip_eval_*.
//
//   cart_eval_kernel   CartPoseErrCalculator / CartPoseJacCalculator and the
//                      DynamicCartPose pair (trajopt/src/kinematic_terms.cpp:58-370):
//                      one wave per problem, lane 0 the unperturbed pose, lane
//                      p + 1 the FK perturbed in dof p (the arithmetic of
//                      sqp_kernel.hip linearize()).
//   coll_eval_kernel   CollisionEvaluator::CalcCollisions + GetGradient +
//                      CalcDistExpressions* for one unit (a free waypoint for
//                      DISCRETE, SingleTimestepCollisionEvaluator
//                      collision_terms.cpp:538-554,646-688; a step pair for
//                      LVS_DISCRETE :817-898 and LVS_CONTINUOUS :1065-1161;
//                      gradient :195-242; expressions :341-386, 463-536): one
//                      256-thread workgroup per (unit, problem) walks the
//                      (sphere, primitive, sub-state) candidates in the
//                      flattened ContactResultMap order (robot link, primitive,
//                      then insertion order sub-state, sphere), 256 at a time;
//                      a ballot + cross-wave prefix gives each contact its rank,
//                      so the list comes out ordered without a sort.  The
//                      arithmetic is oracle/src/collision.cpp's.
//   coll_pack_kernel   concatenates the units' records per problem.
// fp64 throughout; integer/geometry work, no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "collision_device.hpp"
#include "kin_device.hpp"
#include "pair_data.hpp"
#include "self_pairs.hpp"

namespace thip
{
namespace ev
{
constexpr int kEvBlock = 256;
constexpr int kEvWaves = kEvBlock / 64;

// one collision term as the kernels read it
struct CollTerm
{
  int single;      // DISCRETE: one state per unit
  int continuous;  // LVS_CONTINUOUS: casts between consecutive sub-states
  double margin, buffer, lvs;
  // per link-pair margins (pair_data.hpp, [n_spheres][pw][2]; null: `margin` for every pair)
  const double* pmc;
  int pw;
  int contact_test;  // THIP_CONTACT_ALL / FIRST / CLOSEST (trajopt_hip.h)
};

// the contact distance margin of robot sphere s against primitive p (p >= 0)
// or robot sphere -1 - p (CollisionMarginData, collision_terms.cpp:243-332)
__device__ __forceinline__ double pair_margin(const CollTerm& tm, int n_prims, int s, int p)
{
  return tm.pmc ? tm.pmc[2 * (s * tm.pw + (p >= 0 ? p : n_prims + (-1 - p)))] : tm.margin;
}

// per-term unit table: unit u covers waypoint t0 (and t0 + 1 unless single);
// f0 / f1: the ends that are fixed steps of the term
struct Unit
{
  int t0, f0, f1;
};

// the robot spheres grouped by link, ascending (ContactResultMap key order)
struct Spheres
{
  int n_groups;
  int grp_link[THIP_MAX_SPHERES];
  int grp_s0[THIP_MAX_SPHERES];
  int grp_ns[THIP_MAX_SPHERES];
  int sph_order[THIP_MAX_SPHERES];
  double center[THIP_MAX_SPHERES][3];
  double radius[THIP_MAX_SPHERES];
  int link[THIP_MAX_SPHERES];
  // self-collision sphere pairs in key order (self_pairs.hpp)
  int n_self_keys, n_self_sph;
  int self_sa[THIP_MAX_SELF_SPHERE_PAIRS];
  int self_sb[THIP_MAX_SELF_SPHERE_PAIRS];
  int self_kp[THIP_MAX_SELF_PAIRS + 1];
};

__shared__ thip_chain s_chain;

__device__ __forceinline__ void stage_chain_ev(const thip_chain* ch)
{
  const int* src = reinterpret_cast<const int*>(ch);
  int* dst = reinterpret_cast<int*>(&s_chain);
  for (int w = threadIdx.x; w < static_cast<int>(sizeof(thip_chain) / 4); w += blockDim.x)
    dst[w] = src[w];
  __syncthreads();
}

// ------------------------------------------------------------------ CartPose
struct CartArgs
{
  int D;
  int source_link, target_link, has_tol;
  double source_offset[12];
  double lower_tol[6], upper_tol[6];
};

static CartArgs cart_args(const thip_problem_desc& d, int term)
{
  CartArgs a{};
  a.D = d.chain.n_dof;
  a.source_link = d.cart_source_link[term];
  a.target_link = d.cart_target_link[term];
  a.has_tol = d.cart_has_tol[term];
  std::memcpy(a.source_offset, d.cart_source_offset[term], sizeof(a.source_offset));
  std::memcpy(a.lower_tol, d.cart_lower_tol[term], sizeof(a.lower_tol));
  std::memcpy(a.upper_tol, d.cart_upper_tol[term], sizeof(a.upper_tol));
  return a;
}

// One CartPose term at one problem's joint values qb: err[6] and (jac non-null)
// jac[6][D].  One 64-lane wavefront: lane 0 the error, lane p + 1 the FK
// perturbed in dof p.  Shared by the one-term and the all-terms kernels, so
// both give the same bits.
__device__ void cart_eval_one(const thip_chain& ch, const CartArgs& a, const double* qb, const double* to12,
                              double* err, double* jac)
{
  const int D = a.D, lane = threadIdx.x;
  __shared__ Pose s_src, s_tinv;
  if (lane == 0)
  {
    Pose S, So, Ss, Tb, To, Tt, Ti;
    chain_fk(ch, qb, a.source_link, S);
    pose_load(So, a.source_offset);
    pose_mul(S, So, Ss);
    pose_load(To, to12);
    if (a.target_link > 0)
      chain_fk(ch, qb, a.target_link, Tb);  // DynamicCartPose: the active target link
    else
      pose_load(Tb, ch.base_pose);
    pose_mul(Tb, To, Tt);
    pose_inv(Tt, Ti);
    double e[6];
    transform_error(Ti, Ss, e);
    if (a.has_tol)
      apply_tolerances(e, a.lower_tol, a.upper_tol);
    for (int i = 0; i < 6; ++i)
      err[i] = e[i];
    s_src = Ss;
    s_tinv = Ti;
  }
  __syncthreads();
  if (!jac || lane < 1 || lane > D)
    return;
  // forward difference in dof p (CartPoseJacCalculator, eps 1e-5)
  const int p = lane - 1;
  const double eps = 1e-5;
  double qp[THIP_MAX_DOF];
  for (int j = 0; j < D; ++j)
    qp[j] = qb[j];
  qp[p] = qp[p] + eps;
  Pose S, So, Sp;
  chain_fk(ch, qp, a.source_link, S);
  pose_load(So, a.source_offset);
  pose_mul(S, So, Sp);
  const Pose Ss = s_src, Ti = s_tinv;
  Pose pe, ppe;
  pose_mul(Ti, Ss, pe);
  if (a.target_link > 0)
  {
    Pose Tq, To, Tp, Tpi;
    chain_fk(ch, qp, a.target_link, Tq);
    pose_load(To, to12);
    pose_mul(Tq, To, Tp);
    pose_inv(Tp, Tpi);
    pose_mul(Tpi, Sp, ppe);
  }
  else
    pose_mul(Ti, Sp, ppe);
  double diff[6];
  if (a.has_tol)
    transform_error_diff_tol(pe, ppe, a.lower_tol, a.upper_tol, diff);
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
  for (int i = 0; i < 6; ++i)
    jac[i * D + p] = diff[i] / eps;
}

__global__ __launch_bounds__(64) void cart_eval_kernel(const thip_chain* chain, CartArgs a, int batch, int n_cart,
                                                      int term, const double* q, const double* tgt, double* err,
                                                      double* jac)
{
  const int b = blockIdx.x;
  if (b >= batch)
    return;
  stage_chain_ev(chain);
  const long long D = a.D;
  cart_eval_one(s_chain, a, q + b * D, tgt + (static_cast<long long>(b) * n_cart + term) * 12, err + b * 6LL,
                jac ? jac + b * 6 * D : nullptr);
}

// every CartPose term of every problem at its own waypoint of the joint
// trajectories x [batch][N][D]: one workgroup per (problem, term),
// err [batch][n_cart][6], jac [batch][n_cart][6][D] (or null)
__global__ __launch_bounds__(64) void cart_eval_all_kernel(const thip_chain* chain, const CartArgs* args,
                                                          const int* steps, int batch, int n_cart, int N,
                                                          const double* x, const double* tgt, double* err,
                                                          double* jac)
{
  const int item = blockIdx.x;
  if (item >= batch * n_cart)
    return;
  stage_chain_ev(chain);
  const int b = item / n_cart, k = item % n_cart;
  const CartArgs a = args[k];
  const long long D = a.D;
  cart_eval_one(s_chain, a, x + (static_cast<long long>(b) * N + steps[k]) * D, tgt + static_cast<long long>(item) * 12,
                err + item * 6LL, jac ? jac + item * 6 * D : nullptr);
}

// ------------------------------------------------------------------ collision
constexpr int kCCNone = 0, kCCTime0 = 1, kCCTime1 = 2, kCCBetween = 3;

__device__ __forceinline__ void sphere_world(const Pose& T, const double* cl, double* c)
{
  for (int r = 0; r < 3; ++r)
    c[r] = T.r[r * 3 + 0] * cl[0] + T.r[r * 3 + 1] * cl[1] + T.r[r * 3 + 2] * cl[2] + T.t[r];
}

// CollisionEvaluator::GetGradient for one robot link at the waypoint's own
// joint values (oracle/src/collision.cpp contactGradient): sg = -1 for
// link_ids[0], +1 for the second link of a self contact
__device__ void contact_gradient(const thip_chain& ch, const double* dof, int link, const Pose& lt,
                                 const double* p_local, const double* normal, double sg, double* grad)
{
  const int D = ch.n_dof;
  double J[6 * THIP_MAX_DOF];
  chain_jacobian(ch, dof, link, J);
  double r[3];
  for (int i = 0; i < 3; ++i)
    r[i] = lt.r[i * 3 + 0] * p_local[0] + lt.r[i * 3 + 1] * p_local[1] + lt.r[i * 3 + 2] * p_local[2];
  for (int j = 0; j < D; ++j)
  {
    const double wx = J[3 * D + j], wy = J[4 * D + j], wz = J[5 * D + j];
    const double l0 = J[0 * D + j] + (wy * r[2] - wz * r[1]);
    const double l1 = J[1 * D + j] + (wz * r[0] - wx * r[2]);
    const double l2 = J[2 * D + j] + (wx * r[1] - wy * r[0]);
    grad[j] = sg * (normal[0] * l0 + normal[1] * l1 + normal[2] * l2);
  }
}

// records of unit u of problem b: stage [b][u][ucap][W], counts [b][n_units]
__global__ __launch_bounds__(kEvBlock) void coll_eval_kernel(const thip_chain* chain, const Spheres* sph, CollTerm tm,
                                                            const Unit* units, int n_units, int batch, int N,
                                                            const double* x, const double* scene, int n_prims,
                                                            double* stage, int ucap, int* counts)
{
  const int u = blockIdx.x, b = blockIdx.y;
  if (u >= n_units || b >= batch)
    return;
  stage_chain_ev(chain);
  const thip_chain& ch = s_chain;
  const int D = ch.n_dof, W = 8 + 2 * D + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Unit un = units[u];
  const double* q0 = x + (static_cast<long long>(b) * N + un.t0) * D;
  const double* q1 = tm.single ? q0 : q0 + D;
  const double* prims = scene + static_cast<long long>(b) * (n_prims > 0 ? n_prims : 1) * 16;
  // sub-states (DiscreteCollisionEvaluator / CastCollisionEvaluator, collision_terms.cpp:846-852)
  const int cnt = tm.single ? 1 : lvs_count(q0, q1, D, tm.lvs);
  const int n_sub = tm.single ? 1 : (tm.continuous ? cnt - 1 : cnt);
  const int last = cnt - 1;
  const double dt = tm.single ? 0.0 : 1.0 / double(last);
  const Spheres& S = *sph;
  const int n_sph = [&] {
    int n = 0;
    for (int g = 0; g < S.n_groups; ++g)
      n += S.grp_ns[g];
    return n;
  }();
  const long long scene_total = static_cast<long long>(n_sph) * n_prims * n_sub;
  const long long total = scene_total + static_cast<long long>(S.n_self_sph) * n_sub;
  __shared__ int s_wave_cnt[kEvWaves];
  __shared__ int s_base;
  if (tid == 0)
    s_base = 0;
  __syncthreads();
  double* out = stage + (static_cast<long long>(b) * n_units + u) * ucap * W;
  // one candidate (cidx in the flattened ContactResultMap order): its distance and
  // fields; `pre` = contactTest's hit (within the pair's contact distance)
  struct Cand
  {
    bool pre;
    int link[2], p, s, sb, i, cc_type[2];
    double dist, normal[3], pt[2][3], cc_time[2];
    Pose Ta[2], Tb[2];
  };
  auto eval_cand = [&](long long cidx, Cand& cd) {
    cd.link[0] = cd.link[1] = 0;
    cd.p = cd.s = 0;
    cd.sb = -1;
    cd.i = 0;
    cd.cc_type[0] = cd.cc_type[1] = kCCNone;
    cd.cc_time[0] = cd.cc_time[1] = 0.0;
    for (int k = 0; k < 3; ++k)
      cd.normal[k] = cd.pt[0][k] = cd.pt[1][k] = 0.0;
    cd.dist = 0.0;
    int* const link = cd.link;
    int& p = cd.p;
    int& s = cd.s;
    int& sb = cd.sb;
    int& i = cd.i;
    int* const cc_type = cd.cc_type;
    double& dist = cd.dist;
    double* const normal = cd.normal;
    double(&pt)[2][3] = cd.pt;
    double* const cc_time = cd.cc_time;
    Pose* const Ta = cd.Ta;
    Pose* const Tb = cd.Tb;
    {
      double qa[THIP_MAX_DOF], qb[THIP_MAX_DOF];
      auto states = [&]() {
        for (int j = 0; j < D; ++j)
        {
          qa[j] = tm.single ? q0[j] : linspaced(cnt, q0[j], q1[j], i);
          qb[j] = tm.continuous ? linspaced(cnt, q0[j], q1[j], i + 1) : qa[j];
        }
      };
      if (cidx < scene_total)
      {
        // decode (group, primitive, sub-state, sphere of the group) in map order
        long long r = cidx;
        int g = 0;
        for (; g < S.n_groups; ++g)
        {
          const long long sz = static_cast<long long>(S.grp_ns[g]) * n_prims * n_sub;
          if (r < sz)
            break;
          r -= sz;
        }
        const int ng = S.grp_ns[g];
        p = static_cast<int>(r / (static_cast<long long>(n_sub) * ng));
        const int r2 = static_cast<int>(r % (static_cast<long long>(n_sub) * ng));
        i = r2 / ng;
        s = S.sph_order[S.grp_s0[g] + r2 % ng];
        link[0] = S.grp_link[g];
        states();
        chain_fk(ch, qa, link[0], Ta[0]);
        double ca[3];
        sphere_world(Ta[0], S.center[s], ca);
        const double* prim = prims + 16 * p;
        if (tm.continuous)
        {
          chain_fk(ch, qb, link[0], Tb[0]);
          double cb[3], ts = 0;
          sphere_world(Tb[0], S.center[s], cb);
          swept_sphere_prim_distance(ca, cb, S.radius[s], prim, dist, normal, pt[0], ts);
          cc_time[0] = (double(i) + ts) * dt;
          cc_type[0] = (i == 0 && ts == 0.0) ? kCCTime0 : ((i + 1 == last && ts == 1.0) ? kCCTime1 : kCCBetween);
        }
        else
        {
          Tb[0] = Ta[0];
          sphere_prim_distance(ca, S.radius[s], prim, dist, normal, pt[0]);
          if (!tm.single)
          {
            cc_time[0] = double(i) * dt;
            cc_type[0] = (i == 0) ? kCCTime0 : ((i == last) ? kCCTime1 : kCCBetween);
          }
        }
      }
      else
      {
        // a self-collision candidate: key (link pair), sub-state, sphere pair of the key
        int r = static_cast<int>(cidx - scene_total), k = 0;
        for (; k + 1 < S.n_self_keys; ++k)
        {
          const int sz = n_sub * (S.self_kp[k + 1] - S.self_kp[k]);
          if (r < sz)
            break;
          r -= sz;
        }
        const int k0 = S.self_kp[k], npk = S.self_kp[k + 1] - k0;
        i = r / npk;
        const int j = k0 + (r - i * npk);
        s = S.self_sa[j];
        sb = S.self_sb[j];
        p = -1 - sb;
        link[0] = S.link[s];
        link[1] = S.link[sb];
        states();
        double a0[3], a1[3], b0[3], b1[3];
        for (int sd = 0; sd < 2; ++sd)
        {
          chain_fk(ch, qa, link[sd], Ta[sd]);
          if (tm.continuous)
            chain_fk(ch, qb, link[sd], Tb[sd]);
          else
            Tb[sd] = Ta[sd];
        }
        sphere_world(Ta[0], S.center[s], a0);
        sphere_world(Tb[0], S.center[s], a1);
        sphere_world(Ta[1], S.center[sb], b0);
        sphere_world(Tb[1], S.center[sb], b1);
        double t0, t1;
        self_sphere_distance(a0, a1, S.radius[s], b0, b1, S.radius[sb], tm.continuous != 0, dist, normal, pt[0], pt[1],
                             t0, t1);
        if (tm.continuous)
        {
          cc_time[0] = (double(i) + t0) * dt;
          cc_time[1] = (double(i) + t1) * dt;
          cc_type[0] = (i == 0 && t0 == 0.0) ? kCCTime0 : ((i + 1 == last && t0 == 1.0) ? kCCTime1 : kCCBetween);
          cc_type[1] = (i == 0 && t1 == 0.0) ? kCCTime0 : ((i + 1 == last && t1 == 1.0) ? kCCTime1 : kCCBetween);
        }
        else if (!tm.single)
        {
          cc_time[0] = cc_time[1] = double(i) * dt;
          cc_type[0] = cc_type[1] = (i == 0) ? kCCTime0 : ((i == last) ? kCCTime1 : kCCBetween);
        }
      }
    }
    // the pair's contact distance after incrementCollisionMargin(buffer) (a
    // zero-coefficient pair reads margin -inf: it never enters the test)
    const double margin = pair_margin(tm, n_prims, s, p);
    cd.pre = dist < margin + tm.buffer;
  };
  // the evaluator's filter on a tested contact: removeInvalidContactResults
  // (distance beyond the contact distance; at a fixed end keep a contact when one
  // of its active sides is not at that end -- a scene primitive's side is CCType_None)
  auto keep = [&](const Cand& cd) {
    const double margin = pair_margin(tm, n_prims, cd.s, cd.p);
    bool h = cd.pre && !(cd.dist > margin + tm.buffer);
    if (h && (un.f0 || un.f1))
      h = (un.f0 && ((cd.cc_type[0] != kCCNone && cd.cc_type[0] != kCCTime0) ||
                     (cd.cc_type[1] != kCCNone && cd.cc_type[1] != kCCTime0))) ||
          (un.f1 && ((cd.cc_type[0] != kCCNone && cd.cc_type[0] != kCCTime1) ||
                     (cd.cc_type[1] != kCCNone && cd.cc_type[1] != kCCTime1)));
    return h;
  };
  // the contact test type (trajopt_hip.h THIP_CONTACT_*): ALL, one item per
  // candidate; CLOSEST, one item per (key, sub-state) group -- its candidates are
  // contiguous in map order -- keeping the smallest distance (the first on ties);
  // FIRST, one item per sub-state, its first candidate in map order within the
  // contact distance.  The filter runs on what the test returned.
  const int ctest = tm.contact_test;
  long long n_scene_grp = 0;  // CLOSEST: scene groups (link group, primitive, sub-state)
  for (int g = 0; g < S.n_groups; ++g)
    n_scene_grp += static_cast<long long>(n_prims) * n_sub;
  const long long n_items = (ctest == THIP_CONTACT_ALL) ? total
                            : (ctest == THIP_CONTACT_CLOSEST) ? n_scene_grp + static_cast<long long>(S.n_self_keys) * n_sub
                                                              : n_sub;
  // first candidate of scene group g's block (its candidates: primitive-major,
  // then sub-state, then the group's spheres)
  auto grp_base = [&](int g) {
    long long off = 0;
    for (int h = 0; h < g; ++h)
      off += static_cast<long long>(S.grp_ns[h]) * n_prims * n_sub;
    return off;
  };
  auto self_base = [&](int k) {
    long long off = scene_total;
    for (int h = 0; h < k; ++h)
      off += static_cast<long long>(n_sub) * (S.self_kp[h + 1] - S.self_kp[h]);
    return off;
  };
  // FIRST returns one contact per contactTest call (sub-state), but the run's
  // map flattens key-major: pass 1 stores each sub-state's chosen candidate (its
  // index in map order, -1 for none) in a scratch at the tail of this unit's
  // records, pass 2 writes each record at its chosen index's rank.  A unit whose
  // records and scratch do not fit asks for that room (counts > ucap: the host
  // reruns once with it).
  const bool first_t = ctest == THIP_CONTACT_FIRST;
  double* const fscr = out + static_cast<long long>(ucap) * W - n_sub;
  if (first_t)
  {
    const long long need = static_cast<long long>(n_sub) + (n_sub + W - 1) / W;
    if (need > ucap)
    {
      if (tid == 0)
        counts[b * n_units + u] = static_cast<int>(need);
      return;
    }
    for (int ii = tid; ii < n_sub; ii += kEvBlock)
    {
      Cand cd;
      long long chosen = -1;
      bool found = false;
      for (int g = 0; g < S.n_groups && !found; ++g)
      {
        const int ng = S.grp_ns[g];
        for (int pp = 0; pp < n_prims && !found; ++pp)
          for (int e = 0; e < ng && !found; ++e)
          {
            chosen = grp_base(g) + (static_cast<long long>(pp) * n_sub + ii) * ng + e;
            eval_cand(chosen, cd);
            found = cd.pre;
          }
      }
      for (int k = 0; k < S.n_self_keys && !found; ++k)
      {
        const int npk = S.self_kp[k + 1] - S.self_kp[k];
        for (int e = 0; e < npk && !found; ++e)
        {
          chosen = self_base(k) + static_cast<long long>(ii) * npk + e;
          eval_cand(chosen, cd);
          found = cd.pre;
        }
      }
      fscr[ii] = (found && keep(cd)) ? static_cast<double>(chosen) : -1.0;
    }
    __syncthreads();
  }
  for (long long c0 = 0; c0 < n_items; c0 += kEvBlock)
  {
    const long long item = c0 + tid;
    Cand cd;
    cd.pre = false;
    bool hit = false;
    int fpos = 0;
    if (item < n_items)
    {
      if (ctest == THIP_CONTACT_ALL)
      {
        eval_cand(item, cd);
        hit = keep(cd);
      }
      else if (ctest == THIP_CONTACT_CLOSEST)
      {
        long long c_first = 0;
        int c_n = 0;
        if (item < n_scene_grp)
        {
          long long r = item;
          int g = 0;
          for (; g < S.n_groups; ++g)
          {
            const long long sz = static_cast<long long>(n_prims) * n_sub;
            if (r < sz)
              break;
            r -= sz;
          }
          const int ng = S.grp_ns[g];
          // (primitive, sub-state) = r / n_sub, r % n_sub: candidates r * ng .. + ng
          c_first = grp_base(g) + r * ng;
          c_n = ng;
        }
        else
        {
          const long long r = item - n_scene_grp;
          const int k = static_cast<int>(r / n_sub), ii = static_cast<int>(r % n_sub);
          const int npk = S.self_kp[k + 1] - S.self_kp[k];
          c_first = self_base(k) + static_cast<long long>(ii) * npk;
          c_n = npk;
        }
        Cand c2;
        for (int e = 0; e < c_n; ++e)
        {
          eval_cand(c_first + e, c2);
          if (c2.pre && (!cd.pre || c2.dist < cd.dist))
            cd = c2;
        }
        hit = keep(cd);
      }
      else  // FIRST: sub-state item, its pass-1 choice placed at its rank in map order
      {
        const double c = fscr[item];
        hit = c >= 0.0;
        if (hit)
        {
          eval_cand(static_cast<long long>(c), cd);
          for (int i2 = 0; i2 < n_sub; ++i2)
          {
            const double c2 = fscr[i2];
            fpos += (c2 >= 0.0 && c2 < c) ? 1 : 0;
          }
        }
      }
    }
    // the contact's fields for the record below
    int* const link = cd.link;
    const int p = cd.p, s = cd.s, sb = cd.sb, i = cd.i;
    const int* const cc_type = cd.cc_type;
    const double dist = cd.dist;
    const double* const normal = cd.normal;
    const double(&pt)[2][3] = cd.pt;
    const double* const cc_time = cd.cc_time;
    const Pose* const Ta = cd.Ta;
    const Pose* const Tb = cd.Tb;
    const unsigned long long m = __ballot(hit);
    const int lrank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0)
      s_wave_cnt[wave] = __popcll(m);
    __syncthreads();
    int rank = s_base + lrank;
    for (int w = 0; w < wave; ++w)
      rank += s_wave_cnt[w];
    if (first_t)
      rank = fpos;
    if (hit && rank < ucap)
    {
      const int nsides = (sb >= 0) ? 2 : 1;
      // nearest_points_local: each side's point in its link frame of transform
      double pl[2][3];
      for (int sd = 0; sd < nsides; ++sd)
      {
        const double w3[3] = { pt[sd][0] - Ta[sd].t[0], pt[sd][1] - Ta[sd].t[1], pt[sd][2] - Ta[sd].t[2] };
        for (int k = 0; k < 3; ++k)
          pl[sd][k] = Ta[sd].r[0 * 3 + k] * w3[0] + Ta[sd].r[1 * 3 + k] * w3[1] + Ta[sd].r[2 * 3 + k] * w3[2];
      }
      double* rec = out + static_cast<long long>(rank) * W;
      double a0[THIP_MAX_DOF], a1[THIP_MAX_DOF];
      for (int j = 0; j < D; ++j)
        a0[j] = a1[j] = 0.0;
      int mask = 0;
      // one timestep's part: per side scale * g (cleanupAff'd, a variable's side terms
      // summed) and scale * -g.q summed from 0 (oracle contactExpression)
      auto part = [&](const double* qe, bool ts1, double* a, int bit0) {
        double cpart = 0.0;
        for (int sd = 0; sd < nsides; ++sd)
        {
          const bool none = cc_type[sd] == kCCNone;
          const double sc = none ? 1.0 : (ts1 ? cc_time[sd] : 1 - cc_time[sd]);
          const Pose& lt = (ts1 && !none) ? Tb[sd] : Ta[sd];
          double g[THIP_MAX_DOF], gd = 0;
          contact_gradient(ch, qe, link[sd], lt, pl[sd], normal, sd ? 1.0 : -1.0, g);
          for (int j = 0; j < D; ++j)
          {
            const double av = sc * g[j];
            gd += g[j] * qe[j];
            if (fabs(av) > 1e-7)
            {
              const int bit = 1 << (bit0 + j);
              a[j] = (mask & bit) ? a[j] + av : av;
              mask |= bit;
            }
          }
          cpart += sc * -gd;
        }
        return cpart;
      };
      double cst;
      if (tm.single)
      {
        // CalcDistExpressionsSingleTimeStep: 0 + part(x_t), then + d (scale 1, CCType_None)
        cst = 0.0 + part(q0, false, a0, 0);
        cst += dist;
      }
      else
      {
        cst = dist;
        if (!un.f0)
          cst += part(q0, false, a0, 0);
        if (!un.f1)
          cst += part(q1, true, a1, D);
      }
      rec[0] = un.t0;
      rec[1] = link[0];
      rec[2] = p;
      rec[3] = s;
      rec[4] = tm.single ? 0 : i;
      rec[5] = dist;
      rec[6] = cc_time[0];
      rec[7] = __popc(mask);
      for (int j = 0; j < D; ++j)
      {
        rec[8 + j] = a0[j];
        rec[8 + D + j] = a1[j];
      }
      rec[8 + 2 * D] = cst;
    }
    __syncthreads();
    if (tid == 0)
    {
      int t = 0;
      for (int w = 0; w < kEvWaves; ++w)
        t += s_wave_cnt[w];
      s_base += t;
    }
    __syncthreads();
  }
  if (tid == 0)
    counts[b * n_units + u] = s_base;
}

// per problem: the units' records in unit order into out [b][cap][W]
__global__ __launch_bounds__(kEvBlock) void coll_pack_kernel(const double* stage, const int* ucounts, int n_units,
                                                            int ucap, int W, double* out, int cap, int* counts)
{
  const int b = blockIdx.x;
  int off = 0;
  for (int u = 0; u < n_units; ++u)
  {
    const int n = min(ucounts[b * n_units + u], ucap);
    const double* src = stage + (static_cast<long long>(b) * n_units + u) * ucap * W;
    for (int e = threadIdx.x; e < n * W; e += kEvBlock)
    {
      const int r = off + e / W;
      if (r < cap)
        out[(static_cast<long long>(b) * cap + r) * W + e % W] = src[e];
    }
    off += ucounts[b * n_units + u];
  }
  if (threadIdx.x == 0)
    counts[b] = off;
}
}  // namespace ev
}  // namespace thip

using namespace thip::ev;

struct thip_eval
{
  int device = 0, batch = 0;
  thip_problem_desc desc{};
  thip_chain* d_chain = nullptr;
  Spheres* d_sph = nullptr;
  double* d_tgt = nullptr;
  double* d_scene = nullptr;
  double* d_x = nullptr;      // q / x staging
  double* d_err = nullptr;
  double* d_jac = nullptr;
  CartArgs* d_cargs = nullptr;  // per CartPose term (cart_eval_all_kernel)
  int* d_csteps = nullptr;      // per CartPose term: its waypoint
  double* d_err_all = nullptr;  // [batch][n_cart][6]
  double* d_jac_all = nullptr;  // [batch][n_cart][6][D]
  double* d_stage = nullptr;  // collision records per unit
  double* d_out = nullptr;    // packed records
  int* d_counts = nullptr;    // per unit, then per problem
  Unit* d_units = nullptr;
  size_t stage_doubles = 0, out_doubles = 0;
  int ucap = 64;              // records per unit (grows when a unit has more)
  // per collision term: its unit table (offset into d_units) and kernel parameters
  std::vector<int> unit_off, unit_n;
  std::vector<CollTerm> terms;
  std::vector<double*> d_pair;  // per term: its pair table (pair_data.hpp) or null
  int max_units = 0;
  hipStream_t stream = nullptr;
  bool uploaded = false;
  std::string err;
};

static thread_local std::string g_eval_create_err;

namespace
{
int fail(thip_eval* ev, const std::string& m)
{
  ev->err = m;
  return THIP_E_INVALID;
}
int hipfail(thip_eval* ev, const char* what, hipError_t e)
{
  ev->err = std::string(what) + ": " + hipGetErrorString(e);
  return THIP_E_HIP;
}

// the units of a collision term: free waypoints of [first, last] (DISCRETE) or step
// pairs (problem_description.cpp:1735-1858)
bool term_units(int N, int first, int last, int n_fixed, const int* fixed_steps, int cont, std::vector<Unit>& out,
                std::string& why)
{
  if (last < 0)
    last = N - 1;
  if (first < 0 || first >= N || last < first || last >= N)
    return why = "collision: bad first/last step", false;
  auto fixed = [&](int t) {
    for (int k = 0; k < n_fixed; ++k)
      if (fixed_steps[k] == t)
        return true;
    return false;
  };
  if (cont == 2)
  {
    for (int t = first; t <= last; ++t)
      if (!fixed(t))
        out.push_back({ t, 0, 0 });
    return true;
  }
  for (int t = first; t < last; ++t)
  {
    const bool a = fixed(t), b = fixed(t + 1);
    if (a && b)
      return why = "Currently two adjacent fixed steps are not supported in collision term.", false;
    out.push_back({ t, a ? 1 : 0, b ? 1 : 0 });
  }
  return true;
}
}  // namespace

extern "C" {

int thip_eval_create(int device, const thip_problem_desc* desc, int batch, thip_eval** out)
{
  if (!desc || !out || batch <= 0)
  {
    g_eval_create_err = "thip_eval_create: null argument or batch <= 0";
    return THIP_E_INVALID;
  }
  auto reject = [](const std::string& m) {
    g_eval_create_err = "thip_eval_create: " + m;
    return THIP_E_INVALID;
  };
  if (desc->abi_version != THIP_ABI_VERSION)
    return reject("descriptor abi_version " + std::to_string(desc->abi_version) + " != THIP_ABI_VERSION " +
                  std::to_string(THIP_ABI_VERSION));
  const thip_chain& ch = desc->chain;
  const int N = desc->n_steps;
  if (ch.n_dof <= 0 || ch.n_dof > THIP_MAX_DOF || ch.n_links < 1 || ch.n_links > THIP_MAX_LINKS)
    return reject("chain out of range");
  if (N < 1 || N > THIP_EVAL_MAX_STEPS)
    return reject("n_steps out of range");
  for (int k = 1; k < ch.n_links; ++k)
    if ((ch.joint_type[k] < 0 || ch.joint_type[k] > 3) ||
        (ch.joint_type[k] != THIP_JOINT_FIXED && (ch.joint_dof[k] < 0 || ch.joint_dof[k] >= ch.n_dof)) ||
        (ch.is_tree && (ch.parent[k] < 0 || ch.parent[k] >= k)))
      return reject("bad chain joint / parent table");
  if (desc->n_cart < 0 || desc->n_cart > THIP_MAX_CART)
    return reject("n_cart out of range");
  for (int k = 0; k < desc->n_cart; ++k)
    if (desc->cart_step[k] < 0 || desc->cart_step[k] >= N || desc->cart_source_link[k] <= 0 ||
        desc->cart_source_link[k] >= ch.n_links || desc->cart_target_link[k] < 0 ||
        desc->cart_target_link[k] >= ch.n_links)
      return reject("bad CartPose term");
  if (desc->n_coll_extra < 0 || desc->n_coll_extra > THIP_MAX_COLL_EXTRA)
    return reject("n_coll_extra out of range");
  if ((desc->coll_enabled || desc->n_coll_extra > 0) &&
      (desc->n_spheres < 1 || desc->n_spheres > THIP_MAX_SPHERES || desc->n_prims < 0 ||
       desc->n_prims > THIP_EVAL_MAX_PRIMS))
    return reject("collision: spheres / primitives out of range");
  {
    const std::string why = thip::validate_coll_pairs(*desc);
    if (!why.empty())
      return reject(why);
  }
  for (int s = 0; s < (desc->coll_enabled || desc->n_coll_extra > 0 ? desc->n_spheres : 0); ++s)
    if (desc->sphere_link[s] < 1 || desc->sphere_link[s] >= ch.n_links || !(desc->sphere_radius[s] >= 0))
      return reject("collision: bad robot sphere");

  auto* ev = new thip_eval();
  ev->device = device;
  ev->batch = batch;
  ev->desc = *desc;
  if (!ev->desc.chain.is_tree)
    for (int k = 0; k < THIP_MAX_LINKS; ++k)
      ev->desc.chain.parent[k] = k > 0 ? k - 1 : 0;
  const thip_problem_desc& d = ev->desc;
  // collision terms: 0 = coll_*, k = coll_extra[k - 1]
  std::vector<Unit> units;
  const int n_terms = (d.coll_enabled ? 1 : 0) + d.n_coll_extra;
  for (int k = 0; k < n_terms; ++k)
  {
    const bool main = d.coll_enabled && k == 0;
    const thip_coll_term* x = main ? nullptr : &d.coll_extra[k - (d.coll_enabled ? 1 : 0)];
    CollTerm tm;
    const int cont = main ? d.coll_continuous : x->continuous;
    tm.single = cont == 2;
    tm.continuous = cont == 1;
    tm.margin = main ? d.coll_margin : x->margin;
    tm.buffer = main ? d.coll_buffer : x->buffer;
    tm.lvs = main ? d.coll_lvs : x->lvs;
    tm.pmc = nullptr;
    tm.pw = d.n_prims + d.n_spheres;
    tm.contact_test = main ? d.coll_contact_test : x->contact_test;
    const int nf = main ? d.coll_n_fixed : x->n_fixed;
    if (cont < 0 || cont > 2 || nf < 0 || nf > THIP_MAX_STEPS || (!tm.single && !(tm.lvs > 0)) || !(tm.buffer >= 0))
    {
      delete ev;
      return reject("collision term " + std::to_string(k) + ": bad evaluator / lvs / buffer / fixed steps");
    }
    std::string why;
    ev->unit_off.push_back(static_cast<int>(units.size()));
    if (!term_units(N, main ? d.coll_first_step : x->first_step, main ? d.coll_last_step : x->last_step, nf,
                    main ? d.coll_fixed_steps : x->fixed_steps, cont, units, why))
    {
      delete ev;
      return reject(why);
    }
    ev->unit_n.push_back(static_cast<int>(units.size()) - ev->unit_off.back());
    ev->max_units = std::max(ev->max_units, ev->unit_n.back());
    ev->terms.push_back(tm);
  }
  Spheres sp{};
  if (n_terms > 0)
  {
    std::vector<int> order;
    for (int s = 0; s < d.n_spheres; ++s)
      order.push_back(s);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return d.sphere_link[a] < d.sphere_link[b]; });
    for (size_t k = 0; k < order.size(); ++k)
    {
      sp.sph_order[k] = order[k];
      const int link = d.sphere_link[order[k]];
      if (sp.n_groups == 0 || sp.grp_link[sp.n_groups - 1] != link)
      {
        sp.grp_link[sp.n_groups] = link;
        sp.grp_s0[sp.n_groups] = static_cast<int>(k);
        sp.grp_ns[sp.n_groups] = 0;
        sp.n_groups++;
      }
      sp.grp_ns[sp.n_groups - 1]++;
    }
    std::vector<int> ssa, ssb, skp;
    const std::string why = thip::self_sphere_pairs(d, ssa, ssb, skp);
    if (!why.empty())
    {
      delete ev;
      return reject(why);
    }
    sp.n_self_keys = static_cast<int>(skp.size()) - 1;
    sp.n_self_sph = static_cast<int>(ssa.size());
    for (size_t k = 0; k < ssa.size(); ++k)
    {
      sp.self_sa[k] = ssa[k];
      sp.self_sb[k] = ssb[k];
    }
    for (size_t k = 0; k < skp.size(); ++k)
      sp.self_kp[k] = skp[k];
    for (int s = 0; s < d.n_spheres; ++s)
    {
      sp.link[s] = d.sphere_link[s];
      sp.radius[s] = d.sphere_radius[s];
      for (int i = 0; i < 3; ++i)
        sp.center[s][i] = d.sphere_center[s][i];
    }
  }
  auto hfail = [&](const char* what, hipError_t e) {
    g_eval_create_err = std::string("thip_eval_create: ") + what + ": " + hipGetErrorString(e);
    thip_eval_destroy(ev);
    return THIP_E_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess)
    return hfail("hipSetDevice", e);
  const size_t B = static_cast<size_t>(batch), D = static_cast<size_t>(d.chain.n_dof);
  const size_t nc = static_cast<size_t>(std::max(d.n_cart, 1)), np = static_cast<size_t>(std::max(d.n_prims, 1));
  if ((e = hipMalloc(&ev->d_chain, sizeof(thip_chain))) != hipSuccess ||
      (e = hipMalloc(&ev->d_sph, sizeof(Spheres))) != hipSuccess ||
      (e = hipMalloc(&ev->d_tgt, B * nc * 12 * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ev->d_scene, B * np * 16 * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ev->d_x, B * static_cast<size_t>(N) * D * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ev->d_err, B * 6 * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ev->d_jac, B * 6 * D * sizeof(double))) != hipSuccess ||
      (e = hipMalloc(&ev->d_counts, (B * static_cast<size_t>(std::max(ev->max_units, 1)) + B) * sizeof(int))) !=
          hipSuccess ||
      (e = hipMalloc(&ev->d_units, std::max<size_t>(units.size(), 1) * sizeof(Unit))) != hipSuccess)
    return hfail("hipMalloc", e);
  if ((e = hipStreamCreateWithFlags(&ev->stream, hipStreamNonBlocking)) != hipSuccess)
    return hfail("hipStreamCreate", e);
  if ((e = hipMemcpyAsync(ev->d_chain, &d.chain, sizeof(thip_chain), hipMemcpyHostToDevice, ev->stream)) !=
          hipSuccess ||
      (e = hipMemcpyAsync(ev->d_sph, &sp, sizeof(Spheres), hipMemcpyHostToDevice, ev->stream)) != hipSuccess ||
      (!units.empty() && (e = hipMemcpyAsync(ev->d_units, units.data(), units.size() * sizeof(Unit),
                                             hipMemcpyHostToDevice, ev->stream)) != hipSuccess) ||
      (e = hipMemsetAsync(ev->d_tgt, 0, B * nc * 12 * sizeof(double), ev->stream)) != hipSuccess ||
      (e = hipMemsetAsync(ev->d_scene, 0, B * np * 16 * sizeof(double), ev->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(ev->stream)) != hipSuccess)
    return hfail("hipMemcpy", e);
  // every CartPose term's arguments and waypoint (cart_eval_all_kernel)
  if (d.n_cart > 0)
  {
    std::vector<CartArgs> cargs(static_cast<size_t>(d.n_cart));
    std::vector<int> steps(static_cast<size_t>(d.n_cart));
    for (int k = 0; k < d.n_cart; ++k)
    {
      cargs[static_cast<size_t>(k)] = cart_args(d, k);
      steps[static_cast<size_t>(k)] = d.cart_step[k];
      if (d.cart_step[k] < 0 || d.cart_step[k] >= N)
        return reject("CartPose term waypoint out of range");
    }
    if ((e = hipMalloc(&ev->d_cargs, cargs.size() * sizeof(CartArgs))) != hipSuccess ||
        (e = hipMalloc(&ev->d_csteps, steps.size() * sizeof(int))) != hipSuccess ||
        (e = hipMalloc(&ev->d_err_all, B * nc * 6 * sizeof(double))) != hipSuccess ||
        (e = hipMalloc(&ev->d_jac_all, B * nc * 6 * D * sizeof(double))) != hipSuccess)
      return hfail("hipMalloc(CartPose terms)", e);
    if ((e = hipMemcpy(ev->d_cargs, cargs.data(), cargs.size() * sizeof(CartArgs), hipMemcpyHostToDevice)) !=
            hipSuccess ||
        (e = hipMemcpy(ev->d_csteps, steps.data(), steps.size() * sizeof(int), hipMemcpyHostToDevice)) != hipSuccess)
      return hfail("hipMemcpy(CartPose terms)", e);
  }
  // per link-pair margins of each collision term (coefficients are the host's)
  for (size_t k = 0; k < ev->terms.size(); ++k)
  {
    std::vector<double> tab;
    double* dp = nullptr;
    if (thip::coll_pair_table(d, static_cast<int>(k), tab))
    {
      if ((e = hipMalloc(&dp, tab.size() * sizeof(double))) != hipSuccess)
        return hfail("hipMalloc(pair table)", e);
      ev->d_pair.push_back(dp);
      if ((e = hipMemcpy(dp, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
        return hfail("hipMemcpy(pair table)", e);
      ev->terms[k].pmc = dp;
    }
  }
  *out = ev;
  return THIP_OK;
}

int thip_eval_upload(thip_eval* ev, const double* cart_targets, const double* scene)
{
  if (!ev)
    return THIP_E_INVALID;
  const thip_problem_desc& d = ev->desc;
  const size_t B = static_cast<size_t>(ev->batch);
  if (d.n_cart > 0 && !cart_targets)
    return fail(ev, "thip_eval_upload: cart_targets required when n_cart > 0");
  if ((d.coll_enabled || d.n_coll_extra > 0) && d.n_prims > 0 && !scene)
    return fail(ev, "thip_eval_upload: scene required with collision terms");
  hipError_t e;
  if ((e = hipSetDevice(ev->device)) != hipSuccess)
    return hipfail(ev, "hipSetDevice", e);
  if (d.n_cart > 0 &&
      (e = hipMemcpyAsync(ev->d_tgt, cart_targets, B * static_cast<size_t>(d.n_cart) * 12 * sizeof(double),
                          hipMemcpyHostToDevice, ev->stream)) != hipSuccess)
    return hipfail(ev, "hipMemcpy(cart_targets)", e);
  if (scene && d.n_prims > 0 &&
      (e = hipMemcpyAsync(ev->d_scene, scene, B * static_cast<size_t>(d.n_prims) * 16 * sizeof(double),
                          hipMemcpyHostToDevice, ev->stream)) != hipSuccess)
    return hipfail(ev, "hipMemcpy(scene)", e);
  if ((e = hipStreamSynchronize(ev->stream)) != hipSuccess)
    return hipfail(ev, "hipStreamSynchronize", e);
  ev->uploaded = true;
  return THIP_OK;
}

int thip_eval_cart_pose(thip_eval* ev, int term, const double* q, double* err, double* jac)
{
  if (!ev)
    return THIP_E_INVALID;
  const thip_problem_desc& d = ev->desc;
  if (term < 0 || term >= d.n_cart)
    return fail(ev, "thip_eval_cart_pose: term out of range");
  if (!q || !err)
    return fail(ev, "thip_eval_cart_pose: null q / err");
  if (!ev->uploaded)
    return fail(ev, "thip_eval_cart_pose: thip_eval_upload first");
  const int D = d.chain.n_dof;
  const CartArgs a = cart_args(d, term);
  const size_t B = static_cast<size_t>(ev->batch);
  hipError_t e;
  if ((e = hipSetDevice(ev->device)) != hipSuccess)
    return hipfail(ev, "hipSetDevice", e);
  if ((e = hipMemcpyAsync(ev->d_x, q, B * D * sizeof(double), hipMemcpyHostToDevice, ev->stream)) != hipSuccess)
    return hipfail(ev, "hipMemcpy(q)", e);
  hipLaunchKernelGGL(cart_eval_kernel, dim3(ev->batch), dim3(64), 0, ev->stream, ev->d_chain, a, ev->batch, d.n_cart,
                     term, ev->d_x, ev->d_tgt, ev->d_err, jac ? ev->d_jac : nullptr);
  if ((e = hipGetLastError()) != hipSuccess)
    return hipfail(ev, "cart_eval_kernel launch", e);
  if ((e = hipMemcpyAsync(err, ev->d_err, B * 6 * sizeof(double), hipMemcpyDeviceToHost, ev->stream)) !=
          hipSuccess ||
      (jac && (e = hipMemcpyAsync(jac, ev->d_jac, B * 6 * D * sizeof(double), hipMemcpyDeviceToHost, ev->stream)) !=
                  hipSuccess) ||
      (e = hipStreamSynchronize(ev->stream)) != hipSuccess)
    return hipfail(ev, "cart_eval_kernel", e);
  return THIP_OK;
}

int thip_eval_cart_pose_all(thip_eval* ev, const double* x, double* err, double* jac)
{
  if (!ev)
    return THIP_E_INVALID;
  const thip_problem_desc& d = ev->desc;
  if (!x || !err)
    return fail(ev, "thip_eval_cart_pose_all: null x / err");
  if (!ev->uploaded)
    return fail(ev, "thip_eval_cart_pose_all: thip_eval_upload first");
  if (d.n_cart == 0)
    return THIP_OK;
  const int N = d.n_steps, D = d.chain.n_dof;
  const size_t B = static_cast<size_t>(ev->batch), nc = static_cast<size_t>(d.n_cart);
  hipError_t e;
  if ((e = hipSetDevice(ev->device)) != hipSuccess)
    return hipfail(ev, "hipSetDevice", e);
  if ((e = hipMemcpyAsync(ev->d_x, x, B * N * D * sizeof(double), hipMemcpyHostToDevice, ev->stream)) != hipSuccess)
    return hipfail(ev, "hipMemcpy(x)", e);
  hipLaunchKernelGGL(cart_eval_all_kernel, dim3(static_cast<unsigned>(B * nc)), dim3(64), 0, ev->stream, ev->d_chain,
                     ev->d_cargs, ev->d_csteps, ev->batch, d.n_cart, N, ev->d_x, ev->d_tgt, ev->d_err_all,
                     jac ? ev->d_jac_all : nullptr);
  if ((e = hipGetLastError()) != hipSuccess)
    return hipfail(ev, "cart_eval_all_kernel launch", e);
  if ((e = hipMemcpyAsync(err, ev->d_err_all, B * nc * 6 * sizeof(double), hipMemcpyDeviceToHost, ev->stream)) !=
          hipSuccess ||
      (jac && (e = hipMemcpyAsync(jac, ev->d_jac_all, B * nc * 6 * D * sizeof(double), hipMemcpyDeviceToHost,
                                  ev->stream)) != hipSuccess) ||
      (e = hipStreamSynchronize(ev->stream)) != hipSuccess)
    return hipfail(ev, "cart_eval_all_kernel", e);
  return THIP_OK;
}

int thip_eval_collision(thip_eval* ev, int term, const double* x, double* records, int cap, int* counts)
{
  if (!ev)
    return THIP_E_INVALID;
  const thip_problem_desc& d = ev->desc;
  if (term < 0 || term >= static_cast<int>(ev->terms.size()))
    return fail(ev, "thip_eval_collision: term out of range");
  if (!x || !counts || cap < 0 || (cap > 0 && !records))
    return fail(ev, "thip_eval_collision: bad arguments");
  if (!ev->uploaded)
    return fail(ev, "thip_eval_collision: thip_eval_upload first");
  const int N = d.n_steps, D = d.chain.n_dof, W = 8 + 2 * D + 1;
  const size_t B = static_cast<size_t>(ev->batch);
  const int nu = ev->unit_n[static_cast<size_t>(term)];
  const Unit* units = ev->d_units + ev->unit_off[static_cast<size_t>(term)];
  hipError_t e;
  if ((e = hipSetDevice(ev->device)) != hipSuccess)
    return hipfail(ev, "hipSetDevice", e);
  if ((e = hipMemcpyAsync(ev->d_x, x, B * N * D * sizeof(double), hipMemcpyHostToDevice, ev->stream)) != hipSuccess)
    return hipfail(ev, "hipMemcpy(x)", e);
  if (nu == 0)
  {
    std::fill(counts, counts + B, 0);
    return THIP_OK;
  }
  int* ucounts = ev->d_counts;
  int* pcounts = ev->d_counts + B * static_cast<size_t>(std::max(ev->max_units, 1));
  for (int attempt = 0; attempt < 2; ++attempt)
  {
    const size_t need = B * static_cast<size_t>(nu) * ev->ucap * W;
    if (need > ev->stage_doubles)
    {
      hipFree(ev->d_stage);
      ev->d_stage = nullptr;
      if ((e = hipMalloc(&ev->d_stage, need * sizeof(double))) != hipSuccess)
        return hipfail(ev, "hipMalloc(contact records)", e);
      ev->stage_doubles = need;
    }
    hipLaunchKernelGGL(coll_eval_kernel, dim3(nu, ev->batch), dim3(kEvBlock), 0, ev->stream, ev->d_chain, ev->d_sph,
                       ev->terms[static_cast<size_t>(term)], units, nu, ev->batch, N, ev->d_x, ev->d_scene,
                       d.n_prims, ev->d_stage, ev->ucap, ucounts);
    if ((e = hipGetLastError()) != hipSuccess)
      return hipfail(ev, "coll_eval_kernel launch", e);
    std::vector<int> uc(B * static_cast<size_t>(nu));
    if ((e = hipMemcpyAsync(uc.data(), ucounts, uc.size() * sizeof(int), hipMemcpyDeviceToHost, ev->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(ev->stream)) != hipSuccess)
      return hipfail(ev, "coll_eval_kernel", e);
    const int mx = *std::max_element(uc.begin(), uc.end());
    if (mx <= ev->ucap)
      break;
    ev->ucap = mx;  // a unit had more contacts than the staging holds: rerun once with room for all
  }
  const size_t need_out = B * static_cast<size_t>(std::max(cap, 1)) * W;
  if (need_out > ev->out_doubles)
  {
    hipFree(ev->d_out);
    ev->d_out = nullptr;
    if ((e = hipMalloc(&ev->d_out, need_out * sizeof(double))) != hipSuccess)
      return hipfail(ev, "hipMalloc(records)", e);
    ev->out_doubles = need_out;
  }
  hipLaunchKernelGGL(coll_pack_kernel, dim3(ev->batch), dim3(kEvBlock), 0, ev->stream, ev->d_stage, ucounts, nu,
                     ev->ucap, W, ev->d_out, cap, pcounts);
  if ((e = hipGetLastError()) != hipSuccess)
    return hipfail(ev, "coll_pack_kernel launch", e);
  if ((e = hipMemcpyAsync(counts, pcounts, B * sizeof(int), hipMemcpyDeviceToHost, ev->stream)) != hipSuccess ||
      (cap > 0 && (e = hipMemcpyAsync(records, ev->d_out, B * static_cast<size_t>(cap) * W * sizeof(double),
                                      hipMemcpyDeviceToHost, ev->stream)) != hipSuccess) ||
      (e = hipStreamSynchronize(ev->stream)) != hipSuccess)
    return hipfail(ev, "coll_pack_kernel", e);
  return THIP_OK;
}

void thip_eval_destroy(thip_eval* ev)
{
  if (!ev)
    return;
  hipSetDevice(ev->device);
  if (ev->stream)
    hipStreamSynchronize(ev->stream);
  hipFree(ev->d_chain);
  hipFree(ev->d_sph);
  hipFree(ev->d_tgt);
  hipFree(ev->d_scene);
  hipFree(ev->d_x);
  hipFree(ev->d_err);
  hipFree(ev->d_jac);
  hipFree(ev->d_cargs);
  hipFree(ev->d_csteps);
  hipFree(ev->d_err_all);
  hipFree(ev->d_jac_all);
  hipFree(ev->d_stage);
  hipFree(ev->d_out);
  hipFree(ev->d_counts);
  hipFree(ev->d_units);
  for (double* dp : ev->d_pair)
    hipFree(dp);
  if (ev->stream)
    hipStreamDestroy(ev->stream);
  delete ev;
}

const char* thip_eval_last_error(thip_eval* ev) { return ev ? ev->err.c_str() : g_eval_create_err.c_str(); }

}  // extern "C"
