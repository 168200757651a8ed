// Device-side problem layout of the batched SQP (host + device).
//
// One HIP workgroup owns one problem for the whole BasicTrustRegionSQP run.
// The convexified QP is kept in structured (waypoint-blocked) form instead of
// CSC: columns are [x (N*D traj vars) | aux (neg, pos per CartPose row)], rows
// are [fixed-timestep rows | CartPose "abs" rows | one bound row per column],
// the same row/column sets OSQPModel builds from the model
// (trajopt_sco/src/osqp_interface.cpp:170-281), so every OSQP quantity
// (scaling, rho vector, residuals, polish active set) has a 1:1 counterpart.
#pragma once
#include "../../include/trajopt_hip.h"

namespace thip
{
// threads per problem workgroup.  sqp_kernel.hip is compiled twice: the main
// build (256 threads: the register-resident ADMM segment's ownership maps and
// launch bounds need them) and the generic-step build (THIP_GENERIC_ONLY,
// THIP_KBLOCK = kGenBlock, default 256: no segment code, so 17 VGPR spills
// instead of the main build's ~210, and its generic loops adapt their unroll to
// the loop length).  QPs the segment does not take -- blocks wider than 8 dofs
// (config E, JointAcc's waypoint pairs), more than 32 waypoints -- run it
// (round 6; THIP_DEBUG_MAIN_BUILD restores the main build's generic step).
// 512 threads was measured no faster on config E.
#ifndef THIP_KBLOCK
#define THIP_KBLOCK 256
#endif
constexpr int kBlock = THIP_KBLOCK;
constexpr int kWaves = kBlock / 64;
#ifndef THIP_GEN_BLOCK
#define THIP_GEN_BLOCK 256
#endif
constexpr int kGenBlock = THIP_GEN_BLOCK;  // threads of the generic-step build
// 1,024 threads faults on collision problems (HSA aperture violation, config C;
// configs J and B run clean and bitwise at 1,024: DESIGN.md section 4), and 512
// was measured no faster than 256 -- the build refuses anything above 512
static_assert(kGenBlock == 256 || kGenBlock == 512, "the generic-step build runs 256 or 512 threads");
// waves that run the contact scan's per-wave step pairs (their sub-state
// scratch A_CSCR is sized for this many); further waves take part in the
// batched sub-state FK only
constexpr int kScanWaves = 4;
// dynamic LDS a problem may use (160 KB per CU on gfx950, one workgroup per
// CU; the rest is the kernel's static LDS)
constexpr long long kLdsBudgetBytes = 149 * 1024;
// ... for the generic-step build: ~0.5 KB more static LDS at 256 threads (the
// contact scan's FIRST bits), ~2 KB more at 512 (reductions over 8 waves)
constexpr long long kLdsBudgetGenBytes = (kGenBlock == 256) ? 148 * 1024 : 146 * 1024;
// ADMM-segment chain pack (A_CPK), per half h (0: top, 1: bottom) and chain
// step r (distance from the middle block), in the lane order the octet chain
// reads it, zero past the half's length and outside the D x D block:
//   kCpkLM   [2][16][64][2]  (LI, M) pairs of the forward pass (16 B per lane)
//   kCpkNB   [2][16][64]     N' blocks of the backward pass
//   kCpkB    [2][16][8]      right-hand side of the forward pass
//   kCpkBM   [8]             right-hand side of the middle block
//   kCpkYM   [2][8]          the halves' last y, handed to the middle
constexpr int kCpkSteps = 16;
constexpr int kCpkLM = 0, kCpkNB = kCpkLM + 2 * kCpkSteps * 64 * 2, kCpkB = kCpkNB + 2 * kCpkSteps * 64,
              kCpkBM = kCpkB + 2 * kCpkSteps * 8, kCpkYM = kCpkBM + 8, kCpk = kCpkYM + 16;
// CartPose rows per waypoint the register-resident ADMM segment supports
constexpr int kMaxStepRows = 8;
// LVS sub-states per step pair the contact scan supports (sphere-center
// scratch in HBM; lanes loop over the sub-states)
constexpr int kSubCap = 1024;

// per-problem double workspace arrays
enum DArr : int
{
  A_X = 0,   // current SQP iterate (nx)
  A_XN,      // candidate iterate new_x (nx)
  A_INIT,    // initial trajectory (nx)
  A_TGT,     // CartPose target offsets (n_cart*12)
  A_G,       // CartPose rows, weighted, cleaned jacobian (n_abs*D)
  A_GC,      // CartPose rows, weighted constant (n_abs)
  A_COST,    // cost values at X (n_costs)
  A_VIOL,    // constraint violations at X (n_cnts)
  A_NCOST,   // cost values at XN
  A_NVIOL,   // violations at XN
  A_MU,      // merit coefficients (n_cnts)
  A_PD,      // scaled P diagonal (nx)
  A_PO,      // scaled P (t,j)-(t+1,j) coupling (nx)
  A_Q,       // scaled q (n_cols)
  A_DS,      // D scaling (n_cols)
  A_BS,      // scaled bound-row entry (n_cols)
  A_GS,      // scaled CartPose x coefficients (n_abs*D)
  A_WS,      // scaled aux coefficients (n_abs*2)
  A_FS,      // scaled fixed-row coefficient (n_fixed_rows)
  A_E,       // row scaling (m)
  A_L,       // scaled lower bounds (m)
  A_U,       // scaled upper bounds (m)
  A_RHO,     // rho per row (m)
  A_XA0,     // ADMM x, double buffered (n_cols)
  A_XA1,
  A_Z0,      // ADMM z, double buffered (m)
  A_Z1,
  A_Y,       // ADMM y (m)
  A_XT,      // x tilde (n_cols)
  A_ZT,      // z tilde (m)
  A_DX,      // delta x (n_cols)
  A_DY,      // delta y (m)
  A_BA,      // aux right-hand sides (n_cols, aux part used)
  A_MR,      // row multipliers (n_rows)
  A_AX,      // A x (m)
  A_PX,      // P x (n_cols)
  A_ATY,     // A' y (n_cols)
  A_PRV,     // primal residual vector (m)
  A_DRV,     // dual residual vector (n_cols)
  A_DG,      // diagonal of the aux block / x-col diagonal (n_cols)
  A_RE,      // effective rho of CartPose rows after aux elimination (n_rows)
  A_LINV,    // inverse Cholesky factor of the diagonal blocks (N*D*D)
  A_CHM,     // wide blocks (D > 8): the chain matrices M, N in HBM (2*N*D*D; else unused)
  A_KB,      // assembled diagonal blocks (N*D*D)
  A_CV,      // block solve vectors (nx)
  A_YV,      // (nx)
  A_SOLX,    // warm-start solution x, unscaled (n_cols)
  A_SOLY,    // warm-start solution y, unscaled (m)
  A_PB,      // polish rhs (n_cols + m)
  A_PS,      // polish solution (n_cols + m)
  A_PR,      // polish residual (n_cols + m)
  A_PZ,      // polish z (m)
  A_BXW,     // column rhs work (n_cols)
  // collision (LVS-discrete cost, config C); sized 1 when disabled
  A_HC0,     // hinge rows: distance-expression coefficients [h_cap][2D] (x_t, x_t+1), unscaled
  A_HK,      // distance-expression constant (h_cap)
  A_HC,      // scaled row coefficients [h_cap][2D]
  A_HW,      // scaled hinge-variable coefficient (h_cap)
  A_HRE,     // effective rho of hinge rows after eliminating the hinge variable (h_cap)
  A_CPL,     // coupling blocks K_{t+1,t} (N*D*D)
  A_CSCR,    // contact-scan scratch: sphere centers [kScanWaves][kSubCap][n_spheres][3]
  A_HCOST,   // per step-pair collision cost scratch (N)
  A_HDIST,   // contact distance of each hinge row (h_cap)
  A_HCCT,    // contact cc_time of each hinge row (h_cap; diagnostics, thip_collision_rows)
  A_HPK,     // ADMM-segment pack of the hinge rows, field-major [kHPack][n_h] (see admm_segment)
  A_HCHK,    // hinge chunk table: (first row, end row) int pairs, one double per chunk
  A_HPART,   // hinge chunk partial sums [n_chunks][16]
  A_HCT,     // ADMM-segment copy of A_HC, field-major [2D][n_h | 1] (odd stride: no LDS bank conflicts)
  A_CPK,     // ADMM-segment chain pack (kCpk doubles, N <= 32 and D <= 8; see seg_chain_solve)
  A_PO2,     // scaled P (t,j)-(t+2,j) coupling of JointAccEqCost terms (nx; Layout::grp == 2)
  A_COUNT
};

enum IArr : int
{
  I_MASK = 0,  // jacobian drop mask per CartPose row (n_abs)
  I_PMASK,     // mask of the previous QP setup (n_abs)
  I_TYPE,      // constraint type per row: -1 loose, 0 ineq, 1 eq (m)
  I_ACT,       // polish active flags (m)
  I_HT,        // hinge row start waypoint (h_cap)
  I_HMASK,     // kept-coefficient mask of hinge rows (h_cap), current QP
  I_PHMASK,    // ... of the previous QP setup (h_cap)
  I_PHT,       // start waypoints of the previous QP setup (h_cap)
  I_HPTR,      // CSR: hinge rows starting at waypoint t (N+1)
  I_CONT,      // contact list [h_cap][3]: sub-state, sphere, primitive
  I_PCNT,      // contacts per step pair (N)
  I_HKIND,     // hinge row kind: 0 collision (margin - dist), 1 affine (static rows) (h_cap)
  I_HSLOT,     // affine hinge rows: merit slot (constraint) or -1 (cost, objective 1) (h_cap)
  I_HBITS,     // contact scan: hit bit of every candidate of every unit, in the ContactResultMap order
  I_COUNT
};

enum ShKind : int
{
  SH_JP_UP = 0,  // (x - targ - upper) * c
  SH_JP_LO,      // (lower - (x - targ)) * c
  SH_JV_UP,      // -(upper - (vel - targ)) * c
  SH_JV_LO,      // (lower - (vel - targ)) * c
};

struct Layout
{
  // sqp.max_time in wall_clock64() ticks (LLONG_MAX: no limit)
  long long max_ticks;
  int N, D, nx;
  int n_links;
  int n_fixed, n_fixed_rows;
  int n_cart;
  int n_abs;      // CartPose rows (cost rows first, then constraint rows)
  int n_abs_cost; // rows belonging to cost terms
  int n_cols;     // column capacity: nc_base + h_cap
  int n_rows;     // n_fixed_rows + n_abs
  int m;          // row capacity: m_base + 2*h_cap
  // base sizes without collision rows; hinge row h is row m_base + 2h, the
  // bound row of its hinge variable (column nc_base + h) is m_base + 2h + 1
  int nc_base;    // nx + 2*n_abs
  int m_base;     // n_rows + nc_base
  int h_cap;      // hinge-row capacity (0 without collision)
  int coll;       // collision cost enabled
  int coll_first, coll_last;  // collision units [coll_first, coll_last): step pairs, or
                              // waypoints with coll_single
  int coll_single; // DISCRETE (SingleTimestepCollisionEvaluator): one unit per waypoint, its
                   // rows filed in step pair min(t, N - 2) on half t - pair
  int coll_cost0; // cost slot (or, with coll_cnt, constraint slot) of the first step pair
  int coll_cnt;   // collision term is a constraint (CollisionConstraint, ineq rows inflated by mu)
  int n_costs;    // JointVel (0/1) + CartPose cost terms + JointPos cost terms + collision step pairs
  int n_cnts;     // CartPose constraint terms + JointPos constraint terms
  int n_jpos;     // JointPos terms
  int n_jvx;      // further JointVel tolerance terms (static hinge owners n_jpos + 1 + x)
  int jv_first, jv_last;
  int jv_ineq;    // JointVelIneqCost (tolerances) instead of the quadratic JointVelEqCost
  // JointAccEqCost terms (desc jdt_*, thip_jdt_fused): their cost slots; P gains
  // the (t, t+2) coupling A_PO2 and the solve pairs waypoints (grp = 2)
  int n_jacc;
  int jacc_slot[THIP_MAX_JDT];
  int hinge;      // the QP has hinge rows (collision contacts and/or static hinge rows)
  long long dstride;  // doubles per problem
  long long istride;  // ints per problem
  long long doff[A_COUNT];
  long long ioff[I_COUNT];
  // LDS residency plan: offset (doubles) of array k inside the dynamic LDS
  // block, or -1 if it stays in the per-problem HBM workspace.  The first
  // lds_scratch doubles are the block-solve chain matrices / FK staging.
  int loff[A_COUNT];
  int lds_scratch;
  int fac_off;  // doubles: factor()'s 4 D x D scratch blocks, inside lds_scratch
  // D > 8 (e.g. the 14-DoF dual arm): the block solve runs one lane per block
  // row and its chain matrices M, N live in HBM (A_CHM), not in the LDS scratch
  int wide;
  // the chain matrices M, N in HBM (A_CHM) for narrow blocks too: collision
  // problems on the ADMM segment, whose chain runs from the pack (A_CPK), so
  // the LDS they would take holds hinge-row data instead
  int chm_hbm;
  // hinge chunk sums (A_HPART): lanes and doubles per chunk, >= 2 D (16 for
  // the segment's D <= 8, 32 for wider blocks)
  int part_w;
  int lds_doubles;
  int lds_budget;  // doubles of dynamic LDS the launch provides (dynamic plan)
  // register-resident ADMM segment (admm_segment): eligible when every
  // waypoint has <= kMaxStepRows CartPose rows and the hot arrays are LDS
  // resident; seg_slots = column/row slots per thread (1 or 2)
  int seg_ok;
  int seg_slots;
  // middle block of the twisted block factorisation (N / 2)
  int tw_mid;
  // Branches of the block solve.  A kinematic tree whose terms never touch two
  // branches (a dual arm: each CartPose term and each collision sphere moves the
  // dofs of one arm only) has a reduced KKT matrix that is block diagonal over
  // the branches' dof ranges, so the block-tridiagonal solve splits into nbr
  // independent chains of sN / nbr blocks of sD = D / nbr dofs: solve block
  // b * N + t is waypoint t's dofs [b sD, (b + 1) sD) (the dofs of a branch
  // are contiguous).  Each branch gets its own twisted factorisation (top half
  // on wave 2b, bottom half on wave 2b + 1).  nbr = 1: sD = D, sN = N.
  int nbr;
  int sD;
  int sN;
  // Waypoint pairs (JointAccEqCost: P couples t and t + 2, so the reduced KKT
  // matrix is block-tridiagonal over pairs, not over waypoints): grp = 2 makes
  // solve block T waypoints 2T and 2T + 1 (sD = 2 D, sN = N / 2; the solve
  // layout is the column order itself).  grp = 1 otherwise.  sNb: solve blocks
  // per branch (N / grp), the length of each twisted factorisation.
  int grp;
  int sNb;
  // the CartPose rows of every waypoint are contiguous and in order (step_rows
  // is the identity): the generic step reads a waypoint's rows without the
  // step_rows indirection (max_step_rows: the most rows of one waypoint)
  int rows_contig;
  int max_step_rows;
};

// the solve-layout index of column col (t, j): block b * N + t, row j - b sD
__host__ __device__ __forceinline__ int solve_index(const Layout& L, int col)
{
  if (L.nbr == 1)
    return col;
  const int t = col / L.D, j = col - t * L.D, b = j / L.sD;
  return (b * L.N + t) * L.sD + (j - b * L.sD);
}
// the column of solve-layout index v
__host__ __device__ __forceinline__ int solve_column(const Layout& L, int v)
{
  if (L.nbr == 1)
    return v;
  const int T = v / L.sD, i = v - T * L.sD, b = T / L.N, t = T - b * L.N;
  return t * L.D + b * L.sD + i;
}

// shared (batch-wide) tables, device resident
struct Tables
{
  int* row_term;   // CartPose term of each abs row (n_abs)
  int* row_comp;   // error component 0..5 (n_abs)
  int* row_step;   // waypoint (n_abs)
  double* row_w;   // coefficient (n_abs)
  int* step_ptr;   // CSR waypoint -> abs rows (N+1)
  int* step_rows;  // (n_abs)
  int* term_row0;  // first abs row of each CartPose term (n_cart)
  int* term_nrow;  // rows of each term (n_cart)
  int* term_slot;  // cost index or constraint index of each term (n_cart)
  int* fixed_of_step;  // fixed-step slot of each waypoint or -1 (N)
  // abs rows of every source (CartPose rows, JointPos constraint rows)
  int* row_slot;   // merit slot of the row's constraint term, -1 for cost rows (n_abs)
  int* row_jpos;   // 1: JointPos EQ constraint row (row_term = JointPos term, row_comp = joint) (n_abs)
  int* row_off;    // branched solves (Layout::nbr > 1): first dof of the row's branch, whose sD
                   // coefficients are the row's only nonzeros (n_abs; 0 otherwise)
  // JointPos terms (hatch-clamped steps, cost or constraint slot)
  int* jpos_first; // (THIP_MAX_JPOS)
  int* jpos_last;
  int* jpos_slot;
  int* jpos_row0;  // first abs row of a JointPos constraint term
  int* jpos_nrow;
  int* jpos_ineq;  // 1: tolerance (hinge) form (JointPosIneqCost / JointPosIneqConstraint)
  // static hinge rows (JointPos / JointVel tolerance forms, trajectory_costs.cpp:66-135,183-254,303-374),
  // filed under step pairs after the pair's contacts; sorted by pair (CSR sh_ptr)
  int n_sh;
  int* sh_kind;    // ShKind
  int* sh_owner;   // JointPos term k, or n_jpos for the JointVel term
  int* sh_joint;
  int* sh_step;    // waypoint of the row's first variable
  int* sh_pair;    // step pair the row is filed under
  int* sh_slot;    // merit slot of a constraint term (objective mu), -1 for costs (objective 1)
  int* sh_ptr;     // CSR pair -> static rows (N+1)
  // collision model: robot spheres grouped by link in ascending link order
  // (the ContactResultMap key order of the contact scan)
  int n_groups;
  int* grp_link;   // link of group g
  int* grp_s0;     // first entry of the group in sph_order
  int* grp_ns;     // spheres in the group
  int* sph_order;  // sphere indices sorted by (link, index)
  int* coll_fixed; // per waypoint: 1 if a collision fixed step (N)
  int* jvx_first;  // further JointVel terms: clamped steps and cost / constraint slot (THIP_MAX_JVX)
  int* jvx_last;
  int* jvx_slot;
  int* coll_slot;  // per collision unit (step pair, or waypoint for DISCRETE): term slot
                   // relative to coll_cost0, -1 for a fixed waypoint without a term (N)
  // robot self-collision (self_pairs.hpp): sphere pairs in key order, the spheres
  // of link a and of link b, and the first pair of each key (n_self_keys + 1)
  int n_self_keys, n_self_sph;
  int* self_sa;
  int* self_sb;
  int* self_kp;
  // per link-pair margins and coefficients of the collision term (pair_data.hpp:
  // [n_spheres][n_prims + n_spheres][2]); null: every pair takes coll_margin / coll_coeff
  const double* pair_mc;
};

struct KernelArgs
{
  Layout L;
  Tables T;
  const thip_problem_desc* desc;  // device copy
  const double* scene;  // [batch][n_prims][16] (null without collision)
  const double* jpt;    // JointPos targets [batch][max(n_jpos,1)][D]
  double* ws;
  int* iws;
  thip_result* res;
  int batch;
  // diagnostics: per-QP trace records [batch][trace_cap][10] (null = off)
  double* trace;
  int* trace_n;
  int trace_cap;
  // diagnostics: per-problem phase cycle counters [batch][kProfSlots] (null = off)
  long long* prof;
  // sqp_kernel: stage the uploaded inputs into the workspace at entry and gather
  // the final trajectory at exit (null = skip); one launch per run
  const double* stage_init;  // [batch][nx]
  const double* stage_tgt;   // [batch][n_cart][12]
  double* xout;              // [batch][nx]
  // dynamic problem assignment (null = workgroup b solves problem b): the grid
  // holds one workgroup per resident slot and each workgroup takes the next
  // problem from work[0] until the batch is exhausted; the last workgroup to
  // finish (work[1]) resets both to 0 for the next launch on the stream
  int* work;
};

constexpr int kHPack = 14;  // doubles per hinge row in A_HPK
constexpr int kHChunk = 8;  // hinge rows per gather chunk (rows of one step pair)
constexpr int kProfSlots = 40;

}  // namespace thip
