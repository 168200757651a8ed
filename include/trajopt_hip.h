/*
 * trajopt_hip.h — C-ABI of the MI355X batched SQP trajectory optimizer.
 *
 * This is the drop-in boundary between the host layer that mirrors trajopt's
 * plugin surface (ProblemConstructionInfo / TermInfo::hatch / sco::Model /
 * BasicTrustRegionSQP) and the HIP kernels that run the sequential convex
 * optimisation inner loop for a whole batch of structurally identical problems.
 *
 * Plain C: fixed-size structs, plain pointers and sizes, no torch / HIP types
 * in any signature (the stream is passed as an opaque void*).  Every entry point
 * returns 0 on success and a negative THIP_E* code on failure; no exception
 * crosses the ABI.  thip_last_error() gives the message.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference tree):
 *   thip_create / thip_upload   <- trajopt::ConstructProblem(pci) + TrajOptProb ctor
 *                                   (trajopt/src/problem_description.cpp:414-598) and
 *                                   OptProb::createVariables (trajopt_sco/src/modeling.cpp:181-198):
 *                                   the batch of problems is lowered once into SoA device buffers.
 *   thip_sqp_run                <- sco::BasicTrustRegionSQP::optimize
 *                                   (trajopt_sco/src/optimizers.cpp:699-991), the whole penalty /
 *                                   SQP / trust-region loop, device-resident, one workgroup per problem.
 *   thip_linearize              <- the convexify step of that loop for CartPose + JointVel terms:
 *                                   CartPoseErrCalculator / CartPoseJacCalculator
 *                                   (trajopt/src/kinematic_terms.cpp:252-370) and
 *                                   JointVelEqCost::convex (trajopt/src/trajectory_costs.cpp:296-301).
 *   (inside thip_sqp_run)       <- sco::OSQPModel::optimize (trajopt_sco/src/osqp_interface.cpp:440-615):
 *                                   every QP solve with OSQP-1.0 semantics (Ruiz scaling, ADMM, adaptive
 *                                   rho, polish, warm start) on the structured convexified QP.
 *   thip_fwd_kin                <- tesseract JointGroup::calcFwdKin as called at
 *                                   trajopt/src/kinematic_terms.cpp:255,355 (all chain links).
 *   thip_download               <- OptResults (trajopt_sco/include/trajopt_sco/optimizers.hpp:40-59).
 *
 * Data layout: every per-problem array is problem-major and row-major inside a
 * problem: trajectories are [batch][n_steps][n_dof] (the reference's
 * x[t*D + j] layout, problem_description.cpp:557-598), poses are 3x4 row-major
 * [R | t] blocks of 12 doubles.
 */
#ifndef TRAJOPT_HIP_H
#define TRAJOPT_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of the structs below: thip_create rejects a descriptor whose
 * abi_version differs (a caller compiled against another layout).  3: the
 * descriptor carries abi_version, thip_chain.is_tree, thip_sqp_params.max_time.
 * 4: use_time, fixed dofs, time JointVel.  5: TotalTime.  6: further collision
 * terms (thip_coll_term), single-waypoint problems on the generic path.  7: robot
 * self-collision link pairs (n_self_pairs / self_pair).  8: per link-pair collision
 * margins and coefficients (n_coll_pairs / coll_pairs).  9: the collision terms'
 * contact test type (coll_contact_test, thip_coll_term.contact_test). */
#define THIP_ABI_VERSION 9

#define THIP_MAX_DOF 16
#define THIP_MAX_LINKS 32
#define THIP_MAX_STEPS 64
#define THIP_MAX_CART 128
#define THIP_MAX_SPHERES 32
#define THIP_MAX_PRIMS 16
#define THIP_MAX_JPOS 8
#define THIP_MAX_JVX 4
#define THIP_MAX_JDT 8
#define THIP_MAX_JVT 4
#define THIP_MAX_TTT 2
#define THIP_MAX_COLL_EXTRA 3
#define THIP_MAX_SELF_PAIRS 64
#define THIP_MAX_SELF_SPHERE_PAIRS 512
#define THIP_MAX_COLL_PAIRS 64
/* the generic path's device evaluator (thip_eval_*) and the host loop take
 * longer horizons and larger scenes than the fused kernel */
#define THIP_EVAL_MAX_STEPS 4096
#define THIP_EVAL_MAX_PRIMS 1024
#define THIP_MAX_CONTACTS 131072

/* contact test type of a collision term (CollisionTermInfo::contact_test_type,
 * problem_description.cpp:1669-1673, tesseract ContactTestType {FIRST = 0,
 * CLOSEST = 1, ALL = 2}), encoded so that a zero-initialised descriptor means
 * ALL, the reference's default.  Per contactTest call (one LVS sub-state, one
 * cast, or the DISCRETE state), before the evaluator's filter (zero-coefficient
 * pairs, removeInvalidContactResults): ALL keeps every contact within each
 * pair's contact distance; CLOSEST keeps one per link-pair key, the smallest
 * distance (the first in sphere order on ties); FIRST keeps the first contact
 * of the whole test in ContactResultMap order (keys (link, primitive), then the
 * self link pairs; inside a key, sphere order).  The primitive model replaces
 * Bullet's broad phase, so FIRST's choice is parity unpinned against tesseract,
 * as every contact value is.  The fused kernel runs FIRST and CLOSEST in its
 * generic-step build (sqp_kernel_gen: thip_create selects it for such a
 * descriptor, and thip_collision_rows runs that build's scan); the device
 * evaluator (thip_eval_collision) runs all three. */
#define THIP_CONTACT_ALL 0
#define THIP_CONTACT_FIRST 1
#define THIP_CONTACT_CLOSEST 2

/* error codes */
#define THIP_OK 0
#define THIP_E_INVALID (-1)
#define THIP_E_HIP (-2)
#define THIP_E_NOMEM (-3)
#define THIP_E_STATE (-4)

/* joint types (URDF) */
#define THIP_JOINT_FIXED 0
#define THIP_JOINT_REVOLUTE 1
#define THIP_JOINT_CONTINUOUS 2
#define THIP_JOINT_PRISMATIC 3

/* sco::OptStatus (trajopt_sco/include/trajopt_sco/optimizers.hpp:25-33) */
#define THIP_OPT_CONVERGED 0
#define THIP_OPT_SCO_ITERATION_LIMIT 1
#define THIP_OPT_PENALTY_ITERATION_LIMIT 2
#define THIP_OPT_TIME_LIMIT 3
#define THIP_OPT_FAILED 4
#define THIP_OPT_INVALID 5

/* sco::CvxOptStatus (trajopt_sco/include/trajopt_sco/solver_interface.hpp:40-45) */
#define THIP_CVX_SOLVED 0
#define THIP_CVX_INFEASIBLE 1
#define THIP_CVX_FAILED 2

/* scene primitive types (collision, config C).  A primitive record is 16
 * doubles: [0] type, then
 *   SPHERE  [1..3] center, [4] radius
 *   BOX     [1..3] center, [4..12] rotation (row-major, columns = box axes in
 *           world), [13..15] half extents
 *   CAPSULE [1..3] end a, [4..6] end b, [7] radius
 * Distances are closed-form sphere-vs-primitive signed distances (robot
 * links carry spheres), the same arithmetic in the oracle and on the GPU. */
#define THIP_PRIM_SPHERE 0
#define THIP_PRIM_BOX 1
#define THIP_PRIM_CAPSULE 2

/* Kinematic tree (the tesseract JointGroup of the reference, restated): link 0
 * is the root (static, world pose = base_pose); link k >= 1 hangs off link
 * parent[k] < k through joint k with a fixed origin transform followed by the
 * joint motion about/along `joint_axis` (expressed in the joint frame).  A
 * serial chain (the reference's right_arm / left_arm groups) has parent[k] =
 * k - 1; a dual-arm group (both PR2 arms off torso_lift_link) branches at the
 * root.  `parent` is read only when is_tree = 1: a zero-initialised chain is a
 * serial chain (parent[k] = k - 1), never a star.  The segment's
 * register-resident ADMM path takes n_dof <= 8; larger groups (up to
 * THIP_MAX_DOF) run the generic block solve. */
typedef struct thip_chain {
  int n_links;
  int n_dof;
  int is_tree;                            /* 0: serial chain (parent[] ignored); 1: tree, parent[] used */
  double base_pose[12];
  int joint_type[THIP_MAX_LINKS];
  int joint_dof[THIP_MAX_LINKS];          /* dof index for movable joints, -1 for fixed */
  int parent[THIP_MAX_LINKS];             /* is_tree: parent link of link k >= 1 (0 <= parent[k] < k) */
  double joint_origin[THIP_MAX_LINKS][12];
  double joint_axis[THIP_MAX_LINKS][3];
  double lower[THIP_MAX_DOF];             /* joint limits -> variable bounds */
  double upper[THIP_MAX_DOF];
} thip_chain;

/* sco::BasicTrustRegionSQPParameters (optimizers.hpp:92-135), numeric members only */
typedef struct thip_sqp_params {
  double improve_ratio_threshold;   /* 0.25 */
  double min_trust_box_size;        /* 1e-4 */
  double min_approx_improve;        /* 1e-4 */
  double min_approx_improve_frac;   /* -DBL_MAX */
  int max_iter;                     /* 50 */
  double trust_shrink_ratio;        /* 0.1 */
  double trust_expand_ratio;        /* 1.5 */
  double cnt_tolerance;             /* 1e-4 */
  double max_merit_coeff_increases; /* 5 */
  int max_qp_solver_failures;       /* 3 */
  double merit_coeff_increase_ratio;/* 10 */
  double initial_merit_error_coeff; /* 10 */
  int inflate_constraints_individually; /* 1 */
  double trust_box_size;            /* 0.1 */
  double max_time;                  /* seconds, DBL_MAX = no limit (optimizers.hpp:117): checked at the
                                       top of every SQP iteration against the problem's own clock (its
                                       workgroup's start); past it the run ends with OPT_TIME_LIMIT, or
                                       OPT_CONVERGED when no constraint is violated (optimizers.cpp:739-753) */
} thip_sqp_params;

/* OSQP settings as configured by OSQPModelConfig::setDefaultOSQPSettings
 * (trajopt_sco/src/osqp_interface.cpp:78-90) on top of OSQP 1.0 defaults. */
typedef struct thip_osqp_settings {
  double rho;            /* 0.1 */
  double sigma;          /* 1e-6 */
  double alpha;          /* 1.6 */
  int scaling;           /* 10 */
  int adaptive_rho;      /* 1 (iteration based) */
  int adaptive_rho_interval; /* 0 -> 4 * check_termination */
  double adaptive_rho_tolerance; /* 5 */
  int max_iter;          /* 8192 */
  double eps_abs;        /* 1e-4 */
  double eps_rel;        /* 1e-6 */
  double eps_prim_inf;   /* 1e-4 */
  double eps_dual_inf;   /* 1e-4 */
  int check_termination; /* 25 */
  int warm_starting;     /* 1 */
  int polishing;         /* 1 */
  double delta;          /* 1e-6 */
  int polish_refine_iter;/* 3 */
} thip_osqp_settings;

/* One CollisionTermInfo beyond the descriptor's first (coll_* fields):
 * CollisionTermInfo::hatch (problem_description.cpp:1735-1858) with its own
 * evaluator, margin, coefficient and steps over the shared robot spheres and
 * scene.  `continuous` as coll_continuous. */
typedef struct thip_coll_term {
  int is_cnt;
  int first_step;
  int last_step;   /* -1 = the last waypoint */
  int n_fixed;
  int fixed_steps[THIP_MAX_STEPS];
  double margin;   /* dist_pen */
  double coeff;    /* coeffs */
  double buffer;   /* collision_margin_buffer */
  double lvs;      /* longest_valid_segment_length (CONTINUOUS: +inf) */
  int continuous;  /* 0 LVS_DISCRETE, 1 LVS_CONTINUOUS / CONTINUOUS, 2 DISCRETE */
  int contact_test; /* THIP_CONTACT_ALL / FIRST / CLOSEST */
} thip_coll_term;

/* A per link-pair override of one collision term's margin and coefficient:
 * CollisionTermInfo's "pairs" (problem_description.cpp:1686-1719) -- the
 * pair's margin in the contact manager's CollisionMarginData (override type
 * MODIFY) and its coefficient in CollisionCoeffData
 * (trajopt_common/collision_types.h:51-184).  A pair's contacts use its margin
 * for the contact distance (margin + buffer) and the hinge margin - d, and
 * its coefficient for the hinge / constraint weight (collision_terms.cpp:
 * 195-386, 646-688, 817-898, 1065-1161, 1267-1386); a coefficient with
 * |coeff| <= 1e-6 (almostEqualRelativeAndAbs(coeff, 0)) drops the pair's
 * contacts altogether (hasZeroCoeff).  The pair is unordered; a later entry
 * for the same pair and term replaces an earlier one (insert_or_assign). */
typedef struct thip_coll_pair {
  int term;      /* 0: the coll_* term, 1 + x: coll_extra[x] */
  int link;      /* chain link index of one side (a robot link of the group) */
  int other;     /* >= 0: scene primitive index; < 0: -1 - chain link index (a robot link) */
  int pad_;
  double margin; /* the pair's dist_pen */
  double coeff;  /* the pair's coeffs */
} thip_coll_pair;

/* The structure shared by every problem of a batch: chain, horizon, term
 * tables (the lowered TermInfo list), solver parameters.  Per-problem data
 * (initial trajectory, CartPose target poses, scene primitives) is uploaded
 * separately, batched. */
typedef struct thip_problem_desc {
  int abi_version;  /* THIP_ABI_VERSION */
  int n_steps;
  thip_chain chain;

  /* fixed_timesteps: x[t, :] == init[t, :] as persistent model equalities
   * (problem_description.cpp:489-510) */
  int n_fixed;
  int fixed_steps[THIP_MAX_STEPS];

  /* JointVelTermInfo as a cost (problem_description.cpp:1216-1391): zero
   * tolerances -> JointVelEqCost (quadratic, trajectory_costs.cpp:257-301),
   * otherwise JointVelIneqCost (two hinge rows per (step, joint),
   * trajectory_costs.cpp:303-374).  A tolerance counts as zero when
   * |tol| < 1e-5 (trajopt_common::doubleEquals). */
  int jv_enabled;
  int jv_first_step;
  int jv_last_step;
  double jv_coeffs[THIP_MAX_DOF];
  double jv_targets[THIP_MAX_DOF];
  double jv_upper_tols[THIP_MAX_DOF];
  double jv_lower_tols[THIP_MAX_DOF];

  /* CartPoseTermInfo (problem_description.cpp:919-1005): source = chain link
   * (active) with source offset, target = static chain root frame with a
   * per-problem target offset pose. is_cnt: 0 = ABS cost, 1 = EQ constraint. */
  int n_cart;
  int cart_step[THIP_MAX_CART];
  int cart_is_cnt[THIP_MAX_CART];
  int cart_source_link[THIP_MAX_CART];
  double cart_source_offset[THIP_MAX_CART][12];
  double cart_pos_coeffs[THIP_MAX_CART][3];
  double cart_rot_coeffs[THIP_MAX_CART][3];
  /* CartPose tolerance band (CartPoseErrCalculator / CartPoseJacCalculator,
   * kinematic_terms.cpp:189-370): with cart_has_tol the error is
   * applyTolerances(calcTransformError, lower, upper) over the 6 components
   * (x, y, z, rx, ry, rz) and the finite-difference Jacobian uses the
   * tolerance-aware error difference.  0 = no band (empty or equal bounds). */
  int cart_has_tol[THIP_MAX_CART];
  double cart_lower_tol[THIP_MAX_CART][6];
  double cart_upper_tol[THIP_MAX_CART][6];
  /* 0: the target frame is the static chain root (the per-problem target offset
   * is in the root frame).  > 0: DynamicCartPoseTermInfo (problem_description.cpp:
   * 683-842, kinematic_terms.cpp:58-187): the target is this active chain link,
   * the per-problem offset is in its frame, and the FD jacobian perturbs both
   * frames. */
  int cart_target_link[THIP_MAX_CART];

  /* JointPosTermInfo (problem_description.cpp:1097-1196).  Zero tolerances:
   * is_cnt 0 -> JointPosEqCost (quadratic, trajectory_costs.cpp:28-65),
   * is_cnt 1 -> JointPosEqConstraint (one EQ row coeff*(x - target) per
   * (step, joint), trajectory_costs.cpp:137-181).  Nonzero tolerances (|tol| >=
   * 1e-5 for some joint): JointPosIneqCost / JointPosIneqConstraint, two hinge
   * rows per (step, joint) (trajectory_costs.cpp:66-135, 183-254).
   * first/last_step follow the hatch clamping rules (-1 = last step).
   * jpos_targets is the default for every problem; thip_upload_joint_targets
   * sets them per problem. */
  int n_jpos;
  int jpos_is_cnt[THIP_MAX_JPOS];
  int jpos_first_step[THIP_MAX_JPOS];
  int jpos_last_step[THIP_MAX_JPOS];
  double jpos_coeffs[THIP_MAX_JPOS][THIP_MAX_DOF];
  double jpos_targets[THIP_MAX_JPOS][THIP_MAX_DOF];
  double jpos_upper_tols[THIP_MAX_JPOS][THIP_MAX_DOF];
  double jpos_lower_tols[THIP_MAX_JPOS][THIP_MAX_DOF];

  /* Further JointVelTermInfo terms in the tolerance form, besides the jv_*
   * term above: is_cnt 0 -> JointVelIneqCost (trajectory_costs.cpp:303-374),
   * is_cnt 1 -> JointVelIneqConstraint (:426-500); two hinge rows per (step,
   * joint).  Steps clamped as the jv_* term's (problem_description.cpp:1228-1245).
   * Cost terms follow the JointPos cost terms, constraint terms the JointPos
   * constraint terms. */
  int n_jvx;
  int jvx_is_cnt[THIP_MAX_JVX];
  int jvx_first_step[THIP_MAX_JVX];
  int jvx_last_step[THIP_MAX_JVX];
  double jvx_coeffs[THIP_MAX_JVX][THIP_MAX_DOF];
  double jvx_targets[THIP_MAX_JVX][THIP_MAX_DOF];
  double jvx_upper_tols[THIP_MAX_JVX][THIP_MAX_DOF];
  double jvx_lower_tols[THIP_MAX_JVX][THIP_MAX_DOF];

  /* Joint-derivative terms: order 1 JointVelEqConstraint (trajectory_costs.cpp:
   * 376-424), order 2 JointAcc{Eq,Ineq}{Cost,Constraint} (:502-753), order 3
   * JointJerk (:756-1016), zero tolerances -> Eq forms.  Steps after the hatch
   * clamping (problem_description.cpp:1412-1533, 1534-1640).  Costs follow every
   * other cost term but collision, constraints every other constraint but
   * collision.  The fused sqp_kernel lowers JointAccEqCost (order 2, cost, zero
   * tolerances) when thip_jdt_fused() holds: the reduced KKT matrix is then
   * block-tridiagonal over waypoint PAIRS (2 D-wide blocks).  Every other form is
   * refused by thip_create and runs the generic path (sco::BasicTrustRegionSQP
   * on the host with the GpuModel); this table is also the record the oracle
   * reads. */
  int n_jdt;
  int jdt_order[THIP_MAX_JDT];
  int jdt_is_cnt[THIP_MAX_JDT];
  int jdt_first_step[THIP_MAX_JDT];
  int jdt_last_step[THIP_MAX_JDT];
  double jdt_coeffs[THIP_MAX_JDT][THIP_MAX_DOF];
  double jdt_targets[THIP_MAX_JDT][THIP_MAX_DOF];
  double jdt_upper_tols[THIP_MAX_JDT][THIP_MAX_DOF];
  double jdt_lower_tols[THIP_MAX_JDT][THIP_MAX_DOF];

  /* Time parameterisation (basic_info.use_time, problem_description.cpp:557-598,
   * 372-379): one more variable per waypoint, dt_i in [dt_lower, dt_upper]
   * after the waypoint's joints, initialised to init_dt; and the time-
   * parameterised JointVel terms (JointVelTermInfo::hatch with TT_USE_TIME,
   * :1263-1344): per joint j a TrajOptCostFromErrFunc / ConstraintFromErrFunc
   * over (x_j[first..last], dt[first..last]) with JointVelErrCalculator /
   * JointVelJacCalculator (kinematic_terms.cpp:434-475), SQUARED or HINGE
   * (costs) / EQ or INEQ (constraints) by the tolerances, steps clamped as
   * the JointVel hatch.  Costs follow the jdt costs, constraints the jdt
   * constraints.  basic_info.fixed_dofs (:528-546): joint columns pinned to
   * the initial trajectory at every step that is not a fixed timestep.
   * thip_create rejects use_time, n_jvt, n_ttt > 0 and n_fixed_dofs > 0 (the generic
   * path runs them); they are the lowered record the oracle reads. */
  int use_time;
  double dt_lower, dt_upper, init_dt;
  int n_fixed_dofs;
  int fixed_dofs[THIP_MAX_DOF];
  int n_jvt;
  int jvt_is_cnt[THIP_MAX_JVT];
  int jvt_first_step[THIP_MAX_JVT];
  int jvt_last_step[THIP_MAX_JVT];
  double jvt_coeffs[THIP_MAX_JVT][THIP_MAX_DOF];
  double jvt_targets[THIP_MAX_JVT][THIP_MAX_DOF];
  double jvt_upper_tols[THIP_MAX_JVT][THIP_MAX_DOF];
  double jvt_lower_tols[THIP_MAX_JVT][THIP_MAX_DOF];
  /* TotalTimeTermInfo (problem_description.cpp:1860-1913): sum over steps 1..N-1
   * of 1/x[i][W-1] (the last variable column: dt with use_time) minus limit,
   * TimeCostCalculator / TimeCostJacCalculator (kinematic_terms.cpp:579-591);
   * SQUARED / EQ when limit is 0, else HINGE / INEQ.  Costs follow the time
   * JointVel costs, constraints the time JointVel constraints. */
  int n_ttt;
  int ttt_is_cnt[THIP_MAX_TTT];
  double ttt_coeff[THIP_MAX_TTT];
  double ttt_limit[THIP_MAX_TTT];

  /* CollisionTermInfo, LVS_DISCRETE or LVS_CONTINUOUS, cost or constraint
   * (collision_terms.cpp:737-1161,1267-1386):
   * robot collision model = spheres rigidly attached to chain links; the scene
   * is per problem (n_prims primitives of 16 doubles each, see THIP_PRIM_*). */
  int coll_enabled;
  int coll_is_cnt;
  int coll_first_step;
  int coll_last_step;
  int coll_n_fixed;
  int coll_fixed_steps[THIP_MAX_STEPS];
  double coll_margin;      /* dist_pen */
  double coll_coeff;       /* coeffs */
  double coll_buffer;      /* collision_margin_buffer */
  double coll_lvs;         /* longest_valid_segment_length */
  int coll_continuous;     /* 0: LVS_DISCRETE (DiscreteCollisionEvaluator, sub-state contacts);
                              1: LVS_CONTINUOUS / CONTINUOUS (CastCollisionEvaluator,
                              collision_terms.cpp:978-1161): each robot sphere is swept between
                              consecutive sub-states (a capsule) and tested against the scene;
                              CONTINUOUS is LVS_CONTINUOUS with coll_lvs = +inf (one cast per pair) */
  int coll_contact_test;   /* THIP_CONTACT_ALL (0) / FIRST / CLOSEST; the fused kernel takes ALL */
  int n_spheres;
  int sphere_link[THIP_MAX_SPHERES];
  double sphere_center[THIP_MAX_SPHERES][3];  /* in link frame */
  double sphere_radius[THIP_MAX_SPHERES];
  int n_prims;
  /* robot self-collision: the link pairs whose spheres are tested against each
   * other, both links moving -- the contact manager's active-link pairs that the
   * allowed-collision matrix leaves enabled (the SRDF's <disable_collisions>,
   * e.g. pr2.srdf: the two arms of config E, and each arm's shoulder_pan vs its
   * wrist links).  A pair's contacts get gradients on both links
   * (GetGradient's two sides, collision_terms.cpp:195-242) and the scene's
   * margin / coeff.  Key order: a unit's scene keys (link, primitive) first,
   * then these pairs in this order; inside a key, sub-state, then the sphere of
   * link a, then the sphere of link b.  At most THIP_MAX_SELF_SPHERE_PAIRS
   * sphere pairs in all. */
  int n_self_pairs;
  int self_pair[THIP_MAX_SELF_PAIRS][2];
  /* hinge-row (contact) capacity per QP; 0 = automatic: the largest possible
   * contact count (step pairs x 64 LVS sub-states x spheres x primitives),
   * capped at THIP_MAX_CONTACTS and at what fits a 16 GB share of HBM for the
   * batch (~800 B per row and problem), at least 2048.  A QP with more
   * contacts ends the run with OPT_FAILED and THIP_FLAG_CONTACT_OVERFLOW. */
  int coll_max_contacts;
  /* further collision terms (a collision cost and a collision constraint in one
   * problem, simple_collision_test.json:6-37): cost terms follow the first
   * collision term's cost, constraint terms its constraint, each in hatch
   * order.  The generic path evaluates them on the device (thip_eval_*);
   * thip_create rejects n_coll_extra > 0. */
  int n_coll_extra;
  thip_coll_term coll_extra[THIP_MAX_COLL_EXTRA];
  /* per link-pair margins and coefficients of the collision terms (see
   * thip_coll_pair); pairs not listed take their term's coll_margin / coll_coeff */
  int n_coll_pairs;
  thip_coll_pair coll_pairs[THIP_MAX_COLL_PAIRS];

  thip_sqp_params sqp;
  thip_osqp_settings osqp;
} thip_problem_desc;

/* 1 when the descriptor's jdt terms can run in the fused sqp_kernel: every one a
 * JointAccEqCost (order 2, cost, all tolerances zero as JointAccTermInfo::hatch
 * tests them, |tol| < 1e-5), the waypoints pairing into 2 D-wide solve blocks
 * (n_steps even, 2 n_dof <= THIP_MAX_DOF), no time parameterisation.  0 when a
 * jdt term needs the generic path; also 1 without jdt terms. */
int thip_jdt_fused(const thip_problem_desc* d);

/* Per-problem results (sco::OptResults + counters the build adds). */
typedef struct thip_result {
  int status;         /* THIP_OPT_* */
  int n_sqp_iters;    /* executed SQP iterations (outer-loop bodies, all penalty rounds) */
  int n_qp_solves;    /* OptResults::n_qp_solves */
  int n_func_evals;   /* OptResults::n_func_evals */
  long long n_admm_iters; /* ADMM iterations summed over QP solves */
  int n_merit_increases;
  double total_cost;  /* OptResults::total_cost */
  double max_cnt_viol;/* max over constraints of the violation (0 if none) */
  double final_trust_box;
  int n_costs;
  int n_cnts;
  int flags;          /* THIP_FLAG_* */
  /* collision work counters (bench roofline model) */
  long long n_contact_rows;  /* sum over linearisations of the hinge rows built */
  long long n_hinge_admm;    /* sum over QP solves of hinge rows x ADMM iterations */
  long long n_substates;     /* LVS sub-state passes over the scene (all contact scans) */
} thip_result;

/* thip_result.flags */
#define THIP_FLAG_CONTACT_OVERFLOW 1 /* contacts exceeded the hinge-row capacity (or > 1024 LVS
                                        sub-states in a step pair): the run is OPT_FAILED */

typedef struct thip_ctx thip_ctx;

/* Fill defaults (reference default parameters). */
void thip_default_sqp_params(thip_sqp_params* p);
void thip_default_osqp_settings(thip_osqp_settings* s);

/* Validate the descriptor and allocate device buffers for `batch` problems on
 * HIP device `device`. */
int thip_create(int device, const thip_problem_desc* desc, int batch, thip_ctx** out);

/* Use this HIP stream (hipStream_t passed as void*; NULL = the ctx's own). */
int thip_set_stream(thip_ctx* ctx, void* stream);

/* H2D copy of per-problem inputs:
 *   init_traj    [batch][n_steps][n_dof]
 *   cart_targets [batch][n_cart][12]     target-frame offset poses (may be NULL if n_cart == 0)
 *   scene        [batch][n_prims][16]    primitive records (may be NULL if n_prims == 0)  */
int thip_upload(thip_ctx* ctx, const double* init_traj, const double* cart_targets, const double* scene);

/* Per-problem JointPos targets [batch][n_jpos][n_dof] (host pointer); without
 * this call every problem uses desc->jpos_targets.  Replaces the per-problem
 * JointPosTermInfo::targets of the reference (problem_description.cpp:1061-1095). */
int thip_upload_joint_targets(thip_ctx* ctx, const double* jpos_targets);

/* Device-to-device variant: pointers are device pointers (e.g. torch tensors). */
int thip_upload_device(thip_ctx* ctx, const double* d_init_traj, const double* d_cart_targets,
                       const double* d_scene);

/* Run BasicTrustRegionSQP::optimize for every problem (asynchronous on the
 * ctx stream).  Several contexts on their own streams keep several batches in
 * flight: the next batch fills the CUs the current batch's longest problems
 * leave idle. */
int thip_sqp_run(thip_ctx* ctx);

/* Wait for the ctx stream (every run queued on it has finished). */
int thip_synchronize(thip_ctx* ctx);

/* Convexify at trajectory x [batch][n_steps][n_dof] (host pointer): CartPose
 * error rows and forward-difference Jacobians, exactly as the SQP loop does.
 *   err [batch][n_cart][6]   (rows of indices with zero coeff are 0)
 *   jac [batch][n_cart][6][n_dof]
 * Synchronous. */
int thip_linearize(thip_ctx* ctx, const double* x, double* err, double* jac);

/* Forward kinematics of every chain link at x: poses [batch][n_steps][n_links][12]. Synchronous. */
int thip_fwd_kin(thip_ctx* ctx, const double* x, double* poses);

/* Copy results back (synchronises the stream):
 *   x       [batch][n_steps][n_dof]  final trajectory
 *   results [batch]                  (may be NULL) */
int thip_download(thip_ctx* ctx, double* x, thip_result* results);

/* Device pointer of the final trajectories (valid until destroy). */
const double* thip_device_x(thip_ctx* ctx);

/* Per-launch timing of the last thip_sqp_run, measured with HIP events on the
 * ctx stream around the fused kernel (milliseconds). */
double thip_last_kernel_ms(thip_ctx* ctx);

void thip_destroy(thip_ctx* ctx);
const char* thip_last_error(thip_ctx* ctx);

/* Version / build info string. */
const char* thip_build_info(void);

/* sizeof(thip_problem_desc) as compiled into the library (ABI check). */
int thip_sizeof_desc(void);
int thip_sizeof_result(void);

/* Diagnostics: record one 10-double entry per QP solve of every problem
 * (warm_started, rho_initial, admm_iters, osqp_status, polish_status,
 * rho_final, prim_res, dual_res, sum|x*|, trust_box) during thip_sqp_run,
 * up to `capacity` entries per problem (0 disables). */
int thip_debug_trace(thip_ctx* ctx, int capacity);
/* records [batch][capacity][THIP_TRACE_W], counts [batch].  One record per QP
 * solve: [0] warm start, [1] rho at entry, [2] ADMM iterations, [3] status,
 * [4] polish status, [5] rho at exit, [6] primal / [7] dual residual, [8] sum |x*|,
 * [9] trust box size; then the trust-region step that QP served
 * (BasicTrustRegionSQPResults::writeSolver, optimizers.cpp:533-547): [10] old
 * exact merit, [11] new exact merit, [12] approx merit improve, [13] exact merit
 * improve, [14] ratio, [15] decision (1 converged, 2 shrink, 3 accept; 0 none). */
#define THIP_TRACE_W 16
int thip_debug_get_trace(thip_ctx* ctx, double* records, int* counts);

/* Linearised collision rows (config C) of every problem at trajectories x
 * [batch][N][D]: the distance expressions of CollisionCost::convex
 * (trajopt/src/collision_terms.cpp:463-536, 1267-1284), one record per
 * contact in hinge-row order, [t, link, prim, sphere, substate, distance,
 * cc_time, n_kept, a_t[D], a_t+1[D], constant] (8 + 2 D + 1 doubles);
 * records [batch][cap][...], counts[batch] (-1 on contact overflow). */
int thip_collision_rows(thip_ctx* ctx, const double* x, double* records, int cap, int* counts);

/* Diagnostics: per-problem phase cycle counters (32 slots per problem; see
 * the slot list in sqp_kernel.hip).  enable = 0 frees them.  Counters
 * accumulate over runs until re-enabled. */
int thip_debug_profile(thip_ctx* ctx, int enable);
int thip_debug_get_profile(thip_ctx* ctx, long long* counters /* [batch][40] */);
/* Diagnostics: workspace layout (array offsets in doubles / ints, and
 * dims = {N, D, nx, n_fixed_rows, n_abs, n_cols, n_rows, m, dstride, istride,
 * n_double_arrays, n_int_arrays}) and a copy of the device workspace. */
int thip_debug_layout(thip_ctx* ctx, long long* doff, long long* ioff, long long* dims);
/* Diagnostics: force a solve path for every context created after the call
 * (process-wide; 0 restores the automatic choice).  THIP_DEBUG_NO_SEGMENT runs
 * the generic ADMM step instead of the register-resident segment,
 * THIP_DEBUG_FORCE_WIDE the wide-block (D > 8) solve for any D,
 * THIP_DEBUG_NO_BRANCH one block solve over all dofs of a tree whose terms
 * never couple its branches (the dual arm splits into two 7-dof solves).  Same
 * results to the parity bar; for tests and profiling only (the product path
 * never reads the environment). */
#define THIP_DEBUG_NO_SEGMENT 1
#define THIP_DEBUG_FORCE_WIDE 2
#define THIP_DEBUG_NO_BRANCH 4  /* one block solve over all dofs even when the terms split the tree */
#define THIP_DEBUG_STATIC_DISPATCH 8  /* one workgroup per problem instead of persistent workgroups taking
                                         problems from a counter (bitwise the same results) */
#define THIP_DEBUG_GEN_BUILD 16       /* with THIP_DEBUG_NO_SEGMENT: every QP runs the generic-step build
                                         (its own compilation, no segment code) */
#define THIP_DEBUG_MAIN_BUILD 32      /* QPs outside the segment's domain run the main build's generic step
                                         instead of the generic-step build (the default since round 6) */
int thip_debug_set_path(int flags);
int thip_debug_workspace(thip_ctx* ctx, double* dws, int* iws);
/* The solve layout a context chose (diagnostic): out[0] block-solve branches
 * (Layout::nbr), out[1] dofs per block, out[2] wide blocks, out[3] the
 * register-resident segment possible, out[4] the generic-step build,
 * out[5] threads per problem, out[6] waypoints per solve block (Layout::grp:
 * 2 with JointAccEqCost terms), out[7] solve blocks per branch.  n: entries of
 * out (<= 8 written). */
#define THIP_LAYOUT_INFO_N 8
int thip_debug_solve_layout(const thip_ctx* ctx, int* out, int n);

/* ------------------------------------------------------- Term evaluation
 * The kinematic terms of one problem structure evaluated on the device for
 * sco::BasicTrustRegionSQP's host loop (the generic path, which runs what the
 * batched kernel does not lower: single-waypoint problems, several collision
 * terms, CartPose / collision next to JointAcc / JointJerk / time terms or a
 * user sco::Cost).  Replaces the CPU evaluation the reference's term objects
 * do inside the loop:
 *   thip_eval_cart_pose  <- CartPoseErrCalculator / CartPoseJacCalculator
 *                           (trajopt/src/kinematic_terms.cpp:189-370) and the
 *                           DynamicCartPose pair (:58-187), called through
 *                           TrajOptCostFromErrFunc / TrajOptConstraintFromErrFunc
 *                           (CartPoseTermInfo::hatch, problem_description.cpp:919-1005)
 *   thip_eval_collision  <- CollisionEvaluator::CalcCollisions / GetGradient /
 *                           CalcDistExpressions* (collision_terms.cpp:195-554,
 *                           646-688, 817-898, 978-1161), called by
 *                           CollisionCost / CollisionConstraint::value / convex
 *                           (:1267-1386), one term object per unit
 *                           (CollisionTermInfo::hatch, problem_description.cpp:1735-1858)
 * A thip_eval holds a descriptor (any n_steps in [1, THIP_EVAL_MAX_STEPS], up to
 * THIP_EVAL_MAX_PRIMS scene primitives, any term set: only the chain, CartPose and
 * collision fields are read) and the CartPose
 * targets and scenes of `batch` problems.  Synchronous; host arrays. */
typedef struct thip_eval thip_eval;
int thip_eval_create(int device, const thip_problem_desc* desc, int batch, thip_eval** out);
/* cart_targets [batch][n_cart][12], scene [batch][n_prims][16] (NULL when empty) */
int thip_eval_upload(thip_eval* ev, const double* cart_targets, const double* scene);
/* CartPose term `term` (descriptor order) of every problem at its waypoint's joint
 * values q [batch][n_dof]: err [batch][6] the (banded) transform error, jac
 * [batch][6][n_dof] its forward-difference jacobian (eps 1e-5) or NULL for the
 * error alone.  All six components: the caller keeps those whose coefficient is
 * nonzero (CartPoseTermInfo::hatch's indices). */
int thip_eval_cart_pose(thip_eval* ev, int term, const double* q, double* err, double* jac);
/* Every CartPose term of every problem at its own waypoint of the joint
 * trajectories x [batch][n_steps][n_dof], in one launch: err
 * [batch][n_cart][6], jac [batch][n_cart][6][n_dof] or NULL.  Bitwise the
 * values thip_eval_cart_pose gives term by term (the same device function);
 * the host loop evaluates all its CartPose terms at a new x with it instead of
 * one launch per term (sco::OptProb::prefetch). */
int thip_eval_cart_pose_all(thip_eval* ev, const double* x, double* err, double* jac);
/* Collision term `term` (0: the coll_* term when coll_enabled, then coll_extra[])
 * at trajectories x [batch][n_steps][n_dof]: every contact of every unit (a free
 * waypoint of [first, last] for DISCRETE, else a step pair) with its linearised
 * distance expression, in unit order, then ContactResultMap order.  records
 * [batch][cap][8 + 2 n_dof + 1] = [t, link, prim, sphere, substate, distance,
 * cc_time, n_kept, a_t[n_dof], a_t+1[n_dof], constant] as thip_collision_rows
 * (t = the unit's waypoint; a_t+1 = 0 for DISCRETE); counts [batch] = contacts
 * found (records beyond cap are not written). */
int thip_eval_collision(thip_eval* ev, int term, const double* x, double* records, int cap, int* counts);
void thip_eval_destroy(thip_eval* ev);
const char* thip_eval_last_error(thip_eval* ev); /* NULL: the last thip_eval_create failure */

/* ------------------------------------------------------------- Generic QP
 * OSQP 1.0 on an arbitrary sparse QP
 *     minimise 1/2 x'Px + q'x   subject to   l <= A x <= u
 * with OSQPModel's settings and warm start (sco::OSQPModel::optimize,
 * trajopt_sco/src/osqp_interface.cpp:283-615): the QP backend of
 * sco::GpuModel (trajopt-1_amd/host/include/trajopt_sco/gpu_model.hpp), which
 * is the sco::Model a non-lowerable OptProb (custom terms, JointAcc /
 * JointJerk terms, the reference's small-problem tests) is solved with.  A
 * thip_qp holds one sparsity pattern -- P upper-triangular CSC (n x n), A CSC
 * (m x n) -- for `batch` QPs whose values differ; one workgroup per QP, sparse
 * quasi-definite LDL^T of the KKT (minimum-degree order and elimination-tree
 * level schedule computed once per pattern at create), n + m <= THIP_QP_MAX_KKT.
 * Patterns must not repeat an entry. */
#define THIP_QP_MAX_KKT 65536
typedef struct thip_qp thip_qp;
typedef struct thip_qp_info {
  int status;        /* OSQP 1.0 status value (1 solved, 2 solved inaccurate, 3/4 primal infeasible
                        (inaccurate), 5/6 dual infeasible (inaccurate), 7 max iter, 9 non-convex);
                        -1: setup failed (see setup_error) */
  int setup_error;   /* osqp_setup error code when status = -1 (1 data validation, 4 KKT
                        factorisation, 5 non-convex) */
  int polish_status; /* 1 polished, -1 polish failed, 0 not run */
  int iter;          /* ADMM iterations */
  double rho;        /* rho at exit (the warm start of the next solve) */
  double prim_res;
  double dual_res;
} thip_qp_info;
/* Pattern (host arrays, copied): P_colptr[n+1], P_rowind[nnz_P] (rows <= column),
 * A_colptr[n+1], A_rowind[nnz_A]. */
int thip_qp_create(int device, int n, int m, const int* P_colptr, const int* P_rowind, const int* A_colptr,
                   const int* A_rowind, int batch, thip_qp** out);
/* Solve every QP (synchronous; host arrays): P_values [batch][nnz_P], q [batch][n],
 * A_values [batch][nnz_A], l, u [batch][m] (+-1e30 = infinite); warm_x [batch][n],
 * warm_y [batch][m] (both or neither), warm_rho [batch] (or NULL: settings->rho);
 * out: x [batch][n], y [batch][m] (may be NULL), info [batch]. */
int thip_qp_solve(thip_qp* qp, const double* P_values, const double* q, const double* A_values, const double* l,
                  const double* u, const thip_osqp_settings* settings, const double* warm_x, const double* warm_y,
                  const double* warm_rho, double* x, double* y, thip_qp_info* info);
/* thip_qp_solve for the first `count` QPs of the batch (1 <= count <= batch), QP k
 * warm started from warm_x / warm_y only when warm_mask[k] != 0 (warm_mask NULL: all
 * of them, as thip_qp_solve), with warm_rho[k] its initial rho (NULL: settings->rho):
 * one launch for the QPs of many problems' host SQP loops that share a pattern
 * (sco::GpuQPBatcher).  Arrays are [count][...]. */
int thip_qp_solve_some(thip_qp* qp, int count, const double* P_values, const double* q, const double* A_values,
                       const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                       const double* warm_y, const int* warm_mask, const double* warm_rho, double* x, double* y,
                       thip_qp_info* info);
/* thip_qp_solve_some in two halves: thip_qp_submit copies the inputs and
 * launches on the QP object's own stream and returns; thip_qp_collect waits for
 * that launch and returns x, y, info.  Submissions to different QP objects
 * (patterns) run concurrently on the device -- sco::GpuQPBatcher submits every
 * pattern of a round before it collects any.  The host arrays of a submission
 * must stay valid until it is collected; one submission per object at a time. */
int thip_qp_submit(thip_qp* qp, int count, const double* P_values, const double* q, const double* A_values,
                   const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                   const double* warm_y, const int* warm_mask, const double* warm_rho);
int thip_qp_collect(thip_qp* qp, double* x, double* y, thip_qp_info* info);
/* thip_qp_submit without the launch (inputs copied, arguments kept), then one
 * launch for the staged QPs of several objects (patterns) of one device:
 * thip_qp_launch_staged(qps, n) runs them as one grid on qps[0]'s stream (each
 * workgroup finds its pattern), so a round of many patterns is one launch;
 * thip_qp_collect then returns each object's results.  A destroyed qps[0] must
 * be collected first (its stream runs the group). */
int thip_qp_stage(thip_qp* qp, int count, const double* P_values, const double* q, const double* A_values,
                  const double* l, const double* u, const thip_osqp_settings* settings, const double* warm_x,
                  const double* warm_y, const int* warm_mask, const double* warm_rho);
int thip_qp_launch_staged(thip_qp* const* qps, int n);
void thip_qp_destroy(thip_qp* qp);
const char* thip_qp_last_error(thip_qp* qp); /* NULL: the last thip_qp_create failure */
/* Entries of the KKT factor L of the pattern (the symbolic analysis of
 * thip_qp_create): the algorithmic-byte model of the QP solves; -1 for NULL. */
long long thip_qp_factor_nnz(const thip_qp* qp);
/* The pattern's KKT shape (diagnostic): out[0] N = n + m, out[1] entries of L,
 * out[2] elimination-tree levels (the solve's serial depth), out[3] the widest
 * level, out[4] 1 when the factor is staged in LDS, out[5] dynamic LDS bytes. */
int thip_qp_shape(const thip_qp* qp, long long* out);
/* Cycle counters of the first QP of every qp_csc_kernel launch on the current
 * device (diagnostic): out[8] = iterate copies + rhs, KKT solves, updates,
 * checks (residuals, termination, rho updates), ADMM iterations, polish; reset
 * zeroes them after the read. */
int thip_qp_debug_profile(long long* out, int reset);

/* Resident workspace (update in place).  The OSQP 1.0 solver object of every QP
 * of the batch stays on the device between calls, as OsqpEigen::Solver keeps it
 * for trajopt_sqp::OSQPEigenSolver (the QPSolver of the trajopt_sqp front end,
 * trajopt_optimizers/trajopt_sqp/src/osqp_eigen_solver.cpp:73-320, driven by
 * TrustRegionSQPSolver::stepSQPSolver, trust_region_sqp_solver.cpp:202-260):
 * after thip_qp_setup, only the vectors / values that changed are sent, the
 * scaling, rho vector, KKT factor and ADMM iterates persist.  Host arrays,
 * [batch][...], synchronous.  info->status is -1 with setup_error set when a
 * call fails (1 data validation: l > u, the update is rejected; 4 / 5 the
 * refactorisation failed / is not quasi-definite: the workspace is gone, the
 * next call must be thip_qp_setup), 0 otherwise (thip_qp_solve_resident:
 * the OSQP status). */
/* osqp_setup: Ruiz scaling, rho vector, KKT factor; x = z = y = 0 */
int thip_qp_setup(thip_qp* qp, const double* P_values, const double* q, const double* A_values, const double* l,
                  const double* u, const thip_osqp_settings* settings, thip_qp_info* info);
/* osqp_update_data_vec: q and / or (l, u) (NULL = unchanged); the rho vector follows the
 * constraint types, refactored only when a type changed */
int thip_qp_update_vec(thip_qp* qp, const double* q, const double* l, const double* u, thip_qp_info* info);
/* osqp_update_data_mat: all values of P and / or A (same pattern; NULL = unchanged):
 * unscale, replace, rescale, refactor */
int thip_qp_update_mat(thip_qp* qp, const double* P_values, const double* A_values, thip_qp_info* info);
/* osqp_warm_start: x and / or y (unscaled; NULL = unchanged), z = A x; turns warm starting on */
int thip_qp_warm_start(thip_qp* qp, const double* x, const double* y);
/* osqp_solve from the kept iterates (warm_starting) or from zero: x [batch][n], y [batch][m] (may be NULL) */
int thip_qp_solve_resident(thip_qp* qp, double* x, double* y, thip_qp_info* info);

#ifdef __cplusplus
}
#endif

#endif /* TRAJOPT_HIP_H */
