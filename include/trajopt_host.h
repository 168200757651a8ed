/*
 * trajopt_host.h — C entry points of the C++ host front door
 * (trajopt-1_amd/lib/libtrajopt_host.so, sources in trajopt-1_amd/host/).
 *
 * The C++ API (trajopt-1_amd/host/include/trajopt_amd/ headers) mirrors the
 * reference's problem-construction surface: ProblemConstructionInfo::fromJson,
 * the TermInfo registry and hatch(), ConstructProblem
 * (trajopt/src/problem_description.cpp:36-598) and a batch
 * BasicTrustRegionSQP (trajopt_sco/src/optimizers.cpp:699-991).  These C
 * wrappers expose it to ctypes / FFI callers: JSON problem text in the
 * reference's TrajOptRequest format (trajopt_common/data/config/ JSON files) on the
 * built-in environment of the reference's test robots (thost_lower_json).  Return 0 on success, -1 on failure
 * with the message (the reference's std::runtime_error text) in err.
 */
#ifndef TRAJOPT_HOST_H
#define TRAJOPT_HOST_H

#include "trajopt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parse + ConstructProblem for one JSON problem; `scene` holds primitives added
 * to the built-in environment's own ([n_prims][16], THIP_PRIM_* records, may be
 * NULL when n_prims == 0).  The environment is the reference test robot of
 * basic_info.manip: the PR2 (right_arm, left_arm, both_arms; empty scene) or
 * spherebot ("manipulator"; its three static spheres first).  Outputs
 * (caller-sized to the maxima: THIP_EVAL_MAX_STEPS waypoints, THIP_MAX_CART,
 * THIP_MAX_JPOS terms, THIP_EVAL_MAX_PRIMS primitives):
 *   desc          the batch-shared structure (per-problem JointPos targets zeroed)
 *   init          [n_steps][n_dof]                initial trajectory
 *   cart_targets  [n_cart][12]                    CartPose target offsets in the chain root
 *   jpos_targets  [n_jpos][n_dof]                 JointPos targets
 *   scene_out     [desc.n_prims][16]              the scene the collision terms see
 * Any output pointer may be NULL. */
int thost_lower_json(const char* json_text, const double* scene, int n_prims, thip_problem_desc* desc,
                     double* init, double* cart_targets, double* jpos_targets, double* scene_out, char* err,
                     int err_len);

/* ConstructProblem for each of `batch` JSON problems (scenes [batch][n_prims][16])
 * and one BatchTrustRegionSQP on HIP device `device`:
 *   x        [batch][n_steps][n_dof]   final trajectories
 *   results  [batch]                   status and counters (may be NULL) */
int thost_solve_json_batch(const char* const* json_texts, int batch, const double* scenes, int n_prims, int device,
                           double* x, thip_result* results, char* err, int err_len);

/* A batch with problems the fused kernel does not lower runs the problems' host
 * SQP loops on a bounded pool of worker threads (each worker takes the next
 * unsolved problem when its current one ends), every QP round in one launch per
 * sparsity pattern (trajopt::BatchTrustRegionSQP's host-loop mode, sco::GpuQPBatcher);
 * x then holds [batch][n_steps][n_dof (+ 1 with use_time)].  This reports the QP
 * launches and QPs of the calling thread's last batch solve (0 for a fused-kernel batch). */
void thost_last_batch_qp_stats(long long* launches, long long* qps);
/* Worker threads of such host-loop batches (process-wide; n <= 0 restores the
 * default, 64; never more than the batch). */
void thost_set_host_loop_workers(int n);

/* A prepared batch: ConstructProblem for each of `batch` JSON problems
 * (scenes [batch][n_prims][16]) and the trajopt::BatchTrustRegionSQP over them
 * on HIP device `device`, without solving -- so a caller (the bench) times the
 * solve alone.  thost_batch_solve runs it once: x [batch][n_steps][n_dof (+1
 * with use_time)], results [batch] (may be NULL); a host-loop batch's models
 * keep their warm starts, so it is solved at most once (a second call fails).
 * thost_batch_stats: host_loops (1 when the problems run the host loops with
 * batched QPs, 0 for the fused kernel), and for host loops the QP launches, QPs,
 * their algorithmic HBM bytes (sco::GpuQPBatcher::bytes) and the wall seconds
 * spent in the launches.  Every problem's host loop runs at once (one worker
 * per problem), so each QP round of the batch is one launch per pattern. */
typedef struct thost_batch thost_batch;
int thost_batch_create(const char* const* json_texts, int batch, const double* scenes, int n_prims, int device,
                       thost_batch** out, char* err, int err_len);
int thost_batch_solve(thost_batch* b, double* x, thip_result* results, char* err, int err_len);
int thost_batch_stats(const thost_batch* b, int* host_loops, long long* qp_launches, long long* qps, double* qp_bytes,
                      double* qp_seconds);
/* Host-loop batches (diagnostic): out[0] ADMM iterations of all QPs, then the
 * largest KKT's thip_qp_shape (6 entries). */
int thost_batch_qp_shape(const thost_batch* b, long long* out);
void thost_batch_destroy(thost_batch* b);

/* thost_solve_json_batch sharded over n_devices HIP devices of this process
 * (trajopt::MultiDeviceBatchSQP: contiguous shards, sizes differing by at most
 * one, all shards running concurrently; a device may be listed more than once). */
int thost_solve_json_batch_multi(const char* const* json_texts, int batch, const double* scenes, int n_prims,
                                 const int* devices, int n_devices, double* x, thip_result* results, char* err,
                                 int err_len);

/* A stream of n_batches batches of `batch` JSON problems each (json_texts
 * [n_batches * batch], scenes [n_batches * batch][n_prims][16]), every batch
 * sharded over the device entries as thost_solve_json_batch_multi does, with
 * `inflight` batches in flight per device entry
 * (trajopt::MultiDeviceBatchSQP::optimizeStream: the next batches fill the CUs
 * the current batch's tail leaves idle).  x [n_batches * batch][n_steps][n_dof],
 * results [n_batches * batch] (may be NULL), in input order. */
int thost_solve_json_stream(const char* const* json_texts, int n_batches, int batch, const double* scenes, int n_prims,
                            const int* devices, int n_devices, int inflight, double* x, thip_result* results, char* err,
                            int err_len);

/* ConstructProblem for one JSON problem and trajopt::BasicTrustRegionSQP
 * (sco::BasicTrustRegionSQP with the problem's opt_info) on HIP device
 * `device`, as the reference's planning code runs one problem
 * (optimizers.cpp:699-991): a problem whose every term lowered into the
 * batched kernel runs it as a batch of one (*native = 1); one with terms the
 * kernel does not lower (JointAcc / JointJerk, JointVel equality constraints,
 * time-parameterised JointVel, TotalTime, fixed dofs) runs the SQP loop on the
 * host with every QP on the GPU (GpuModel, *native = 0).
 * x: [n_steps][n_dof (+ 1: the dt column with basic_info.use_time)];
 * result and native may be NULL. */
int thost_solve_json(const char* json_text, const double* scene, int n_prims, int device, double* x,
                     thip_result* result, int* native, char* err, int err_len);

/* ---------------------------------------------------------- trajopt_sqp
 * The second SQP front end (the ifopt stack):
 * trajopt_sqp::TrustRegionSQPSolver over a trajopt_sqp::TrajOptQPProblem whose
 * QP keeps one sparsity pattern and is updated in place on the GPU
 * (trajopt_sqp::GpuQPSolver over thip_qp's resident workspace).  The C++ API is
 * trajopt-1_amd/host/include/trajopt_sqp/ and trajopt_ifopt/; this flat spec
 * drives it from FFI callers and the tests: a joint trajectory of n_nodes
 * nodes (one trajopt_ifopt::Var of n_dof positions each) with joint
 * position / velocity / acceleration / jerk terms as constraints or costs. */
#define TSQP_MAX_NODES 64
#define TSQP_MAX_TERMS 16
enum { TSQP_JOINT_POS = 0, TSQP_JOINT_VEL = 1, TSQP_JOINT_ACC = 2, TSQP_JOINT_JERK = 3 };
/* addConstraintSet, or addCostSet with CostPenaltyType kSquared / kAbsolute / kHinge */
enum { TSQP_CONSTRAINT = 0, TSQP_SQUARED = 1, TSQP_ABSOLUTE = 2, TSQP_HINGE = 3 };
/* trajopt_sqp::SQPStatus (types.h) */
enum {
  TSQP_STATUS_RUNNING = 0,
  TSQP_STATUS_CONVERGED = 1,
  TSQP_STATUS_ITERATION_LIMIT = 2,
  TSQP_STATUS_PENALTY_ITERATION_LIMIT = 3,
  TSQP_STATUS_TIME_LIMIT = 4,
  TSQP_STATUS_QP_SOLVE_FAILED = 5,
  TSQP_STATUS_STOPPED_BY_CALLBACK = 6
};
typedef struct tsqp_term {
  int kind;        /* TSQP_JOINT_* */
  int penalty;     /* TSQP_CONSTRAINT / SQUARED / ABSOLUTE / HINGE */
  int first, last; /* nodes first..last (JointPos: the node `first`) */
  int n_coeffs;    /* 0, 1 or n_dof coefficients */
  double coeffs[THIP_MAX_DOF];
  /* JointPos: per-dof bounds (lower == upper: a target; a range splits into two
   * inequalities, RangeBoundHandling::kSplitToTwoInequalities); JointVel / Acc /
   * Jerk: per-dof targets in `lower` */
  double lower[THIP_MAX_DOF], upper[THIP_MAX_DOF];
} tsqp_term;
typedef struct tsqp_spec {
  int n_nodes, n_dof;
  double init[TSQP_MAX_NODES * THIP_MAX_DOF]; /* [n_nodes][n_dof] */
  double var_lower[THIP_MAX_DOF], var_upper[THIP_MAX_DOF]; /* variable bounds (+-inf allowed) */
  int n_terms;
  tsqp_term terms[TSQP_MAX_TERMS];
  /* trajopt_sqp::SQPParameters (types.h) */
  double improve_ratio_threshold, min_trust_box_size, min_approx_improve, min_approx_improve_frac;
  int max_iterations;
  double trust_shrink_ratio, trust_expand_ratio, cnt_tolerance, max_merit_coeff_increases;
  int max_qp_solver_failures;
  double merit_coeff_increase_ratio, max_time, initial_merit_error_coeff;
  int inflate_constraints_individually;
  double initial_trust_box_size;
  thip_osqp_settings osqp; /* OSQPEigenSolver::setDefaultOSQPSettings + the test's overrides */
} tsqp_spec;
typedef struct tsqp_result {
  int status;             /* TSQP_STATUS_* */
  int overall_iteration;  /* QP solves of the trust-region loop (SQPResults::overall_iteration) */
  int penalty_iteration;
  int qp_setups;          /* full QP setups (first solve, pattern or size change) */
  int qp_updates;         /* convexifications applied in place (update_data_mat / _vec) */
  int qp_solves;
  long long admm_iters;
  double best_exact_merit;
} tsqp_result;
/* SQPParameters / OSQP settings defaults into a spec (terms untouched) */
void thost_tsqp_defaults(tsqp_spec* spec);
/* solve on HIP device `device`: x [n_nodes][n_dof] (the best variables) */
int thost_tsqp_solve(const tsqp_spec* spec, int device, double* x, tsqp_result* result, char* err, int err_len);
/* sizeof(tsqp_spec) / sizeof(tsqp_result) as compiled into the library (FFI layout check) */
int thost_tsqp_sizeof_spec(void);
int thost_tsqp_sizeof_result(void);

#ifdef __cplusplus
}
#endif

#endif /* TRAJOPT_HOST_H */
