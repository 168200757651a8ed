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
 * built-in PR2 "right_arm" environment.  Return 0 on success, -1 on failure
 * with the message (the reference's std::runtime_error text) in err.
 */
#ifndef TRAJOPT_HOST_H
#define TRAJOPT_HOST_H

#include "trajopt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parse + ConstructProblem for one JSON problem; `scene` holds the
 * environment's primitives ([n_prims][16], THIP_PRIM_* records, may be NULL
 * when n_prims == 0).  Outputs (caller-sized to the maxima):
 *   desc          the batch-shared structure (per-problem JointPos targets zeroed)
 *   init          [n_steps][n_dof]                initial trajectory
 *   cart_targets  [n_cart][12]                    CartPose target offsets in the chain root
 *   jpos_targets  [n_jpos][n_dof]                 JointPos targets
 * Any output pointer may be NULL. */
int thost_lower_json(const char* json_text, const double* scene, int n_prims, thip_problem_desc* desc,
                     double* init, double* cart_targets, double* jpos_targets, char* err, int err_len);

/* ConstructProblem for each of `batch` JSON problems (scenes [batch][n_prims][16])
 * and one BatchTrustRegionSQP on HIP device `device`:
 *   x        [batch][n_steps][n_dof]   final trajectories
 *   results  [batch]                   status and counters (may be NULL) */
int thost_solve_json_batch(const char* const* json_texts, int batch, const double* scenes, int n_prims, int device,
                           double* x, thip_result* results, char* err, int err_len);

/* thost_solve_json_batch sharded over n_devices HIP devices of this process
 * (trajopt::MultiDeviceBatchSQP: contiguous shards, sizes differing by at most
 * one, all shards running concurrently; a device may be listed more than once). */
int thost_solve_json_batch_multi(const char* const* json_texts, int batch, const double* scenes, int n_prims,
                                 const int* devices, int n_devices, double* x, thip_result* results, char* err,
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

#ifdef __cplusplus
}
#endif

#endif /* TRAJOPT_HOST_H */
