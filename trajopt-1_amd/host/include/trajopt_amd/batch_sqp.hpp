// BatchTrustRegionSQP: sco::BasicTrustRegionSQP::optimize
// (trajopt_sco/src/optimizers.cpp:699-991) for a batch of TrajOptProbs that
// share one structure, on one HIP device, through the C-ABI of
// include/trajopt_hip.h (SURVEY.md §8b tier ii).  Not thread-safe per object;
// use one per host thread and device.
#pragma once
#include <memory>
#include <vector>

#include "trajopt_amd/problem_description.hpp"

namespace trajopt
{
class BatchTrustRegionSQP
{
public:
  // Lowerable problems (every term in the descriptor): checks that every problem
  // shares problem 0's structure (steps, chain, terms, parameters, scene size)
  // and allocates the fused kernel's device workspace.  A batch with problems
  // the kernel does not lower (JointAcc / JointJerk, time terms, custom terms,
  // single waypoints, several collision terms) runs every problem's host loop
  // (sco::BasicTrustRegionSQP) on its own host thread, the kinematic terms
  // evaluated on the device and the QPs of all loops batched into one launch
  // per sparsity pattern (sco::GpuQPBatcher); results are each problem's own.
  explicit BatchTrustRegionSQP(const std::vector<TrajOptProb::Ptr>& probs, int device = 0);
  explicit BatchTrustRegionSQP(std::vector<LoweredProblem> probs, int device = 0);
  ~BatchTrustRegionSQP();
  BatchTrustRegionSQP(const BatchTrustRegionSQP&) = delete;
  BatchTrustRegionSQP& operator=(const BatchTrustRegionSQP&) = delete;

  // Run on the caller's HIP stream (hipStream_t as void*).
  void setStream(void* stream);
  // Upload, run every problem's SQP loop, download.
  std::vector<sco::OptResults> optimize();
  // optimize() in two halves: submit() uploads and queues the fused kernel on
  // the context's stream and returns; collect() waits for it and downloads.
  void submit();
  std::vector<sco::OptResults> collect();
  // submit() for another batch of the same structure and size on this context
  // (its device workspace is reused; collect() the previous batch first)
  void submit(std::vector<LoweredProblem> probs);
  // HIP-event duration of the last fused launch (ms).
  double lastKernelMs() const;
  // Per-QP records of the next optimize() (thip_debug_trace, THIP_TRACE_W doubles each).
  void enableTrace(int capacity);
  std::vector<std::vector<double>> trace() const;  // [problem][n_records * THIP_TRACE_W]
  // After a traced optimize(): problem b's solver log in the reference's
  // writeSolver format (trajopt_solver.log, optimizers.cpp:533-547) at `path`.
  // (A single problem observed through sco::BasicTrustRegionSQP -- callbacks or
  // log_results -- runs the host loop, which writes all four logs.)
  void writeSolverLog(int b, const std::string& path) const;
  int batch() const { return static_cast<int>(generic_.empty() ? probs_.size() : generic_.size()); }
  // true: the batch runs the host loops with batched QPs (see the constructor)
  bool hostLoops() const { return !generic_.empty(); }
  // host-loop batches: QP launches and QPs of the last optimize() (sco::GpuQPBatcher)
  long long qpLaunches() const { return qp_launches_; }
  long long qpSolves() const { return qp_solves_; }
  // host-loop batches: the QP solves' algorithmic HBM bytes (sco::GpuQPBatcher::bytes)
  double qpBytes() const { return qp_bytes_; }
  double qpLaunchSeconds() const { return qp_launch_s_; }
  long long qpAdmmIters() const { return qp_admm_; }
  const long long* qpMaxShape() const { return qp_shape_; }
  // host-loop batches: worker threads (problems solved at once); 0 = the
  // process default (setDefaultHostLoopWorkers, initially 64), never more
  // than the batch
  void setHostLoopWorkers(int n) { workers_ = n; }
  int hostLoopWorkers() const;
  static void setDefaultHostLoopWorkers(int n);

private:
  void init(int device);
  void check(int rc, const char* what) const;
  std::vector<sco::OptResults> optimizeHostLoops();
  std::vector<LoweredProblem> probs_;
  struct thip_ctx* ctx_ = nullptr;
  int trace_cap_ = 0;
  std::vector<TrajOptProb::Ptr> generic_;  // host-loop batch
  int device_ = 0;
  std::vector<sco::OptResults> generic_results_;
  long long qp_launches_ = 0, qp_solves_ = 0;
  double qp_bytes_ = 0, qp_launch_s_ = 0;
  long long qp_admm_ = 0, qp_shape_[6] = { 0, 0, 0, 0, 0, 0 };
  int workers_ = 0;
};

// One batch sharded over several HIP devices of this process (SURVEY.md §8e:
// the problems are independent, so there is no collective): contiguous shards
// whose sizes differ by at most one, one BatchTrustRegionSQP per device entry
// (a device may be listed more than once: several contexts on their own
// streams), every shard submitted before any is collected, so the devices run
// concurrently.  Results come back in the batch's order.
class MultiDeviceBatchSQP
{
public:
  MultiDeviceBatchSQP(const std::vector<TrajOptProb::Ptr>& probs, const std::vector<int>& devices);
  std::vector<sco::OptResults> optimize();
  // host-loop shards: QP launches and QPs of the last optimize(), summed over the shards
  long long qpLaunches() const;
  long long qpSolves() const;
  // problems per device entry (0 for an entry beyond the batch size)
  const std::vector<int>& shardSizes() const { return sizes_; }

  // A stream of batches (each sharded over `devices` as above) with `inflight`
  // batches in flight per device entry: one context per (device entry, slot)
  // on its own stream, batch j in slot j % inflight, a slot's previous batch
  // collected just before the slot is reused.  The next batch's problems take
  // the CUs the current batch's longest problems leave idle, so
  // a stream runs at the pipelined rate instead of lone-batch latency.  Every
  // batch of the stream must share batch 0's structure and size.  Results are
  // per batch, in order, bitwise those of each batch solved alone.
  static std::vector<std::vector<sco::OptResults>> optimizeStream(
      const std::vector<std::vector<TrajOptProb::Ptr>>& batches, const std::vector<int>& devices, int inflight);

private:
  std::vector<std::unique_ptr<BatchTrustRegionSQP>> shards_;
  std::vector<int> sizes_;
};

// Per-problem drop-in for the reference's optimizer usage (SURVEY.md §8b tier i):
//   BasicTrustRegionSQP opt(prob);                 optimizers.hpp:142-194
//   opt.initialize(trajToDblVec(prob->GetInitTraj()));
//   opt.optimize();                                optimizers.cpp:699-991
//   getTraj(opt.x(), ...), opt.results()           (planning_unit.cpp:83-124)
// sco::BasicTrustRegionSQP with the problem's own opt_info as the parameters
// and the HIP device of both paths (the fused kernel for a lowerable problem,
// the GpuModel's QPs otherwise).
class BasicTrustRegionSQP : public sco::BasicTrustRegionSQP
{
public:
  explicit BasicTrustRegionSQP(const TrajOptProb::Ptr& prob, int device = 0);
  // the reference's host loop whatever the problem (optimizers.cpp:699-991)
  sco::OptStatus optimizeHostLoop() { return optimizeGeneric(); }
};

// Upper bound on the per-QP trace records of one problem under param (the
// batched path's trajopt_solver.log: enableTrace(traceCapacity(param)))
int traceCapacity(const sco::BasicTrustRegionSQPParameters& param);

// trajopt/src/utils.cpp:13-24: the trajectory as one row-major vector
DblVec trajToDblVec(const std::vector<DblVec>& traj);
}  // namespace trajopt
