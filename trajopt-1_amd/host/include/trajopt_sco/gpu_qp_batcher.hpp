// GpuQPBatcher: the convex subproblems of many host SQP loops (one
// sco::BasicTrustRegionSQP per problem, each on its own host thread) solved in
// one GPU launch per sparsity pattern.  The reference solves each problem's
// QPs one at a time (OSQPModel::optimize, trajopt_sco/src/osqp_interface.cpp:
// 283-615); here every GpuModel attached to a batcher hands its QP to
// solve(), which blocks, and the call that completes the round -- every
// running client waiting -- launches all pending QPs, grouped by (device,
// sizes, P / A pattern, settings), through thip_qp_solve_some (one workgroup
// per QP; each QP keeps its own warm start and rho).  A QP's result does not
// depend on what it is grouped with.  Clients are counted by enter() / leave()
// (one per problem thread).
#pragma once
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "trajopt_hip.h"

namespace sco
{
class GpuQPBatcher
{
public:
  using Ptr = std::shared_ptr<GpuQPBatcher>;
  GpuQPBatcher() = default;
  ~GpuQPBatcher();
  GpuQPBatcher(const GpuQPBatcher&) = delete;
  GpuQPBatcher& operator=(const GpuQPBatcher&) = delete;

  // one QP: upper-triangular CSC P (n x n), CSC A (m x n), OSQP settings
  struct Request
  {
    int device = 0, n = 0, m = 0;
    const std::vector<int>*Pp = nullptr, *Pi = nullptr, *Ap = nullptr, *Ai = nullptr;
    const std::vector<double>*Px = nullptr, *Ax = nullptr, *q = nullptr, *l = nullptr, *u = nullptr;
    thip_osqp_settings settings{};
    bool warm = false;  // warm start from wx / wy with rho = settings.rho (the previous rho)
    const std::vector<double>*wx = nullptr, *wy = nullptr;
    std::vector<double>*x = nullptr, *y = nullptr;  // out: n, m
    thip_qp_info* info = nullptr;                     // out
    // internal
    bool done = false;
    std::string error;
  };

  void enter();
  void leave();
  // blocks until r is solved; throws std::runtime_error on a device failure
  void solve(Request& r);

  // launches and QPs so far (diagnostics)
  long long launches() const { return launches_; }
  long long qps() const { return qps_; }
  // algorithmic HBM bytes of the solves so far (the bench's roofline model of
  // qp_csc.hip, per QP: each ADMM iteration streams the factor L twice -- the
  // forward and backward solves, value and index -- plus D, A x and A'y, P x
  // and the iterate vectors; each factorisation reads the KKT values and writes
  // L; polish adds one factorisation and 1 + polish_refine_iter solves).  A
  // pattern staged in LDS (thip_qp_shape out[4]) keeps L out of HBM: its
  // factor and solve terms count only the vectors
  double bytes() const { return bytes_; }
  long long admmIters() const { return admm_iters_; }
  // wall seconds of the rounds on the device: first submission to last collection
  // (the launches of a round run concurrently, each pattern on its own stream)
  double launchSeconds() const { return launch_s_; }
  // the largest KKT seen: N, entries of L, elimination-tree levels, widest level
  const long long* maxShape() const { return shape_; }

private:
  void flushLocked();
  std::mutex mu_;
  std::condition_variable cv_;
  int active_ = 0;
  std::vector<Request*> pending_;
  struct Slot
  {
    thip_qp* qp = nullptr;
    int capacity = 0;
    long long last_round = 0;
  };
  std::map<std::string, Slot> cache_;
  long long round_ = 0, launches_ = 0, qps_ = 0, admm_iters_ = 0;
  double bytes_ = 0, launch_s_ = 0;
  long long shape_[6] = { 0, 0, 0, 0, 0, 0 };
};

// RAII: a client of the batcher for its lifetime
class GpuQPBatcherClient
{
public:
  explicit GpuQPBatcherClient(GpuQPBatcher::Ptr b) : b_(std::move(b))
  {
    if (b_)
      b_->enter();
  }
  ~GpuQPBatcherClient()
  {
    if (b_)
      b_->leave();
  }
  GpuQPBatcherClient(const GpuQPBatcherClient&) = delete;
  GpuQPBatcherClient& operator=(const GpuQPBatcherClient&) = delete;

private:
  GpuQPBatcher::Ptr b_;
};
}  // namespace sco
