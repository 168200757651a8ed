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
  // Checks that every problem shares problem 0's structure (steps, chain,
  // terms, parameters, scene size) and allocates the device workspace.
  explicit BatchTrustRegionSQP(std::vector<TrajOptProb::Ptr> probs, int device = 0);
  ~BatchTrustRegionSQP();
  BatchTrustRegionSQP(const BatchTrustRegionSQP&) = delete;
  BatchTrustRegionSQP& operator=(const BatchTrustRegionSQP&) = delete;

  // Run on the caller's HIP stream (hipStream_t as void*).
  void setStream(void* stream);
  // Upload, run every problem's SQP loop, download.
  std::vector<sco::OptResults> optimize();
  // HIP-event duration of the last fused launch (ms).
  double lastKernelMs() const;
  int batch() const { return static_cast<int>(probs_.size()); }

private:
  void check(int rc, const char* what) const;
  std::vector<TrajOptProb::Ptr> probs_;
  struct thip_ctx* ctx_ = nullptr;
};
}  // namespace trajopt
