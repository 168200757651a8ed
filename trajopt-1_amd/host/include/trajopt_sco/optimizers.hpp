// sco::Optimizer / BasicTrustRegionSQP (trajopt_sco/include/trajopt_sco/
// optimizers.hpp:63-219) over the MI355X build.
//
// optimize() first offers the problem to its native batched path
// (OptProb::solveNative: a TrajOptProb whose terms all lowered runs the fused
// sqp_kernel as a batch of one); otherwise it runs the reference's loop
// (optimizers.cpp:699-991) on the host over getCosts() / getConstraints(), every
// convex subproblem solved on the GPU by the problem's Model (GpuModel):
// penalty loop, SQP loop with the time limit (max_time), convexify,
// cntsToCosts, the trust-region loop with the QP-failure policy and the
// /tmp/fail.lp dump, BasicTrustRegionSQPResults::update, the four CSV logs
// (log_results), penalty adjustment, callbacks.
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "trajopt_sco/modeling.hpp"
#include "trajopt_sco/optimizers_fwd.hpp"

namespace sco
{
class Optimizer
{
public:
  using Ptr = std::shared_ptr<Optimizer>;
  using Callback = std::function<void(OptProb*, OptResults&)>;
  Optimizer() = default;
  virtual ~Optimizer() = default;
  virtual OptStatus optimize() = 0;
  virtual void setProblem(OptProb::Ptr prob) { prob_ = std::move(prob); }
  void initialize(const DblVec& x);
  DblVec& x() { return results_.x; }
  OptResults& results() { return results_; }
  void addCallback(const Callback& cb);

protected:
  std::vector<Callback> callbacks_;
  void callCallbacks();
  OptProb::Ptr prob_;
  OptResults results_;
};

class BasicTrustRegionSQP : public Optimizer
{
public:
  using Ptr = std::shared_ptr<BasicTrustRegionSQP>;
  BasicTrustRegionSQP() = default;
  explicit BasicTrustRegionSQP(const OptProb::Ptr& prob);
  void setProblem(OptProb::Ptr prob) override;
  OptStatus optimize() override;

  void setParameters(const BasicTrustRegionSQPParameters& param) { param_ = param; }
  const BasicTrustRegionSQPParameters& getParameters() const { return param_; }
  BasicTrustRegionSQPParameters& getParameters() { return param_; }

  virtual DblVec evaluateCosts(const std::vector<Cost::Ptr>& costs, const DblVec& x) const;
  virtual DblVec evaluateConstraintViols(const std::vector<Constraint::Ptr>& cnts, const DblVec& x) const;
  virtual std::vector<ConvexObjective::Ptr> convexifyCosts(const std::vector<Cost::Ptr>& costs, const DblVec& x,
                                                           Model* model) const;
  virtual std::vector<ConvexConstraints::Ptr> convexifyConstraints(const std::vector<Constraint::Ptr>& cnts,
                                                                   const DblVec& x, Model* model) const;
  virtual DblVec evaluateModelCosts(const std::vector<ConvexObjective::Ptr>& costs, const DblVec& x) const;
  virtual DblVec evaluateModelCntViols(const std::vector<ConvexConstraints::Ptr>& cnts, const DblVec& x) const;
  virtual std::vector<std::string> getCostNames(const std::vector<Cost::Ptr>& costs) const;
  virtual std::vector<std::string> getCntNames(const std::vector<Constraint::Ptr>& cnts) const;
  virtual std::vector<std::string> getVarNames(const VarVector& vars) const;

protected:
  void ctor(const OptProb::Ptr& prob);
  void adjustTrustRegion(double ratio) { param_.trust_box_size *= ratio; }
  void setTrustRegionSize(double size) { param_.trust_box_size = size; }
  void setTrustBoxConstraints(const DblVec& x);
  OptStatus optimizeGeneric();

  Model::Ptr model_;
  BasicTrustRegionSQPParameters param_;
};

// optimizers.hpp:196-219: convexification over OpenMP threads in the
// reference; here the terms of the native path already run in parallel on the
// device and the generic path convexifies serially (same results).
class BasicTrustRegionSQPMultiThreaded : public BasicTrustRegionSQP
{
public:
  using Ptr = std::shared_ptr<BasicTrustRegionSQPMultiThreaded>;
  using BasicTrustRegionSQP::BasicTrustRegionSQP;
};

// optimizers.cpp:59-81: constraint models become costs with merit coefficients
std::vector<ConvexObjective::Ptr> cntsToCosts(const std::vector<ConvexConstraints::Ptr>& cnts, const DblVec& err_coeffs,
                                              Model* model);
}  // namespace sco
