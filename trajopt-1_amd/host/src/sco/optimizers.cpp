// BasicTrustRegionSQP over the MI355X build (optimizers.hpp): the native
// batched path when the problem has one, else the reference's loop
// (trajopt_sco/src/optimizers.cpp:699-991) on the host with the GpuModel.
#include "trajopt_sco/optimizers.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"
#include "trajopt_sco/gpu_model.hpp"

namespace sco
{
std::string toString(OptStatus status)
{
  static const char* names[] = { "OPT_CONVERGED",  "OPT_SCO_ITERATION_LIMIT", "OPT_PENALTY_ITERATION_LIMIT",
                                 "OPT_TIME_LIMIT", "OPT_FAILED",              "INVALID" };
  const int k = static_cast<int>(status);
  return (k >= 0 && k <= 5) ? names[k] : "INVALID";
}

std::vector<ConvexObjective::Ptr> cntsToCosts(const std::vector<ConvexConstraints::Ptr>& cnts, const DblVec& err_coeffs,
                                              Model* model)
{
  std::vector<ConvexObjective::Ptr> out;
  out.reserve(cnts.size());
  for (std::size_t c = 0; c < cnts.size(); ++c)
  {
    auto obj = std::make_shared<ConvexObjective>(model);
    for (const AffExpr& aff : cnts[c]->eqs_)
      obj->addAbs(aff, err_coeffs[c]);
    for (const AffExpr& aff : cnts[c]->ineqs_)
      obj->addHinge(aff, err_coeffs[c]);
    out.push_back(obj);
  }
  return out;
}

// ------------------------------------------------------------------ Optimizer
void Optimizer::initialize(const DblVec& x)
{
  if (!prob_)
    throw std::runtime_error("need to set the problem before initializing");
  if (prob_->getVars().size() != x.size())
    throw std::runtime_error("initialization vector has wrong length. expected " +
                             std::to_string(prob_->getVars().size()) + " got " + std::to_string(x.size()));
  results_.clear();
  results_.x = x;
}
void Optimizer::addCallback(const Callback& cb) { callbacks_.push_back(cb); }
void Optimizer::callCallbacks()
{
  for (auto& cb : callbacks_)
    cb(prob_.get(), results_);
}

// ------------------------------------------------------------------ BasicTrustRegionSQP
BasicTrustRegionSQP::BasicTrustRegionSQP(const OptProb::Ptr& prob) { ctor(prob); }
void BasicTrustRegionSQP::setProblem(OptProb::Ptr prob) { ctor(prob); }
void BasicTrustRegionSQP::ctor(const OptProb::Ptr& prob)
{
  Optimizer::setProblem(prob);
  model_ = prob->getModel();
}

void BasicTrustRegionSQP::setTrustBoxConstraints(const DblVec& x)
{
  // optimizers.cpp:151-170 (quirk Q6: x clamped into [lb, ub] first)
  const VarVector& vars = prob_->getVars();
  const DblVec& lb = prob_->getLowerBounds();
  const DblVec& ub = prob_->getUpperBounds();
  DblVec lo(x.size()), hi(x.size());
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    const double xi = std::min(std::max(x[i], lb[i]), ub[i]);
    lo[i] = std::max(xi - param_.trust_box_size, lb[i]);
    hi[i] = std::min(xi + param_.trust_box_size, ub[i]);
  }
  model_->setVarBounds(vars, lo, hi);
}

DblVec BasicTrustRegionSQP::evaluateCosts(const std::vector<Cost::Ptr>& costs, const DblVec& x) const
{
  prob_->prefetch(x);
  DblVec out(costs.size());
  for (std::size_t i = 0; i < costs.size(); ++i)
    out[i] = costs[i]->value(x);
  return out;
}
DblVec BasicTrustRegionSQP::evaluateConstraintViols(const std::vector<Constraint::Ptr>& cnts, const DblVec& x) const
{
  prob_->prefetch(x);
  DblVec out(cnts.size());
  for (std::size_t i = 0; i < cnts.size(); ++i)
    out[i] = cnts[i]->violation(x);
  return out;
}
std::vector<ConvexObjective::Ptr> BasicTrustRegionSQP::convexifyCosts(const std::vector<Cost::Ptr>& costs,
                                                                      const DblVec& x, Model* model) const
{
  prob_->prefetch(x);
  std::vector<ConvexObjective::Ptr> out(costs.size());
  for (std::size_t i = 0; i < costs.size(); ++i)
    out[i] = costs[i]->convex(x, model);
  return out;
}
std::vector<ConvexConstraints::Ptr> BasicTrustRegionSQP::convexifyConstraints(const std::vector<Constraint::Ptr>& cnts,
                                                                              const DblVec& x, Model* model) const
{
  prob_->prefetch(x);
  std::vector<ConvexConstraints::Ptr> out(cnts.size());
  for (std::size_t i = 0; i < cnts.size(); ++i)
    out[i] = cnts[i]->convex(x, model);
  return out;
}
DblVec BasicTrustRegionSQP::evaluateModelCosts(const std::vector<ConvexObjective::Ptr>& costs, const DblVec& x) const
{
  DblVec out(costs.size());
  for (std::size_t i = 0; i < costs.size(); ++i)
    out[i] = costs[i]->value(x);
  return out;
}
DblVec BasicTrustRegionSQP::evaluateModelCntViols(const std::vector<ConvexConstraints::Ptr>& cnts,
                                                  const DblVec& x) const
{
  DblVec out(cnts.size());
  for (std::size_t i = 0; i < cnts.size(); ++i)
    out[i] = cnts[i]->violation(x);
  return out;
}
std::vector<std::string> BasicTrustRegionSQP::getCostNames(const std::vector<Cost::Ptr>& costs) const
{
  std::vector<std::string> out;
  for (const auto& c : costs)
    out.push_back(c->name());
  return out;
}
std::vector<std::string> BasicTrustRegionSQP::getCntNames(const std::vector<Constraint::Ptr>& cnts) const
{
  std::vector<std::string> out;
  for (const auto& c : cnts)
    out.push_back(c->name());
  return out;
}
std::vector<std::string> BasicTrustRegionSQP::getVarNames(const VarVector& vars) const
{
  std::vector<std::string> out;
  for (const auto& v : vars)
    out.push_back(v.var_rep->name);
  return out;
}

OptStatus BasicTrustRegionSQP::optimize()
{
  if (results_.x.empty())
    throw std::runtime_error("you forgot to initialize!");
  if (!prob_)
    throw std::runtime_error("you forgot to set the optimization problem");
  // The batched kernel runs the whole loop on the device.  A caller that observes
  // the iterations -- callbacks at every SQP iteration (optimizers.cpp:754), the
  // four CSV logs (:533-647, 858-871) -- gets the reference's host loop instead, over
  // the same terms (the kinematic ones evaluated on the device), so the observed
  // behaviour is the reference's whichever path solves the problem.
  OptResults native;
  if (callbacks_.empty() && !param_.log_results && prob_->solveNative(param_, results_.x, native))
  {
    results_ = native;
    return results_.status;
  }
  return optimizeGeneric();
}

namespace
{
// BasicTrustRegionSQPResults (optimizers.hpp:221-319, optimizers.cpp:380-647):
// one trust-region step's model / exact values and the four CSV log lines
struct StepResults
{
  std::vector<std::string> var_names, cost_names, cnt_names;
  DblVec model_var_vals, model_cost_vals, model_cnt_viols, new_x, old_cost_vals, old_cnt_viols, new_cost_vals,
      new_cnt_viols, merit_error_coeffs;
  double old_merit = 0, model_merit = 0, new_merit = 0, approx_merit_improve = 0, exact_merit_improve = 0,
         merit_improve_ratio = 0;

  void writeSolver(std::FILE* f, bool header) const
  {
    if (header)
      std::fprintf(f, "%s,%s,%s,%s,%s,%s\n", "DESCRIPTION", "oldexact", "new_exact", "dapprox", "dexact", "ratio");
    std::fprintf(f, "%s,%10.3e,%10.3e,%10.3e,%10.3e,%10.3e\n", "Solver", old_merit, new_merit, approx_merit_improve,
                 exact_merit_improve, merit_improve_ratio);
    std::fflush(f);
  }
  void writeVars(std::FILE* f, bool header) const
  {
    if (header)
    {
      std::fprintf(f, "%s", "NAMES");
      for (const auto& v : var_names)
        std::fprintf(f, ",%s", v.c_str());
      std::fprintf(f, "\n");
    }
    std::fprintf(f, "%s", "VALUES");
    for (double v : new_x)
      std::fprintf(f, ",%e", v);
    std::fprintf(f, "\n");
    std::fflush(f);
  }
  static void writeTerms(std::FILE* f, bool header, const char* title, const char* row,
                         const std::vector<std::string>& names, const DblVec& olds, const DblVec& models,
                         const DblVec& news, const DblVec* scale)
  {
    if (header)
    {
      std::fprintf(f, "%s", title);
      for (const auto& n : names)
        std::fprintf(f, ",%s,%s,%s,%s", n.c_str(), n.c_str(), n.c_str(), n.c_str());
      std::fprintf(f, "\n%s", "DESCRIPTION");
      for (std::size_t i = 0; i < names.size(); ++i)
        std::fprintf(f, ",%s,%s,%s,%s", "oldexact", "dapprox", "dexact", "ratio");
      std::fprintf(f, "\n");
    }
    std::fprintf(f, "%s", row);
    for (std::size_t i = 0; i < olds.size(); ++i)
    {
      const double s = scale ? (*scale)[i] : 1.0;
      const double approx = olds[i] - models[i], exact = olds[i] - news[i];
      if (std::fabs(approx) > 1e-8)
        std::fprintf(f, ",%e,%e,%e,%e", s * olds[i], s * approx, s * exact, exact / approx);
      else
        std::fprintf(f, ",%e,%e,%e,%s", s * olds[i], s * approx, s * exact, "nan");
    }
    std::fprintf(f, "\n");
    std::fflush(f);
  }
};
}  // namespace

OptStatus BasicTrustRegionSQP::optimizeGeneric()
{
  StepResults it;
  it.var_names = getVarNames(prob_->getVars());
  it.cost_names = getCostNames(prob_->getCosts());
  const std::vector<Constraint::Ptr> constraints = prob_->getConstraints();
  it.cnt_names = getCntNames(constraints);
  DblVec merit_error_coeffs(constraints.size(), param_.initial_merit_error_coeff);
  std::FILE *log_solver = nullptr, *log_vars = nullptr, *log_costs = nullptr, *log_cnts = nullptr;
  if (param_.log_results)
  {
    log_solver = std::fopen((param_.log_dir + "/trajopt_solver.log").c_str(), "w");
    log_vars = std::fopen((param_.log_dir + "/trajopt_vars.log").c_str(), "w");
    log_costs = std::fopen((param_.log_dir + "/trajopt_costs.log").c_str(), "w");
    log_cnts = std::fopen((param_.log_dir + "/trajopt_constraints.log").c_str(), "w");
  }
  results_.x = prob_->getClosestFeasiblePoint(results_.x);
  OptStatus retval = INVALID;
  const auto start_time = std::chrono::high_resolution_clock::now();
  auto max_viol = [&]() { return results_.cnt_viols.empty() ? -HUGE_VAL : vecMax(results_.cnt_viols); };

  for (int merit_increases = 0; merit_increases < param_.max_merit_coeff_increases; ++merit_increases)
  {
    bool to_penalty = false;
    for (int iter = 1;; ++iter)
    {
      const double elapsed =
          std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - start_time).count() /
          1000.0;
      if (elapsed > param_.max_time)
      {
        retval = OPT_TIME_LIMIT;
        if (results_.cnt_viols.empty() || max_viol() < param_.cnt_tolerance)
          retval = OPT_CONVERGED;
        goto cleanup;
      }
      callCallbacks();
      ++results_.n_sqp_iters;
      if (results_.cost_vals.empty() && results_.cnt_viols.empty())
      {
        results_.cnt_viols = evaluateConstraintViols(constraints, results_.x);
        results_.cost_vals = evaluateCosts(prob_->getCosts(), results_.x);
        ++results_.n_func_evals;
      }
      {
        const std::vector<ConvexObjective::Ptr> cost_models = convexifyCosts(prob_->getCosts(), results_.x, model_.get());
        const std::vector<ConvexConstraints::Ptr> cnt_models = convexifyConstraints(constraints, results_.x, model_.get());
        const std::vector<ConvexObjective::Ptr> cnt_cost_models = cntsToCosts(cnt_models, merit_error_coeffs, model_.get());
        model_->update();
        for (const auto& c : cost_models)
          c->addConstraintsToModel();
        for (const auto& c : cnt_cost_models)
          c->addConstraintsToModel();
        model_->update();
        QuadExpr objective;
        for (const auto& c : cost_models)
          exprInc(objective, c->quad_);
        for (const auto& c : cnt_cost_models)
          exprInc(objective, c->quad_);
        model_->setObjective(objective);

        int qp_solver_failures = 0;
        while (param_.trust_box_size >= param_.min_trust_box_size)
        {
          setTrustBoxConstraints(results_.x);
          const CvxOptStatus status = model_->optimize();
          ++results_.n_qp_solves;
          if (status != CVX_SOLVED)
          {
            model_->writeToFile("/tmp/fail.lp");  // optimizers.cpp:821-822
            if (qp_solver_failures < (param_.max_qp_solver_failures - 1))
            {
              adjustTrustRegion(param_.trust_shrink_ratio);
              ++qp_solver_failures;
              continue;
            }
            if (qp_solver_failures == (param_.max_qp_solver_failures - 1))
            {
              setTrustRegionSize(param_.min_trust_box_size);
              ++qp_solver_failures;
              continue;
            }
            retval = OPT_FAILED;
            goto cleanup;
          }
          // BasicTrustRegionSQPResults::update (optimizers.cpp:380-426)
          it.merit_error_coeffs = merit_error_coeffs;
          it.model_var_vals = model_->getVarValues(model_->getVars());
          it.model_cost_vals = evaluateModelCosts(cost_models, it.model_var_vals);
          it.model_cnt_viols = evaluateModelCntViols(cnt_models, it.model_var_vals);
          it.new_x = DblVec(it.model_var_vals.begin(), it.model_var_vals.begin() + static_cast<long>(results_.x.size()));
          it.old_cost_vals = results_.cost_vals;
          it.old_cnt_viols = results_.cnt_viols;
          it.new_cost_vals = evaluateCosts(prob_->getCosts(), it.new_x);
          it.new_cnt_viols = evaluateConstraintViols(constraints, it.new_x);
          it.old_merit = vecSum(it.old_cost_vals) + vecDot(it.old_cnt_viols, merit_error_coeffs);
          it.model_merit = vecSum(it.model_cost_vals) + vecDot(it.model_cnt_viols, merit_error_coeffs);
          it.new_merit = vecSum(it.new_cost_vals) + vecDot(it.new_cnt_viols, merit_error_coeffs);
          it.approx_merit_improve = it.old_merit - it.model_merit;
          it.exact_merit_improve = it.old_merit - it.new_merit;
          it.merit_improve_ratio = it.exact_merit_improve / it.approx_merit_improve;
          if (param_.log_results)
          {
            const bool header = results_.n_func_evals == 1;
            if (log_solver)
              it.writeSolver(log_solver, header);
            if (log_vars)
              it.writeVars(log_vars, header);
            if (log_costs)
              StepResults::writeTerms(log_costs, header, "COST NAMES", "COSTS", it.cost_names, it.old_cost_vals,
                                      it.model_cost_vals, it.new_cost_vals, nullptr);
            if (log_cnts)
              StepResults::writeTerms(log_cnts, header, "CONSTRAINT NAMES", "CONSTRAINTS", it.cnt_names,
                                      it.old_cnt_viols, it.model_cnt_viols, it.new_cnt_viols, &it.merit_error_coeffs);
          }
          ++results_.n_func_evals;
          if (it.approx_merit_improve < param_.min_approx_improve)
          {
            retval = OPT_CONVERGED;
            to_penalty = true;
            break;
          }
          if (it.approx_merit_improve / it.old_merit < param_.min_approx_improve_frac)
          {
            retval = OPT_CONVERGED;
            to_penalty = true;
            break;
          }
          if (it.exact_merit_improve < 0 || it.merit_improve_ratio < param_.improve_ratio_threshold)
            adjustTrustRegion(param_.trust_shrink_ratio);
          else
          {
            results_.x = it.new_x;
            results_.cost_vals = it.new_cost_vals;
            results_.cnt_viols = it.new_cnt_viols;
            adjustTrustRegion(param_.trust_expand_ratio);
            break;
          }
        }
      }  // the convex models leave the Model here
      if (to_penalty)
        break;
      if (param_.trust_box_size < param_.min_trust_box_size)
      {
        retval = OPT_CONVERGED;
        break;
      }
      if (iter >= param_.max_iter)
      {
        retval = OPT_SCO_ITERATION_LIMIT;
        if (results_.cnt_viols.empty() || max_viol() < param_.cnt_tolerance)
          retval = OPT_CONVERGED;
        goto cleanup;
      }
    }
    // penalty adjustment (optimizers.cpp:938-968)
    if (results_.cnt_viols.empty() || max_viol() < param_.cnt_tolerance)
      goto cleanup;
    for (std::size_t i = 0; i < merit_error_coeffs.size(); ++i)
      if (!param_.inflate_constraints_individually || results_.cnt_viols[i] > param_.cnt_tolerance)
        merit_error_coeffs[i] *= param_.merit_coeff_increase_ratio;
    param_.trust_box_size = std::fmax(param_.trust_box_size, param_.min_trust_box_size / param_.trust_shrink_ratio * 1.5);
  }
  retval = OPT_PENALTY_ITERATION_LIMIT;

cleanup:
  results_.status = retval;
  results_.total_cost = vecSum(results_.cost_vals);
  results_.max_cnt_viol = results_.cnt_viols.empty() ? 0.0 : vecMax(results_.cnt_viols);
  if (const auto* gm = dynamic_cast<const GpuModel*>(model_.get()))
    results_.n_admm_iters = gm->admmItersTotal();
  callCallbacks();
  for (std::FILE* f : { log_solver, log_vars, log_costs, log_cnts })
    if (f)
      std::fclose(f);
  return retval;
}
}  // namespace sco
