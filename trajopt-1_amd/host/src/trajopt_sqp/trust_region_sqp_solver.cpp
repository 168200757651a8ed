// trajopt_sqp::TrustRegionSQPSolver: behaviour of
// trajopt_optimizers/trajopt_sqp/src/trust_region_sqp_solver.cpp (init :44-64,
// solve :84-168, adjustPenalty :180-200, stepSQPSolver :202-260,
// runTrustRegionLoop :262-383, solveQPProblem :385-470) and types.cpp
// (toString :119-140).  The QP of every convexification is updated in place in
// the QPSolver when its dimensions are unchanged.
#include "trajopt_sqp/trust_region_sqp_solver.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>

namespace trajopt_sqp
{
namespace
{
double sum(const VectorXd& v)
{
  double s = 0;
  for (double e : v)
    s += e;
  return s;
}
double dot(const VectorXd& a, const VectorXd& b)
{
  double s = 0;
  for (std::size_t i = 0; i < a.size(); ++i)
    s += a[i] * b[i];
  return s;
}
double maxCoeff(const VectorXd& v)
{
  double m = -std::numeric_limits<double>::infinity();
  for (double e : v)
    m = std::max(m, e);
  return m;
}
}  // namespace

std::string toString(SQPStatus status)
{
  switch (status)
  {
    case SQPStatus::kRunning:
      return "SQP_RUNNING";
    case SQPStatus::kConverged:
      return "SQP_CONVERGED";
    case SQPStatus::kIterationLimit:
      return "SQP_ITERATION_LIMIT";
    case SQPStatus::kPenaltyIterationLimit:
      return "SQP_PENALTY_ITERATION_LIMIT";
    case SQPStatus::kTimeLimit:
      return "SQP_TIME_LIMIT";
    case SQPStatus::kQPSolveFailed:
      return "SQP_FAILED";
    case SQPStatus::kStoppedByCallback:
      return "SQP_STOPPED_BY_CALLBACK";
  }
  return "SQP_STATUS_UNKNOWN";
}

SQPResults::SQPResults(long num_vars, long num_cnts, long num_costs)
{
  const auto nv = static_cast<std::size_t>(num_vars), nc = static_cast<std::size_t>(num_cnts),
             nk = static_cast<std::size_t>(num_costs);
  best_var_vals.assign(nv, 0.0);
  new_var_vals.assign(nv, 0.0);
  box_size.assign(nv, 0.0);
  merit_error_coeffs.assign(nc, 0.0);
  best_constraint_violations.assign(nc, 0.0);
  new_constraint_violations.assign(nc, 0.0);
  best_approx_constraint_violations.assign(nc, 0.0);
  new_approx_constraint_violations.assign(nc, 0.0);
  best_costs.assign(nk, 0.0);
  new_costs.assign(nk, 0.0);
  best_approx_costs.assign(nk, 0.0);
  new_approx_costs.assign(nk, 0.0);
}

TrustRegionSQPSolver::TrustRegionSQPSolver(std::shared_ptr<QPSolver> solver) : qp_solver(std::move(solver)) {}

void TrustRegionSQPSolver::registerCallback(const SQPCallback::Ptr& callback) { callbacks_.push_back(callback); }
const SQPStatus& TrustRegionSQPSolver::getStatus() { return status_; }
const SQPResults& TrustRegionSQPSolver::getResults() { return results_; }

bool TrustRegionSQPSolver::init(QPProblem::Ptr qp_prob)
{
  qp_problem = std::move(qp_prob);
  results_ = SQPResults(qp_problem->getNumNLPVars(), qp_problem->getNumNLPConstraints(), qp_problem->getNumNLPCosts());
  results_.best_var_vals = qp_problem->getVariableValues();
  results_.merit_error_coeffs.assign(static_cast<std::size_t>(qp_problem->getNumNLPConstraints()),
                                     params.initial_merit_error_coeff);
  // the exact (expensive) evaluations at the start point
  results_.best_costs = qp_problem->getExactCosts();
  results_.best_constraint_violations = qp_problem->getExactConstraintViolations();
  setBoxSize(params.initial_trust_box_size);
  constraintMeritCoeffChanged();
  return true;
}

void TrustRegionSQPSolver::setBoxSize(double box_size)
{
  qp_problem->setBoxSize(VectorXd(static_cast<std::size_t>(qp_problem->getNumNLPVars()), box_size));
  results_.box_size = qp_problem->getBoxSize();
}

void TrustRegionSQPSolver::constraintMeritCoeffChanged()
{
  qp_problem->setConstraintMeritCoeff(results_.merit_error_coeffs);
  // the best merit under the new coefficients
  results_.best_exact_merit =
      sum(results_.best_costs) + dot(results_.best_constraint_violations, results_.merit_error_coeffs);
}

void TrustRegionSQPSolver::solve(const QPProblem::Ptr& qp_prob)
{
  status_ = SQPStatus::kRunning;
  using Clock = std::chrono::steady_clock;
  const auto start = Clock::now();
  init(qp_prob);
  for (int penalty_iteration = 0; penalty_iteration < params.max_merit_coeff_increases; ++penalty_iteration)
  {
    results_.penalty_iteration = penalty_iteration;
    results_.convexify_iteration = 0;
    for (int convex_iteration = 1; convex_iteration < 100; ++convex_iteration)
    {
      const double elapsed = std::chrono::duration<double, std::milli>(Clock::now() - start).count() / 1000.0;
      if (elapsed > params.max_time)
      {
        status_ = SQPStatus::kTimeLimit;
        break;
      }
      if (results_.overall_iteration >= params.max_iterations)
      {
        status_ = SQPStatus::kIterationLimit;
        break;
      }
      if (stepSQPSolver())
        break;
    }
    if (verifySQPSolverConvergence())
    {
      status_ = SQPStatus::kConverged;
      break;
    }
    if (status_ == SQPStatus::kIterationLimit || status_ == SQPStatus::kTimeLimit)
      break;
    status_ = SQPStatus::kRunning;
    adjustPenalty();  // constraints not yet satisfied
  }
  if (status_ == SQPStatus::kRunning)
    status_ = SQPStatus::kPenaltyIterationLimit;
  qp_problem->setVariables(results_.best_var_vals.data());
}

bool TrustRegionSQPSolver::verifySQPSolverConvergence()
{
  if (results_.best_constraint_violations.empty())
    return true;
  return maxCoeff(results_.best_constraint_violations) < params.cnt_tolerance;
}

void TrustRegionSQPSolver::adjustPenalty()
{
  if (params.inflate_constraints_individually)
  {
    for (std::size_t i = 0; i < results_.best_constraint_violations.size(); ++i)
      if (results_.best_constraint_violations[i] > params.cnt_tolerance)
        results_.merit_error_coeffs[i] *= params.merit_coeff_increase_ratio;
  }
  else
    for (double& c : results_.merit_error_coeffs)
      c *= params.merit_coeff_increase_ratio;
  setBoxSize(std::fmax(results_.box_size[0], params.min_trust_box_size / params.trust_shrink_ratio * 1.5));
  constraintMeritCoeffChanged();
}

bool TrustRegionSQPSolver::stepSQPSolver()
{
  ++results_.convexify_iteration;
  const long prev_nv = qp_problem->getNumQPVars(), prev_nc = qp_problem->getNumQPConstraints();
  qp_problem->convexify();
  const long nv = qp_problem->getNumQPVars(), nc = qp_problem->getNumQPConstraints();
  auto rebuild = [&]() {
    qp_solver->clear();
    qp_solver->init(nv, nc);
    qp_solver->updateHessianMatrix(qp_problem->getHessian());
    qp_solver->updateGradient(qp_problem->getGradient());
    qp_solver->updateLinearConstraintsMatrix(qp_problem->getConstraintMatrix());
    qp_solver->updateBounds(qp_problem->getBoundsLower(), qp_problem->getBoundsUpper());
    qp_solver->setWarmStart(*qp_problem);
  };
  if (qp_solver->getSolverStatus() == QPSolverStatus::kUninitialized || nv != prev_nv || nc != prev_nc)
    rebuild();
  else if (!qp_solver->updateHessianMatrix(qp_problem->getHessian()) ||
           !qp_solver->updateGradient(qp_problem->getGradient()) ||
           !qp_solver->updateLinearConstraintsMatrix(qp_problem->getConstraintMatrix()) ||
           !qp_solver->updateBounds(qp_problem->getBoundsLower(), qp_problem->getBoundsUpper()))
    rebuild();  // the in-place update was refused
  runTrustRegionLoop();
  if (status_ == SQPStatus::kConverged)
    return true;
  if (maxCoeff(results_.box_size) < params.min_trust_box_size)
  {
    status_ = SQPStatus::kConverged;  // the trust region is tiny
    return true;
  }
  return false;
}

void TrustRegionSQPSolver::runTrustRegionLoop()
{
  results_.trust_region_iteration = 0;
  int failures = 0;
  auto pushBox = [&]() {
    qp_solver->updateBounds(qp_problem->getBoundsLower(), qp_problem->getBoundsUpper());
    results_.box_size = qp_problem->getBoxSize();
  };
  while (maxCoeff(results_.box_size) >= params.min_trust_box_size)
  {
    ++results_.overall_iteration;
    ++results_.trust_region_iteration;
    status_ = solveQPProblem();
    if (status_ == SQPStatus::kStoppedByCallback)
      return;
    if (status_ != SQPStatus::kRunning)
    {
      ++failures;
      if (failures < params.max_qp_solver_failures)
      {
        double s = params.trust_shrink_ratio;
        qp_problem->scaleBoxSize(s);
        pushBox();
        continue;
      }
      if (failures == params.max_qp_solver_failures)
      {
        // the last attempt: the smallest trust region
        qp_problem->setBoxSize(VectorXd(static_cast<std::size_t>(qp_problem->getNumNLPVars()), params.min_trust_box_size));
        pushBox();
        continue;
      }
      return;  // the QP solver failed too many times
    }
    if (results_.approx_merit_improve < -1e-5 && verbose)
      std::printf("Approximate merit function got worse (%.3e)\n", results_.approx_merit_improve);
    if (results_.approx_merit_improve < params.min_approx_improve)
    {
      status_ = SQPStatus::kConverged;
      return;
    }
    const double denom = std::max(std::abs(results_.best_exact_merit), 1e-12);
    if (results_.approx_merit_improve / denom < params.min_approx_improve_frac)
    {
      status_ = SQPStatus::kConverged;
      return;
    }
    if (results_.exact_merit_improve < 0 || results_.merit_improve_ratio < params.improve_ratio_threshold)
    {
      double s = params.trust_shrink_ratio;
      qp_problem->scaleBoxSize(s);
      pushBox();
    }
    else
    {
      // accept the step and grow the trust region
      results_.best_var_vals = results_.new_var_vals;
      results_.best_exact_merit = results_.new_exact_merit;
      results_.best_constraint_violations = results_.new_constraint_violations;
      results_.best_costs = results_.new_costs;
      results_.best_approx_merit = results_.new_approx_merit;
      results_.best_approx_constraint_violations = results_.new_approx_constraint_violations;
      results_.best_approx_costs = results_.new_approx_costs;
      qp_problem->setVariables(results_.best_var_vals.data());
      double s = params.trust_expand_ratio;
      qp_problem->scaleBoxSize(s);
      pushBox();
      return;
    }
  }
}

SQPStatus TrustRegionSQPSolver::solveQPProblem()
{
  if (!qp_solver->solve())
  {
    qp_problem->setVariables(results_.best_var_vals.data());
    return SQPStatus::kQPSolveFailed;
  }
  results_.new_var_vals = qp_solver->getSolution();
  qp_problem->setVariables(results_.new_var_vals.data());
  // model (convexified) merit at the QP solution
  results_.new_approx_constraint_violations = qp_problem->evaluateConvexConstraintViolations(results_.new_var_vals);
  results_.new_approx_costs = qp_problem->evaluateConvexCosts(results_.new_var_vals);
  results_.new_approx_merit =
      sum(results_.new_approx_costs) + dot(results_.new_approx_constraint_violations, results_.merit_error_coeffs);
  results_.approx_merit_improve = results_.best_exact_merit - results_.new_approx_merit;
  // exact merit at the QP solution
  results_.new_costs = qp_problem->getExactCosts();
  results_.new_constraint_violations = qp_problem->getExactConstraintViolations();
  results_.new_exact_merit =
      sum(results_.new_costs) + dot(results_.new_constraint_violations, results_.merit_error_coeffs);
  results_.exact_merit_improve = results_.best_exact_merit - results_.new_exact_merit;
  results_.merit_improve_ratio = (std::abs(results_.approx_merit_improve) < 1e-12) ?
                                     0.0 :
                                     results_.exact_merit_improve / results_.approx_merit_improve;
  // the problem stays at the best point until the step is accepted
  qp_problem->setVariables(results_.best_var_vals.data());
  if (verbose)
    printStepInfo();
  if (!callCallbacks())
    return SQPStatus::kStoppedByCallback;
  return SQPStatus::kRunning;
}

bool TrustRegionSQPSolver::callCallbacks()
{
  bool ok = true;
  for (const auto& cb : callbacks_)
    ok &= cb->execute(*qp_problem, results_);
  return ok;
}

void TrustRegionSQPSolver::printStepInfo() const
{
  std::printf("| overall %d | convexify %d | trust region %d | penalty %d | box %.6f |\n", results_.overall_iteration,
              results_.convexify_iteration, results_.trust_region_iteration, results_.penalty_iteration,
              results_.box_size.empty() ? 0.0 : results_.box_size[0]);
  std::printf("| merit %.6e -> exact %.6e, approx %.6e | improve exact %.3e approx %.3e ratio %.3e |\n",
              results_.best_exact_merit, results_.new_exact_merit, results_.new_approx_merit,
              results_.exact_merit_improve, results_.approx_merit_improve, results_.merit_improve_ratio);
}
}  // namespace trajopt_sqp
