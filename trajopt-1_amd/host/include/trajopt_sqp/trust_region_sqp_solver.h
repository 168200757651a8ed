// trajopt_sqp::TrustRegionSQPSolver (src/trust_region_sqp_solver.cpp): penalty
// loop -> convexification loop -> trust-region loop over one QPProblem, the QP
// updated in place between convexifications (stepSQPSolver).
#pragma once
#include <memory>
#include <vector>

#include "trajopt_sqp/qp_problem.h"
#include "trajopt_sqp/qp_solver.h"
#include "trajopt_sqp/sqp_callback.h"
#include "trajopt_sqp/types.h"

namespace trajopt_sqp
{
class TrustRegionSQPSolver
{
public:
  explicit TrustRegionSQPSolver(std::shared_ptr<QPSolver> qp_solver);
  bool init(QPProblem::Ptr qp_prob);
  void solve(const QPProblem::Ptr& qp_prob);
  bool stepSQPSolver();
  bool verifySQPSolverConvergence();
  void adjustPenalty();
  void runTrustRegionLoop();
  SQPStatus solveQPProblem();
  bool callCallbacks();
  void printStepInfo() const;
  void registerCallback(const SQPCallback::Ptr& callback);
  const SQPStatus& getStatus();
  const SQPResults& getResults();

  bool verbose = false;
  SQPParameters params;
  std::shared_ptr<QPSolver> qp_solver;
  std::shared_ptr<QPProblem> qp_problem;

protected:
  void setBoxSize(double box_size);
  void constraintMeritCoeffChanged();
  SQPStatus status_ = SQPStatus::kRunning;
  SQPResults results_;
  std::vector<SQPCallback::Ptr> callbacks_;
};
}  // namespace trajopt_sqp
