// trajopt_sqp::TrajOptQPProblem (src/trajopt_qp_problem.cpp): constraint and cost
// sets linearised into one QP whose sparsity pattern stays fixed across
// convexifications (small jacobian entries are stored as zeros, not dropped):
//   variables  [NLP variables | slacks: two per equality row, one per inequality row]
//   rows       [hinge-cost rows | absolute-cost rows | constraint rows | identity over
//               every variable (trust box on the NLP block, slack >= 0)]
//   objective  squared costs as a quadratic on the NLP block, slacks weighted by
//              the row coefficient (x the merit coefficient for constraints)
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_ifopt/variable_sets/nodes_variables.h"
#include "trajopt_sqp/qp_problem.h"

namespace trajopt_sqp
{
class TrajOptQPProblem : public QPProblem
{
public:
  using Ptr = std::shared_ptr<TrajOptQPProblem>;
  explicit TrajOptQPProblem(std::shared_ptr<trajopt_ifopt::NodesVariables> variables);
  ~TrajOptQPProblem() override;
  void addConstraintSet(std::shared_ptr<trajopt_ifopt::ConstraintSet> constraint_set) override;
  void addCostSet(std::shared_ptr<trajopt_ifopt::ConstraintSet> constraint_set, CostPenaltyType penalty_type) override;
  void setup() override;
  void setVariables(const double* x) override;
  VectorXd getVariableValues() const override;
  void convexify() override;
  double evaluateTotalConvexCost(const VectorXd& var_vals) const override;
  VectorXd evaluateConvexCosts(const VectorXd& var_vals) const override;
  double getTotalExactCost() const override;
  VectorXd getExactCosts() const override;
  VectorXd evaluateConvexConstraintViolations(const VectorXd& var_vals) const override;
  VectorXd getExactConstraintViolations() const override;
  void scaleBoxSize(double& scale) override;
  void setBoxSize(const VectorXd& box_size) override;
  void setConstraintMeritCoeff(const VectorXd& merit_coeff) override;
  void print() const override;
  long getNumNLPVars() const override;
  long getNumNLPConstraints() const override;
  long getNumNLPCosts() const override;
  long getNumQPVars() const override;
  long getNumQPConstraints() const override;
  const std::vector<std::string>& getNLPConstraintNames() const override;
  const std::vector<std::string>& getNLPCostNames() const override;
  const VectorXd& getBoxSize() const override;
  const VectorXd& getConstraintMeritCoeff() const override;
  const trajopt_ifopt::Jacobian& getHessian() const override;
  const VectorXd& getGradient() const override;
  const trajopt_ifopt::Jacobian& getConstraintMatrix() const override;
  const VectorXd& getBoundsLower() const override;
  const VectorXd& getBoundsUpper() const override;

private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};
}  // namespace trajopt_sqp
