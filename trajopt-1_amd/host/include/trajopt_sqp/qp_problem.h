// trajopt_sqp::QPProblem (include/trajopt_sqp/qp_problem.h): what the trust-region
// solver asks of a convexifiable problem.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_ifopt/core/constraint_set.h"
#include "trajopt_sqp/types.h"

namespace trajopt_sqp
{
class QPProblem
{
public:
  using Ptr = std::shared_ptr<QPProblem>;
  virtual ~QPProblem() = default;
  virtual void addConstraintSet(std::shared_ptr<trajopt_ifopt::ConstraintSet> constraint_set) = 0;
  virtual void addCostSet(std::shared_ptr<trajopt_ifopt::ConstraintSet> constraint_set,
                          CostPenaltyType penalty_type) = 0;
  virtual void setup() = 0;
  virtual void setVariables(const double* x) = 0;
  virtual VectorXd getVariableValues() const = 0;
  virtual void convexify() = 0;
  virtual double evaluateTotalConvexCost(const VectorXd& var_vals) const = 0;
  virtual VectorXd evaluateConvexCosts(const VectorXd& var_vals) const = 0;
  virtual double getTotalExactCost() const = 0;
  virtual VectorXd getExactCosts() const = 0;
  virtual VectorXd evaluateConvexConstraintViolations(const VectorXd& var_vals) const = 0;
  virtual VectorXd getExactConstraintViolations() const = 0;
  virtual void scaleBoxSize(double& scale) = 0;
  virtual void setBoxSize(const VectorXd& box_size) = 0;
  virtual void setConstraintMeritCoeff(const VectorXd& merit_coeff) = 0;
  virtual void print() const = 0;
  virtual long getNumNLPVars() const = 0;
  virtual long getNumNLPConstraints() const = 0;
  virtual long getNumNLPCosts() const = 0;
  virtual long getNumQPVars() const = 0;
  virtual long getNumQPConstraints() const = 0;
  virtual const std::vector<std::string>& getNLPConstraintNames() const = 0;
  virtual const std::vector<std::string>& getNLPCostNames() const = 0;
  virtual const VectorXd& getBoxSize() const = 0;
  virtual const VectorXd& getConstraintMeritCoeff() const = 0;
  virtual const trajopt_ifopt::Jacobian& getHessian() const = 0;
  virtual const VectorXd& getGradient() const = 0;
  virtual const trajopt_ifopt::Jacobian& getConstraintMatrix() const = 0;
  virtual const VectorXd& getBoundsLower() const = 0;
  virtual const VectorXd& getBoundsUpper() const = 0;
};
}  // namespace trajopt_sqp
