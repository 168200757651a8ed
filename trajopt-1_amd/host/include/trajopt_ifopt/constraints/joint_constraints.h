// The joint-space terms of trajopt_ifopt (src/constraints/joint_*_constraint.cpp):
// position (per-dof bounds or targets), velocity q_{i+1} - q_i, acceleration
// q_{i+2} - 2 q_{i+1} + q_i (backward differences at the last two nodes) and
// jerk -q_i + 3 q_{i+1} - 3 q_{i+2} + q_{i+3} (backward at the last three), each
// with the reference's coefficient expansion and argument checks.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_ifopt/core/constraint_set.h"

namespace trajopt_ifopt
{
class JointPosConstraint : public ConstraintSet
{
public:
  JointPosConstraint(const VectorXd& target, const std::shared_ptr<const Var>& position_var, const VectorXd& coeffs,
                     std::string name = "JointPos",
                     RangeBoundHandling range_bound_handling = RangeBoundHandling::kSplitToTwoInequalities);
  JointPosConstraint(const std::vector<Bounds>& bounds, const std::shared_ptr<const Var>& position_var,
                     const VectorXd& coeffs, std::string name = "JointPos",
                     RangeBoundHandling range_bound_handling = RangeBoundHandling::kSplitToTwoInequalities);
  VectorXd getValues() const override;
  Jacobian getJacobian() const override;
  std::vector<Bounds> getBounds() const override { return bounds_; }
  VectorXd getCoefficients() const override { return coeffs_; }

private:
  Index n_dof_ = 0;
  VectorXd coeffs_;
  std::vector<Bounds> bounds_;
  std::vector<Index> indices_;  // dof of each row (a split range bound has two rows)
  std::shared_ptr<const Var> position_var_;
};

// JointVel / JointAccel / JointJerk share one shape: row (i, k) is a fixed
// stencil over dof k of a few consecutive nodes
class JointDiffConstraint : public ConstraintSet
{
public:
  VectorXd getValues() const override;
  Jacobian getJacobian() const override;
  std::vector<Bounds> getBounds() const override { return bounds_; }
  VectorXd getCoefficients() const override { return coeffs_; }

protected:
  // rows: per stencil row the nodes it reads and their weights (in the
  // reference's evaluation order)
  JointDiffConstraint(const VectorXd& targets, const std::vector<std::shared_ptr<const Var>>& position_vars,
                      const VectorXd& coeffs, std::string name, int rows_per_dof, double default_coeff,
                      const char* who, std::size_t min_vars, const char* min_msg);
  void addStencil(std::vector<int> nodes, std::vector<double> weights);
  Index n_dof_ = 0;
  std::vector<std::shared_ptr<const Var>> position_vars_;
  VectorXd coeffs_;
  std::vector<Bounds> bounds_;
  std::vector<std::vector<int>> stencil_nodes_;
  std::vector<std::vector<double>> stencil_w_;
};

class JointVelConstraint : public JointDiffConstraint
{
public:
  JointVelConstraint(const VectorXd& targets, const std::vector<std::shared_ptr<const Var>>& position_vars,
                     const VectorXd& coeffs, std::string name = "JointVel");
};
class JointAccelConstraint : public JointDiffConstraint
{
public:
  JointAccelConstraint(const VectorXd& targets, const std::vector<std::shared_ptr<const Var>>& position_vars,
                       const VectorXd& coeffs, std::string name = "JointAccel");
};
class JointJerkConstraint : public JointDiffConstraint
{
public:
  JointJerkConstraint(const VectorXd& targets, const std::vector<std::shared_ptr<const Var>>& position_vars,
                      const VectorXd& coeffs, std::string name = "JointJerk");
};
}  // namespace trajopt_ifopt
