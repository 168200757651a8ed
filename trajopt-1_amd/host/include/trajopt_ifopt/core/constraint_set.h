// trajopt_ifopt::ConstraintSet (core/constraint_set.h, component.h): the plugin
// surface of the trajopt_sqp front end.  A term is a set of `rows` functions of
// the variables with their bounds and penalty coefficients; TrajOptQPProblem
// adds it as a constraint (addConstraintSet) or a cost (addCostSet) and calls
// getValues / getJacobian at every convexification.  Subclass it for a custom
// term, as with the reference.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_ifopt/core/bounds.h"
#include "trajopt_ifopt/core/eigen_types.h"
#include "trajopt_ifopt/variable_sets/nodes_variables.h"

namespace trajopt_ifopt
{
enum class RangeBoundHandling
{
  kKeepAsIs,
  kSplitToTwoInequalities
};

class ConstraintSet
{
public:
  using Ptr = std::shared_ptr<ConstraintSet>;
  ConstraintSet(std::string name, int rows) : name_(std::move(name)), rows_(rows) {}
  virtual ~ConstraintSet() = default;
  virtual VectorXd getValues() const = 0;
  virtual Jacobian getJacobian() const = 0;
  virtual std::vector<Bounds> getBounds() const = 0;
  // penalty coefficient of every row (ones by default)
  virtual VectorXd getCoefficients() const { return VectorXd(static_cast<std::size_t>(rows_), 1.0); }
  // dynamic sets may change their row count at update() (the collision terms)
  virtual bool isDynamic() const { return false; }
  virtual int update() { return rows_; }
  void linkWithVariables(const std::shared_ptr<NodesVariables>& vars) { variables_ = vars; }
  int getRows() const { return rows_; }
  Index getNonZeros() const { return non_zeros_; }
  const std::string& getName() const { return name_; }

protected:
  std::string name_;
  int rows_;
  Index non_zeros_ = 0;
  std::shared_ptr<NodesVariables> variables_;
};
using Differentiable = ConstraintSet;
}  // namespace trajopt_ifopt
