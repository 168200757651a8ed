// trajopt_ifopt pieces of the trajopt_sqp front end: bounds, node variables and
// the joint-space constraint sets (behaviour of trajopt_ifopt/src/core/bounds.cpp,
// src/variable_sets/*.cpp, src/constraints/joint_*_constraint.cpp,
// src/utils/ifopt_utils.cpp:122-145).
#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <stdexcept>

#include "trajopt_ifopt/constraints/joint_constraints.h"
#include "trajopt_ifopt/utils/ifopt_utils.h"

namespace trajopt_ifopt
{
bool isFinite(double value) { return std::isfinite(value) && value < 1e20 && value > -1e20; }

Bounds::Bounds(double lower, double upper) : lower_(lower), upper_(upper) { updateType(); }
void Bounds::set(double lower, double upper)
{
  lower_ = lower;
  upper_ = upper;
  updateType();
}
void Bounds::setLower(double lower)
{
  lower_ = lower;
  updateType();
}
void Bounds::setUpper(double upper)
{
  upper_ = upper;
  updateType();
}
void Bounds::operator+=(double scalar)
{
  lower_ += scalar;
  upper_ += scalar;
  updateType();
}
void Bounds::operator-=(double scalar)
{
  lower_ -= scalar;
  upper_ -= scalar;
  updateType();
}
void Bounds::updateType()
{
  const bool lf = isFinite(lower_), uf = isFinite(upper_);
  if (!lf && !uf)
    type_ = BoundsType::kUnbounded;
  else if (lf && uf)
    type_ = (std::abs(upper_ - lower_) < 1e-8) ? BoundsType::kEquality : BoundsType::kRangeBound;
  else
    type_ = lf ? BoundsType::kLowerBound : BoundsType::kUpperBound;
}

const Bounds NoBound = Bounds(-std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity());
const Bounds BoundZero = Bounds(0.0, 0.0);
const Bounds BoundGreaterZero = Bounds(0.0, std::numeric_limits<double>::infinity());
const Bounds BoundSmallerZero = Bounds(-std::numeric_limits<double>::infinity(), 0.0);

void calcBoundsViolations(VectorXd& out, const VectorXd& input, const std::vector<Bounds>& bounds)
{
  if (input.size() != bounds.size())
    throw std::runtime_error("calcBoundsViolations: size mismatch");
  out.assign(input.size(), 0.0);
  for (std::size_t i = 0; i < input.size(); ++i)
  {
    const double x = input[i], lb = bounds[i].getLower(), ub = bounds[i].getUpper();
    if (x < lb)
      out[i] = std::abs(x - lb);
    else if (x > ub)
      out[i] = std::abs(x - ub);
  }
}

// ---------------------------------------------------------------- variables
Var::Var(std::string name, std::vector<std::string> child_names, VectorXd values, std::vector<Bounds> bounds)
  : name_(std::move(name)), child_names_(std::move(child_names)), values_(std::move(values)), bounds_(std::move(bounds))
{
  if (child_names_.size() != values_.size() || bounds_.size() != values_.size())
    throw std::runtime_error("Var: names, values and bounds must have the same size");
}

std::shared_ptr<const Var> Node::addVar(const std::string& name, const std::vector<std::string>& child_names,
                                        const VectorXd& values, const std::vector<Bounds>& bounds)
{
  vars_.push_back(std::make_shared<Var>(name, child_names, values, bounds));
  return vars_.back();
}

NodesVariables::NodesVariables(std::string name, std::vector<std::unique_ptr<Node>> nodes)
  : name_(std::move(name)), nodes_(std::move(nodes))
{
  for (const auto& n : nodes_)
    for (const auto& v : n->getVars())
    {
      v->index_ = rows_;
      rows_ += v->size();
      vars_.push_back(v);
    }
  setVariables(getValues());
}

VectorXd NodesVariables::getValues() const
{
  VectorXd x;
  x.reserve(static_cast<std::size_t>(rows_));
  for (const auto& v : vars_)
    x.insert(x.end(), v->values_.begin(), v->values_.end());
  return x;
}

void NodesVariables::setVariables(const VectorXd& x)
{
  if (static_cast<Index>(x.size()) < rows_)
    throw std::runtime_error("NodesVariables::setVariables: too few values");
  std::size_t h = 1469598103934665603ull;
  std::size_t k = 0;
  for (const auto& v : vars_)
    for (double& e : v->values_)
    {
      e = x[k++];
      h = (h ^ std::hash<double>()(e)) * 1099511628211ull;
    }
  hash_ = h;
}

std::vector<Bounds> NodesVariables::getBounds() const
{
  std::vector<Bounds> b;
  for (const auto& v : vars_)
    b.insert(b.end(), v->bounds_.begin(), v->bounds_.end());
  return b;
}

// ------------------------------------------------------------ joint position
namespace
{
void checkCoeffs(const VectorXd& c, const char* who)
{
  for (double v : c)
    if (!(v > 0))
      throw std::runtime_error(std::string(who) + ", coeff must be greater than zero.");
}
}  // namespace

JointPosConstraint::JointPosConstraint(const VectorXd& target, const std::shared_ptr<const Var>& position_var,
                                       const VectorXd& coeffs, std::string name, RangeBoundHandling)
  : ConstraintSet(std::move(name), static_cast<int>(target.size())), n_dof_(static_cast<Index>(target.size())),
    coeffs_(coeffs), position_var_(position_var)
{
  if (n_dof_ <= 0)
    throw std::runtime_error("JointPosConstraint: empty target");
  checkCoeffs(coeffs_, "JointPosConstraint");
  if (coeffs_.size() == 1)
    coeffs_.assign(static_cast<std::size_t>(n_dof_), coeffs[0]);
  if (static_cast<Index>(coeffs_.size()) != n_dof_)
    throw std::runtime_error("JointPosConstraint, coeff must be the same size of the joint postion.");
  if (static_cast<Index>(target.size()) != position_var->size())
    throw std::runtime_error("JointPosConstraint: targets size does not align with variables provided");
  for (Index i = 0; i < n_dof_; ++i)
  {
    bounds_.emplace_back(target[static_cast<std::size_t>(i)], target[static_cast<std::size_t>(i)]);
    indices_.push_back(i);
  }
  non_zeros_ = static_cast<Index>(indices_.size());
}

JointPosConstraint::JointPosConstraint(const std::vector<Bounds>& bounds, const std::shared_ptr<const Var>& position_var,
                                       const VectorXd& coeffs, std::string name, RangeBoundHandling handling)
  : ConstraintSet(std::move(name), static_cast<int>(bounds.size())), n_dof_(static_cast<Index>(bounds.size())),
    coeffs_(coeffs), position_var_(position_var)
{
  if (n_dof_ <= 0)
    throw std::runtime_error("JointPosConstraint: empty bounds");
  checkCoeffs(coeffs_, "JointPosConstraint");
  if (coeffs_.empty())
    coeffs_.assign(static_cast<std::size_t>(n_dof_), 1.0);
  else if (coeffs_.size() == 1)
    coeffs_.assign(static_cast<std::size_t>(n_dof_), coeffs[0]);
  else if (static_cast<Index>(coeffs_.size()) != n_dof_)
    throw std::runtime_error("JointPosConstraint, coeff must be the same size of the joint postion.");
  if (n_dof_ != position_var->size())
    throw std::runtime_error("JointPosConstraint: bounds size does not align with variables provided");
  if (handling == RangeBoundHandling::kSplitToTwoInequalities)
  {
    // a range bound becomes [lower, inf) and (-inf, upper] on two rows with the
    // dof's coefficient (the reference indexes the caller's coeffs here, which
    // is only defined for per-dof coefficients; the expanded ones give the same)
    const double inf = std::numeric_limits<double>::infinity();
    VectorXd split;
    for (Index i = 0; i < n_dof_; ++i)
    {
      const Bounds& b = bounds[static_cast<std::size_t>(i)];
      const double c = coeffs_[static_cast<std::size_t>(i)];
      if (b.getType() == BoundsType::kRangeBound)
      {
        bounds_.emplace_back(b.getLower(), inf);
        bounds_.emplace_back(-inf, b.getUpper());
        indices_.push_back(i);
        indices_.push_back(i);
        split.push_back(c);
        split.push_back(c);
      }
      else
      {
        bounds_.push_back(b);
        indices_.push_back(i);
        split.push_back(c);
      }
    }
    coeffs_ = split;
    rows_ = static_cast<int>(indices_.size());
  }
  else
  {
    bounds_ = bounds;
    for (Index i = 0; i < n_dof_; ++i)
      indices_.push_back(i);
  }
  non_zeros_ = static_cast<Index>(indices_.size());
}

VectorXd JointPosConstraint::getValues() const
{
  VectorXd v(indices_.size());
  const VectorXd& q = position_var_->value();
  for (std::size_t r = 0; r < indices_.size(); ++r)
    v[r] = q[static_cast<std::size_t>(indices_[r])];
  return v;
}

Jacobian JointPosConstraint::getJacobian() const
{
  Jacobian j(rows_, variables_->getRows());
  j.reserve(non_zeros_);
  for (int r = 0; r < rows_; ++r)
  {
    j.startVec(r);
    j.insertBack(r, position_var_->getIndex() + indices_[static_cast<std::size_t>(r)]) = 1.0;
  }
  j.finalize();
  return j;
}

// ------------------------------------------------- velocity / accel / jerk
JointDiffConstraint::JointDiffConstraint(const VectorXd& targets,
                                         const std::vector<std::shared_ptr<const Var>>& position_vars,
                                         const VectorXd& coeffs, std::string name, int rows_per_dof,
                                         double default_coeff, const char* who, std::size_t min_vars,
                                         const char* min_msg)
  : ConstraintSet(std::move(name), static_cast<int>(targets.size()) * rows_per_dof),
    n_dof_(static_cast<Index>(targets.size())), position_vars_(position_vars)
{
  if (position_vars.size() < min_vars)
    throw std::runtime_error(min_msg);
  if (n_dof_ <= 0)
    throw std::runtime_error(std::string(who) + ": empty targets");
  for (const auto& v : position_vars_)
    if (v->size() != n_dof_)
      throw std::runtime_error(std::string(who) + ": targets size does not align with variables provided");
  checkCoeffs(coeffs, who);
  const std::size_t rows = static_cast<std::size_t>(rows_);
  if (coeffs.empty())
    coeffs_.assign(rows, default_coeff);
  else if (coeffs.size() == 1)
    coeffs_.assign(rows, coeffs[0]);
  else if (static_cast<Index>(coeffs.size()) == n_dof_)
    for (std::size_t r = 0; r < rows; ++r)
      coeffs_.push_back(coeffs[r % static_cast<std::size_t>(n_dof_)]);
  else
    throw std::runtime_error(std::string(who) + ", coeff must be the same size of the joint position.");
  for (std::size_t r = 0; r < rows; ++r)
  {
    const double t = targets[r % static_cast<std::size_t>(n_dof_)];
    bounds_.emplace_back(t, t);
  }
}

void JointDiffConstraint::addStencil(std::vector<int> nodes, std::vector<double> weights)
{
  stencil_nodes_.push_back(std::move(nodes));
  stencil_w_.push_back(std::move(weights));
  non_zeros_ += n_dof_ * static_cast<Index>(stencil_w_.back().size());
}

VectorXd JointDiffConstraint::getValues() const
{
  VectorXd v(static_cast<std::size_t>(rows_));
  for (std::size_t s = 0; s < stencil_nodes_.size(); ++s)
  {
    const auto& nd = stencil_nodes_[s];
    const auto& w = stencil_w_[s];
    for (Index k = 0; k < n_dof_; ++k)
    {
      // left to right in the reference's expression order
      double a = w[0] * position_vars_[static_cast<std::size_t>(nd[0])]->value()[static_cast<std::size_t>(k)];
      for (std::size_t e = 1; e < nd.size(); ++e)
        a += w[e] * position_vars_[static_cast<std::size_t>(nd[e])]->value()[static_cast<std::size_t>(k)];
      v[s * static_cast<std::size_t>(n_dof_) + static_cast<std::size_t>(k)] = a;
    }
  }
  return v;
}

Jacobian JointDiffConstraint::getJacobian() const
{
  Jacobian j(rows_, variables_->getRows());
  j.reserve(non_zeros_);
  for (std::size_t s = 0; s < stencil_nodes_.size(); ++s)
  {
    // entries by ascending column: the stencil's nodes sorted by their variable index
    std::vector<std::pair<Index, double>> e;
    for (std::size_t q = 0; q < stencil_nodes_[s].size(); ++q)
      e.emplace_back(position_vars_[static_cast<std::size_t>(stencil_nodes_[s][q])]->getIndex(), stencil_w_[s][q]);
    std::sort(e.begin(), e.end());
    for (Index k = 0; k < n_dof_; ++k)
    {
      const Index row = static_cast<Index>(s) * n_dof_ + k;
      j.startVec(row);
      for (const auto& p : e)
        j.insertBack(row, p.first + k) = p.second;
    }
  }
  j.finalize();
  return j;
}

JointVelConstraint::JointVelConstraint(const VectorXd& targets,
                                       const std::vector<std::shared_ptr<const Var>>& position_vars,
                                       const VectorXd& coeffs, std::string name)
  : JointDiffConstraint(targets, position_vars, coeffs, std::move(name),
                        static_cast<int>(position_vars.size()) - 1, 5.0, "JointVelConstraint", 2,
                        "JointVelConstraint, requires minimum of three position variables!")
{
  for (int s = 0; s + 1 < static_cast<int>(position_vars.size()); ++s)
    addStencil({ s + 1, s }, { 1.0, -1.0 });  // q_{s+1} - q_s
}

JointAccelConstraint::JointAccelConstraint(const VectorXd& targets,
                                           const std::vector<std::shared_ptr<const Var>>& position_vars,
                                           const VectorXd& coeffs, std::string name)
  : JointDiffConstraint(targets, position_vars, coeffs, std::move(name), static_cast<int>(position_vars.size()), 1.0,
                        "JointAccelConstraint", 4, "JointAccelConstraint requires a minimum of four position variables!")
{
  const int n = static_cast<int>(position_vars.size());
  for (int i = 0; i < n; ++i)
  {
    if (i < n - 2)
      addStencil({ i + 2, i + 1, i }, { 1.0, -2.0, 1.0 });  // q_{i+2} - 2 q_{i+1} + q_i
    else
      addStencil({ i - 2, i - 1, i }, { 1.0, -2.0, 1.0 });  // q_{i-2} - 2 q_{i-1} + q_i
  }
}

JointJerkConstraint::JointJerkConstraint(const VectorXd& targets,
                                         const std::vector<std::shared_ptr<const Var>>& position_vars,
                                         const VectorXd& coeffs, std::string name)
  : JointDiffConstraint(targets, position_vars, coeffs, std::move(name), static_cast<int>(position_vars.size()), 1.0,
                        "JointJerkConstraint", 6, "JointJerkConstraint requires a minimum of six position variables!")
{
  const int n = static_cast<int>(position_vars.size());
  for (int i = 0; i < n; ++i)
  {
    if (i < n - 3)
      addStencil({ i, i + 1, i + 2, i + 3 }, { -1.0, 3.0, -3.0, 1.0 });
    else
      addStencil({ i, i - 1, i - 2, i - 3 }, { 1.0, -3.0, 3.0, -1.0 });
  }
}
}  // namespace trajopt_ifopt
