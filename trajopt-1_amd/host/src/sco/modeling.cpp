// Convex modelling + OptProb (restating trajopt_sco/src/modeling.cpp:16-295).
#include "trajopt_sco/modeling.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"

namespace sco
{
// ------------------------------------------------------------------ ConvexObjective
void ConvexObjective::addAffExpr(const AffExpr& a) { exprInc(quad_, a); }
void ConvexObjective::addQuadExpr(const QuadExpr& q) { exprInc(quad_, q); }

void ConvexObjective::addHinge(const AffExpr& aff, double coeff)
{
  const Var h = model_->addVar("hinge", 0, HUGE_VAL);
  vars_.push_back(h);
  AffExpr row = aff;  // aff - h <= 0
  exprDec(row, h);
  ineqs_.push_back(std::move(row));
  exprInc(quad_, exprMult(AffExpr(h), coeff));
}

void ConvexObjective::addAbs(const AffExpr& aff, double coeff)
{
  const Var neg = model_->addVar("neg", 0, HUGE_VAL);
  const Var pos = model_->addVar("pos", 0, HUGE_VAL);
  vars_.push_back(neg);
  vars_.push_back(pos);
  AffExpr cost;  // coeff * (neg + pos)
  cost.coeffs = { coeff, coeff };
  cost.vars = { neg, pos };
  exprInc(quad_, cost);
  AffExpr row = aff;  // aff + neg - pos = 0
  row.coeffs.push_back(1);
  row.vars.push_back(neg);
  row.coeffs.push_back(-1);
  row.vars.push_back(pos);
  eqs_.push_back(std::move(row));
}

void ConvexObjective::addHinges(const AffExprVector& ev)
{
  for (const auto& e : ev)
    addHinge(e, 1);
}
void ConvexObjective::addL1Norm(const AffExprVector& ev)
{
  for (const auto& e : ev)
    addAbs(e, 1);
}
void ConvexObjective::addL2Norm(const AffExprVector& ev)
{
  for (const auto& e : ev)
    exprInc(quad_, exprSquare(e));
}
void ConvexObjective::addMax(const AffExprVector& ev)
{
  // (as the reference: the "max" variable is not recorded in vars_)
  const Var mx = model_->addVar("max", -HUGE_VAL, HUGE_VAL);
  for (const auto& e : ev)
  {
    ineqs_.push_back(e);
    exprDec(ineqs_.back(), mx);
  }
}

void ConvexObjective::addConstraintsToModel()
{
  for (const AffExpr& a : eqs_)
    cnts_.push_back(model_->addEqCnt(a, ""));
  for (const AffExpr& a : ineqs_)
    cnts_.push_back(model_->addIneqCnt(a, ""));
}
void ConvexObjective::removeFromModel()
{
  model_->removeCnts(cnts_);
  model_->removeVars(vars_);
  model_ = nullptr;
}
ConvexObjective::~ConvexObjective()
{
  if (inModel())
    removeFromModel();
}
double ConvexObjective::value(const DblVec& x) const { return quad_.value(x); }

// ------------------------------------------------------------------ ConvexConstraints
void ConvexConstraints::addEqCnt(const AffExpr& a) { eqs_.push_back(a); }
void ConvexConstraints::addIneqCnt(const AffExpr& a) { ineqs_.push_back(a); }
void ConvexConstraints::addConstraintsToModel()
{
  for (const AffExpr& a : eqs_)
    cnts_.push_back(model_->addEqCnt(a, ""));
  for (const AffExpr& a : ineqs_)
    cnts_.push_back(model_->addIneqCnt(a, ""));
}
void ConvexConstraints::removeFromModel()
{
  model_->removeCnts(cnts_);
  model_ = nullptr;
}
DblVec ConvexConstraints::violations(const DblVec& x)
{
  DblVec out;
  out.reserve(eqs_.size() + ineqs_.size());
  for (const AffExpr& a : eqs_)
    out.push_back(std::fabs(a.value(x.data())));
  for (const AffExpr& a : ineqs_)
    out.push_back(pospart(a.value(x.data())));
  return out;
}
double ConvexConstraints::violation(const DblVec& x) { return vecSum(violations(x)); }
ConvexConstraints::~ConvexConstraints()
{
  if (inModel())
    removeFromModel();
}

// ------------------------------------------------------------------ Constraint
DblVec Constraint::violations(const DblVec& x)
{
  DblVec v = value(x);
  const bool eq = type() == EQ;
  for (double& a : v)
    a = eq ? std::fabs(a) : pospart(a);
  return v;
}
double Constraint::violation(const DblVec& x) { return vecSum(violations(x)); }

// ------------------------------------------------------------------ OptProb
OptProb::OptProb(ModelType convex_solver, const ModelConfig::ConstPtr& convex_solver_config)
  : model_(createModel(convex_solver, convex_solver_config))
{
}

VarVector OptProb::createVariables(const std::vector<std::string>& names)
{
  return createVariables(names, DblVec(names.size(), -HUGE_VAL), DblVec(names.size(), HUGE_VAL));
}

VarVector OptProb::createVariables(const std::vector<std::string>& names, const DblVec& lb, const DblVec& ub)
{
  if (lb.size() != names.size() || ub.size() != names.size())
    throw std::runtime_error("OptProb::createVariables: bounds and names differ in size");
  const std::size_t first = vars_.size();
  for (std::size_t k = 0; k < names.size(); ++k)
  {
    vars_.push_back(model_->addVar(names[k], lb[k], ub[k]));
    lower_bounds_.push_back(lb[k]);
    upper_bounds_.push_back(ub[k]);
  }
  model_->update();
  return VarVector(vars_.begin() + static_cast<long>(first), vars_.end());
}

void OptProb::setLowerBounds(const DblVec& lb) { lower_bounds_ = lb; }
void OptProb::setUpperBounds(const DblVec& ub) { upper_bounds_ = ub; }
void OptProb::setLowerBounds(const DblVec& lb, const VarVector& vars) { setVec(lower_bounds_, vars, lb); }
void OptProb::setUpperBounds(const DblVec& ub, const VarVector& vars) { setVec(upper_bounds_, vars, ub); }
void OptProb::addCost(Cost::Ptr cost) { costs_.push_back(std::move(cost)); }
void OptProb::addConstraint(Constraint::Ptr cnt)
{
  if (cnt->type() == EQ)
    addEqConstraint(std::move(cnt));
  else
    addIneqConstraint(std::move(cnt));
}
void OptProb::addEqConstraint(Constraint::Ptr cnt) { eqcnts_.push_back(std::move(cnt)); }
void OptProb::addIneqConstraint(Constraint::Ptr cnt) { ineqcnts_.push_back(std::move(cnt)); }

std::vector<Constraint::Ptr> OptProb::getConstraints() const
{
  std::vector<Constraint::Ptr> out(eqcnts_);
  out.insert(out.end(), ineqcnts_.begin(), ineqcnts_.end());
  return out;
}

void OptProb::addLinearConstraint(const AffExpr& expr, ConstraintType type)
{
  if (type == EQ)
    model_->addEqCnt(expr, "");
  else
    model_->addIneqCnt(expr, "");
}

DblVec OptProb::getClosestFeasiblePoint(const DblVec& x, const double& delta)
{
  DblVec y(x.size());
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    const double inset = std::min(delta, (upper_bounds_[i] - lower_bounds_[i]) / 2);
    y[i] = std::min(std::max(x[i], lower_bounds_[i] + inset), upper_bounds_[i] - inset);
  }
  return y;
}

bool OptProb::solveNative(const BasicTrustRegionSQPParameters&, const DblVec&, OptResults&) { return false; }
}  // namespace sco
