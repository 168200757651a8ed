// Costs / constraints from error functions (restating trajopt_sco/src/
// modeling_utils.cpp:31-269 and num_diff.cpp without Eigen).
#include "trajopt_sco/modeling_utils.hpp"

#include <cmath>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"

namespace sco
{
namespace
{
struct FnScalar : ScalarOfVector
{
  func f;
  explicit FnScalar(func g) : f(std::move(g)) {}
  double operator()(const DblVec& x) const override { return f(x); }
};
struct FnVector : VectorOfVector
{
  func f;
  explicit FnVector(func g) : f(std::move(g)) {}
  DblVec operator()(const DblVec& x) const override { return f(x); }
};
struct FnMatrix : MatrixOfVector
{
  func f;
  explicit FnMatrix(func g) : f(std::move(g)) {}
  Mat operator()(const DblVec& x) const override { return f(x); }
};
}  // namespace

ScalarOfVector::Ptr ScalarOfVector::construct(func f) { return std::make_shared<FnScalar>(std::move(f)); }
VectorOfVector::Ptr VectorOfVector::construct(func f) { return std::make_shared<FnVector>(std::move(f)); }
MatrixOfVector::Ptr MatrixOfVector::construct(func f) { return std::make_shared<FnMatrix>(std::move(f)); }

Mat calcForwardNumJac(const VectorOfVector& f, const DblVec& x, double epsilon)
{
  const DblVec y = f(x);
  Mat J(static_cast<int>(y.size()), static_cast<int>(x.size()));
  DblVec xp = x;
  for (std::size_t j = 0; j < x.size(); ++j)
  {
    xp[j] = x[j] + epsilon;
    const DblVec yp = f(xp);
    for (std::size_t i = 0; i < y.size(); ++i)
      J(static_cast<int>(i), static_cast<int>(j)) = (yp[i] - y[i]) / epsilon;
    xp[j] = x[j];
  }
  return J;
}

AffExpr affFromValGrad(double y, const DblVec& x, const DblVec& dydx, const VarVector& vars)
{
  AffExpr aff;
  double dot = 0;
  for (std::size_t k = 0; k < x.size(); ++k)
    dot += dydx[k] * x[k];
  aff.constant = y - dot;
  aff.coeffs = dydx;
  aff.vars = vars;
  return cleanupAff(aff);
}

CostFromErrFunc::CostFromErrFunc(VectorOfVector::Ptr f, VarVector vars, DblVec coeffs, PenaltyType pen_type,
                                 const std::string& name)
  : Cost(name), f_(std::move(f)), vars_(std::move(vars)), coeffs_(std::move(coeffs)), pen_type_(pen_type)
{
}
CostFromErrFunc::CostFromErrFunc(VectorOfVector::Ptr f, MatrixOfVector::Ptr dfdx, VarVector vars, DblVec coeffs,
                                 PenaltyType pen_type, const std::string& name)
  : Cost(name)
  , f_(std::move(f))
  , dfdx_(std::move(dfdx))
  , vars_(std::move(vars))
  , coeffs_(std::move(coeffs))
  , pen_type_(pen_type)
{
}

double CostFromErrFunc::value(const DblVec& x)
{
  DblVec err = f_->call(getDblVec(x, vars_));
  double total = 0;
  for (std::size_t i = 0; i < err.size(); ++i)
  {
    double e = err[i];
    e = (pen_type_ == SQUARED) ? e * e : (pen_type_ == ABS) ? std::fabs(e) : std::fmax(e, 0.0);
    if (!coeffs_.empty())
      e *= coeffs_[i];
    total += e;
  }
  return total;
}

ConvexObjective::Ptr CostFromErrFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xv = getDblVec(x, vars_);
  const Mat jac = dfdx_ ? dfdx_->call(xv) : calcForwardNumJac(*f_, xv, epsilon_);
  auto out = std::make_shared<ConvexObjective>(model);
  const DblVec y = f_->call(xv);
  for (int i = 0; i < jac.rows; ++i)
  {
    AffExpr aff = affFromValGrad(y[static_cast<std::size_t>(i)], xv, jac.row(i), vars_);
    double w = 1;
    if (!coeffs_.empty())
    {
      if (coeffs_[static_cast<std::size_t>(i)] == 0)
        continue;
      w = coeffs_[static_cast<std::size_t>(i)];
    }
    if (pen_type_ == SQUARED)
    {
      QuadExpr quad = exprSquare(aff);
      exprScale(quad, w);
      out->addQuadExpr(quad);
    }
    else
    {
      exprScale(aff, w);
      if (pen_type_ == ABS)
        out->addAbs(aff, 1);
      else
        out->addHinge(aff, 1);
    }
  }
  return out;
}

ConstraintFromErrFunc::ConstraintFromErrFunc(VectorOfVector::Ptr f, VarVector vars, DblVec coeffs, ConstraintType type,
                                             const std::string& name)
  : Constraint(name), f_(std::move(f)), vars_(std::move(vars)), coeffs_(std::move(coeffs)), type_(type)
{
}
ConstraintFromErrFunc::ConstraintFromErrFunc(VectorOfVector::Ptr f, MatrixOfVector::Ptr dfdx, VarVector vars,
                                             DblVec coeffs, ConstraintType type, const std::string& name)
  : Constraint(name)
  , f_(std::move(f))
  , dfdx_(std::move(dfdx))
  , vars_(std::move(vars))
  , coeffs_(std::move(coeffs))
  , type_(type)
{
}

DblVec ConstraintFromErrFunc::value(const DblVec& x)
{
  DblVec err = f_->call(getDblVec(x, vars_));
  if (!coeffs_.empty())
    for (std::size_t i = 0; i < err.size(); ++i)
      err[i] *= coeffs_[i];
  return err;
}

ConvexConstraints::Ptr ConstraintFromErrFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xv = getDblVec(x, vars_);
  const Mat jac = dfdx_ ? dfdx_->call(xv) : calcForwardNumJac(*f_, xv, epsilon_);
  auto out = std::make_shared<ConvexConstraints>(model);
  const DblVec y = f_->call(xv);
  for (int i = 0; i < jac.rows; ++i)
  {
    AffExpr aff = affFromValGrad(y[static_cast<std::size_t>(i)], xv, jac.row(i), vars_);
    if (!coeffs_.empty())
    {
      if (coeffs_[static_cast<std::size_t>(i)] == 0)
        continue;
      exprScale(aff, coeffs_[static_cast<std::size_t>(i)]);
    }
    if (type_ == INEQ)
      out->addIneqCnt(aff);
    else
      out->addEqCnt(aff);
  }
  return out;
}
}  // namespace sco
