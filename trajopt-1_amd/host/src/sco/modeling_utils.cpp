// Costs / constraints from error functions (restating trajopt_sco/src/
// modeling_utils.cpp:31-269 and num_diff.cpp without Eigen).
#include "trajopt_sco/modeling_utils.hpp"

#include <algorithm>
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

DblVec calcForwardNumGrad(const ScalarOfVector& f, const DblVec& x, double epsilon)
{
  const double y = f(x);
  DblVec g(x.size());
  DblVec xp = x;
  for (std::size_t j = 0; j < x.size(); ++j)
  {
    xp[j] = x[j] + epsilon;
    g[j] = (f(xp) - y) / epsilon;
    xp[j] = x[j];
  }
  return g;
}

void calcGradAndDiagHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad,
                         DblVec& hess)
{
  y = f(x);
  grad.assign(x.size(), 0.0);
  hess.assign(x.size(), 0.0);
  DblVec xp = x;
  for (std::size_t j = 0; j < x.size(); ++j)
  {
    xp[j] = x[j] + epsilon / 2;
    const double yplus = f(xp);
    xp[j] = x[j] - epsilon / 2;
    const double yminus = f(xp);
    grad[j] = (yplus - yminus) / epsilon;
    hess[j] = (yplus + yminus - 2 * y) / (epsilon * epsilon / 4);
    xp[j] = x[j];
  }
}

void calcGradHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad, Mat& hess)
{
  y = f(x);
  const auto gradient = VectorOfVector::construct([&](const DblVec& z) { return calcForwardNumGrad(f, z, epsilon); });
  grad = gradient->call(x);
  const Mat h = calcForwardNumJac(*gradient, x, epsilon);
  hess = Mat(h.rows, h.cols);
  for (int i = 0; i < h.rows; ++i)
    for (int j = 0; j < h.cols; ++j)
      hess(i, j) = (h(i, j) + h(j, i)) / 2;
}

namespace
{
// eigen-decomposition of a small symmetric matrix by cyclic Jacobi rotations
// (stands in for Eigen::SelfAdjointEigenSolver): A = V diag(w) V^T
void symmetricEigen(const Mat& A, DblVec& w, Mat& V)
{
  const int n = A.rows;
  Mat a = A;
  V = Mat(n, n);
  for (int i = 0; i < n; ++i)
    V(i, i) = 1;
  for (int sweep = 0; sweep < 64; ++sweep)
  {
    double off = 0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q)
        off += a(p, q) * a(p, q);
    if (off < 1e-30)
      break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q)
      {
        if (a(p, q) == 0.0)
          continue;
        // rotation that zeroes a(p, q): tan(phi) = t
        const double zeta = (a(q, q) - a(p, p)) / (2 * a(p, q));
        const double t = std::copysign(1.0, zeta) / (std::fabs(zeta) + std::hypot(1.0, zeta));
        const double c = 1 / std::hypot(1.0, t), s = t * c;
        for (int k = 0; k < n; ++k)
        {
          const double kp = a(k, p), kq = a(k, q);
          a(k, p) = c * kp - s * kq;
          a(k, q) = s * kp + c * kq;
        }
        for (int k = 0; k < n; ++k)
        {
          const double pk = a(p, k), qk = a(q, k);
          a(p, k) = c * pk - s * qk;
          a(q, k) = s * pk + c * qk;
        }
        for (int k = 0; k < n; ++k)
        {
          const double kp = V(k, p), kq = V(k, q);
          V(k, p) = c * kp - s * kq;
          V(k, q) = s * kp + c * kq;
        }
      }
  }
  w.resize(static_cast<std::size_t>(n));
  for (int i = 0; i < n; ++i)
    w[static_cast<std::size_t>(i)] = a(i, i);
}
}  // namespace

CostFromFunc::CostFromFunc(ScalarOfVector::Ptr f, VarVector vars, const std::string& name, bool full_hessian)
  : Cost(name), f_(std::move(f)), vars_(std::move(vars)), full_hessian_(full_hessian)
{
}

double CostFromFunc::value(const DblVec& x) { return f_->call(getDblVec(x, vars_)); }

ConvexObjective::Ptr CostFromFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xv = getDblVec(x, vars_);
  const std::size_t n = xv.size();
  const int ni = static_cast<int>(n);
  auto out = std::make_shared<ConvexObjective>(model);
  QuadExpr& quad = out->quad_;
  double val = 0;
  DblVec grad;
  Mat H(ni, ni);  // the positive part of the Hessian
  if (!full_hessian_)
  {
    DblVec diag;
    calcGradAndDiagHess(*f_, xv, epsilon_, val, grad, diag);
    for (int i = 0; i < ni; ++i)
      H(i, i) = std::max(diag[static_cast<std::size_t>(i)], 0.0);
  }
  else
  {
    Mat hess;
    calcGradHess(*f_, xv, epsilon_, val, grad, hess);
    DblVec w;
    Mat V;
    symmetricEigen(hess, w, V);
    for (int k = 0; k < ni; ++k)
      if (w[static_cast<std::size_t>(k)] > 0)
        for (int i = 0; i < ni; ++i)
          for (int j = 0; j < ni; ++j)
            H(i, j) += w[static_cast<std::size_t>(k)] * V(i, k) * V(j, k);
  }
  DblVec Hx(n, 0.0);
  for (int i = 0; i < ni; ++i)
    for (int j = 0; j < ni; ++j)
      Hx[static_cast<std::size_t>(i)] += H(i, j) * xv[static_cast<std::size_t>(j)];
  double gx = 0, xHx = 0;
  for (std::size_t i = 0; i < n; ++i)
  {
    gx += grad[i] * xv[i];
    xHx += xv[i] * Hx[i];
  }
  // f(x0) + g.(x - x0) + 1/2 (x - x0)' H (x - x0)
  quad.affexpr.constant = val - gx + .5 * xHx;
  quad.affexpr.vars = vars_;
  quad.affexpr.coeffs.resize(n);
  for (std::size_t i = 0; i < n; ++i)
    quad.affexpr.coeffs[i] = grad[i] - Hx[i];
  if (!full_hessian_)
  {
    quad.vars1 = vars_;
    quad.vars2 = vars_;
    for (int i = 0; i < ni; ++i)
      quad.coeffs.push_back(H(i, i) * .5);
  }
  else
    for (int i = 0; i < ni; ++i)
    {
      quad.vars1.push_back(vars_[static_cast<std::size_t>(i)]);
      quad.vars2.push_back(vars_[static_cast<std::size_t>(i)]);
      quad.coeffs.push_back(H(i, i) / 2);
      for (int j = i + 1; j < ni; ++j)
      {
        quad.vars1.push_back(vars_[static_cast<std::size_t>(i)]);
        quad.vars2.push_back(vars_[static_cast<std::size_t>(j)]);
        quad.coeffs.push_back(H(i, j));
      }
    }
  return out;
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
