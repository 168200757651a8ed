// Joint-space trajectory terms (restating trajopt/src/trajectory_costs.cpp:28-1016
// over one difference-order parameter).
#include "trajopt_amd/trajectory_costs.hpp"

#include <cmath>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"

namespace trajopt
{
namespace
{
const double* stencil(int order)
{
  static const double s0[] = { 1 }, s1[] = { -1, 1 }, s2[] = { 1, -2, 1 }, s3[] = { -1, 3, -3, 1 };
  switch (order)
  {
    case 0:
      return s0;
    case 1:
      return s1;
    case 2:
      return s2;
    default:
      return s3;
  }
}

void checkLength(const JointDiffSpec& s, const std::string& what)
{
  if (s.order < 0 || s.order > 3)
    throw std::runtime_error(what + ": difference order must be 0..3");
  if (s.order > 0 && ((s.last_step - s.order) - s.first_step) < 0)
    throw std::runtime_error(what + ", trajectory is too short!");
}

// d-th difference minus target at (i, j), as the ctors build it: sum of
// exprMult(x_{i+k, j}, stencil_k) in k order, then exprDec(target)
sco::AffExpr diffExpr(const JointDiffSpec& s, int i, int j)
{
  sco::AffExpr d;
  const double* st = stencil(s.order);
  for (int k = 0; k <= s.order; ++k)
    sco::exprInc(d, sco::exprMult(sco::AffExpr(s.vars(i + k, j)), st[k]));
  sco::exprDec(d, s.targets[static_cast<std::size_t>(j)]);
  return d;
}

// Eigen's diffAxis0 applied `order` times to the trajectory block, minus the target
double diffValue(const JointDiffSpec& s, const DblVec& x, int i, int j)
{
  double v[4];
  for (int k = 0; k <= s.order; ++k)
    v[k] = s.vars(i + k, j).value(x);
  for (int o = 0; o < s.order; ++o)
    for (int k = 0; k < s.order - o; ++k)
      v[k] = v[k + 1] - v[k];
  return v[0] - s.targets[static_cast<std::size_t>(j)];
}

int lastIndex(const JointDiffSpec& s) { return s.last_step - s.order; }
}  // namespace

JointDiffEqCost::JointDiffEqCost(JointDiffSpec s, const std::string& name) : sco::Cost(name), s_(std::move(s))
{
  checkLength(s_, name + "Cost");
  for (int i = s_.first_step; i <= lastIndex(s_); ++i)
    for (int j = 0; j < s_.vars.cols(); ++j)
      sco::exprInc(expr_, sco::exprMult(sco::exprSquare(diffExpr(s_, i, j)), s_.coeffs[static_cast<std::size_t>(j)]));
}

double JointDiffEqCost::value(const DblVec& x)
{
  // (diff^2 * diag(coeffs)).sum(), column-major
  double sum = 0;
  for (int j = 0; j < s_.vars.cols(); ++j)
    for (int i = s_.first_step; i <= lastIndex(s_); ++i)
    {
      const double d = diffValue(s_, x, i, j);
      sum += (d * d) * s_.coeffs[static_cast<std::size_t>(j)];
    }
  return sum;
}

sco::ConvexObjective::Ptr JointDiffEqCost::convex(const DblVec&, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexObjective>(model);
  out->addQuadExpr(expr_);
  return out;
}

JointDiffIneqCost::JointDiffIneqCost(JointDiffSpec s, const std::string& name) : sco::Cost(name), s_(std::move(s))
{
  checkLength(s_, name + "Cost");
  for (int i = s_.first_step; i <= lastIndex(s_); ++i)
    for (int j = 0; j < s_.vars.cols(); ++j)
    {
      const auto jj = static_cast<std::size_t>(j);
      const sco::AffExpr d = diffExpr(s_, i, j);
      sco::AffExpr up, lo;
      if (s_.order == 0)
      {
        // JointPosIneq: (pos - upper) * coeff, (lower - pos) * coeff
        sco::exprInc(up, d);
        sco::exprDec(up, s_.upper_tols[jj]);
        sco::exprScale(up, s_.coeffs[jj]);
      }
      else
      {
        // velocity / acceleration / jerk: -(upper - d) * coeff, (lower - d) * coeff
        sco::exprInc(up, s_.upper_tols[jj]);
        sco::exprDec(up, d);
        sco::exprScale(up, -s_.coeffs[jj]);
      }
      exprs_.push_back(up);
      sco::exprInc(lo, s_.lower_tols[jj]);
      sco::exprDec(lo, d);
      sco::exprScale(lo, s_.coeffs[jj]);
      exprs_.push_back(lo);
    }
}

DblVec JointDiffIneqCost::blockValues(const DblVec& x) const
{
  DblVec out;
  for (int blk = 0; blk < 2; ++blk)
    for (int j = 0; j < s_.vars.cols(); ++j)
      for (int i = s_.first_step; i <= lastIndex(s_); ++i)
      {
        const auto jj = static_cast<std::size_t>(j);
        const double d = diffValue(s_, x, i, j);
        out.push_back(blk == 0 ? (d - s_.upper_tols[jj]) * s_.coeffs[jj]
                               : ((d * -1) + s_.lower_tols[jj]) * s_.coeffs[jj]);
      }
  return out;
}

double JointDiffIneqCost::value(const DblVec& x)
{
  const DblVec v = blockValues(x);
  const std::size_t half = v.size() / 2;
  double s1 = 0, s2 = 0;
  for (std::size_t k = 0; k < half; ++k)
    s1 += std::fmax(v[k], 0.0);
  for (std::size_t k = half; k < v.size(); ++k)
    s2 += std::fmax(v[k], 0.0);
  return s1 + s2;
}

sco::ConvexObjective::Ptr JointDiffIneqCost::convex(const DblVec&, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexObjective>(model);
  for (const sco::AffExpr& e : exprs_)
    out->addHinge(e, 1);
  return out;
}

JointDiffEqConstraint::JointDiffEqConstraint(JointDiffSpec s, const std::string& name)
  : sco::EqConstraint(name), s_(std::move(s))
{
  checkLength(s_, name + "Constraint");
  for (int i = s_.first_step; i <= lastIndex(s_); ++i)
    for (int j = 0; j < s_.vars.cols(); ++j)
      exprs_.push_back(sco::exprMult(diffExpr(s_, i, j), s_.coeffs[static_cast<std::size_t>(j)]));
}

DblVec JointDiffEqConstraint::value(const DblVec& x)
{
  DblVec out;
  for (int j = 0; j < s_.vars.cols(); ++j)
    for (int i = s_.first_step; i <= lastIndex(s_); ++i)
    {
      const double d = diffValue(s_, x, i, j);
      out.push_back((d * d) * s_.coeffs[static_cast<std::size_t>(j)]);
    }
  return out;
}

sco::ConvexConstraints::Ptr JointDiffEqConstraint::convex(const DblVec&, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexConstraints>(model);
  for (const sco::AffExpr& e : exprs_)
    out->addEqCnt(e);
  return out;
}

JointDiffIneqConstraint::JointDiffIneqConstraint(JointDiffSpec s, const std::string& name)
  : sco::IneqConstraint(name), rows_(s, name), clamp_(s.order != 0)
{
}

DblVec JointDiffIneqConstraint::value(const DblVec& x)
{
  DblVec v = rows_.blockValues(x);
  if (clamp_)
    for (double& a : v)
      a = std::fmax(a, 0.0);
  return v;
}

sco::ConvexConstraints::Ptr JointDiffIneqConstraint::convex(const DblVec&, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexConstraints>(model);
  for (const sco::AffExpr& e : rows_.exprs())
    out->addIneqCnt(e);
  return out;
}

sco::VectorOfVector::Ptr jointVelTimeErr(double target, double upper_tol, double lower_tol)
{
  return sco::VectorOfVector::construct([target, upper_tol, lower_tol](const DblVec& v) {
    const std::size_t half = v.size() / 2, nv = half - 1;
    DblVec out(2 * nv);
    for (std::size_t i = 0; i < nv; ++i)
    {
      const double vel = (v[i + 1] - v[i]) * v[half + i + 1];
      out[i] = -(upper_tol - (vel - target));
      out[nv + i] = lower_tol - (vel - target);
    }
    return out;
  });
}

sco::MatrixOfVector::Ptr jointVelTimeJac()
{
  return sco::MatrixOfVector::construct([](const DblVec& v) {
    const int n = static_cast<int>(v.size()), half = n / 2, nv = half - 1;
    sco::Mat J(2 * nv, n);
    for (int i = 0; i < nv; ++i)
    {
      const int ti = i + half + 1;  // the dt of the velocity's second waypoint
      J(i, i) = -1.0 * v[static_cast<std::size_t>(ti)];
      J(i, i + 1) = 1.0 * v[static_cast<std::size_t>(ti)];
      J(i, ti) = v[static_cast<std::size_t>(i + 1)] - v[static_cast<std::size_t>(i)];
    }
    for (int i = 0; i < nv; ++i)  // the bottom half: the negative velocities
      for (int c = 0; c < n; ++c)
        J(nv + i, c) = -J(i, c);
    return J;
  });
}

sco::VectorOfVector::Ptr totalTimeErr(double limit)
{
  return sco::VectorOfVector::construct([limit](const DblVec& v) {
    double s = 0;
    for (const double x : v)
      s += 1.0 / x;
    return DblVec{ s - limit };
  });
}

sco::MatrixOfVector::Ptr totalTimeJac()
{
  return sco::MatrixOfVector::construct([](const DblVec& v) {
    sco::Mat J(1, static_cast<int>(v.size()));
    for (int c = 0; c < static_cast<int>(v.size()); ++c)
      J(0, c) = -1.0 / (v[static_cast<std::size_t>(c)] * v[static_cast<std::size_t>(c)]);
    return J;
  });
}

}  // namespace trajopt
