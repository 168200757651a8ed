// ORACLE — test infrastructure only (see sco_expr.hpp header).
#include "terms.hpp"
#include "jitter.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

#include "collision.hpp"

namespace orc
{
OsqpSettings toOsqpSettings(const thip_osqp_settings& s)
{
  OsqpSettings o;
  o.rho = s.rho;
  o.sigma = s.sigma;
  o.alpha = s.alpha;
  o.scaling = s.scaling;
  o.adaptive_rho = s.adaptive_rho;
  o.adaptive_rho_interval = s.adaptive_rho_interval;
  o.adaptive_rho_tolerance = s.adaptive_rho_tolerance;
  o.max_iter = s.max_iter;
  o.eps_abs = s.eps_abs;
  o.eps_rel = s.eps_rel;
  o.eps_prim_inf = s.eps_prim_inf;
  o.eps_dual_inf = s.eps_dual_inf;
  o.check_termination = s.check_termination;
  o.warm_starting = s.warm_starting;
  o.polishing = s.polishing;
  o.delta = s.delta;
  o.polish_refine_iter = s.polish_refine_iter;
  return o;
}

BasicTrustRegionSQPParameters toSqpParams(const thip_sqp_params& p)
{
  BasicTrustRegionSQPParameters o;
  o.improve_ratio_threshold = p.improve_ratio_threshold;
  o.min_trust_box_size = p.min_trust_box_size;
  o.min_approx_improve = p.min_approx_improve;
  o.min_approx_improve_frac = p.min_approx_improve_frac;
  o.max_iter = p.max_iter;
  o.trust_shrink_ratio = p.trust_shrink_ratio;
  o.trust_expand_ratio = p.trust_expand_ratio;
  o.cnt_tolerance = p.cnt_tolerance;
  o.max_merit_coeff_increases = p.max_merit_coeff_increases;
  o.max_qp_solver_failures = p.max_qp_solver_failures;
  o.merit_coeff_increase_ratio = p.merit_coeff_increase_ratio;
  o.initial_merit_error_coeff = p.initial_merit_error_coeff;
  o.inflate_constraints_individually = p.inflate_constraints_individually != 0;
  o.trust_box_size = p.trust_box_size;
  o.max_time = p.max_time;
  return o;
}

// ------------------------------------------------------------ JointVelEqCost
namespace
{
class JointVelEqCost : public Cost
{
public:
  JointVelEqCost(std::vector<VarVector> rows, DblVec coeffs, DblVec targets, int first_step, int last_step)
    : Cost("JointVelEq")
    , rows_(std::move(rows))
    , coeffs_(std::move(coeffs))
    , targets_(std::move(targets))
    , first_(first_step)
    , last_(last_step)
  {
    if (((last_ - 1) - first_) < 0)
      throw std::runtime_error("JointVelEqCost, trajectory is too short!");
    for (int i = first_; i <= last_ - 1; ++i)
      for (std::size_t j = 0; j < coeffs_.size(); ++j)
      {
        AffExpr vel;
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i)][j], -1));
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i + 1)][j], 1));
        exprDec(vel, targets_[j]);
        exprInc(expr_, exprMult(exprSquare(vel), coeffs_[j]));
      }
  }
  double value(const DblVec& x) override
  {
    // (diffAxis0(traj) - targets)^2 * diag(coeffs), summed column-major
    double s = 0;
    for (std::size_t j = 0; j < coeffs_.size(); ++j)
      for (int i = first_; i <= last_ - 1; ++i)
      {
        const double d = (rows_[static_cast<std::size_t>(i + 1)][j].value(x) - rows_[static_cast<std::size_t>(i)][j].value(x)) -
                         targets_[j];
        s += (d * d) * coeffs_[j];
      }
    return s;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    out->addQuadExpr(expr_);
    return out;
  }
  VarVector getVars() override
  {
    VarVector v;
    for (auto& r : rows_)
      v.insert(v.end(), r.begin(), r.end());
    return v;
  }

private:
  std::vector<VarVector> rows_;
  DblVec coeffs_, targets_;
  int first_, last_;
  QuadExpr expr_;
};
// JointVelIneqCost (trajectory_costs.cpp:303-374): hinge rows
// -(upper - (vel - targ)) * c and (lower - (vel - targ)) * c per (step, joint)
class JointVelIneqCost : public Cost
{
public:
  JointVelIneqCost(std::vector<VarVector> rows, DblVec coeffs, DblVec targets, DblVec upper, DblVec lower,
                   int first_step, int last_step)
    : Cost("JointVelIneq")
    , rows_(std::move(rows))
    , coeffs_(std::move(coeffs))
    , targets_(std::move(targets))
    , upper_(std::move(upper))
    , lower_(std::move(lower))
    , first_(first_step)
    , last_(last_step)
  {
    if (((last_ - 1) - first_) < 0)
      throw std::runtime_error("JointVelIneqCost, trajectory is too short!");
    for (int i = first_; i <= last_ - 1; ++i)
      for (std::size_t j = 0; j < coeffs_.size(); ++j)
      {
        AffExpr vel, expr, expr_neg;
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i)][j], -1));
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i + 1)][j], 1));
        exprDec(vel, targets_[j]);
        exprInc(expr, upper_[j]);
        exprDec(expr, vel);
        exprScale(expr, -coeffs_[j]);
        exprs_.push_back(expr);
        exprInc(expr_neg, lower_[j]);
        exprDec(expr_neg, vel);
        exprScale(expr_neg, coeffs_[j]);
        exprs_.push_back(expr_neg);
      }
  }
  double value(const DblVec& x) override
  {
    double s1 = 0, s2 = 0;
    for (std::size_t j = 0; j < coeffs_.size(); ++j)
      for (int i = first_; i <= last_ - 1; ++i)
      {
        const double vel = rows_[static_cast<std::size_t>(i + 1)][j].value(x) - rows_[static_cast<std::size_t>(i)][j].value(x);
        const double d0 = vel - targets_[j];
        s1 += std::max((d0 - upper_[j]) * coeffs_[j], 0.0);
        s2 += std::max(((d0 * -1) + lower_[j]) * coeffs_[j], 0.0);
      }
    return s1 + s2;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    for (const AffExpr& e : exprs_)
      out->addHinge(e, 1);
    return out;
  }
  VarVector getVars() override
  {
    VarVector v;
    for (auto& r : rows_)
      v.insert(v.end(), r.begin(), r.end());
    return v;
  }
  // JointVelIneqConstraint::value (trajectory_costs.cpp:472-487): [diff1, diff2] hinged,
  // column-major over the [step x joint] blocks
  DblVec values(const DblVec& x) const
  {
    DblVec up, lo;
    for (std::size_t j = 0; j < coeffs_.size(); ++j)
      for (int i = first_; i <= last_ - 1; ++i)
      {
        const double vel = rows_[static_cast<std::size_t>(i + 1)][j].value(x) - rows_[static_cast<std::size_t>(i)][j].value(x);
        const double d0 = vel - targets_[j];
        up.push_back(std::max((d0 - upper_[j]) * coeffs_[j], 0.0));
        lo.push_back(std::max(((d0 * -1) + lower_[j]) * coeffs_[j], 0.0));
      }
    up.insert(up.end(), lo.begin(), lo.end());
    return up;
  }
  const AffExprVector& exprs() const { return exprs_; }

private:
  std::vector<VarVector> rows_;
  DblVec coeffs_, targets_, upper_, lower_;
  int first_, last_;
  AffExprVector exprs_;
};

// JointVelIneqConstraint (trajectory_costs.cpp:426-500): the same rows as
// JointVelIneqCost, as inequality constraints
class JointVelIneqConstraint : public Constraint
{
public:
  JointVelIneqConstraint(std::vector<VarVector> rows, DblVec coeffs, DblVec targets, DblVec upper, DblVec lower,
                         int first_step, int last_step)
    : Constraint("JointVelIneq"), rows_(rows, coeffs, targets, upper, lower, first_step, last_step)
  {
  }
  ConstraintType type() override { return INEQ; }
  DblVec value(const DblVec& x) override { return rows_.values(x); }
  ConvexConstraints::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    for (const AffExpr& e : rows_.exprs())
      out->addIneqCnt(e);
    return out;
  }
  VarVector getVars() override { return rows_.getVars(); }

private:
  JointVelIneqCost rows_;
};

// ------------------------------------------------------------ JointPos
// JointPosEqCost / JointPosIneqCost / JointPosEqConstraint / JointPosIneqConstraint
// (trajopt/src/trajectory_costs.cpp:28-254).  value() sums follow the Eigen
// expressions' element order only up to rounding (column-major over the
// [step x joint] block).
struct JointPosData
{
  std::vector<VarVector> rows;
  DblVec coeffs, targets, upper, lower;
  int first = 0, last = 0;
  double diff(const DblVec& x, int i, std::size_t j) const
  {
    return rows[static_cast<std::size_t>(i)][j].value(x) - targets[j];
  }
  VarVector vars() const
  {
    VarVector v;
    for (auto& r : rows)
      v.insert(v.end(), r.begin(), r.end());
    return v;
  }
  // expr_ / expr_vec_ of the ctors
  AffExpr pos(int i, std::size_t j) const
  {
    AffExpr p;
    exprInc(p, exprMult(rows[static_cast<std::size_t>(i)][j], 1));
    exprDec(p, targets[j]);
    return p;
  }
  AffExprVector ineqExprs() const
  {
    AffExprVector out;
    for (int i = first; i <= last; ++i)
      for (std::size_t j = 0; j < coeffs.size(); ++j)
      {
        const AffExpr p = pos(i, j);
        AffExpr e;  // (pos - upper_tol) * coeff
        exprInc(e, p);
        exprDec(e, upper[j]);
        exprScale(e, coeffs[j]);
        out.push_back(e);
        AffExpr en;  // (lower_tol - pos) * coeff
        exprInc(en, lower[j]);
        exprDec(en, p);
        exprScale(en, coeffs[j]);
        out.push_back(en);
      }
    return out;
  }
  // [diff1 | diff2] of the Ineq value(): (d - upper) c and (lower - d) c
  void ineqValues(const DblVec& x, DblVec& up, DblVec& lo) const
  {
    for (std::size_t j = 0; j < coeffs.size(); ++j)
      for (int i = first; i <= last; ++i)
      {
        const double d = diff(x, i, j);
        up.push_back((d - upper[j]) * coeffs[j]);
        lo.push_back(((d * -1) + lower[j]) * coeffs[j]);
      }
  }
};

class JointPosEqCost : public Cost
{
public:
  explicit JointPosEqCost(JointPosData d) : Cost("JointPosEq"), d_(std::move(d))
  {
    for (int i = d_.first; i <= d_.last; ++i)
      for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
        exprInc(expr_, exprMult(exprSquare(d_.pos(i, j)), d_.coeffs[j]));
  }
  double value(const DblVec& x) override
  {
    double s = 0;
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last; ++i)
      {
        const double dd = d_.diff(x, i, j);
        s += (dd * dd) * d_.coeffs[j];
      }
    return s;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    out->addQuadExpr(expr_);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointPosData d_;
  QuadExpr expr_;
};

class JointPosIneqCost : public Cost
{
public:
  explicit JointPosIneqCost(JointPosData d) : Cost("JointPosIneq"), d_(std::move(d)), exprs_(d_.ineqExprs()) {}
  double value(const DblVec& x) override
  {
    DblVec up, lo;
    d_.ineqValues(x, up, lo);
    double s1 = 0, s2 = 0;
    for (double v : up)
      s1 += std::max(v, 0.0);
    for (double v : lo)
      s2 += std::max(v, 0.0);
    return s1 + s2;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    for (const AffExpr& e : exprs_)
      out->addHinge(e, 1);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointPosData d_;
  AffExprVector exprs_;
};

class JointPosEqConstraint : public Constraint
{
public:
  explicit JointPosEqConstraint(JointPosData d) : Constraint("JointPosEq"), d_(std::move(d))
  {
    for (int i = d_.first; i <= d_.last; ++i)
      for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
        exprs_.push_back(exprMult(d_.pos(i, j), d_.coeffs[j]));
  }
  ConstraintType type() override { return EQ; }
  // quirk (trajectory_costs.cpp:162-171): the value is the *squared* error times coeff
  DblVec value(const DblVec& x) override
  {
    DblVec out;
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last; ++i)
      {
        const double dd = d_.diff(x, i, j);
        out.push_back((dd * dd) * d_.coeffs[j]);
      }
    return out;
  }
  ConvexConstraints::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    for (const AffExpr& e : exprs_)
      out->addEqCnt(e);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointPosData d_;
  AffExprVector exprs_;
};

class JointPosIneqConstraint : public Constraint
{
public:
  explicit JointPosIneqConstraint(JointPosData d)
    : Constraint("JointPosIneq"), d_(std::move(d)), exprs_(d_.ineqExprs())
  {
  }
  ConstraintType type() override { return INEQ; }
  DblVec value(const DblVec& x) override
  {
    DblVec up, lo;
    d_.ineqValues(x, up, lo);
    up.insert(up.end(), lo.begin(), lo.end());
    return up;
  }
  ConvexConstraints::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    for (const AffExpr& e : exprs_)
      out->addIneqCnt(e);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointPosData d_;
  AffExprVector exprs_;
};
}  // namespace

// JointPosTermInfo::hatch (problem_description.cpp:1097-1196) for term k of the descriptor.
static void addJointPosTerm(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d, int k,
                            const double* targets)
{
  const int N = d.n_steps, D = d.chain.n_dof;
  JointPosData jd;
  jd.rows = rows;
  jd.coeffs.assign(d.jpos_coeffs[k], d.jpos_coeffs[k] + D);
  jd.targets.assign(targets, targets + D);
  jd.upper.assign(d.jpos_upper_tols[k], d.jpos_upper_tols[k] + D);
  jd.lower.assign(d.jpos_lower_tols[k], d.jpos_lower_tols[k] + D);
  int first = d.jpos_first_step[k], last = d.jpos_last_step[k];
  if (last <= -1)
    last = N - 1;
  if ((N - 1) <= first)
    first = N - 1;
  if ((N - 1) <= last)
    last = N - 1;
  if (last < first)
    std::swap(first, last);
  jd.first = first;
  jd.last = last;
  bool zero_tols = true;  // trajopt_common::doubleEquals(tol, 0.)
  for (int j = 0; j < D; ++j)
    zero_tols = zero_tols && std::fabs(jd.upper[static_cast<std::size_t>(j)]) < 1e-5 &&
                std::fabs(jd.lower[static_cast<std::size_t>(j)]) < 1e-5;
  if (!d.jpos_is_cnt[k])
  {
    if (zero_tols)
      tp.prob->addCost(std::make_shared<JointPosEqCost>(jd));
    else
      tp.prob->addCost(std::make_shared<JointPosIneqCost>(jd));
  }
  else
  {
    if (zero_tols)
      tp.prob->addConstraint(std::make_shared<JointPosEqConstraint>(jd));
    else
      tp.prob->addConstraint(std::make_shared<JointPosIneqConstraint>(jd));
  }
}

// ------------------------------------------------------------ CartPose
void cartPoseIndices(const thip_problem_desc& d, int term, std::vector<int>& indices, DblVec& coeffs)
{
  indices.clear();
  coeffs.clear();
  for (int i = 0; i < 3; ++i)
    if (std::fabs(d.cart_pos_coeffs[term][i]) > 1e-5)
    {
      indices.push_back(i);
      coeffs.push_back(d.cart_pos_coeffs[term][i]);
    }
  for (int i = 0; i < 3; ++i)
    if (std::fabs(d.cart_rot_coeffs[term][i]) > 1e-5)
    {
      indices.push_back(i + 3);
      coeffs.push_back(d.cart_rot_coeffs[term][i]);
    }
}

void setCartPoseTolerances(const thip_problem_desc& d, int term, CartPoseCalc& c)
{
  c.has_tol = d.cart_has_tol[term] != 0;
  c.target_link = d.cart_target_link[term];
  for (int i = 0; i < 6; ++i)
  {
    c.lower_tol[i] = d.cart_lower_tol[term][i];
    c.upper_tol[i] = d.cart_upper_tol[term][i];
    if (c.has_tol && c.lower_tol[i] > c.upper_tol[i])
      throw std::runtime_error("CartPoseErrCalculator: Inverted tolerance band");
  }
}

DblVec CartPoseCalc::operator()(const DblVec& q) const
{
  std::vector<Iso3> fk;
  chainFwdKin(*chain, q.data(), fk);
  const Iso3 source_tf = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
  const Iso3 target_tf = mul(fk[static_cast<std::size_t>(target_link)], target_offset);
  double err[6];
  calcTransformError(target_tf, source_tf, err);
  if (has_tol)
    applyTolerances(err, lower_tol, upper_tol, 6);
  DblVec out(indices.size());
  for (std::size_t i = 0; i < indices.size(); ++i)
    out[i] = err[indices[i]];
  return out;
}

Mat CartPoseCalc::jac(const DblVec& q) const
{
  const double eps = 1e-5;
  std::vector<Iso3> fk;
  chainFwdKin(*chain, q.data(), fk);
  const Iso3 source_tf = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
  const Iso3 target_tf = mul(fk[static_cast<std::size_t>(target_link)], target_offset);
  Mat J(static_cast<int>(indices.size()), static_cast<int>(q.size()));
  DblVec qp = q;
  for (std::size_t i = 0; i < q.size(); ++i)
  {
    qp[i] = q[i] + eps;
    chainFwdKin(*chain, qp.data(), fk);
    const Iso3 sp = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
    // the static root frame does not move under the perturbation
    const Iso3 tp = target_link > 0 ? mul(fk[static_cast<std::size_t>(target_link)], target_offset) : target_tf;
    double diff[6];
    if (has_tol)
      calcJacobianTransformErrorDiffTol(target_tf, tp, source_tf, sp, lower_tol, upper_tol, diff);
    else
      calcJacobianTransformErrorDiff(target_tf, tp, source_tf, sp, diff);
    for (std::size_t r = 0; r < indices.size(); ++r)
    {
      J(static_cast<int>(r), static_cast<int>(i)) = diff[indices[r]] / eps;
      if (g_jitter.jac_abs > 0)  // parity-gate rounding jitter (jitter.hpp)
        J(static_cast<int>(r), static_cast<int>(i)) += g_jitter.jac_abs * jitterU();
    }
    qp[i] = q[i];
  }
  return J;
}

// ------------------------------------------------------------ JointVel cnt / JointAcc / JointJerk
// JointVelEqConstraint (trajectory_costs.cpp:376-424), JointAcc{Eq,Ineq}{Cost,
// Constraint} (:502-753), JointJerk{...} (:756-1016): the k-th forward difference
// of the trajectory (stencils [-1 1], [1 -2 1], [-1 3 -3 1], expressions built in
// the ctors' exprInc order), minus the target, per (step, joint), i-major.
// value(): Eigen's diffAxis0 applied k times (repeated differences), summed
// column-major.
struct JointDiffData
{
  std::vector<VarVector> rows;
  DblVec coeffs, targets, upper, lower;
  int order = 2, first = 0, last = 0;
  static const double* stencil(int order)
  {
    static const double s1[] = { -1, 1 }, s2[] = { 1, -2, 1 }, s3[] = { -1, 3, -3, 1 };
    return order == 1 ? s1 : order == 2 ? s2 : s3;
  }
  int count() const { return last - order - first + 1; }  // steps i = first .. last - order
  AffExpr diffExpr(int i, std::size_t j) const
  {
    AffExpr d;
    const double* st = stencil(order);
    for (int k = 0; k <= order; ++k)
      exprInc(d, exprMult(rows[static_cast<std::size_t>(i + k)][j], st[k]));
    exprDec(d, targets[j]);
    return d;
  }
  // (diffAxis0^order(traj block) - targets)[i - first][j]
  double diffValue(const DblVec& x, int i, std::size_t j) const
  {
    double v[4];
    for (int k = 0; k <= order; ++k)
      v[k] = rows[static_cast<std::size_t>(i + k)][j].value(x);
    for (int o = 0; o < order; ++o)
      for (int k = 0; k < order - o; ++k)
        v[k] = v[k + 1] - v[k];
    return v[0] - targets[j];
  }
  AffExprVector ineqExprs() const
  {
    AffExprVector out;
    for (int i = first; i <= last - order; ++i)
      for (std::size_t j = 0; j < coeffs.size(); ++j)
      {
        const AffExpr d = diffExpr(i, j);
        AffExpr up, lo;
        exprInc(up, upper[j]);  // -(upper_tol - (d - targ)) * coeff
        exprDec(up, d);
        exprScale(up, -coeffs[j]);
        out.push_back(up);
        exprInc(lo, lower[j]);  // (lower_tol - (d - targ)) * coeff
        exprDec(lo, d);
        exprScale(lo, coeffs[j]);
        out.push_back(lo);
      }
    return out;
  }
  VarVector vars() const
  {
    VarVector v;
    for (auto& r : rows)
      v.insert(v.end(), r.begin(), r.end());
    return v;
  }
  void check(const char* what) const
  {
    if (((last - order) - first) < 0)
      throw std::runtime_error(std::string(what) + ", trajectory is too short!");
  }
};

class JointDiffEqCost : public Cost
{
public:
  explicit JointDiffEqCost(JointDiffData d) : Cost(d.order == 2 ? "JointAccEq" : "JointJerkEq"), d_(std::move(d))
  {
    d_.check(d_.order == 2 ? "JointAccEqCost" : "JointJerkEqCost");
    for (int i = d_.first; i <= d_.last - d_.order; ++i)
      for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
        exprInc(expr_, exprMult(exprSquare(d_.diffExpr(i, j)), d_.coeffs[j]));
  }
  double value(const DblVec& x) override
  {
    double s = 0;
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last - d_.order; ++i)
      {
        const double v = d_.diffValue(x, i, j);
        s += (v * v) * d_.coeffs[j];
      }
    return s;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    out->addQuadExpr(expr_);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointDiffData d_;
  QuadExpr expr_;
};

// hinge form: upper/lower rows; value sums pospart of both blocks column-major
class JointDiffIneqCost : public Cost
{
public:
  explicit JointDiffIneqCost(JointDiffData d) : Cost(d.order == 2 ? "JointAccIneq" : "JointJerkIneq"), d_(std::move(d))
  {
    d_.check(d_.order == 2 ? "JointAccIneqCost" : "JointJerkIneqCost");
    exprs_ = d_.ineqExprs();
  }
  double value(const DblVec& x) override
  {
    double s1 = 0, s2 = 0;
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last - d_.order; ++i)
      {
        const double v = d_.diffValue(x, i, j);
        s1 += std::fmax((v - d_.upper[j]) * d_.coeffs[j], 0.0);
      }
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last - d_.order; ++i)
      {
        const double v = d_.diffValue(x, i, j);
        s2 += std::fmax(((v * -1) + d_.lower[j]) * d_.coeffs[j], 0.0);
      }
    return s1 + s2;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    for (const AffExpr& e : exprs_)
      out->addHinge(e, 1);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }
  const AffExprVector& exprs() const { return exprs_; }
  DblVec values(const DblVec& x) const
  {
    // [diff1 | diff2] flattened column-major, pospart (the IneqConstraint value)
    DblVec out;
    for (int blk = 0; blk < 2; ++blk)
      for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
        for (int i = d_.first; i <= d_.last - d_.order; ++i)
        {
          const double v = d_.diffValue(x, i, j);
          const double e = blk == 0 ? (v - d_.upper[j]) * d_.coeffs[j] : ((v * -1) + d_.lower[j]) * d_.coeffs[j];
          out.push_back(std::fmax(e, 0.0));
        }
    return out;
  }

private:
  JointDiffData d_;
  AffExprVector exprs_;
};

class JointDiffEqConstraint : public Constraint
{
public:
  explicit JointDiffEqConstraint(JointDiffData d)
    : Constraint(d.order == 1 ? "JointVelEq" : d.order == 2 ? "JointAccEq" : "JointJerkEq"), d_(std::move(d))
  {
    d_.check(d_.order == 1 ? "JointVelEqConstraint" : d_.order == 2 ? "JointAccEqConstraint" : "JointJerkEqConstraint");
    for (int i = d_.first; i <= d_.last - d_.order; ++i)
      for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
        exprs_.push_back(exprMult(d_.diffExpr(i, j), d_.coeffs[j]));
  }
  ConstraintType type() override { return EQ; }
  // quirk Q3: the value is the SQUARED difference times the coefficient (column-major)
  DblVec value(const DblVec& x) override
  {
    DblVec out;
    for (std::size_t j = 0; j < d_.coeffs.size(); ++j)
      for (int i = d_.first; i <= d_.last - d_.order; ++i)
      {
        const double v = d_.diffValue(x, i, j);
        out.push_back((v * v) * d_.coeffs[j]);
      }
    return out;
  }
  ConvexConstraints::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    for (const AffExpr& e : exprs_)
      out->addEqCnt(e);
    return out;
  }
  VarVector getVars() override { return d_.vars(); }

private:
  JointDiffData d_;
  AffExprVector exprs_;
};

class JointDiffIneqConstraint : public Constraint
{
public:
  explicit JointDiffIneqConstraint(JointDiffData d)
    : Constraint(d.order == 2 ? "JointAccIneq" : "JointJerkIneq"), rows_(std::move(d))
  {
  }
  ConstraintType type() override { return INEQ; }
  DblVec value(const DblVec& x) override { return rows_.values(x); }
  ConvexConstraints::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    for (const AffExpr& e : rows_.exprs())
      out->addIneqCnt(e);
    return out;
  }
  VarVector getVars() override { return rows_.getVars(); }

private:
  JointDiffIneqCost rows_;
};

void addJointDiffTerm(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d, int k)
{
  const int D = d.chain.n_dof;
  JointDiffData jd;
  jd.rows = rows;
  jd.order = d.jdt_order[k];
  jd.first = d.jdt_first_step[k];
  jd.last = d.jdt_last_step[k];
  jd.coeffs.assign(d.jdt_coeffs[k], d.jdt_coeffs[k] + D);
  jd.targets.assign(d.jdt_targets[k], d.jdt_targets[k] + D);
  jd.upper.assign(d.jdt_upper_tols[k], d.jdt_upper_tols[k] + D);
  jd.lower.assign(d.jdt_lower_tols[k], d.jdt_lower_tols[k] + D);
  bool zero = true;
  for (int j = 0; j < D; ++j)
    zero = zero && std::fabs(jd.upper[static_cast<std::size_t>(j)]) < 1e-5 &&
           std::fabs(jd.lower[static_cast<std::size_t>(j)]) < 1e-5;
  if (jd.order < 1 || jd.order > 3)
    throw std::runtime_error("jdt_order must be 1, 2 or 3");
  if (d.jdt_is_cnt[k])
  {
    if (zero)
      tp.prob->addConstraint(std::make_shared<JointDiffEqConstraint>(jd));
    else if (jd.order == 1)
      throw std::runtime_error("a JointVel tolerance constraint is a jvx term");
    else
      tp.prob->addConstraint(std::make_shared<JointDiffIneqConstraint>(jd));
  }
  else
  {
    if (jd.order == 1)
    {
      // a JointVel cost beyond the jv term: JointVelEqCost (trajectory_costs.cpp:257-301)
      // over the hatch-clamped steps (tolerance forms are jvx terms)
      if (!zero)
        throw std::runtime_error("a JointVel tolerance cost is a jvx term");
      tp.prob->addCost(std::make_shared<JointVelEqCost>(rows, jd.coeffs, jd.targets, jd.first, jd.last));
      return;
    }
    if (zero)
      tp.prob->addCost(std::make_shared<JointDiffEqCost>(jd));
    else
      tp.prob->addCost(std::make_shared<JointDiffIneqCost>(jd));
  }
}

// ------------------------------------------------------------ time-parameterised JointVel
// JointVelErrCalculator (kinematic_terms.cpp:434-449) over v = (x_first..x_last,
// dt_first..dt_last): vel_i = (x_{i+1} - x_i) * dt_{i+1}; the error is
// [-(upper - (vel - target)); lower - (vel - target)]
static DblVec jointVelTimeErr(const DblVec& v, double target, double upper, double lower)
{
  const int half = static_cast<int>(v.size() / 2), nv = half - 1;
  DblVec out(static_cast<std::size_t>(2 * nv));
  for (int i = 0; i < nv; ++i)
  {
    const double vel = (v[static_cast<std::size_t>(i + 1)] - v[static_cast<std::size_t>(i)]) *
                       v[static_cast<std::size_t>(half + i + 1)];
    out[static_cast<std::size_t>(i)] = -(upper - (vel - target));
    out[static_cast<std::size_t>(nv + i)] = lower - (vel - target);
  }
  return out;
}

// JointVelJacCalculator (kinematic_terms.cpp:451-475)
static Mat jointVelTimeJac(const DblVec& v)
{
  const int n = static_cast<int>(v.size()), half = n / 2, nv = half - 1;
  Mat J(2 * nv, n);
  for (int i = 0; i < nv; ++i)
  {
    const int ti = i + half + 1;
    J(i, i) = -1.0 * v[static_cast<std::size_t>(ti)];
    J(i, i + 1) = 1.0 * v[static_cast<std::size_t>(ti)];
    J(i, ti) = v[static_cast<std::size_t>(i + 1)] - v[static_cast<std::size_t>(i)];
  }
  for (int i = 0; i < nv; ++i)
    for (int c = 0; c < n; ++c)
      J(nv + i, c) = -J(i, c);
  return J;
}

// JointVelTermInfo::hatch with TT_USE_TIME (problem_description.cpp:1263-1344):
// one term per joint over (x_j, dt) on steps [first, last] (already clamped)
void addJointVelTimeTerm(TrajProblem& tp, const thip_problem_desc& d, int k)
{
  const int D = d.chain.n_dof, W = tp.n_cols;
  const int first = d.jvt_first_step[k], last = d.jvt_last_step[k];
  const int nv = last - first;
  bool zero = true;
  for (int j = 0; j < D; ++j)
    zero = zero && std::fabs(d.jvt_upper_tols[k][j]) < 1e-5 && std::fabs(d.jvt_lower_tols[k][j]) < 1e-5;
  for (int j = 0; j < D; ++j)
  {
    VarVector vars;
    for (int i = first; i <= last; ++i)
      vars.push_back(tp.traj_vars[static_cast<std::size_t>(i * W + j)]);
    for (int i = first; i <= last; ++i)
      vars.push_back(tp.traj_vars[static_cast<std::size_t>(i * W + D)]);
    const double targ = d.jvt_targets[k][j], up = d.jvt_upper_tols[k][j], lo = d.jvt_lower_tols[k][j];
    VectorOfVector f = [targ, up, lo](const DblVec& v) { return jointVelTimeErr(v, targ, up, lo); };
    MatrixOfVector dfdx = [](const DblVec& v) { return jointVelTimeJac(v); };
    const DblVec coeffs(static_cast<std::size_t>(nv * 2), d.jvt_coeffs[k][j]);
    const std::string name = "joint_vel_time_" + std::to_string(k) + "_j" + std::to_string(j);
    if (!d.jvt_is_cnt[k])
      tp.prob->addCost(std::make_shared<CostFromErrFunc>(f, dfdx, vars, coeffs, zero ? SQUARED : HINGE, name));
    else
      tp.prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(f, dfdx, vars, coeffs, zero ? EQ : INEQ, name));
  }
}

// ------------------------------------------------------------ TotalTime
// TotalTimeTermInfo::hatch (problem_description.cpp:1872-1913) over the last
// variable column of steps 1..N-1; TimeCostCalculator / TimeCostJacCalculator
// (kinematic_terms.cpp:579-591): sum(1/v) - limit, d/dv = -1/v^2
void addTotalTimeTerm(TrajProblem& tp, const thip_problem_desc& d, int k)
{
  const int N = tp.n_steps, W = tp.n_cols;
  VarVector vars;
  for (int i = 1; i < N; ++i)
    vars.push_back(tp.traj_vars[static_cast<std::size_t>(i * W + W - 1)]);
  const double limit = d.ttt_limit[k];
  VectorOfVector f = [limit](const DblVec& v) {
    double s = 0;
    for (double x : v)
      s += 1.0 / x;
    return DblVec{ s - limit };
  };
  MatrixOfVector dfdx = [](const DblVec& v) {
    Mat J(1, static_cast<int>(v.size()));
    for (int c = 0; c < static_cast<int>(v.size()); ++c)
      J(0, c) = -1.0 / (v[static_cast<std::size_t>(c)] * v[static_cast<std::size_t>(c)]);
    return J;
  };
  const bool zero = std::fabs(limit) < 1e-5;  // doubleEquals(limit, 0)
  const DblVec coeffs{ d.ttt_coeff[k] };
  const std::string name = "total_time_" + std::to_string(k);
  if (!d.ttt_is_cnt[k])
    tp.prob->addCost(std::make_shared<CostFromErrFunc>(f, dfdx, vars, coeffs, zero ? SQUARED : HINGE, name));
  else
    tp.prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(f, dfdx, vars, coeffs, zero ? EQ : INEQ, name));
}

// ------------------------------------------------------------ construction
TrajProblem constructProblem(const thip_problem_desc& d, const double* init_traj, const double* cart_targets,
                             const double* scene, const double* jpos_targets)
{
  auto jposTargets = [&](int k) {
    return jpos_targets ? jpos_targets + static_cast<std::size_t>(k) * d.chain.n_dof : d.jpos_targets[k];
  };
  TrajProblem tp;
  const int N = d.n_steps, D = d.chain.n_dof;
  tp.n_steps = N;
  tp.n_dof = D;
  tp.prob = std::make_shared<OptProb>(toOsqpSettings(d.osqp));
  // TrajOptProb ctor: variables j_i_j with joint-limit bounds, and with use_time
  // dt_i in [dt_lower, dt_upper] after each waypoint's joints
  // (problem_description.cpp:557-598); generateInitTraj appends the constant
  // init dt column (:372-379)
  const int ut = d.use_time ? 1 : 0, W = D + ut;
  tp.n_cols = W;
  std::vector<std::string> names;
  DblVec lb, ub;
  for (int i = 0; i < N; ++i)
  {
    for (int j = 0; j < D; ++j)
    {
      names.push_back("j_" + std::to_string(i) + "_" + std::to_string(j));
      lb.push_back(d.chain.lower[j]);
      ub.push_back(d.chain.upper[j]);
    }
    if (ut)
    {
      names.push_back("dt_" + std::to_string(i));
      lb.push_back(d.dt_lower);
      ub.push_back(d.dt_upper);
    }
  }
  tp.traj_vars = tp.prob->createVariables(names, lb, ub);
  for (int i = 0; i < N; ++i)
  {
    tp.init.insert(tp.init.end(), init_traj + i * D, init_traj + (i + 1) * D);
    if (ut)
      tp.init.push_back(d.init_dt);
  }
  std::vector<VarVector> rows(static_cast<std::size_t>(N));  // the joint variables of each waypoint
  for (int i = 0; i < N; ++i)
    rows[static_cast<std::size_t>(i)] =
        VarVector(tp.traj_vars.begin() + i * W, tp.traj_vars.begin() + i * W + D);

  // fixed timesteps: persistent linear equalities (problem_description.cpp:489-510)
  for (int f = 0; f < d.n_fixed; ++f)
  {
    const int t = d.fixed_steps[f];
    for (int j = 0; j < D; ++j)
      tp.prob->addLinearConstraint(exprSub(AffExpr(rows[static_cast<std::size_t>(t)][static_cast<std::size_t>(j)]),
                                           init_traj[t * D + j]),
                                   EQ);
  }
  // fixed dofs: the joint pinned to the initial trajectory at every step that is
  // not a fixed timestep (problem_description.cpp:528-546)
  for (int k = 0; k < d.n_fixed_dofs; ++k)
  {
    const int j = d.fixed_dofs[k];
    for (int i = 0; i < N; ++i)
    {
      bool fixed = false;
      for (int f = 0; f < d.n_fixed; ++f)
        fixed = fixed || d.fixed_steps[f] == i;
      if (fixed)
        continue;
      tp.prob->addLinearConstraint(exprSub(AffExpr(rows[static_cast<std::size_t>(i)][static_cast<std::size_t>(j)]),
                                           AffExpr(init_traj[i * D + j])),
                                   EQ);
    }
  }

  // cost_infos: JointVel, CartPose costs, collision cost
  if (d.jv_enabled)
  {
    int first = d.jv_first_step, last = d.jv_last_step;
    if (last <= -1)
      last = N - 1;
    if ((N - 2) <= first)
      first = N - 2;
    if ((N - 1) <= last)
      last = N - 1;
    if (last == first)
      last += 1;
    if (last < first)
      std::swap(first, last);
    bool zero_tols = true;
    for (int j = 0; j < D; ++j)
      zero_tols = zero_tols && std::fabs(d.jv_upper_tols[j]) < 1e-5 && std::fabs(d.jv_lower_tols[j]) < 1e-5;
    if (zero_tols)
      tp.prob->addCost(std::make_shared<JointVelEqCost>(rows, DblVec(d.jv_coeffs, d.jv_coeffs + D),
                                                        DblVec(d.jv_targets, d.jv_targets + D), first, last));
    else
      tp.prob->addCost(std::make_shared<JointVelIneqCost>(
          rows, DblVec(d.jv_coeffs, d.jv_coeffs + D), DblVec(d.jv_targets, d.jv_targets + D),
          DblVec(d.jv_upper_tols, d.jv_upper_tols + D), DblVec(d.jv_lower_tols, d.jv_lower_tols + D), first, last));
  }
  auto makeCalc = [&](int k) {
    auto calc = std::make_shared<CartPoseCalc>();
    calc->chain = &d.chain;
    calc->source_link = d.cart_source_link[k];
    calc->source_offset = Iso3::from12(d.cart_source_offset[k]);
    calc->target_offset = Iso3::from12(cart_targets + 12 * k);
    DblVec coeffs;
    cartPoseIndices(d, k, calc->indices, coeffs);
    setCartPoseTolerances(d, k, *calc);
    return std::make_pair(calc, coeffs);
  };
  for (int k = 0; k < d.n_cart; ++k)
  {
    if (d.cart_is_cnt[k])
      continue;
    auto [calc, coeffs] = makeCalc(k);
    tp.prob->addCost(std::make_shared<CostFromErrFunc>([calc](const DblVec& q) { return (*calc)(q); },
                                                       [calc](const DblVec& q) { return calc->jac(q); },
                                                       rows[static_cast<std::size_t>(d.cart_step[k])], coeffs, ABS,
                                                       "cart_pose_" + std::to_string(k)));
  }
  for (int k = 0; k < d.n_jpos; ++k)
    if (!d.jpos_is_cnt[k])
      addJointPosTerm(tp, rows, d, k, jposTargets(k));
  // further JointVel tolerance terms (JointVelTermInfo::hatch with tolerances,
  // problem_description.cpp:1346-1391), steps clamped as the first term's
  auto jvxArgs = [&](int x, int& first, int& last) {
    first = d.jvx_first_step[x];
    last = d.jvx_last_step[x];
    if (last <= -1)
      last = N - 1;
    if ((N - 2) <= first)
      first = N - 2;
    if ((N - 1) <= last)
      last = N - 1;
    if (last == first)
      last += 1;
    if (last < first)
      std::swap(first, last);
  };
  auto dv = [&](const double* p) { return DblVec(p, p + D); };
  for (int x = 0; x < d.n_jvx; ++x)
    if (!d.jvx_is_cnt[x])
    {
      int f, l;
      jvxArgs(x, f, l);
      tp.prob->addCost(std::make_shared<JointVelIneqCost>(rows, dv(d.jvx_coeffs[x]), dv(d.jvx_targets[x]),
                                                          dv(d.jvx_upper_tols[x]), dv(d.jvx_lower_tols[x]), f, l));
    }
  for (int k = 0; k < d.n_jdt; ++k)
    if (!d.jdt_is_cnt[k])
      addJointDiffTerm(tp, rows, d, k);
  for (int k = 0; k < d.n_jvt; ++k)
    if (!d.jvt_is_cnt[k])
      addJointVelTimeTerm(tp, d, k);
  for (int k = 0; k < d.n_ttt; ++k)
    if (!d.ttt_is_cnt[k])
      addTotalTimeTerm(tp, d, k);
  if (d.coll_enabled && !d.coll_is_cnt)
    addCollisionTerms(tp, rows, d, scene);
  for (int k = 0; k < d.n_coll_extra; ++k)  // further collision terms, in hatch order
    if (!d.coll_extra[k].is_cnt)
      addCollisionTerms(tp, rows, d, scene, 1 + k);
  // cnt_infos: CartPose constraints, collision constraint
  for (int k = 0; k < d.n_cart; ++k)
  {
    if (!d.cart_is_cnt[k])
      continue;
    auto [calc, coeffs] = makeCalc(k);
    tp.prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(
        [calc](const DblVec& q) { return (*calc)(q); }, [calc](const DblVec& q) { return calc->jac(q); },
        rows[static_cast<std::size_t>(d.cart_step[k])], coeffs, EQ, "cart_pose_cnt_" + std::to_string(k)));
  }
  for (int k = 0; k < d.n_jpos; ++k)
    if (d.jpos_is_cnt[k])
      addJointPosTerm(tp, rows, d, k, jposTargets(k));
  for (int x = 0; x < d.n_jvx; ++x)
    if (d.jvx_is_cnt[x])
    {
      int f, l;
      jvxArgs(x, f, l);
      tp.prob->addConstraint(std::make_shared<JointVelIneqConstraint>(
          rows, dv(d.jvx_coeffs[x]), dv(d.jvx_targets[x]), dv(d.jvx_upper_tols[x]), dv(d.jvx_lower_tols[x]), f, l));
    }
  for (int k = 0; k < d.n_jdt; ++k)
    if (d.jdt_is_cnt[k])
      addJointDiffTerm(tp, rows, d, k);
  for (int k = 0; k < d.n_jvt; ++k)
    if (d.jvt_is_cnt[k])
      addJointVelTimeTerm(tp, d, k);
  for (int k = 0; k < d.n_ttt; ++k)
    if (d.ttt_is_cnt[k])
      addTotalTimeTerm(tp, d, k);
  if (d.coll_enabled && d.coll_is_cnt)
    addCollisionTerms(tp, rows, d, scene);
  for (int k = 0; k < d.n_coll_extra; ++k)
    if (d.coll_extra[k].is_cnt)
      addCollisionTerms(tp, rows, d, scene, 1 + k);
  return tp;
}

}  // namespace orc
