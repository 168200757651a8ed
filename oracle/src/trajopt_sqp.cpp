// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// Restatement of the trajopt_sqp front end; file:line citations at each piece
// (the header lists the files).
#include "trajopt_sqp.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace orc
{
namespace tsqp
{
namespace
{
// trajopt_ifopt::isFinite (bounds.cpp:24)
bool isFiniteB(double v) { return std::isfinite(v) && v < 1e20 && v > -1e20; }
}  // namespace

// Bounds::updateType (bounds.cpp:74-84)
Bound::Bound(double l, double u) : lo(l), up(u)
{
  if (!isFiniteB(lo) && !isFiniteB(up))
    type = BoundsType::kUnbounded;
  else if (isFiniteB(lo) && isFiniteB(up))
    type = (std::abs(up - lo) < 1e-8) ? BoundsType::kEquality : BoundsType::kRangeBound;
  else
    type = isFiniteB(lo) ? BoundsType::kLowerBound : BoundsType::kUpperBound;
}

std::vector<double> Term::values(const std::vector<double>& x) const
{
  std::vector<double> v(static_cast<std::size_t>(rows));
  for (int r = 0; r < rows; ++r)
  {
    // the terms' getValues(): q2 - 2 q1 + q0, -q0 + 3 q1 - 3 q2 + q3, q1 - q0, q
    // (joint_*_constraint.cpp), evaluated left to right in the source's order
    const auto& c = cols[static_cast<std::size_t>(r)];
    const auto& ww = w[static_cast<std::size_t>(r)];
    double s = ww[0] * x[static_cast<std::size_t>(c[0])];
    for (std::size_t k = 1; k < c.size(); ++k)
      s += ww[k] * x[static_cast<std::size_t>(c[k])];
    v[static_cast<std::size_t>(r)] = s;
  }
  return v;
}

Rm Term::jacobian(int n_vars) const
{
  Rm j;
  j.rows = rows;
  j.cols = n_vars;
  for (int r = 0; r < rows; ++r)
  {
    // entries in ascending column order (insertBack)
    std::vector<std::pair<int, double>> e;
    for (std::size_t k = 0; k < cols[static_cast<std::size_t>(r)].size(); ++k)
      e.emplace_back(cols[static_cast<std::size_t>(r)][k], w[static_cast<std::size_t>(r)][k]);
    std::sort(e.begin(), e.end());
    for (const auto& p : e)
      j.push(p.first, p.second);
    j.endRow();
  }
  return j;
}

namespace
{
constexpr double kInf = std::numeric_limits<double>::infinity();

// coefficient expansion shared by the joint terms (joint_*_constraint.cpp ctors)
std::vector<double> expandCoeffs(const tsqp_term& t, int n_dof, int rows, double dflt)
{
  std::vector<double> c(static_cast<std::size_t>(rows));
  for (int r = 0; r < rows; ++r)
    c[static_cast<std::size_t>(r)] = (t.n_coeffs == 0)   ? dflt :
                                     (t.n_coeffs == 1) ? t.coeffs[0] :
                                                         t.coeffs[r % n_dof];
  return c;
}

Term makeTerm(const tsqp_spec& s, const tsqp_term& t)
{
  const int D = s.n_dof;
  for (int k = 0; k < t.n_coeffs; ++k)
    if (!(t.coeffs[k] > 0))
      throw std::runtime_error("coeff must be greater than zero.");
  if (t.n_coeffs != 0 && t.n_coeffs != 1 && t.n_coeffs != D)
    throw std::runtime_error("coeff must be the same size of the joint position.");
  Term m;
  if (t.kind == TSQP_JOINT_POS)
  {
    // JointPosConstraint (joint_position_constraint.cpp:78-137): a range bound
    // splits into [lo, inf) and (-inf, up] with the dof's coefficient twice
    m.name = "JointPos";
    const std::vector<double> c0 = expandCoeffs(t, D, D, 1.0);
    for (int i = 0; i < D; ++i)
    {
      const Bound b(t.lower[i], t.upper[i]);
      const int col = t.first * D + i;
      if (b.type == BoundsType::kRangeBound)
      {
        m.bounds.emplace_back(b.lo, kInf);
        m.bounds.emplace_back(-kInf, b.up);
        for (int u = 0; u < 2; ++u)
        {
          m.cols.push_back({ col });
          m.w.push_back({ 1.0 });
          m.coeffs.push_back(c0[static_cast<std::size_t>(i)]);
        }
      }
      else
      {
        m.bounds.push_back(b);
        m.cols.push_back({ col });
        m.w.push_back({ 1.0 });
        m.coeffs.push_back(c0[static_cast<std::size_t>(i)]);
      }
    }
    m.rows = static_cast<int>(m.cols.size());
    return m;
  }
  const int n = t.last - t.first + 1;  // position vars
  auto node = [&](int k) { return (t.first + k) * D; };
  if (t.kind == TSQP_JOINT_VEL)
  {
    // JointVelConstraint (joint_velocity_constraint.cpp:36-149): v = q_{s+1} - q_s
    if (n < 2)
      throw std::runtime_error("JointVelConstraint, requires minimum of three position variables!");
    m.name = "JointVel";
    m.rows = D * (n - 1);
    m.coeffs = expandCoeffs(t, D, m.rows, 5.0);
    for (int sgi = 0; sgi < n - 1; ++sgi)
      for (int k = 0; k < D; ++k)
      {
        m.cols.push_back({ node(sgi + 1) + k, node(sgi) + k });
        m.w.push_back({ 1.0, -1.0 });
        m.bounds.emplace_back(t.lower[k], t.lower[k]);
      }
    return m;
  }
  if (t.kind == TSQP_JOINT_ACC)
  {
    // JointAccelConstraint (joint_acceleration_constraint.cpp:36-175): forward
    // q2 - 2 q1 + q0 for i <= n - 3, backward for the last two
    if (n < 4)
      throw std::runtime_error("JointAccelConstraint requires a minimum of four position variables!");
    m.name = "JointAccel";
    m.rows = D * n;
    m.coeffs = expandCoeffs(t, D, m.rows, 1.0);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < D; ++k)
      {
        if (i < n - 2)
          m.cols.push_back({ node(i + 2) + k, node(i + 1) + k, node(i) + k });
        else
          m.cols.push_back({ node(i - 2) + k, node(i - 1) + k, node(i) + k });
        m.w.push_back({ 1.0, -2.0, 1.0 });
        m.bounds.emplace_back(t.lower[k], t.lower[k]);
      }
    return m;
  }
  if (t.kind == TSQP_JOINT_JERK)
  {
    // JointJerkConstraint (joint_jerk_constraint.cpp:36-184)
    if (n < 6)
      throw std::runtime_error("JointJerkConstraint requires a minimum of six position variables!");
    m.name = "JointJerk";
    m.rows = D * n;
    m.coeffs = expandCoeffs(t, D, m.rows, 1.0);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < D; ++k)
      {
        if (i < n - 3)
        {
          m.cols.push_back({ node(i) + k, node(i + 1) + k, node(i + 2) + k, node(i + 3) + k });
          m.w.push_back({ -1.0, 3.0, -3.0, 1.0 });
        }
        else
        {
          m.cols.push_back({ node(i) + k, node(i - 1) + k, node(i - 2) + k, node(i - 3) + k });
          m.w.push_back({ 1.0, -3.0, 3.0, -1.0 });
        }
        m.bounds.emplace_back(t.lower[k], t.lower[k]);
      }
    return m;
  }
  throw std::runtime_error("unknown term kind");
}

// calcBoundsViolations (ifopt_utils.cpp:122-145)
double violationSum(const std::vector<double>& v, const std::vector<Bound>& b, std::size_t off = 0)
{
  double s = 0;
  for (std::size_t i = 0; i < b.size(); ++i)
  {
    const double x = v[off + i];
    double e = 0;
    if (x < b[i].lo)
      e = std::abs(x - b[i].lo);
    else if (x > b[i].up)
      e = std::abs(x - b[i].up);
    s += e;
  }
  return s;
}

// row-major sparse product: res_r = sum over the row's entries in order
std::vector<double> rmMul(const Rm& a, const std::vector<double>& x)
{
  std::vector<double> r(static_cast<std::size_t>(a.rows), 0.0);
  for (int i = 0; i < a.rows; ++i)
  {
    double t = 0;
    for (int e = a.outer[static_cast<std::size_t>(i)]; e < a.outer[static_cast<std::size_t>(i) + 1]; ++e)
      t += a.val[static_cast<std::size_t>(e)] * x[static_cast<std::size_t>(a.inner[static_cast<std::size_t>(e)])];
    r[static_cast<std::size_t>(i)] = t;
  }
  return r;
}

struct Trip
{
  int r, c;
  double v;
};

// the convex problem of TrajOptQPProblem::convexify (trajopt_qp_problem.cpp:720-973)
struct Qp
{
  int n_nlp = 0, n_slack = 0, nv = 0, nc = 0, n_pen_rows = 0, n_merit_rows = 0;
  std::vector<Trip> A;       // constraint matrix triplets (setFromTriplets: unique here)
  std::vector<Trip> H;       // hessian (row-major, full symmetric)
  std::vector<double> g;     // gradient
  std::vector<double> lo, up;
  std::vector<double> cconst;  // constraint constants (rows of the penalty + merit terms)
  Rm Arm;                      // A row-major (rows of the penalty + merit terms)
  // squared objective (QuadExprs squared_objective_nlp)
  std::vector<double> sq_const;
  Rm sq_lin;                            // rows x n_nlp
  std::vector<std::vector<std::pair<int, double>>> sq_q;  // q_i rows
};

class Problem
{
public:
  Problem(const tsqp_spec& s) : spec_(s)
  {
    n_ = s.n_nodes * s.n_dof;
    x_.assign(s.init, s.init + n_);
    for (int i = 0; i < n_; ++i)
    {
      vlo_.push_back(s.var_lower[i % s.n_dof]);
      vup_.push_back(s.var_upper[i % s.n_dof]);
    }
    // setup(): objective (squared), penalty (hinge, then absolute), merit constraints
    for (int k = 0; k < s.n_terms; ++k)
    {
      const tsqp_term& t = s.terms[k];
      Term m = makeTerm(s, t);
      if (t.penalty == TSQP_SQUARED || t.penalty == TSQP_ABSOLUTE)
        for (const Bound& b : m.bounds)
          if (b.type != BoundsType::kEquality)
            throw std::runtime_error("TrajOpt Ifopt squared / absolute cost must have equality bounds!");
      if (t.penalty == TSQP_HINGE)
        for (const Bound& b : m.bounds)
          if (b.type != BoundsType::kLowerBound && b.type != BoundsType::kUpperBound)
            throw std::runtime_error("TrajOpt Ifopt hinge cost must have inequality bounds!");
      if (t.penalty == TSQP_SQUARED)
        sq_.push_back(m);
      else if (t.penalty == TSQP_HINGE)
        hinge_.push_back(m);
      else if (t.penalty == TSQP_ABSOLUTE)
        abs_.push_back(m);
      else
        cnt_.push_back(m);
    }
    pen_ = hinge_;
    pen_.insert(pen_.end(), abs_.begin(), abs_.end());
    box_.assign(static_cast<std::size_t>(n_), 1e-1);
    merit_.assign(cnt_.size(), 10.0);
  }
  int nNlp() const { return n_; }
  int nCnts() const { return static_cast<int>(cnt_.size()); }
  int nCosts() const { return static_cast<int>(sq_.size() + pen_.size()); }
  const std::vector<double>& x() const { return x_; }
  void setVariables(const double* x) { x_.assign(x, x + n_); }
  void setMerit(const std::vector<double>& m) { merit_ = m; }
  const std::vector<double>& box() const { return box_; }
  void setBox(const std::vector<double>& b)
  {
    box_ = b;
    updateBounds();
  }
  void scaleBox(double s)
  {
    for (double& b : box_)
      b = b * s;
    updateBounds();
  }
  const Qp& qp() const { return qp_; }

  // getExactCosts (trajopt_qp_problem.cpp:977-1020): squared costs sum(err^2 * coeff);
  // hinge / absolute costs sum(err) (coefficients not applied)
  std::vector<double> exactCosts() const
  {
    std::vector<double> c;
    for (const Term& t : sq_)
    {
      const std::vector<double> v = t.values(x_);
      double s = 0;
      for (int i = 0; i < t.rows; ++i)
      {
        const double x = v[static_cast<std::size_t>(i)];
        double e = 0;
        if (x < t.bounds[static_cast<std::size_t>(i)].lo)
          e = std::abs(x - t.bounds[static_cast<std::size_t>(i)].lo);
        else if (x > t.bounds[static_cast<std::size_t>(i)].up)
          e = std::abs(x - t.bounds[static_cast<std::size_t>(i)].up);
        s += (e * e) * t.coeffs[static_cast<std::size_t>(i)];
      }
      c.push_back(s);
    }
    for (const Term& t : pen_)
      c.push_back(violationSum(t.values(x_), t.bounds));
    return c;
  }
  std::vector<double> exactViolations() const
  {
    std::vector<double> v;
    for (const Term& t : cnt_)
      v.push_back(violationSum(t.values(x_), t.bounds));
    return v;
  }

  // convexify (trajopt_qp_problem.cpp:720-973)
  void convexify()
  {
    Qp q;
    q.n_nlp = n_;
    const std::vector<double>& x0 = x_;
    std::vector<double> slack_g;
    int row = 0, var = n_, mi = 0;
    std::vector<const Term*> cterms;
    for (const Term& t : pen_)
      cterms.push_back(&t);
    for (const Term& t : cnt_)
      cterms.push_back(&t);
    for (std::size_t ti = 0; ti < cterms.size(); ++ti)
    {
      const Term& t = *cterms[ti];
      const bool merit = ti >= pen_.size();
      if (t.rows == 0)
        continue;
      const Rm jac = t.jacobian(n_);
      const std::vector<double> val = t.values(x0);
      const std::vector<double> jx = rmMul(jac, x0);
      const double mc = merit ? merit_[static_cast<std::size_t>(mi++)] : 1.0;
      for (int k = 0; k < t.rows; ++k)
      {
        const double cc = val[static_cast<std::size_t>(k)] - jx[static_cast<std::size_t>(k)];
        q.cconst.push_back(cc);
        for (int e = jac.outer[static_cast<std::size_t>(k)]; e < jac.outer[static_cast<std::size_t>(k) + 1]; ++e)
        {
          const double v = jac.val[static_cast<std::size_t>(e)];
          q.A.push_back({ row + k, jac.inner[static_cast<std::size_t>(e)], std::abs(v) < 1e-7 ? 0.0 : v });
        }
        const Bound& b = t.bounds[static_cast<std::size_t>(k)];
        q.lo.push_back(b.lo - cc);
        q.up.push_back(b.up - cc);
        const double coeff = mc * t.coeffs[static_cast<std::size_t>(k)];
        if (b.type == BoundsType::kEquality)
        {
          slack_g.push_back(coeff);
          slack_g.push_back(coeff);
          q.A.push_back({ row + k, var++, 1.0 });
          q.A.push_back({ row + k, var++, -1.0 });
        }
        else if (b.type == BoundsType::kLowerBound)
        {
          slack_g.push_back(coeff);
          q.A.push_back({ row + k, var++, 1.0 });
        }
        else if (b.type == BoundsType::kUpperBound)
        {
          slack_g.push_back(coeff);
          q.A.push_back({ row + k, var++, -1.0 });
        }
        else
          throw std::runtime_error("Unsupported bounds type!");
      }
      if (merit)
        q.n_merit_rows += t.rows;
      else
        q.n_pen_rows += t.rows;
      row += t.rows;
    }
    q.n_slack = var - n_;
    q.nv = var;
    q.nc = row + q.nv;
    q.g.assign(static_cast<std::size_t>(q.nv), 0.0);
    for (int k = 0; k < q.n_slack; ++k)
      q.g[static_cast<std::size_t>(n_ + k)] = slack_g[static_cast<std::size_t>(k)];
    // squared costs (expressions.cpp:13-24, 26-102): each term's column sums and
    // Bw^T Bw (rows in order) first, then added to the running totals in term order
    std::vector<double> obj_lin(static_cast<std::size_t>(n_), 0.0);
    std::vector<std::pair<std::pair<int, int>, double>> htot;
    q.sq_lin.rows = 0;
    q.sq_lin.cols = n_;
    for (const Term& t : sq_)
    {
      const Rm jac = t.jacobian(n_);
      const std::vector<double> val = t.values(x0);
      const std::vector<double> jx = rmMul(jac, x0);
      // cache_aff_expr: constants = f - J x0, then target - constants, linear = -J
      std::vector<double> a(static_cast<std::size_t>(t.rows));
      for (int r = 0; r < t.rows; ++r)
        a[static_cast<std::size_t>(r)] =
            t.bounds[static_cast<std::size_t>(r)].lo - (val[static_cast<std::size_t>(r)] - jx[static_cast<std::size_t>(r)]);
      std::vector<double> tlin(static_cast<std::size_t>(n_), 0.0);
      std::vector<std::pair<std::pair<int, int>, double>> hent;
      for (int r = 0; r < t.rows; ++r)
      {
        const double wgt = t.coeffs[static_cast<std::size_t>(r)];
        const double ar = a[static_cast<std::size_t>(r)];
        q.sq_const.push_back((ar * ar) * wgt);
        const double sr = 2.0 * (ar * wgt);
        const double sw = std::sqrt(wgt);
        std::vector<std::pair<int, double>> qi;
        for (int e = jac.outer[static_cast<std::size_t>(r)]; e < jac.outer[static_cast<std::size_t>(r) + 1]; ++e)
        {
          const int c = jac.inner[static_cast<std::size_t>(e)];
          const double b = -jac.val[static_cast<std::size_t>(e)];
          const double lv = b * sr;
          q.sq_lin.push(c, lv);
          tlin[static_cast<std::size_t>(c)] += lv;
          qi.emplace_back(c, b * sw);
        }
        q.sq_lin.endRow();
        ++q.sq_lin.rows;
        for (const auto& e1 : qi)
          for (const auto& e2 : qi)
            hent.push_back({ { e1.first, e2.first }, e1.second * e2.second });
        q.sq_q.push_back(qi);
      }
      for (int j = 0; j < n_; ++j)
        obj_lin[static_cast<std::size_t>(j)] += tlin[static_cast<std::size_t>(j)];
      // this term's Bw^T Bw (sum over its rows in order), added to the total
      std::stable_sort(hent.begin(), hent.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      std::vector<std::pair<std::pair<int, int>, double>> acc;
      for (const auto& e : hent)
      {
        if (!acc.empty() && acc.back().first == e.first)
          acc.back().second += e.second;
        else
          acc.push_back(e);
      }
      std::vector<std::pair<std::pair<int, int>, double>> merged;
      std::size_t i1 = 0, i2 = 0;
      while (i1 < htot.size() || i2 < acc.size())
      {
        if (i2 >= acc.size() || (i1 < htot.size() && htot[i1].first < acc[i2].first))
          merged.push_back(htot[i1++]);
        else if (i1 >= htot.size() || acc[i2].first < htot[i1].first)
          merged.push_back(acc[i2++]);
        else
        {
          merged.push_back({ htot[i1].first, htot[i1].second + acc[i2].second });
          ++i1;
          ++i2;
        }
      }
      htot.swap(merged);
    }
    // the stored pattern keeps zeros (|v| < 1e-7 -> 0)
    for (const auto& e : htot)
      q.H.push_back({ e.first.first, e.first.second, std::abs(e.second) < 1e-7 ? 0.0 : e.second });
    for (int j = 0; j < n_; ++j)
      q.g[static_cast<std::size_t>(j)] = obj_lin[static_cast<std::size_t>(j)];
    // identity rows below the constraints; slack bounds [0, inf)
    for (int i = 0; i < q.nv; ++i)
      q.A.push_back({ row + i, i, 1.0 });
    q.lo.resize(static_cast<std::size_t>(q.nc), 0.0);
    q.up.resize(static_cast<std::size_t>(q.nc), kInf);
    for (int i = row + n_; i < q.nc; ++i)
    {
      q.lo[static_cast<std::size_t>(i)] = 0.0;
      q.up[static_cast<std::size_t>(i)] = kInf;
    }
    {
      // row-major copy of the term rows (entries in ascending column order)
      std::vector<Trip> t;
      for (const Trip& e : q.A)
        if (e.r < row)
          t.push_back(e);
      std::stable_sort(t.begin(), t.end(), [](const Trip& a, const Trip& b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
      q.Arm.rows = row;
      q.Arm.cols = q.nv;
      std::size_t k = 0;
      for (int r = 0; r < row; ++r)
      {
        for (; k < t.size() && t[k].r == r; ++k)
          q.Arm.push(t[k].c, t[k].v);
        q.Arm.endRow();
      }
    }
    qp_ = std::move(q);
    updateBounds();
  }

  // updateNLPVariableBounds (trajopt_qp_problem.cpp:1094-1118)
  void updateBounds()
  {
    if (qp_.nv == 0)
      return;
    const int idx = qp_.n_pen_rows + qp_.n_merit_rows;
    for (int i = 0; i < n_; ++i)
    {
      const double bi = box_[static_cast<std::size_t>(i)];
      const double lb = vlo_[static_cast<std::size_t>(i)], ub = vup_[static_cast<std::size_t>(i)];
      const double xi = std::clamp(x_[static_cast<std::size_t>(i)], lb, ub);
      qp_.lo[static_cast<std::size_t>(idx + i)] = std::max(xi - bi, lb);
      qp_.up[static_cast<std::size_t>(idx + i)] = std::min(xi + bi, ub);
    }
  }

  // ConvexProblem::evaluateConvexCosts (trajopt_qp_problem.cpp:131-200): squared
  // costs from the quadratic expressions at the nlp block, penalty costs from
  // the constraint rows at ALL QP variables (slacks included)
  std::vector<double> convexCosts(const std::vector<double>& v) const
  {
    std::vector<double> c;
    std::size_t r = 0;
    for (const Term& t : sq_)
    {
      double s = 0;
      for (int k = 0; k < t.rows; ++k, ++r)
      {
        double o = qp_.sq_const[r];
        double lin = 0;
        for (int e = qp_.sq_lin.outer[r]; e < qp_.sq_lin.outer[r + 1]; ++e)
          lin += qp_.sq_lin.val[static_cast<std::size_t>(e)] * v[static_cast<std::size_t>(qp_.sq_lin.inner[static_cast<std::size_t>(e)])];
        o += lin;
        double tq = 0.0;
        for (const auto& e : qp_.sq_q[r])
          tq += e.second * v[static_cast<std::size_t>(e.first)];
        o += tq * tq;
        s += o;
      }
      c.push_back(s);
    }
    int row = 0;
    for (const Term& t : pen_)
    {
      c.push_back(rowViolation(v, t, row, qp_.nv));
      row += t.rows;
    }
    return c;
  }
  // evaluateConvexConstraintViolations (:202-243): merit rows, nlp columns only
  std::vector<double> convexViolations(const std::vector<double>& v) const
  {
    std::vector<double> c;
    int row = qp_.n_pen_rows;
    for (const Term& t : cnt_)
    {
      c.push_back(rowViolation(v, t, row, n_));
      row += t.rows;
    }
    return c;
  }

private:
  // violation sum of rows [row, row + t.rows) of constant + A x over columns < ncols
  double rowViolation(const std::vector<double>& v, const Term& t, int row, int ncols) const
  {
    std::vector<double> val(static_cast<std::size_t>(t.rows));
    for (int k = 0; k < t.rows; ++k)
    {
      double s = 0;
      const Rm& A = qp_.Arm;
      for (int e = A.outer[static_cast<std::size_t>(row + k)]; e < A.outer[static_cast<std::size_t>(row + k) + 1]; ++e)
        if (A.inner[static_cast<std::size_t>(e)] < ncols)
          s += A.val[static_cast<std::size_t>(e)] * v[static_cast<std::size_t>(A.inner[static_cast<std::size_t>(e)])];
      val[static_cast<std::size_t>(k)] = qp_.cconst[static_cast<std::size_t>(row + k)] + s;
    }
    return violationSum(val, t.bounds);
  }
  tsqp_spec spec_;
  int n_ = 0;
  std::vector<double> x_, vlo_, vup_, box_, merit_;
  std::vector<Term> sq_, hinge_, abs_, pen_, cnt_;
  Qp qp_;
};

// CSC (column-major, rows ascending) of triplets restricted by `keep`
Csc toCsc(int m, int n, const std::vector<Trip>& t, bool upper_only, double scale)
{
  std::vector<std::vector<std::pair<int, double>>> col(static_cast<std::size_t>(n));
  for (const Trip& e : t)
    if (!upper_only || e.r <= e.c)
      col[static_cast<std::size_t>(e.c)].emplace_back(e.r, e.v * scale);
  Csc c;
  c.m = m;
  c.n = n;
  c.p.assign(static_cast<std::size_t>(n) + 1, 0);
  for (int j = 0; j < n; ++j)
  {
    auto& cc = col[static_cast<std::size_t>(j)];
    std::stable_sort(cc.begin(), cc.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& e : cc)
    {
      c.i.push_back(e.first);
      c.x.push_back(e.second);
    }
    c.p[static_cast<std::size_t>(j) + 1] = static_cast<OsqpInt>(c.i.size());
  }
  return c;
}

OsqpSettings toSettings(const thip_osqp_settings& s)
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

// OSQPEigenSolver over OsqpEigen::Solver (osqp_eigen_solver.cpp:38-326)
class EigenSolverLike
{
public:
  explicit EigenSolverLike(const thip_osqp_settings& s) : settings_(toSettings(s)) {}
  int status = 0;  // 0 uninitialized, 1 initialized, 2 failed
  int setups = 0, updates = 0, solves = 0;
  long long admm = 0;

  void clear()
  {
    initialized_ = false;
    status = 0;
  }
  void init(int nv, int nc)
  {
    nv_ = nv;
    nc_ = nc;
    x0_.assign(static_cast<std::size_t>(nv), 0.0);
    y0_.assign(static_cast<std::size_t>(nc), 0.0);
    status = 1;
  }
  // the data of one convexification; in place when the solver exists and the
  // patterns are unchanged (OsqpEigen::Solver::updateHessianMatrix /
  // updateLinearConstraintsMatrix: osqp_update_data_mat, else a new setup that keeps
  // the primal / dual solution)
  bool setData(const Qp& q, bool in_place)
  {
    P_ = toCsc(q.nv, q.nv, q.H, true, 2.0);  // OSQPEigenSolver::updateHessianMatrix: 2 H
    A_ = toCsc(q.nc, q.nv, q.A, false, 1.0);
    g_.assign(q.g.begin(), q.g.end());
    for (double& v : g_)
      if (std::abs(v) < 1e-7)
        v = 0.0;
    setBounds(q);
    if (!in_place)
      return true;
    if (!initialized_)
      return false;  // OsqpEigen: no solver to update -> the caller rebuilds
    const bool same = P_.p == oP_.p && P_.i == oP_.i && A_.p == oA_.p && A_.i == oA_.i;
    if (!same)
    {
      // pattern changed: a new solver warm started from the last solution
      const std::vector<double> xs = osqp_.sol_x, ys = osqp_.sol_y;
      if (setupNow())
        osqp_.warm_start(xs.data(), ys.data());
      return true;
    }
    ++updates;
    // updateHessianMatrix, updateGradient, updateLinearConstraintsMatrix, updateBounds
    if (osqp_.update_data_mat(P_.x.data(), nullptr) != 0 || osqp_.update_data_vec(g_.data(), nullptr, nullptr) != 0 ||
        osqp_.update_data_mat(nullptr, A_.x.data()) != 0)
    {
      initialized_ = false;
      return false;
    }
    updateBoundsNow();
    oP_ = P_;
    oA_ = A_;
    return true;
  }
  void setBounds(const Qp& q)
  {
    lo_.assign(q.lo.begin(), q.lo.end());
    up_.assign(q.up.begin(), q.up.end());
    for (double& v : lo_)
      v = std::max(v, -OSQP_INFTY);
    for (double& v : up_)
      v = std::min(v, OSQP_INFTY);
  }
  void updateBoundsNow()
  {
    if (initialized_)
      osqp_.update_data_vec(nullptr, lo_.data(), up_.data());
  }
  // setWarmStart (osqp_eigen_solver.cpp:267-324): x0 = [nlp vars; slacks from the
  // merit violations], y0 = 0
  void setWarmStart(const Problem& p)
  {
    const int nn = p.nNlp();
    x0_.assign(static_cast<std::size_t>(nv_), 0.0);
    for (int i = 0; i < nn; ++i)
      x0_[static_cast<std::size_t>(i)] = p.x()[static_cast<std::size_t>(i)];
    if (nv_ > nn)
    {
      const std::vector<double> viol = p.convexViolations(p.x());
      // (the reference walks constraint-matrix row k for violation k)
      const Rm& A = p.qp().Arm;
      for (std::size_t k = 0; k < viol.size() && static_cast<int>(k) < A.rows; ++k)
        for (int e = A.outer[k]; e < A.outer[k + 1]; ++e)
          if (A.inner[static_cast<std::size_t>(e)] >= nn && std::abs(A.val[static_cast<std::size_t>(e)]) > 1e-14)
            x0_[static_cast<std::size_t>(A.inner[static_cast<std::size_t>(e)])] =
                std::max(0.0, viol[k] / A.val[static_cast<std::size_t>(e)]);
    }
    y0_.assign(static_cast<std::size_t>(nc_), 0.0);
  }
  bool solve()
  {
    if (!initialized_)
    {
      if (!setupNow())
      {
        status = 2;
        return false;
      }
      if (settings_.warm_starting == 1)
        osqp_.warm_start(x0_.data(), y0_.data());
    }
    osqp_.solve();
    ++solves;
    admm += osqp_.iter;
    const int st = osqp_.status_val;
    if (st == OSQP_SOLVED || st == OSQP_SOLVED_INACCURATE)
      return true;
    status = 2;
    return false;
  }
  const std::vector<double>& solution() const { return osqp_.sol_x; }

private:
  bool setupNow()
  {
    ++setups;
    initialized_ = osqp_.setup(P_, g_.data(), A_, lo_.data(), up_.data(), nc_, nv_, settings_) == 0;
    oP_ = P_;
    oA_ = A_;
    return initialized_;
  }
  OsqpSettings settings_;
  OsqpSolver osqp_;
  bool initialized_ = false;
  int nv_ = 0, nc_ = 0;
  Csc P_, A_, oP_, oA_;
  std::vector<double> g_, lo_, up_, x0_, y0_;
};
}  // namespace

// TrustRegionSQPSolver::solve (trust_region_sqp_solver.cpp:84-168) with
// stepSQPSolver (:202-260), runTrustRegionLoop (:262-383), solveQPProblem
// (:385-470), adjustPenalty (:180-200)
Result solve(const tsqp_spec& s)
{
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now();
  Problem prob(s);
  EigenSolverLike qps(s.osqp);
  Result res;
  int status = TSQP_STATUS_RUNNING;
  // init (:44-64)
  std::vector<double> best_x = prob.x();
  std::vector<double> merit(static_cast<std::size_t>(prob.nCnts()), s.initial_merit_error_coeff);
  std::vector<double> best_costs = prob.exactCosts(), best_viol = prob.exactViolations();
  std::vector<double> new_x, new_costs, new_viol;
  prob.setBox(std::vector<double>(static_cast<std::size_t>(prob.nNlp()), s.initial_trust_box_size));
  auto sum = [](const std::vector<double>& v) {
    double a = 0;
    for (double e : v)
      a += e;
    return a;
  };
  auto dot = [](const std::vector<double>& a, const std::vector<double>& b) {
    double r = 0;
    for (std::size_t i = 0; i < a.size(); ++i)
      r += a[i] * b[i];
    return r;
  };
  auto maxv = [](const std::vector<double>& v) {
    double m = -std::numeric_limits<double>::infinity();
    for (double e : v)
      m = std::max(m, e);
    return m;
  };
  prob.setMerit(merit);
  double best_merit = sum(best_costs) + dot(best_viol, merit);
  int overall = 0, prev_nv = 0, prev_nc = 0;
  double approx_improve = 0, exact_improve = 0, ratio = 0, new_merit = 0;
  auto box_max = [&]() { return maxv(prob.box()); };

  auto solveQp = [&]() -> int {
    if (!qps.solve())
    {
      prob.setVariables(best_x.data());
      return TSQP_STATUS_QP_SOLVE_FAILED;
    }
    new_x = qps.solution();
    prob.setVariables(new_x.data());
    const std::vector<double> av = prob.convexViolations(new_x);
    const std::vector<double> ac = prob.convexCosts(new_x);
    const double approx_merit = sum(ac) + dot(av, merit);
    approx_improve = best_merit - approx_merit;
    new_costs = prob.exactCosts();
    new_viol = prob.exactViolations();
    new_merit = sum(new_costs) + dot(new_viol, merit);
    exact_improve = best_merit - new_merit;
    ratio = (std::abs(approx_improve) < 1e-12) ? 0.0 : exact_improve / approx_improve;
    prob.setVariables(best_x.data());
    return TSQP_STATUS_RUNNING;
  };

  auto trustLoop = [&]() {
    int failures = 0;
    while (box_max() >= s.min_trust_box_size)
    {
      ++overall;
      status = solveQp();
      if (status != TSQP_STATUS_RUNNING)
      {
        ++failures;
        if (failures < s.max_qp_solver_failures)
        {
          prob.scaleBox(s.trust_shrink_ratio);
          qps.setBounds(prob.qp());
          qps.updateBoundsNow();
          continue;
        }
        if (failures == s.max_qp_solver_failures)
        {
          prob.setBox(std::vector<double>(static_cast<std::size_t>(prob.nNlp()), s.min_trust_box_size));
          qps.setBounds(prob.qp());
          qps.updateBoundsNow();
          continue;
        }
        return;
      }
      if (approx_improve < s.min_approx_improve)
      {
        status = TSQP_STATUS_CONVERGED;
        return;
      }
      const double denom = std::max(std::abs(best_merit), 1e-12);
      if (approx_improve / denom < s.min_approx_improve_frac)
      {
        status = TSQP_STATUS_CONVERGED;
        return;
      }
      if (exact_improve < 0 || ratio < s.improve_ratio_threshold)
      {
        prob.scaleBox(s.trust_shrink_ratio);
        qps.setBounds(prob.qp());
        qps.updateBoundsNow();
      }
      else
      {
        best_x = new_x;
        best_x.resize(static_cast<std::size_t>(prob.nNlp()));
        best_merit = new_merit;
        best_viol = new_viol;
        best_costs = new_costs;
        prob.setVariables(best_x.data());
        prob.scaleBox(s.trust_expand_ratio);
        qps.setBounds(prob.qp());
        qps.updateBoundsNow();
        return;
      }
    }
  };

  auto step = [&]() -> bool {
    prob.convexify();
    const int nv = prob.qp().nv, nc = prob.qp().nc;
    const bool first = qps.status == 0;
    const bool dims = nv != prev_nv || nc != prev_nc;
    prev_nv = nv;
    prev_nc = nc;
    if (first || dims)
    {
      qps.clear();
      qps.init(nv, nc);
      qps.setData(prob.qp(), false);
      qps.setWarmStart(prob);
    }
    else if (!qps.setData(prob.qp(), true))
    {
      // update in place failed: full rebuild (trust_region_sqp_solver.cpp:229-243)
      qps.clear();
      qps.init(nv, nc);
      qps.setData(prob.qp(), false);
      qps.setWarmStart(prob);
    }
    trustLoop();
    if (status == TSQP_STATUS_CONVERGED)
      return true;
    if (box_max() < s.min_trust_box_size)
    {
      status = TSQP_STATUS_CONVERGED;
      return true;
    }
    return false;
  };

  int penalty = 0;
  for (penalty = 0; penalty < s.max_merit_coeff_increases; ++penalty)
  {
    res.penalty_iteration = penalty;
    for (int ci = 1; ci < 100; ++ci)
    {
      const double el = std::chrono::duration<double>(Clock::now() - t0).count();
      if (el > s.max_time)
      {
        status = TSQP_STATUS_TIME_LIMIT;
        break;
      }
      if (overall >= s.max_iterations)
      {
        status = TSQP_STATUS_ITERATION_LIMIT;
        break;
      }
      if (step())
        break;
    }
    if (best_viol.empty() || maxv(best_viol) < s.cnt_tolerance)
    {
      status = TSQP_STATUS_CONVERGED;
      break;
    }
    if (status == TSQP_STATUS_ITERATION_LIMIT || status == TSQP_STATUS_TIME_LIMIT)
      break;
    status = TSQP_STATUS_RUNNING;
    // adjustPenalty
    if (s.inflate_constraints_individually)
    {
      for (std::size_t i = 0; i < best_viol.size(); ++i)
        if (best_viol[i] > s.cnt_tolerance)
          merit[i] *= s.merit_coeff_increase_ratio;
    }
    else
      for (double& m : merit)
        m *= s.merit_coeff_increase_ratio;
    prob.setBox(std::vector<double>(static_cast<std::size_t>(prob.nNlp()),
                                    std::fmax(prob.box()[0], s.min_trust_box_size / s.trust_shrink_ratio * 1.5)));
    prob.setMerit(merit);
    best_merit = sum(best_costs) + dot(best_viol, merit);
  }
  if (status == TSQP_STATUS_RUNNING)
    status = TSQP_STATUS_PENALTY_ITERATION_LIMIT;
  prob.setVariables(best_x.data());
  res.x = best_x;
  res.status = status;
  res.overall_iteration = overall;
  res.qp_setups = qps.setups;
  res.qp_updates = qps.updates;
  res.qp_solves = qps.solves;
  res.admm_iters = qps.admm;
  res.best_exact_merit = best_merit;
  return res;
}

}  // namespace tsqp
}  // namespace orc
