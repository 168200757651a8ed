// trajopt_sqp::TrajOptQPProblem: behaviour of
// trajopt_optimizers/trajopt_sqp/src/trajopt_qp_problem.cpp (ConvexProblem
// evaluation :131-243, setup / update :405-698, convexify :720-973, exact
// values :975-1044, trust box :1046-1118) and of the squared-cost expressions
// (src/expressions.cpp:6-102: AffExprs::create / square, QuadExprs::values).
#include "trajopt_sqp/trajopt_qp_problem.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <map>
#include <stdexcept>

#include "trajopt_ifopt/utils/ifopt_utils.h"

namespace trajopt_sqp
{
using trajopt_ifopt::BoundsType;
using trajopt_ifopt::ConstraintSet;
using trajopt_ifopt::Jacobian;

namespace
{
constexpr double kInf = std::numeric_limits<double>::infinity();

// row-major product J x (each row summed over its entries in order)
VectorXd mul(const Jacobian& J, const VectorXd& x)
{
  VectorXd r(static_cast<std::size_t>(J.rows()), 0.0);
  for (long i = 0; i < J.rows(); ++i)
  {
    double t = 0;
    for (long e = J.rowBegin(i); e < J.rowEnd(i); ++e)
      t += J.value(e) * x[static_cast<std::size_t>(J.col(e))];
    r[static_cast<std::size_t>(i)] = t;
  }
  return r;
}

struct Entry
{
  long r, c;
  double v;
};

// row-major matrix from entries with unique (row, col) (Eigen setFromTriplets)
Jacobian fromEntries(long rows, long cols, std::vector<Entry> e)
{
  std::stable_sort(e.begin(), e.end(), [](const Entry& a, const Entry& b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
  Jacobian J(rows, cols);
  J.reserve(static_cast<long>(e.size()));
  std::size_t k = 0;
  for (long r = 0; r < rows; ++r)
  {
    J.startVec(r);
    for (; k < e.size() && e[k].r == r; ++k)
      J.insertBack(r, e[k].c) = e[k].v;
  }
  J.finalize();
  return J;
}
}  // namespace

struct TrajOptQPProblem::Impl
{
  std::shared_ptr<trajopt_ifopt::NodesVariables> variables;
  std::vector<std::shared_ptr<ConstraintSet>> squared, hinge, absolute, constraints;
  std::vector<std::shared_ptr<ConstraintSet>> penalty;  // hinge then absolute costs
  std::vector<std::string> cost_names, cnt_names;
  bool initialized = false;
  long n_nlp = 0, n_slack = 0, n_qp_vars = 0, n_qp_cnts = 0, n_pen_rows = 0, n_merit_rows = 0;
  VectorXd box, merit, var_lo, var_up;
  // the convex problem
  Jacobian hessian, cmat;
  VectorXd gradient, lo, up, cconst;
  // squared objective: per row constant, linear row (NLP columns), q_i row
  VectorXd sq_const;
  Jacobian sq_lin;
  std::vector<std::vector<std::pair<long, double>>> sq_q;

  void updateNLPVariableBounds(const VectorXd& x)
  {
    const long idx = n_pen_rows + n_merit_rows;
    if (static_cast<long>(lo.size()) < idx + n_nlp)
      return;
    for (long i = 0; i < n_nlp; ++i)
    {
      const auto u = static_cast<std::size_t>(i);
      const double xi = std::clamp(x[u], var_lo[u], var_up[u]);
      lo[static_cast<std::size_t>(idx + i)] = std::max(xi - box[u], var_lo[u]);
      up[static_cast<std::size_t>(idx + i)] = std::min(xi + box[u], var_up[u]);
    }
  }

  // violation sum of matrix rows [row, row + rows) + constant over columns < ncols
  double rowsViolation(const VectorXd& v, const ConstraintSet& t, long row, long ncols) const
  {
    VectorXd val(static_cast<std::size_t>(t.getRows())), err;
    for (long k = 0; k < t.getRows(); ++k)
    {
      double s = 0;
      for (long e = cmat.rowBegin(row + k); e < cmat.rowEnd(row + k); ++e)
        if (cmat.col(e) < ncols)
          s += cmat.value(e) * v[static_cast<std::size_t>(cmat.col(e))];
      val[static_cast<std::size_t>(k)] = cconst[static_cast<std::size_t>(row + k)] + s;
    }
    trajopt_ifopt::calcBoundsViolations(err, val, t.getBounds());
    double a = 0;
    for (double e : err)
      a += e;
    return a;
  }
};

TrajOptQPProblem::TrajOptQPProblem(std::shared_ptr<trajopt_ifopt::NodesVariables> variables)
  : impl_(std::make_unique<Impl>())
{
  impl_->variables = std::move(variables);
}
TrajOptQPProblem::~TrajOptQPProblem() = default;

void TrajOptQPProblem::addConstraintSet(std::shared_ptr<ConstraintSet> constraint_set)
{
  constraint_set->linkWithVariables(impl_->variables);
  impl_->constraints.push_back(std::move(constraint_set));
  impl_->initialized = false;
}

void TrajOptQPProblem::addCostSet(std::shared_ptr<ConstraintSet> constraint_set, CostPenaltyType penalty_type)
{
  constraint_set->linkWithVariables(impl_->variables);
  const auto bounds = constraint_set->getBounds();
  switch (penalty_type)
  {
    case CostPenaltyType::kSquared:
      for (const auto& b : bounds)
        if (b.getType() != BoundsType::kEquality)
          throw std::runtime_error("TrajOpt Ifopt squared cost must have equality bounds!");
      impl_->squared.push_back(std::move(constraint_set));
      break;
    case CostPenaltyType::kAbsolute:
      for (const auto& b : bounds)
        if (b.getType() != BoundsType::kEquality)
          throw std::runtime_error("TrajOpt Ifopt absolute cost must have equality bounds!");
      impl_->absolute.push_back(std::move(constraint_set));
      break;
    case CostPenaltyType::kHinge:
      for (const auto& b : bounds)
        if (b.getType() != BoundsType::kLowerBound && b.getType() != BoundsType::kUpperBound)
          throw std::runtime_error("TrajOpt Ifopt hinge cost must have inequality bounds!");
      impl_->hinge.push_back(std::move(constraint_set));
      break;
  }
  impl_->initialized = false;
}

void TrajOptQPProblem::setup()
{
  Impl& I = *impl_;
  I.penalty = I.hinge;
  I.penalty.insert(I.penalty.end(), I.absolute.begin(), I.absolute.end());
  for (auto* v : { &I.squared, &I.penalty, &I.constraints })
    for (auto& c : *v)
      c->update();
  I.n_nlp = I.variables->getRows();
  I.box.assign(static_cast<std::size_t>(I.n_nlp), 1e-1);
  I.cost_names.clear();
  for (const auto& c : I.squared)
    I.cost_names.push_back(c->getName());
  for (const auto& c : I.penalty)
    I.cost_names.push_back(c->getName());
  I.cnt_names.clear();
  for (const auto& c : I.constraints)
    I.cnt_names.push_back(c->getName());
  I.merit.assign(I.constraints.size(), 10.0);
  I.var_lo.clear();
  I.var_up.clear();
  for (const auto& b : I.variables->getBounds())
  {
    I.var_lo.push_back(b.getLower());
    I.var_up.push_back(b.getUpper());
  }
  I.initialized = true;
}

void TrajOptQPProblem::setVariables(const double* x)
{
  Impl& I = *impl_;
  const std::size_t h = I.variables->getHash();
  I.variables->setVariables(VectorXd(x, x + I.n_nlp));
  if (h == I.variables->getHash())
    return;  // unchanged: no term update
  for (auto* v : { &I.squared, &I.penalty, &I.constraints })
    for (auto& c : *v)
      c->update();
}

VectorXd TrajOptQPProblem::getVariableValues() const { return impl_->variables->getValues(); }

void TrajOptQPProblem::convexify()
{
  Impl& I = *impl_;
  if (!I.initialized)
    throw std::runtime_error("TrajOptQPProblem::convexify: call setup() first");
  const VectorXd x0 = I.variables->getValues();
  std::vector<Entry> a;
  VectorXd slack_g;
  I.lo.clear();
  I.up.clear();
  I.cconst.clear();
  long row = 0, var = I.n_nlp;
  std::size_t merit_idx = 0;
  I.n_pen_rows = I.n_merit_rows = 0;
  // hinge / absolute cost rows, then the constraint rows: the linearisation with
  // its constant (value - J x0, the merit's model), bounds relative to it and
  // the row's slack variables
  for (int pass = 0; pass < 2; ++pass)
  {
    const auto& terms = (pass == 0) ? I.penalty : I.constraints;
    for (const auto& t : terms)
    {
      if (t->getRows() == 0)
        continue;
      const Jacobian jac = t->getJacobian();
      const VectorXd val = t->getValues(), jx = mul(jac, x0), coeffs = t->getCoefficients();
      const auto bounds = t->getBounds();
      const double mc = (pass == 1) ? I.merit[merit_idx++] : 1.0;
      for (long k = 0; k < jac.outerSize(); ++k)
      {
        const auto uk = static_cast<std::size_t>(k);
        for (long e = jac.rowBegin(k); e < jac.rowEnd(k); ++e)
          a.push_back({ row + k, jac.col(e), std::abs(jac.value(e)) < 1e-7 ? 0.0 : jac.value(e) });  // kept as zeros
        const double cc = val[uk] - jx[uk];
        I.cconst.push_back(cc);
        I.lo.push_back(bounds[uk].getLower() - cc);
        I.up.push_back(bounds[uk].getUpper() - cc);
        const double coeff = mc * coeffs[uk];
        switch (bounds[uk].getType())
        {
          case BoundsType::kEquality:
            slack_g.push_back(coeff);
            slack_g.push_back(coeff);
            a.push_back({ row + k, var++, 1.0 });
            a.push_back({ row + k, var++, -1.0 });
            break;
          case BoundsType::kLowerBound:
            slack_g.push_back(coeff);
            a.push_back({ row + k, var++, 1.0 });
            break;
          case BoundsType::kUpperBound:
            slack_g.push_back(coeff);
            a.push_back({ row + k, var++, -1.0 });
            break;
          default:
            throw std::runtime_error("Unsupported bounds type!");
        }
      }
      (pass == 0 ? I.n_pen_rows : I.n_merit_rows) += t->getRows();
      row += t->getRows();
    }
  }
  I.n_slack = var - I.n_nlp;
  I.n_qp_vars = var;
  I.n_qp_cnts = row + I.n_qp_vars;
  I.gradient.assign(static_cast<std::size_t>(I.n_qp_vars), 0.0);
  for (long k = 0; k < I.n_slack; ++k)
    I.gradient[static_cast<std::size_t>(I.n_nlp + k)] = slack_g[static_cast<std::size_t>(k)];
  // squared costs: residual target - (f(x0) + J (x - x0)) = a - J x with
  // a = target - (f(x0) - J x0); per row a^2 w + 2 a w (-J x) + w (J x)^2.  Each
  // term's column sums and (sqrt(w) J)'(sqrt(w) J) are formed first and then
  // added to the totals in term order.
  VectorXd obj_lin(static_cast<std::size_t>(I.n_nlp), 0.0);
  std::map<std::pair<long, long>, double> H;
  std::vector<Entry> lin;
  I.sq_const.clear();
  I.sq_q.clear();
  long srow = 0;
  for (const auto& t : I.squared)
  {
    const Jacobian jac = t->getJacobian();
    const VectorXd val = t->getValues(), jx = mul(jac, x0), w = t->getCoefficients();
    const auto bounds = t->getBounds();
    VectorXd tlin(static_cast<std::size_t>(I.n_nlp), 0.0);
    std::map<std::pair<long, long>, double> th;
    for (long r = 0; r < t->getRows(); ++r)
    {
      const auto ur = static_cast<std::size_t>(r);
      const double ar = bounds[ur].getLower() - (val[ur] - jx[ur]);
      I.sq_const.push_back((ar * ar) * w[ur]);
      const double sr = 2.0 * (ar * w[ur]), sw = std::sqrt(w[ur]);
      std::vector<std::pair<long, double>> qi;
      for (long e = jac.rowBegin(r); e < jac.rowEnd(r); ++e)
      {
        const double b = -jac.value(e);
        const double lv = b * sr;
        lin.push_back({ srow, jac.col(e), lv });
        tlin[static_cast<std::size_t>(jac.col(e))] += lv;
        qi.emplace_back(jac.col(e), b * sw);
      }
      for (const auto& e1 : qi)
        for (const auto& e2 : qi)
        {
          auto it = th.find({ e1.first, e2.first });
          if (it == th.end())
            th.emplace(std::make_pair(e1.first, e2.first), e1.second * e2.second);
          else
            it->second += e1.second * e2.second;
        }
      I.sq_q.push_back(qi);
      ++srow;
    }
    for (long j = 0; j < I.n_nlp; ++j)
      obj_lin[static_cast<std::size_t>(j)] += tlin[static_cast<std::size_t>(j)];
    for (const auto& e : th)
    {
      auto it = H.find(e.first);
      if (it == H.end())
        H.emplace(e.first, e.second);
      else
        it->second += e.second;
    }
  }
  I.sq_lin = fromEntries(srow, I.n_nlp, lin);
  for (long j = 0; j < I.n_nlp; ++j)
    I.gradient[static_cast<std::size_t>(j)] = obj_lin[static_cast<std::size_t>(j)];
  std::vector<Entry> he;
  for (const auto& e : H)
    he.push_back({ e.first.first, e.first.second, std::abs(e.second) < 1e-7 ? 0.0 : e.second });
  I.hessian = fromEntries(I.n_qp_vars, I.n_qp_vars, he);
  // identity block over every QP variable; slack bounds [0, inf)
  for (long i = 0; i < I.n_qp_vars; ++i)
    a.push_back({ row + i, i, 1.0 });
  I.cmat = fromEntries(I.n_qp_cnts, I.n_qp_vars, a);
  I.lo.resize(static_cast<std::size_t>(I.n_qp_cnts), 0.0);
  I.up.resize(static_cast<std::size_t>(I.n_qp_cnts), kInf);
  I.updateNLPVariableBounds(x0);
}

double TrajOptQPProblem::evaluateTotalConvexCost(const VectorXd& var_vals) const
{
  double s = 0;
  for (double c : evaluateConvexCosts(var_vals))
    s += c;
  return s;
}

// squared costs from the quadratic model over the NLP block; hinge / absolute
// costs from their matrix rows over every QP variable, slacks included (as the
// reference, trajopt_qp_problem.cpp:133)
VectorXd TrajOptQPProblem::evaluateConvexCosts(const VectorXd& var_vals) const
{
  const Impl& I = *impl_;
  VectorXd costs;
  long r = 0;
  for (const auto& t : I.squared)
  {
    double s = 0;
    for (long k = 0; k < t->getRows(); ++k, ++r)
    {
      double o = I.sq_const[static_cast<std::size_t>(r)];
      double l = 0;
      for (long e = I.sq_lin.rowBegin(r); e < I.sq_lin.rowEnd(r); ++e)
        l += I.sq_lin.value(e) * var_vals[static_cast<std::size_t>(I.sq_lin.col(e))];
      o += l;
      double q = 0;
      for (const auto& e : I.sq_q[static_cast<std::size_t>(r)])
        q += e.second * var_vals[static_cast<std::size_t>(e.first)];
      o += q * q;
      s += o;
    }
    costs.push_back(s);
  }
  long row = 0;
  for (const auto& t : I.penalty)
  {
    costs.push_back(t->getRows() == 0 ? 0.0 : I.rowsViolation(var_vals, *t, row, I.n_qp_vars));
    row += t->getRows();
  }
  return costs;
}

// constraint rows over the NLP columns only
VectorXd TrajOptQPProblem::evaluateConvexConstraintViolations(const VectorXd& var_vals) const
{
  const Impl& I = *impl_;
  VectorXd v;
  long row = I.n_pen_rows;
  for (const auto& t : I.constraints)
  {
    v.push_back(t->getRows() == 0 ? 0.0 : I.rowsViolation(var_vals, *t, row, I.n_nlp));
    row += t->getRows();
  }
  return v;
}

double TrajOptQPProblem::getTotalExactCost() const
{
  double s = 0;
  for (double c : getExactCosts())
    s += c;
  return s;
}

// squared costs: sum(err^2 * coeff); hinge / absolute costs: sum(err), without the
// coefficients (trajopt_qp_problem.cpp:977-1020)
VectorXd TrajOptQPProblem::getExactCosts() const
{
  const Impl& I = *impl_;
  VectorXd g;
  VectorXd err;
  for (const auto& c : I.squared)
  {
    trajopt_ifopt::calcBoundsViolations(err, c->getValues(), c->getBounds());
    const VectorXd w = c->getCoefficients();
    double s = 0;
    for (std::size_t i = 0; i < err.size(); ++i)
      s += (err[i] * err[i]) * w[i];
    g.push_back(s);
  }
  for (const auto& c : I.penalty)
  {
    trajopt_ifopt::calcBoundsViolations(err, c->getValues(), c->getBounds());
    double s = 0;
    for (double e : err)
      s += e;
    g.push_back(s);
  }
  return g;
}

VectorXd TrajOptQPProblem::getExactConstraintViolations() const
{
  VectorXd v, err;
  for (const auto& c : impl_->constraints)
  {
    trajopt_ifopt::calcBoundsViolations(err, c->getValues(), c->getBounds());
    double s = 0;
    for (double e : err)
      s += e;
    v.push_back(s);
  }
  return v;
}

void TrajOptQPProblem::scaleBoxSize(double& scale)
{
  for (double& b : impl_->box)
    b = b * scale;
  impl_->updateNLPVariableBounds(impl_->variables->getValues());
}

void TrajOptQPProblem::setBoxSize(const VectorXd& box_size)
{
  if (static_cast<long>(box_size.size()) != impl_->n_nlp)
    throw std::runtime_error("TrajOptQPProblem::setBoxSize: size mismatch");
  impl_->box = box_size;
  impl_->updateNLPVariableBounds(impl_->variables->getValues());
}

void TrajOptQPProblem::setConstraintMeritCoeff(const VectorXd& merit_coeff)
{
  if (merit_coeff.size() != impl_->constraints.size())
    throw std::runtime_error("TrajOptQPProblem::setConstraintMeritCoeff: size mismatch");
  impl_->merit = merit_coeff;
}

void TrajOptQPProblem::print() const
{
  const Impl& I = *impl_;
  std::printf("-------------- QPProblem::print() --------------\n");
  std::printf("Num NLP Vars: %ld\nNum QP Vars: %ld\nNum QP Constraints: %ld\n", I.n_nlp, I.n_qp_vars, I.n_qp_cnts);
}

long TrajOptQPProblem::getNumNLPVars() const { return impl_->n_nlp; }
long TrajOptQPProblem::getNumNLPConstraints() const { return static_cast<long>(impl_->constraints.size()); }
long TrajOptQPProblem::getNumNLPCosts() const
{
  return static_cast<long>(impl_->squared.size() + impl_->penalty.size());
}
long TrajOptQPProblem::getNumQPVars() const { return impl_->n_qp_vars; }
long TrajOptQPProblem::getNumQPConstraints() const { return impl_->n_qp_cnts; }
const std::vector<std::string>& TrajOptQPProblem::getNLPConstraintNames() const { return impl_->cnt_names; }
const std::vector<std::string>& TrajOptQPProblem::getNLPCostNames() const { return impl_->cost_names; }
const VectorXd& TrajOptQPProblem::getBoxSize() const { return impl_->box; }
const VectorXd& TrajOptQPProblem::getConstraintMeritCoeff() const { return impl_->merit; }
const Jacobian& TrajOptQPProblem::getHessian() const { return impl_->hessian; }
const VectorXd& TrajOptQPProblem::getGradient() const { return impl_->gradient; }
const Jacobian& TrajOptQPProblem::getConstraintMatrix() const { return impl_->cmat; }
const VectorXd& TrajOptQPProblem::getBoundsLower() const { return impl_->lo; }
const VectorXd& TrajOptQPProblem::getBoundsUpper() const { return impl_->up; }
}  // namespace trajopt_sqp
