// ORACLE — test infrastructure only (see sco_expr.hpp header).
// Restatement of trajopt_sco modelling + OSQPModel + BasicTrustRegionSQP.
#include <chrono>
#include "sco.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace orc
{
// ============================================================ sparse helpers
Csc cscFromTriplets(OsqpInt m, OsqpInt n, const std::vector<Triplet>& t)
{
  // bucket by column keeping input order, then stable-sort rows inside a column,
  // summing duplicates in input order (Eigen setFromTriplets + collapseDuplicates)
  std::vector<std::vector<std::pair<OsqpInt, double>>> cols(static_cast<std::size_t>(n));
  for (const auto& e : t)
    cols[e.c].push_back({ e.r, e.v });
  Csc A;
  A.m = m;
  A.n = n;
  A.p.assign(static_cast<std::size_t>(n + 1), 0);
  for (OsqpInt j = 0; j < n; ++j)
  {
    auto& c = cols[j];
    std::stable_sort(c.begin(), c.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    OsqpInt last = -1;
    for (const auto& e : c)
    {
      if (e.first == last)
        A.x.back() += e.second;
      else
      {
        A.i.push_back(e.first);
        A.x.push_back(e.second);
        last = e.first;
      }
    }
    A.p[j + 1] = static_cast<OsqpInt>(A.i.size());
  }
  return A;
}

void exprToDense(const AffExpr& expr, std::vector<double>& v, OsqpInt n_vars)
{
  v.assign(static_cast<std::size_t>(n_vars), 0.0);
  std::vector<std::pair<OsqpInt, double>> d;
  for (std::size_t i = 0; i < expr.size(); ++i)
  {
    const auto idx = static_cast<OsqpInt>(expr.vars[i].var_rep->index);
    if (idx >= n_vars)
      throw std::runtime_error("exprToEigen: variable index out of range");
    if (expr.coeffs[i] != 0.)
      d.push_back({ idx, expr.coeffs[i] });
  }
  std::stable_sort(d.begin(), d.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  for (const auto& e : d)
    v[e.first] += e.second;
}

static Csc quadUpperTriplets(const QuadExpr& expr, OsqpInt n_vars, bool force_diagonal)
{
  std::vector<Triplet> t;
  for (std::size_t i = 0; i < expr.coeffs.size(); ++i)
  {
    if (expr.coeffs[i] == 0.0)
      continue;
    const auto a = static_cast<OsqpInt>(expr.vars1[i].var_rep->index);
    const auto b = static_cast<OsqpInt>(expr.vars2[i].var_rep->index);
    if (a == b)
      t.push_back({ a, b, expr.coeffs[i] });
    else if (a < b)
      t.push_back({ a, b, expr.coeffs[i] });
    else
      t.push_back({ b, a, expr.coeffs[i] });
  }
  if (force_diagonal)
    for (OsqpInt k = 0; k < n_vars; ++k)
      t.push_back({ k, k, 0.0 });
  return cscFromTriplets(n_vars, n_vars, t);
}

void quadToCsc(const QuadExpr& expr, Csc& P, std::vector<double>& q, OsqpInt n_vars, bool halved, bool force_diagonal)
{
  exprToDense(expr.affexpr, q, n_vars);
  Csc sm = quadUpperTriplets(expr, n_vars, force_diagonal);
  // upper triangle of (sm + sm^T) [* 0.5]
  P = sm;
  for (OsqpInt j = 0; j < P.n; ++j)
    for (OsqpInt p = P.p[j]; p < P.p[j + 1]; ++p)
    {
      double v = (P.i[p] == j) ? (P.x[p] + P.x[p]) : P.x[p];
      if (!halved)
        v = 0.5 * v;
      P.x[p] = v;
    }
}

void quadToCscFull(const QuadExpr& expr, Csc& F, std::vector<double>& q, OsqpInt n_vars, bool halved,
                   bool force_diagonal)
{
  exprToDense(expr.affexpr, q, n_vars);
  Csc sm = quadUpperTriplets(expr, n_vars, force_diagonal);
  std::vector<Triplet> t;
  for (OsqpInt j = 0; j < sm.n; ++j)
    for (OsqpInt p = sm.p[j]; p < sm.p[j + 1]; ++p)
    {
      t.push_back({ sm.i[p], j, sm.x[p] });
      t.push_back({ j, sm.i[p], sm.x[p] });
    }
  F = cscFromTriplets(n_vars, n_vars, t);
  if (!halved)
    for (auto& v : F.x)
      v *= 0.5;
}

void affVecToCsc(const AffExprVector& exprs, Csc& A, std::vector<double>& rhs, OsqpInt n_vars)
{
  rhs.assign(exprs.size(), 0.0);
  std::vector<Triplet> t;
  for (std::size_t i = 0; i < exprs.size(); ++i)
  {
    const AffExpr& e = exprs[i];
    rhs[i] = -e.constant;
    for (std::size_t j = 0; j < e.size(); ++j)
    {
      const auto idx = static_cast<OsqpInt>(e.vars[j].var_rep->index);
      if (idx >= n_vars)
        throw std::runtime_error("exprToEigen: variable index out of range");
      if (e.coeffs[j] != 0.)
        t.push_back({ static_cast<OsqpInt>(i), idx, e.coeffs[j] });
    }
  }
  A = cscFromTriplets(static_cast<OsqpInt>(exprs.size()), n_vars, t);
}

// ==================================================================== model
Var Model::addVar(const std::string& name, double lb, double ub)
{
  Var v = addVar(name);
  setVarBounds(v, lb, ub);
  return v;
}
void Model::setVarBounds(const Var& var, double lower, double upper)
{
  setVarBounds(VarVector(1, var), DblVec(1, lower), DblVec(1, upper));
}
double Model::getVarValue(const Var& var) const { return getVarValues(VarVector(1, var))[0]; }

OSQPModel::OSQPModel(const OsqpSettings& settings) : settings_(settings) {}
OSQPModel::~OSQPModel()
{
  for (const Var& v : vars_)
    v.var_rep->removed = true;
  for (const Cnt& c : cnts_)
    c.cnt_rep->removed = true;
  OSQPModel::update();
}

Var OSQPModel::addVar(const std::string& name)
{
  std::scoped_lock lock(mutex_);
  vars_.emplace_back(std::make_shared<VarRep>(vars_.size(), name, this));
  lbs_.push_back(-OSQP_INFTY);
  ubs_.push_back(OSQP_INFTY);
  return vars_.back();
}
Cnt OSQPModel::addEqCnt(const AffExpr& expr, const std::string&)
{
  std::scoped_lock lock(mutex_);
  cnts_.emplace_back(std::make_shared<CntRep>(cnts_.size(), this));
  cnt_exprs_.push_back(expr);
  cnt_types_.push_back(EQ);
  return cnts_.back();
}
Cnt OSQPModel::addIneqCnt(const AffExpr& expr, const std::string&)
{
  std::scoped_lock lock(mutex_);
  cnts_.emplace_back(std::make_shared<CntRep>(cnts_.size(), this));
  cnt_exprs_.push_back(expr);
  cnt_types_.push_back(INEQ);
  return cnts_.back();
}
void OSQPModel::removeVars(const VarVector& vars)
{
  std::scoped_lock lock(mutex_);
  for (const auto& v : vars)
    v.var_rep->removed = true;
}
void OSQPModel::removeCnts(const CntVector& cnts)
{
  std::scoped_lock lock(mutex_);
  for (const auto& c : cnts)
    c.cnt_rep->removed = true;
}

void OSQPModel::update()
{
  std::size_t inew = 0;
  for (std::size_t iold = 0; iold < vars_.size(); ++iold)
  {
    Var& var = vars_[iold];
    if (!var.var_rep->removed)
    {
      vars_[inew] = var;
      lbs_[inew] = lbs_[iold];
      ubs_[inew] = ubs_[iold];
      vars_[inew].var_rep->index = inew;
      ++inew;
    }
  }
  vars_.resize(inew);
  lbs_.resize(inew);
  ubs_.resize(inew);
  inew = 0;
  for (std::size_t iold = 0; iold < cnts_.size(); ++iold)
  {
    Cnt& cnt = cnts_[iold];
    if (!cnt.cnt_rep->removed)
    {
      cnts_[inew] = cnt;
      cnt_exprs_[inew] = cnt_exprs_[iold];
      cnt_types_[inew] = cnt_types_[iold];
      cnts_[inew].cnt_rep->index = inew;
      ++inew;
    }
  }
  cnts_.resize(inew);
  cnt_exprs_.resize(inew);
  cnt_types_.resize(inew);
}

void OSQPModel::setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper)
{
  for (std::size_t i = 0; i < vars.size(); ++i)
  {
    const std::size_t k = vars[i].var_rep->index;
    lbs_[k] = lower[i];
    ubs_[k] = upper[i];
  }
}

DblVec OSQPModel::getVarValues(const VarVector& vars) const
{
  DblVec out(vars.size());
  for (std::size_t i = 0; i < vars.size(); ++i)
    out[i] = solution_[vars[i].var_rep->index];
  return out;
}

// osqp_interface.cpp:170-211 incl. quirk Q2 (memcmp over n+1 / nzmax BYTES)
bool OSQPModel::updateObjective(bool check_sparsity)
{
  const auto n = static_cast<OsqpInt>(vars_.size());
  Csc P;
  quadToCsc(objective_, P, q_, n, true);
  bool eq = false;
  if (check_sparsity && has_P_ && P_.n == n && P_.m == n && P_.nnz() == P.nnz())
  {
    eq = true;
    eq = eq && std::memcmp(P_.p.data(), P.p.data(), static_cast<std::size_t>(P_.n) + 1) == 0;
    // (an empty P compares equal; memcmp is not called on its null data)
    eq = eq && (P_.nnz() == 0 || std::memcmp(P_.i.data(), P.i.data(), static_cast<std::size_t>(P_.nnz())) == 0);
  }
  n_ = n;
  P_ = std::move(P);
  has_P_ = true;
  return eq;
}

// osqp_interface.cpp:213-281
bool OSQPModel::updateConstraints(bool check_sparsity)
{
  const auto n = static_cast<OsqpInt>(vars_.size());
  const auto m = static_cast<OsqpInt>(cnts_.size());
  m_ = m + n;
  Csc sm;
  DblVec v;
  affVecToCsc(cnt_exprs_, sm, v, n);
  l_.assign(static_cast<std::size_t>(m + n), -OSQP_INFTY);
  u_.assign(static_cast<std::size_t>(m + n), OSQP_INFTY);
  for (OsqpInt i = 0; i < m; ++i)
  {
    l_[i] = (cnt_types_[i] == INEQ) ? -OSQP_INFTY : v[i];
    u_[i] = v[i];
  }
  // append the identity block (rows m..m+n-1)
  Csc A;
  A.m = m + n;
  A.n = n;
  A.p.assign(static_cast<std::size_t>(n + 1), 0);
  for (OsqpInt j = 0; j < n; ++j)
  {
    for (OsqpInt p = sm.p[j]; p < sm.p[j + 1]; ++p)
    {
      A.i.push_back(sm.i[p]);
      A.x.push_back(sm.x[p]);
    }
    A.i.push_back(m + j);
    A.x.push_back(1.0);
    A.p[j + 1] = static_cast<OsqpInt>(A.i.size());
  }
  for (OsqpInt i = 0; i < n; ++i)
  {
    l_[m + i] = std::fmax(lbs_[i], -OSQP_INFTY);
    u_[m + i] = std::fmin(ubs_[i], OSQP_INFTY);
  }
  bool eq = false;
  if (check_sparsity && has_A_ && A_.n == A.n && A_.m == A.m && A_.nnz() == A.nnz())
  {
    eq = true;
    eq = eq && std::memcmp(A_.p.data(), A.p.data(), static_cast<std::size_t>(A_.n) + 1) == 0;
    eq = eq && std::memcmp(A_.i.data(), A.i.data(), static_cast<std::size_t>(A_.nnz())) == 0;
  }
  A_ = std::move(A);
  has_A_ = true;
  return eq;
}

// osqp_interface.cpp:283-370
void OSQPModel::createOrUpdateSolver()
{
  bool allow_update = false, allow_ws = false;
  if (ws_)
  {
    const int st = ws_->status_val;
    if (st == OSQP_SOLVED || st == OSQP_SOLVED_INACCURATE)
    {
      if (update_workspace)
        allow_update = true;
      else if (settings_.warm_starting != 0)
        allow_ws = true;
    }
  }
  const bool P_eq = updateObjective(allow_update || allow_ws);
  const bool A_eq = updateConstraints(P_eq);
  allow_ws = allow_ws && P_eq && A_eq;
  OsqpSettings settings = settings_;
  DblVec prev_x, prev_y;
  if (ws_)
  {
    if (allow_ws)
    {
      prev_x.assign(ws_->sol_x.begin(), ws_->sol_x.begin() + n_);
      prev_y.assign(ws_->sol_y.begin(), ws_->sol_y.begin() + m_);
      settings.rho = ws_->settings().rho;
    }
    ws_.reset();
  }
  auto ws = std::make_unique<OsqpSolver>();
  const int ret = ws->setup(P_, q_.data(), A_, l_.data(), u_.data(), m_, n_, settings);
  if (ret != 0)
    throw std::runtime_error("Could not initialize OSQP: error " + std::to_string(ret));
  last_warm_started = false;
  if (!prev_x.empty() && !prev_y.empty())
  {
    ws->warm_start(prev_x.data(), prev_y.data());
    last_warm_started = true;
  }
  ws_ = std::move(ws);
}

CvxOptStatus OSQPModel::optimize()
{
  update();
  try
  {
    createOrUpdateSolver();
  }
  catch (const std::exception&)
  {
    if (trace)
      trace->push_back({ 0, 0, 0, -1, 0, 0, 0, 0, 0, trace_trust, trace_tie_cleanup, 0 });
    return CVX_FAILED;
  }
  const double rho0 = ws_->settings().rho;
  const int ret = ws_->solve();
  admm_iters_total += ws_->iter;
  if (trace)
  {
    double xs = 0;
    for (double v : ws_->sol_x)
      xs += std::fabs(v);
    trace->push_back({ last_warm_started ? 1.0 : 0.0, rho0, static_cast<double>(ws_->iter),
                       static_cast<double>(ws_->status_val), static_cast<double>(ws_->status_polish),
                       ws_->settings().rho, ws_->prim_res, ws_->dual_res, xs, trace_trust, trace_tie_cleanup,
                       ws_->polish_margin });
  }
  last_osqp_status = ws_->status_val;
  last_polish_status = ws_->status_polish;
  if (ret == 0)
  {
    solution_.assign(ws_->sol_x.begin(), ws_->sol_x.begin() + static_cast<long>(vars_.size()));
    const int st = ws_->status_val;
    if (st == OSQP_SOLVED || st == OSQP_SOLVED_INACCURATE)
      return CVX_SOLVED;
    if (st == OSQP_PRIMAL_INFEASIBLE || st == OSQP_PRIMAL_INFEASIBLE_INACCURATE || st == OSQP_DUAL_INFEASIBLE ||
        st == OSQP_DUAL_INFEASIBLE_INACCURATE)
      return CVX_INFEASIBLE;
  }
  return CVX_FAILED;
}

void OSQPModel::setObjective(const AffExpr& expr) { objective_.affexpr = expr; }
void OSQPModel::setObjective(const QuadExpr& expr) { objective_ = expr; }

// ================================================================ modelling
void ConvexObjective::addAffExpr(const AffExpr& a) { exprInc(quad_, a); }
void ConvexObjective::addQuadExpr(const QuadExpr& q) { exprInc(quad_, q); }
void ConvexObjective::addHinge(const AffExpr& affexpr, double coeff)
{
  Var hinge = model_->addVar("hinge", 0, INFINITY);
  vars_.push_back(hinge);
  ineqs_.push_back(affexpr);
  exprDec(ineqs_.back(), hinge);
  AffExpr hinge_cost = exprMult(AffExpr(hinge), coeff);
  exprInc(quad_, hinge_cost);
}
void ConvexObjective::addAbs(const AffExpr& affexpr, double coeff)
{
  Var neg = model_->addVar("neg", 0, INFINITY);
  Var pos = model_->addVar("pos", 0, INFINITY);
  vars_.push_back(neg);
  vars_.push_back(pos);
  AffExpr neg_plus_pos;
  neg_plus_pos.coeffs = DblVec(2, coeff);
  neg_plus_pos.vars.push_back(neg);
  neg_plus_pos.vars.push_back(pos);
  exprInc(quad_, neg_plus_pos);
  AffExpr affeq = affexpr;
  affeq.vars.push_back(neg);
  affeq.vars.push_back(pos);
  affeq.coeffs.push_back(1);
  affeq.coeffs.push_back(-1);
  eqs_.push_back(affeq);
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
  Var m = model_->addVar("max", -INFINITY, INFINITY);
  for (const auto& e : ev)
  {
    ineqs_.push_back(e);
    exprDec(ineqs_.back(), m);
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

DblVec Constraint::violations(const DblVec& x)
{
  DblVec val = value(x);
  DblVec out(val.size());
  if (type() == EQ)
    for (std::size_t i = 0; i < val.size(); ++i)
      out[i] = std::fabs(val[i]);
  else
    for (std::size_t i = 0; i < val.size(); ++i)
      out[i] = pospart(val[i]);
  return out;
}
double Constraint::violation(const DblVec& x) { return vecSum(violations(x)); }

OptProb::OptProb(const OsqpSettings& s) : model_(std::make_shared<OSQPModel>(s)) {}
VarVector OptProb::createVariables(const std::vector<std::string>& names)
{
  return createVariables(names, DblVec(names.size(), -INFINITY), DblVec(names.size(), INFINITY));
}
VarVector OptProb::createVariables(const std::vector<std::string>& names, const DblVec& lb, const DblVec& ub)
{
  const std::size_t n_add = names.size();
  for (std::size_t i = 0; i < n_add; ++i)
  {
    vars_.push_back(model_->addVar(names[i], lb[i], ub[i]));
    lower_bounds_.push_back(lb[i]);
    upper_bounds_.push_back(ub[i]);
  }
  model_->update();
  return VarVector(vars_.end() - static_cast<long>(n_add), vars_.end());
}
void OptProb::addConstraint(Constraint::Ptr c)
{
  if (c->type() == EQ)
    eqcnts_.push_back(std::move(c));
  else
    ineqcnts_.push_back(std::move(c));
}
void OptProb::addLinearConstraint(const AffExpr& expr, ConstraintType type)
{
  if (type == EQ)
    model_->addEqCnt(expr, "");
  else
    model_->addIneqCnt(expr, "");
}
std::vector<Constraint::Ptr> OptProb::getConstraints() const
{
  std::vector<Constraint::Ptr> out;
  out.insert(out.end(), eqcnts_.begin(), eqcnts_.end());
  out.insert(out.end(), ineqcnts_.begin(), ineqcnts_.end());
  return out;
}
// modeling.cpp:261-273
DblVec OptProb::getClosestFeasiblePoint(const DblVec& x, const double& delta)
{
  DblVec y(x.size());
  for (std::size_t i = 0; i < x.size(); i++)
  {
    const double inset = std::min(delta, (upper_bounds_[i] - lower_bounds_[i]) / 2);
    y[i] = std::min(std::max(x[i], lower_bounds_[i] + inset), upper_bounds_[i] - inset);
  }
  return y;
}

// ============================================================ num diff etc.
Mat calcForwardNumJac(const VectorOfVector& f, const DblVec& x, double epsilon)
{
  const DblVec y = f(x);
  Mat out(static_cast<int>(y.size()), static_cast<int>(x.size()));
  DblVec xpert = x;
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    xpert[i] = x[i] + epsilon;
    const DblVec yp = f(xpert);
    for (std::size_t r = 0; r < y.size(); ++r)
      out(static_cast<int>(r), static_cast<int>(i)) = (yp[r] - y[r]) / epsilon;
    xpert[i] = x[i];
  }
  return out;
}
DblVec calcForwardNumGrad(const ScalarOfVector& f, const DblVec& x, double epsilon)
{
  DblVec out(x.size());
  DblVec xpert = x;
  const double y = f(x);
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    xpert[i] = x[i] + epsilon;
    const double yp = f(xpert);
    out[i] = (yp - y) / epsilon;
    xpert[i] = x[i];
  }
  return out;
}
void calcGradAndDiagHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad,
                         DblVec& hess)
{
  y = f(x);
  grad.resize(x.size());
  hess.resize(x.size());
  DblVec xpert = x;
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    xpert[i] = x[i] + epsilon / 2;
    const double yplus = f(xpert);
    xpert[i] = x[i] - epsilon / 2;
    const double yminus = f(xpert);
    grad[i] = (yplus - yminus) / epsilon;
    hess[i] = (yplus + yminus - 2 * y) / (epsilon * epsilon / 4);
    xpert[i] = x[i];
  }
}
void calcGradHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad, Mat& hess)
{
  y = f(x);
  auto grad_func = [&](const DblVec& xx) { return calcForwardNumGrad(f, xx, epsilon); };
  grad = grad_func(x);
  Mat h = calcForwardNumJac(grad_func, x, epsilon);
  hess = Mat(h.rows, h.cols);
  for (int i = 0; i < h.rows; ++i)
    for (int j = 0; j < h.cols; ++j)
      hess(i, j) = (h(i, j) + h(j, i)) / 2;
}

DblVec getDblVec(const DblVec& x, const VarVector& vars)
{
  DblVec out(vars.size());
  for (std::size_t i = 0; i < vars.size(); ++i)
    out[i] = x[vars[i].var_rep->index];
  return out;
}

AffExpr affFromValGrad(double y, const DblVec& x, const DblVec& dydx, const VarVector& vars)
{
  AffExpr aff;
  double dot = 0;
  for (std::size_t i = 0; i < x.size(); ++i)
    dot += dydx[i] * x[i];
  aff.constant = y - dot;
  aff.coeffs = dydx;
  aff.vars = vars;
  return cleanupAff(aff);
}

// ---- symmetric eigen-decomposition (Jacobi) for CostFromFunc full_hessian
static void symEig(const Mat& A, DblVec& evals, Mat& evecs)
{
  const int n = A.rows;
  Mat a = A;
  evecs = Mat(n, n);
  for (int i = 0; i < n; ++i)
    evecs(i, i) = 1;
  for (int sweep = 0; sweep < 100; ++sweep)
  {
    double off = 0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j)
        off += a(i, j) * a(i, j);
    if (off < 1e-30)
      break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q)
      {
        if (std::fabs(a(p, q)) < 1e-300)
          continue;
        const double theta = (a(q, q) - a(p, p)) / (2 * a(p, q));
        const double t = (theta >= 0 ? 1 : -1) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; ++k)
        {
          const double akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - s * akq;
          a(k, q) = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k)
        {
          const double apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - s * aqk;
          a(q, k) = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k)
        {
          const double vkp = evecs(k, p), vkq = evecs(k, q);
          evecs(k, p) = c * vkp - s * vkq;
          evecs(k, q) = s * vkp + c * vkq;
        }
      }
  }
  evals.resize(static_cast<std::size_t>(n));
  for (int i = 0; i < n; ++i)
    evals[static_cast<std::size_t>(i)] = a(i, i);
}

CostFromFunc::CostFromFunc(ScalarOfVector f, VarVector vars, const std::string& name, bool full_hessian)
  : Cost(name), f_(std::move(f)), vars_(std::move(vars)), full_hessian_(full_hessian), epsilon_(1e-5)
{
}
double CostFromFunc::value(const DblVec& x) { return f_(getDblVec(x, vars_)); }
ConvexObjective::Ptr CostFromFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xe = getDblVec(x, vars_);
  const std::size_t n = xe.size();
  auto out = std::make_shared<ConvexObjective>(model);
  QuadExpr& quad = out->quad_;
  if (!full_hessian_)
  {
    double val;
    DblVec grad, hess;
    calcGradAndDiagHess(f_, xe, epsilon_, val, grad, hess);
    for (double& h : hess)
      h = std::max(h, 0.0);
    double gx = 0, xhx = 0;
    for (std::size_t i = 0; i < n; ++i)
    {
      gx += grad[i] * xe[i];
      xhx += xe[i] * (hess[i] * xe[i]);
    }
    quad.affexpr.constant = val - gx + .5 * xhx;
    quad.affexpr.vars = vars_;
    quad.affexpr.coeffs.resize(n);
    for (std::size_t i = 0; i < n; ++i)
      quad.affexpr.coeffs[i] = grad[i] - hess[i] * xe[i];
    quad.vars1 = vars_;
    quad.vars2 = vars_;
    quad.coeffs.resize(n);
    for (std::size_t i = 0; i < n; ++i)
      quad.coeffs[i] = hess[i] * .5;
  }
  else
  {
    double val;
    DblVec grad;
    Mat hess;
    calcGradHess(f_, xe, epsilon_, val, grad, hess);
    DblVec evals;
    Mat evecs;
    symEig(hess, evals, evecs);
    const int ni = static_cast<int>(n);
    Mat pos(ni, ni);
    for (int k = 0; k < ni; ++k)
      if (evals[static_cast<std::size_t>(k)] > 0)
        for (int i = 0; i < ni; ++i)
          for (int j = 0; j < ni; ++j)
            pos(i, j) += evals[static_cast<std::size_t>(k)] * evecs(i, k) * evecs(j, k);
    DblVec px(n, 0.0);
    for (int i = 0; i < ni; ++i)
      for (int j = 0; j < ni; ++j)
        px[static_cast<std::size_t>(i)] += pos(i, j) * xe[static_cast<std::size_t>(j)];
    double gx = 0, xpx = 0;
    for (std::size_t i = 0; i < n; ++i)
    {
      gx += grad[i] * xe[i];
      xpx += xe[i] * px[i];
    }
    quad.affexpr.constant = val - gx + .5 * xpx;
    quad.affexpr.vars = vars_;
    quad.affexpr.coeffs.resize(n);
    for (std::size_t i = 0; i < n; ++i)
      quad.affexpr.coeffs[i] = grad[i] - px[i];
    for (int i = 0; i < ni; ++i)
    {
      quad.vars1.push_back(vars_[static_cast<std::size_t>(i)]);
      quad.vars2.push_back(vars_[static_cast<std::size_t>(i)]);
      quad.coeffs.push_back(pos(i, i) / 2);
      for (int j = i + 1; j < ni; ++j)
      {
        quad.vars1.push_back(vars_[static_cast<std::size_t>(i)]);
        quad.vars2.push_back(vars_[static_cast<std::size_t>(j)]);
        quad.coeffs.push_back(pos(i, j));
      }
    }
  }
  return out;
}

CostFromErrFunc::CostFromErrFunc(VectorOfVector f, MatrixOfVector dfdx, VarVector vars, DblVec coeffs,
                                 PenaltyType pen_type, const std::string& name)
  : Cost(name)
  , f_(std::move(f))
  , dfdx_(std::move(dfdx))
  , vars_(std::move(vars))
  , coeffs_(std::move(coeffs))
  , pen_type_(pen_type)
  , epsilon_(1e-5)
{
}
double CostFromErrFunc::value(const DblVec& x)
{
  DblVec err = f_(getDblVec(x, vars_));
  for (double& e : err)
  {
    switch (pen_type_)
    {
      case SQUARED:
        e = e * e;
        break;
      case ABS:
        e = std::fabs(e);
        break;
      case HINGE:
        e = std::max(e, 0.0);
        break;
    }
  }
  if (!coeffs_.empty())
    for (std::size_t i = 0; i < err.size(); ++i)
      err[i] *= coeffs_[i];
  return vecSum(err);
}
ConvexObjective::Ptr CostFromErrFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xe = getDblVec(x, vars_);
  Mat jac = dfdx_ ? dfdx_(xe) : calcForwardNumJac(f_, xe, epsilon_);
  auto out = std::make_shared<ConvexObjective>(model);
  const DblVec y = f_(xe);
  for (int i = 0; i < jac.rows; ++i)
  {
    DblVec row(jac.a.begin() + i * jac.cols, jac.a.begin() + (i + 1) * jac.cols);
    AffExpr aff = affFromValGrad(y[static_cast<std::size_t>(i)], xe, row, vars_);
    double weight = 1;
    if (!coeffs_.empty())
    {
      if (coeffs_[static_cast<std::size_t>(i)] == 0)
        continue;
      weight = coeffs_[static_cast<std::size_t>(i)];
    }
    switch (pen_type_)
    {
      case SQUARED:
      {
        QuadExpr quad = exprSquare(aff);
        exprScale(quad, weight);
        out->addQuadExpr(quad);
        break;
      }
      case ABS:
        exprScale(aff, weight);
        out->addAbs(aff, 1);
        break;
      case HINGE:
        exprScale(aff, weight);
        out->addHinge(aff, 1);
        break;
    }
  }
  return out;
}

ConstraintFromErrFunc::ConstraintFromErrFunc(VectorOfVector f, MatrixOfVector dfdx, VarVector vars, DblVec coeffs,
                                             ConstraintType type, const std::string& name)
  : Constraint(name)
  , f_(std::move(f))
  , dfdx_(std::move(dfdx))
  , vars_(std::move(vars))
  , coeffs_(std::move(coeffs))
  , type_(type)
  , epsilon_(1e-5)
{
}
DblVec ConstraintFromErrFunc::value(const DblVec& x)
{
  DblVec err = f_(getDblVec(x, vars_));
  if (!coeffs_.empty())
    for (std::size_t i = 0; i < err.size(); ++i)
      err[i] *= coeffs_[i];
  return err;
}
ConvexConstraints::Ptr ConstraintFromErrFunc::convex(const DblVec& x, Model* model)
{
  const DblVec xe = getDblVec(x, vars_);
  Mat jac = dfdx_ ? dfdx_(xe) : calcForwardNumJac(f_, xe, epsilon_);
  auto out = std::make_shared<ConvexConstraints>(model);
  const DblVec y = f_(xe);
  for (int i = 0; i < jac.rows; ++i)
  {
    DblVec row(jac.a.begin() + i * jac.cols, jac.a.begin() + (i + 1) * jac.cols);
    AffExpr aff = affFromValGrad(y[static_cast<std::size_t>(i)], xe, row, vars_);
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

// ================================================================ optimizer
namespace
{
std::vector<ConvexObjective::Ptr> cntsToCosts(const std::vector<ConvexConstraints::Ptr>& cnts,
                                              const DblVec& err_coeffs, Model* model)
{
  std::vector<ConvexObjective::Ptr> out;
  for (std::size_t c = 0; c < cnts.size(); ++c)
  {
    auto obj = std::make_shared<ConvexObjective>(model);
    for (const AffExpr& aff : cnts[c]->eqs_)
      obj->addAbs(aff, err_coeffs[c]);
    for (const AffExpr& aff : cnts[c]->ineqs_)
      obj->addHinge(aff, err_coeffs[c]);
    out.push_back(obj);
  }
  return out;
}
}  // namespace

void BasicTrustRegionSQP::setTrustBoxConstraints(const DblVec& x)
{
  const VarVector& vars = prob_->getVars();
  const DblVec& lb = prob_->getLowerBounds();
  const DblVec& ub = prob_->getUpperBounds();
  DblVec lbt(x.size()), ubt(x.size());
  for (std::size_t i = 0; i < x.size(); ++i)
  {
    const double xi = std::clamp(x[i], lb[i], ub[i]);
    lbt[i] = std::max(xi - param_.trust_box_size, lb[i]);
    ubt[i] = std::min(xi + param_.trust_box_size, ub[i]);
  }
  model_->setVarBounds(vars, lbt, ubt);
}

// optimizers.cpp:699-991
OptStatus BasicTrustRegionSQP::optimize()
{
  auto* osqp_model = dynamic_cast<OSQPModel*>(model_.get());
  const std::vector<Constraint::Ptr> constraints = prob_->getConstraints();
  std::vector<Cost::Ptr>& costs = prob_->getCosts();
  DblVec merit_error_coeffs(constraints.size(), param_.initial_merit_error_coeff);
  if (results_.x.empty())
    throw std::runtime_error("you forgot to initialize!");
  results_.x = prob_->getClosestFeasiblePoint(results_.x);
  OptStatus retval = INVALID;
  const auto start_time = std::chrono::steady_clock::now();

  auto evalCosts = [&](const DblVec& x) {
    DblVec out(costs.size());
    for (std::size_t i = 0; i < costs.size(); ++i)
      out[i] = costs[i]->value(x);
    return out;
  };
  auto evalViols = [&](const DblVec& x) {
    DblVec out(constraints.size());
    for (std::size_t i = 0; i < constraints.size(); ++i)
      out[i] = constraints[i]->violation(x);
    return out;
  };

  for (int merit_increases = 0; merit_increases < param_.max_merit_coeff_increases; ++merit_increases)
  {
    for (int iter = 1;; ++iter)
    {
      // time limit (optimizers.cpp:739-753): checked before the iteration body runs
      const double elapsed_time =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start_time).count() / 1000.0;
      if (elapsed_time > param_.max_time)
      {
        retval = OPT_TIME_LIMIT;
        if (results_.cnt_viols.empty() || vecMax(results_.cnt_viols) < param_.cnt_tolerance)
          retval = OPT_CONVERGED;
        goto cleanup;
      }
      ++results_.n_sqp_iters;
      if (results_.cost_vals.empty() && results_.cnt_viols.empty())
      {
        results_.cnt_viols = evalViols(results_.x);
        results_.cost_vals = evalCosts(results_.x);
        ++results_.n_func_evals;
      }
      bool converged_inner = false;
      bool failed = false;
      {
        t_cleanup_margin = 1e300;
        std::vector<ConvexObjective::Ptr> cost_models(costs.size());
        for (std::size_t i = 0; i < costs.size(); ++i)
          cost_models[i] = costs[i]->convex(results_.x, model_.get());
        std::vector<ConvexConstraints::Ptr> cnt_models(constraints.size());
        for (std::size_t i = 0; i < constraints.size(); ++i)
          cnt_models[i] = constraints[i]->convex(results_.x, model_.get());
        std::vector<ConvexObjective::Ptr> cnt_cost_models =
            cntsToCosts(cnt_models, merit_error_coeffs, model_.get());
        model_->update();
        for (auto& c : cost_models)
          c->addConstraintsToModel();
        for (auto& c : cnt_cost_models)
          c->addConstraintsToModel();
        model_->update();
        QuadExpr objective;
        for (auto& c : cost_models)
          exprInc(objective, c->quad_);
        for (auto& c : cnt_cost_models)
          exprInc(objective, c->quad_);
        model_->setObjective(objective);
        if (osqp_model)
          osqp_model->trace_tie_cleanup = t_cleanup_margin;

        int qp_solver_failures = 0;
        while (param_.trust_box_size >= param_.min_trust_box_size)
        {
          setTrustBoxConstraints(results_.x);
          if (osqp_model)
            osqp_model->trace_trust = param_.trust_box_size;
          const CvxOptStatus status = model_->optimize();
          ++results_.n_qp_solves;
          if (osqp_model)
            results_.n_admm_iters = osqp_model->admm_iters_total;
          if (status != CVX_SOLVED)
          {
            if (qp_solver_failures < (param_.max_qp_solver_failures - 1))
            {
              param_.trust_box_size *= param_.trust_shrink_ratio;
              qp_solver_failures++;
              continue;
            }
            if (qp_solver_failures == (param_.max_qp_solver_failures - 1))
            {
              param_.trust_box_size = param_.min_trust_box_size;
              qp_solver_failures++;
              continue;
            }
            failed = true;
            break;
          }
          // BasicTrustRegionSQPResults::update (optimizers.cpp:380-426)
          const DblVec model_var_vals = model_->getVarValues(model_->getVars());
          DblVec model_cost_vals(cost_models.size());
          for (std::size_t i = 0; i < cost_models.size(); ++i)
            model_cost_vals[i] = cost_models[i]->value(model_var_vals);
          DblVec model_cnt_viols(cnt_models.size());
          for (std::size_t i = 0; i < cnt_models.size(); ++i)
            model_cnt_viols[i] = cnt_models[i]->violation(model_var_vals);
          const DblVec new_x(model_var_vals.begin(), model_var_vals.begin() + static_cast<long>(results_.x.size()));
          const DblVec new_cost_vals = evalCosts(new_x);
          const DblVec new_cnt_viols = evalViols(new_x);
          const double old_merit = vecSum(results_.cost_vals) + vecDot(results_.cnt_viols, merit_error_coeffs);
          const double model_merit = vecSum(model_cost_vals) + vecDot(model_cnt_viols, merit_error_coeffs);
          const double new_merit = vecSum(new_cost_vals) + vecDot(new_cnt_viols, merit_error_coeffs);
          const double approx_merit_improve = old_merit - model_merit;
          const double exact_merit_improve = old_merit - new_merit;
          const double merit_improve_ratio = exact_merit_improve / approx_merit_improve;
          ++results_.n_func_evals;

          if (approx_merit_improve < param_.min_approx_improve)
          {
            retval = OPT_CONVERGED;
            converged_inner = true;
            break;
          }
          if (approx_merit_improve / old_merit < param_.min_approx_improve_frac)
          {
            retval = OPT_CONVERGED;
            converged_inner = true;
            break;
          }
          if (exact_merit_improve < 0 || merit_improve_ratio < param_.improve_ratio_threshold)
          {
            param_.trust_box_size *= param_.trust_shrink_ratio;
          }
          else
          {
            results_.x = new_x;
            results_.cost_vals = new_cost_vals;
            results_.cnt_viols = new_cnt_viols;
            param_.trust_box_size *= param_.trust_expand_ratio;
            break;
          }
        }
      }  // models destroyed here (removed from the model)
      if (failed)
      {
        retval = OPT_FAILED;
        goto cleanup;
      }
      if (converged_inner)
        goto penaltyadjustment;
      if (param_.trust_box_size < param_.min_trust_box_size)
      {
        retval = OPT_CONVERGED;
        goto penaltyadjustment;
      }
      else if (iter >= param_.max_iter)
      {
        retval = OPT_SCO_ITERATION_LIMIT;
        if (results_.cnt_viols.empty() || vecMax(results_.cnt_viols) < param_.cnt_tolerance)
          retval = OPT_CONVERGED;
        goto cleanup;
      }
    }
  penaltyadjustment:
    if (results_.cnt_viols.empty() || vecMax(results_.cnt_viols) < param_.cnt_tolerance)
      goto cleanup;
    if (param_.inflate_constraints_individually)
    {
      for (std::size_t idx = 0; idx < results_.cnt_viols.size(); idx++)
        if (results_.cnt_viols[idx] > param_.cnt_tolerance)
          merit_error_coeffs[idx] *= param_.merit_coeff_increase_ratio;
    }
    else
    {
      for (auto& c : merit_error_coeffs)
        c *= param_.merit_coeff_increase_ratio;
    }
    param_.trust_box_size =
        std::fmax(param_.trust_box_size, param_.min_trust_box_size / param_.trust_shrink_ratio * 1.5);
    ++results_.n_merit_increases;
  }
  retval = OPT_PENALTY_ITERATION_LIMIT;

cleanup:
  results_.status = retval;
  results_.total_cost = vecSum(results_.cost_vals);
  if (osqp_model)
    results_.n_admm_iters = osqp_model->admm_iters_total;
  return retval;
}

}  // namespace orc
