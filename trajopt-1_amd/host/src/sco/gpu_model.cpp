// GpuModel (see gpu_model.hpp): OSQPModel's bookkeeping and QP assembly
// (trajopt_sco/src/osqp_interface.cpp:73-640, solver_utils.cpp:12-183),
// solved on the GPU by thip_qp_solve.
#include <cstdio>
#include "trajopt_sco/gpu_model.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <utility>

namespace sco
{
namespace
{
constexpr double kOsqpInfty = 1e30;  // OSQP_INFTY

struct Trip
{
  int r, c;
  double v;
};

// Eigen setFromTriplets semantics: column buckets in input order, rows sorted
// stably inside a column, duplicates summed in input order
void cscFromTriplets(int m, int n, const std::vector<Trip>& t, std::vector<int>& p, std::vector<int>& idx,
                     std::vector<double>& x)
{
  std::vector<std::vector<std::pair<int, double>>> col(static_cast<std::size_t>(n));
  for (const Trip& e : t)
    col[static_cast<std::size_t>(e.c)].emplace_back(e.r, e.v);
  p.assign(static_cast<std::size_t>(n) + 1, 0);
  idx.clear();
  x.clear();
  (void)m;
  for (int j = 0; j < n; ++j)
  {
    auto& c = col[static_cast<std::size_t>(j)];
    std::stable_sort(c.begin(), c.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (std::size_t k = 0; k < c.size(); ++k)
    {
      if (k > 0 && c[k].first == c[k - 1].first)
        x.back() += c[k].second;
      else
      {
        idx.push_back(c[k].first);
        x.push_back(c[k].second);
      }
    }
    p[static_cast<std::size_t>(j) + 1] = static_cast<int>(idx.size());
  }
}
}  // namespace

GpuModelConfig::GpuModelConfig()
{
  thip_default_osqp_settings(&settings);
}

GpuModel::GpuModel(const GpuModelConfig& config) : config_(config) {}

GpuModel::~GpuModel()
{
  for (const Var& v : vars_)
    v.var_rep->removed = true;
  for (const Cnt& c : cnts_)
    c.cnt_rep->removed = true;
  thip_qp_destroy(qp_);
}

void GpuModel::setDevice(int device)
{
  if (device == config_.device)
    return;
  thip_qp_destroy(qp_);
  qp_ = nullptr;
  qp_Pp_.clear();
  config_.device = device;
}

Var GpuModel::addVar(const std::string& name)
{
  std::scoped_lock lock(mutex_);
  vars_.emplace_back(std::make_shared<VarRep>(vars_.size(), name, this));
  lbs_.push_back(-kOsqpInfty);
  ubs_.push_back(kOsqpInfty);
  return vars_.back();
}

Cnt GpuModel::addEqCnt(const AffExpr& expr, const std::string&)
{
  std::scoped_lock lock(mutex_);
  cnts_.emplace_back(std::make_shared<CntRep>(cnts_.size(), this));
  cnt_exprs_.push_back(expr);
  cnt_types_.push_back(EQ);
  return cnts_.back();
}

Cnt GpuModel::addIneqCnt(const AffExpr& expr, const std::string&)
{
  std::scoped_lock lock(mutex_);
  cnts_.emplace_back(std::make_shared<CntRep>(cnts_.size(), this));
  cnt_exprs_.push_back(expr);
  cnt_types_.push_back(INEQ);
  return cnts_.back();
}

Cnt GpuModel::addIneqCnt(const QuadExpr&, const std::string&)
{
  throw std::runtime_error("Not implemented");  // as OSQPModel (osqp_interface.cpp:146-149)
}

void GpuModel::removeVars(const VarVector& vars)
{
  std::scoped_lock lock(mutex_);
  for (const Var& v : vars)
    v.var_rep->removed = true;
}

void GpuModel::removeCnts(const CntVector& cnts)
{
  std::scoped_lock lock(mutex_);
  for (const Cnt& c : cnts)
    c.cnt_rep->removed = true;
}

void GpuModel::update()
{
  // compact removed variables / constraints and renumber (osqp_interface.cpp:372-418)
  std::size_t w = 0;
  for (std::size_t r = 0; r < vars_.size(); ++r)
    if (!vars_[r].var_rep->removed)
    {
      vars_[w] = vars_[r];
      lbs_[w] = lbs_[r];
      ubs_[w] = ubs_[r];
      vars_[w].var_rep->index = w;
      ++w;
    }
  vars_.resize(w);
  lbs_.resize(w);
  ubs_.resize(w);
  w = 0;
  for (std::size_t r = 0; r < cnts_.size(); ++r)
    if (!cnts_[r].cnt_rep->removed)
    {
      cnts_[w] = cnts_[r];
      cnt_exprs_[w] = cnt_exprs_[r];
      cnt_types_[w] = cnt_types_[r];
      cnts_[w].cnt_rep->index = w;
      ++w;
    }
  cnts_.resize(w);
  cnt_exprs_.resize(w);
  cnt_types_.resize(w);
}

void GpuModel::setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper)
{
  for (std::size_t k = 0; k < vars.size(); ++k)
  {
    const std::size_t i = vars[k].var_rep->index;
    lbs_[i] = lower[k];
    ubs_[i] = upper[k];
  }
}

DblVec GpuModel::getVarValues(const VarVector& vars) const
{
  DblVec out(vars.size());
  for (std::size_t k = 0; k < vars.size(); ++k)
    out[k] = solution_[vars[k].var_rep->index];
  return out;
}

void GpuModel::setObjective(const AffExpr& expr) { objective_.affexpr = expr; }
void GpuModel::setObjective(const QuadExpr& expr) { objective_ = expr; }
VarVector GpuModel::getVars() const { return vars_; }

// exprToEigen(QuadExpr, ..., matrix_is_halved = true) + upper triangle (solver_utils.cpp:49-109):
// the quadratic terms into an upper-triangular pattern, duplicates summed, then sm + sm^T
// restricted to the upper triangle, i.e. P_ii = 2 c_ii and P_ij = c_ij
void GpuModel::buildObjective(Csc& P, DblVec& q) const
{
  const int n = static_cast<int>(vars_.size());
  q.assign(static_cast<std::size_t>(n), 0.0);
  {
    std::vector<std::pair<int, double>> lin;
    for (std::size_t k = 0; k < objective_.affexpr.size(); ++k)
    {
      const int i = static_cast<int>(objective_.affexpr.vars[k].var_rep->index);
      if (i >= n)
        throw std::runtime_error("exprToEigen: variable index out of range");
      if (objective_.affexpr.coeffs[k] != 0.)
        lin.emplace_back(i, objective_.affexpr.coeffs[k]);
    }
    std::stable_sort(lin.begin(), lin.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& e : lin)
      q[static_cast<std::size_t>(e.first)] += e.second;
  }
  std::vector<Trip> t;
  for (std::size_t k = 0; k < objective_.size(); ++k)
  {
    const double c = objective_.coeffs[k];
    if (c == 0.0)
      continue;
    int a = static_cast<int>(objective_.vars1[k].var_rep->index), b = static_cast<int>(objective_.vars2[k].var_rep->index);
    if (a > b)
      std::swap(a, b);
    t.push_back({ a, b, c });
  }
  P.n = P.m = n;
  cscFromTriplets(n, n, t, P.p, P.i, P.x);
  for (int j = 0; j < n; ++j)
    for (int e = P.p[static_cast<std::size_t>(j)]; e < P.p[static_cast<std::size_t>(j) + 1]; ++e)
      if (P.i[static_cast<std::size_t>(e)] == j)
        P.x[static_cast<std::size_t>(e)] = P.x[static_cast<std::size_t>(e)] + P.x[static_cast<std::size_t>(e)];
}

// updateConstraints (osqp_interface.cpp:213-281): constraint rows (EQ: l = u = -c,
// INEQ: l = -inf, u = -c) and below them the identity block of variable bounds
void GpuModel::buildConstraints(Csc& A, DblVec& l, DblVec& u) const
{
  const int n = static_cast<int>(vars_.size()), mc = static_cast<int>(cnts_.size());
  std::vector<Trip> t;
  DblVec rhs(static_cast<std::size_t>(mc));
  for (int r = 0; r < mc; ++r)
  {
    const AffExpr& e = cnt_exprs_[static_cast<std::size_t>(r)];
    rhs[static_cast<std::size_t>(r)] = -e.constant;
    for (std::size_t k = 0; k < e.size(); ++k)
    {
      const int j = static_cast<int>(e.vars[k].var_rep->index);
      if (j >= n)
        throw std::runtime_error("exprToEigen: variable index out of range");
      if (e.coeffs[k] != 0.)
        t.push_back({ r, j, e.coeffs[k] });
    }
  }
  Csc C;
  cscFromTriplets(mc, n, t, C.p, C.i, C.x);
  A.m = mc + n;
  A.n = n;
  A.p.assign(static_cast<std::size_t>(n) + 1, 0);
  A.i.clear();
  A.x.clear();
  for (int j = 0; j < n; ++j)
  {
    for (int e = C.p[static_cast<std::size_t>(j)]; e < C.p[static_cast<std::size_t>(j) + 1]; ++e)
    {
      A.i.push_back(C.i[static_cast<std::size_t>(e)]);
      A.x.push_back(C.x[static_cast<std::size_t>(e)]);
    }
    A.i.push_back(mc + j);
    A.x.push_back(1.0);
    A.p[static_cast<std::size_t>(j) + 1] = static_cast<int>(A.i.size());
  }
  l.assign(static_cast<std::size_t>(mc + n), -kOsqpInfty);
  u.assign(static_cast<std::size_t>(mc + n), kOsqpInfty);
  for (int r = 0; r < mc; ++r)
  {
    l[static_cast<std::size_t>(r)] = (cnt_types_[static_cast<std::size_t>(r)] == INEQ) ? -kOsqpInfty : rhs[static_cast<std::size_t>(r)];
    u[static_cast<std::size_t>(r)] = rhs[static_cast<std::size_t>(r)];
  }
  for (int j = 0; j < n; ++j)
  {
    l[static_cast<std::size_t>(mc + j)] = std::fmax(lbs_[static_cast<std::size_t>(j)], -kOsqpInfty);
    u[static_cast<std::size_t>(mc + j)] = std::fmin(ubs_[static_cast<std::size_t>(j)], kOsqpInfty);
  }
}

// quirk Q2 (osqp_interface.cpp:199-201, 268-271): sizes equal and the first
// n + 1 / nnz BYTES of the column pointers / row indices equal
bool GpuModel::bytesEqual(const Csc& a, const Csc& b)
{
  if (a.n != b.n || a.m != b.m || a.p.back() != b.p.back())
    return false;
  // OSQPInt is 64-bit: compare the first bytes of 8-byte index arrays
  std::vector<long long> ap(a.p.begin(), a.p.end()), bp(b.p.begin(), b.p.end());
  std::vector<long long> ai(a.i.begin(), a.i.end()), bi(b.i.begin(), b.i.end());
  const std::size_t nb_p = static_cast<std::size_t>(a.n) + 1, nb_i = static_cast<std::size_t>(a.p.back());
  if (nb_p && std::memcmp(ap.data(), bp.data(), std::min(nb_p, ap.size() * 8)) != 0)
    return false;
  if (nb_i && std::memcmp(ai.data(), bi.data(), std::min(nb_i, ai.size() * 8)) != 0)
    return false;
  return true;
}

CvxOptStatus GpuModel::optimize()
{
  update();
  Csc P, A;
  DblVec q, l, u;
  try
  {
    buildObjective(P, q);
    buildConstraints(A, l, u);
  }
  catch (const std::exception&)
  {
    return CVX_FAILED;
  }
  const int n = P.n, m = A.m;
  // createOrUpdateSolver (osqp_interface.cpp:283-370): warm start only after a
  // solved / solved-inaccurate previous workspace with the "same" sparsity
  bool allow_ws = have_prev_ && (prev_status_ == 1 || prev_status_ == 2) && config_.settings.warm_starting != 0;
  if (allow_ws)
  {
    const bool p_eq = bytesEqual(prev_P_, P);
    const bool a_eq = p_eq && bytesEqual(prev_A_, A);
    allow_ws = p_eq && a_eq;
  }
  thip_osqp_settings s = config_.settings;
  if (allow_ws)
    s.rho = prev_rho_;
  if (n + m > THIP_QP_MAX_KKT)
  {
    // beyond the GPU QP solver's capacity: a failed solve, so the reference's
    // failure handling applies to this problem alone (trust-box shrink and
    // retry, then /tmp/fail.lp and OPT_FAILED, optimizers.cpp:790-822)
    std::fprintf(stderr,
                 "GpuModel: the convex subproblem has %d variables and %d constraints; the GPU QP solver takes "
                 "n + m <= THIP_QP_MAX_KKT (%d): CVX_FAILED\n",
                 n, m, THIP_QP_MAX_KKT);
    prev_status_ = 0;
    return CVX_FAILED;
  }
  DblVec x(static_cast<std::size_t>(n)), y(static_cast<std::size_t>(std::max(m, 1)));
  const bool ws = allow_ws && static_cast<int>(prev_x_.size()) >= n && static_cast<int>(prev_y_.size()) >= m;
  if (batcher_)
  {
    GpuQPBatcher::Request r;
    r.device = config_.device;
    r.n = n;
    r.m = m;
    r.Pp = &P.p;
    r.Pi = &P.i;
    r.Ap = &A.p;
    r.Ai = &A.i;
    r.Px = &P.x;
    r.Ax = &A.x;
    r.q = &q;
    r.l = &l;
    r.u = &u;
    r.settings = s;
    r.warm = ws;
    r.wx = &prev_x_;
    r.wy = &prev_y_;
    r.x = &x;
    r.y = &y;
    r.info = &info_;
    batcher_->solve(r);
    y.resize(static_cast<std::size_t>(std::max(m, 1)));
  }
  else
    solveDirect(P, A, q, l, u, s, ws, x, y);
  if (trace_)
  {
    double xs = 0;
    for (double v : x)
      xs += std::fabs(v);
    trace_->push_back({ ws ? 1.0 : 0.0, s.rho, static_cast<double>(info_.iter), static_cast<double>(info_.status),
                        static_cast<double>(info_.polish_status), info_.rho, info_.prim_res, info_.dual_res, xs });
  }
  return finishSolve(std::move(P), std::move(A), x, y);
}

void GpuModel::solveDirect(const Csc& P, const Csc& A, const DblVec& q, const DblVec& l, const DblVec& u,
                           const thip_osqp_settings& s, bool ws, DblVec& x, DblVec& y)
{
  const int n = P.n, m = A.m;
  // device pattern: rebuilt when it changes
  if (!qp_ || qp_Pp_ != P.p || qp_Pi_ != P.i || qp_Ap_ != A.p || qp_Ai_ != A.i)
  {
    thip_qp_destroy(qp_);
    qp_ = nullptr;
    if (thip_qp_create(config_.device, n, m, P.p.data(), P.i.data(), A.p.data(), A.i.data(), 1, &qp_) != THIP_OK)
      throw std::runtime_error(std::string("GpuModel: ") + thip_qp_last_error(nullptr));
    qp_Pp_ = P.p;
    qp_Pi_ = P.i;
    qp_Ap_ = A.p;
    qp_Ai_ = A.i;
  }
  const int rc = thip_qp_solve(qp_, P.x.data(), q.data(), A.x.data(), l.data(), u.data(), &s, ws ? prev_x_.data() : nullptr,
                               ws ? prev_y_.data() : nullptr, nullptr, x.data(), y.data(), &info_);
  if (rc != THIP_OK)
    throw std::runtime_error(std::string("GpuModel: thip_qp_solve: ") + thip_qp_last_error(qp_));
}

CvxOptStatus GpuModel::finishSolve(Csc&& P, Csc&& A, const DblVec& x, const DblVec& y)
{
  // the next solve's warm start
  prev_P_ = std::move(P);
  prev_A_ = std::move(A);
  have_prev_ = true;
  prev_status_ = info_.status;
  if (info_.status == -1)
  {
    have_prev_ = false;  // osqp_setup threw: the workspace is gone
    return CVX_FAILED;
  }
  admm_total_ += info_.iter;
  prev_x_ = x;
  prev_y_ = y;
  prev_rho_ = info_.rho;
  solution_.assign(x.begin(), x.begin() + static_cast<long>(vars_.size()));
  if (info_.status == 1 || info_.status == 2)
    return CVX_SOLVED;
  if (info_.status >= 3 && info_.status <= 6)
    return CVX_INFEASIBLE;
  return CVX_FAILED;
}

void GpuModel::writeToFile(const std::string& fname) const
{
  std::ofstream out(fname);
  out << "\\ Generated by trajopt_sco with backend OSQP\n";
  out << "Minimize\n";
  out << objective_;
  out << "Subject To\n";
  for (std::size_t r = 0; r < cnt_exprs_.size(); ++r)
    out << cnt_exprs_[r] << ((cnt_types_[r] == INEQ) ? " <= " : " = ") << 0 << "\n";
  out << "Bounds\n";
  for (std::size_t i = 0; i < vars_.size(); ++i)
    out << lbs_[i] << " <= " << vars_[i] << " <= " << ubs_[i] << "\n";
  out << "End";
}
}  // namespace sco
