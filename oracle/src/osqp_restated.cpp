// ORACLE — test infrastructure only (see sco_expr.hpp header).
// OSQP 1.0.0 restatement; see osqp_restated.hpp for provenance.
#include "osqp_restated.hpp"
#include "jitter.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <set>
#include <utility>

namespace orc
{
// ---------------------------------------------------------------- CSC helpers
void csc_axpy(const Csc& A, const double* x, double* y, double alpha, double beta)
{
  for (OsqpInt r = 0; r < A.m; ++r)
    y[r] = (beta == 0.0) ? 0.0 : beta * y[r];
  for (OsqpInt j = 0; j < A.n; ++j)
    for (OsqpInt p = A.p[j]; p < A.p[j + 1]; ++p)
      y[A.i[p]] += alpha * A.x[p] * x[j];
}

void csc_atxpy(const Csc& A, const double* x, double* y, double alpha, double beta)
{
  for (OsqpInt j = 0; j < A.n; ++j)
  {
    double s = 0;
    for (OsqpInt p = A.p[j]; p < A.p[j + 1]; ++p)
      s += A.x[p] * x[A.i[p]];
    y[j] = ((beta == 0.0) ? 0.0 : beta * y[j]) + alpha * s;
  }
}

void csc_sym_triu_axpy(const Csc& P, const double* x, double* y, double alpha, double beta)
{
  for (OsqpInt r = 0; r < P.n; ++r)
    y[r] = (beta == 0.0) ? 0.0 : beta * y[r];
  for (OsqpInt j = 0; j < P.n; ++j)
    for (OsqpInt p = P.p[j]; p < P.p[j + 1]; ++p)
    {
      const OsqpInt i = P.i[p];
      y[i] += alpha * P.x[p] * x[j];
      if (i != j)
        y[j] += alpha * P.x[p] * x[i];
    }
}

Csc csc_transpose(const Csc& A)
{
  Csc T;
  T.m = A.n;
  T.n = A.m;
  T.p.assign(static_cast<std::size_t>(A.m + 1), 0);
  const OsqpInt nnz = A.nnz();
  T.i.resize(static_cast<std::size_t>(nnz));
  T.x.resize(static_cast<std::size_t>(nnz));
  for (OsqpInt k = 0; k < nnz; ++k)
    T.p[A.i[k] + 1]++;
  for (OsqpInt r = 0; r < A.m; ++r)
    T.p[r + 1] += T.p[r];
  std::vector<OsqpInt> next(T.p.begin(), T.p.end() - 1);
  for (OsqpInt j = 0; j < A.n; ++j)
    for (OsqpInt p = A.p[j]; p < A.p[j + 1]; ++p)
    {
      const OsqpInt q = next[A.i[p]]++;
      T.i[q] = j;
      T.x[q] = A.x[p];
    }
  return T;
}

static double norm_inf(const std::vector<double>& v)
{
  double m = 0;
  for (double a : v)
    m = std::max(m, std::fabs(a));
  return m;
}
static double scaled_norm_inf(const std::vector<double>& s, const std::vector<double>& v)
{
  double m = 0;
  for (std::size_t i = 0; i < v.size(); ++i)
    m = std::max(m, std::fabs(s[i] * v[i]));
  return m;
}

// ------------------------------------------------------------------ LDL solver
// Minimum-degree ordering on the symmetric pattern (exact external degree,
// smallest index breaks ties). AMD in QDLDL; only affects fill and rounding.
void LdlSolver::order(const Csc& a)
{
  const OsqpInt n = a.n;
  std::vector<std::vector<OsqpInt>> adj(static_cast<std::size_t>(n));
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = a.p[j]; p < a.p[j + 1]; ++p)
    {
      const OsqpInt i = a.i[p];
      if (i != j)
        adj[j].push_back(i);
    }
  for (auto& v : adj)
  {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
  }
  std::set<std::pair<std::size_t, OsqpInt>> pq;
  for (OsqpInt j = 0; j < n; ++j)
    pq.insert({ adj[j].size(), j });
  std::vector<char> done(static_cast<std::size_t>(n), 0);
  perm_.clear();
  perm_.reserve(static_cast<std::size_t>(n));
  std::vector<OsqpInt> merged;
  while (!pq.empty())
  {
    const OsqpInt v = pq.begin()->second;
    pq.erase(pq.begin());
    done[v] = 1;
    perm_.push_back(v);
    const std::vector<OsqpInt> nv = adj[v];
    for (OsqpInt u : nv)
    {
      if (done[u])
        continue;
      pq.erase({ adj[u].size(), u });
      merged.clear();
      std::set_union(adj[u].begin(), adj[u].end(), nv.begin(), nv.end(), std::back_inserter(merged));
      adj[u].clear();
      for (OsqpInt w : merged)
        if (w != u && w != v && !done[w])
          adj[u].push_back(w);
      pq.insert({ adj[u].size(), u });
    }
    adj[v].clear();
  }
  pinv_.assign(static_cast<std::size_t>(n), 0);
  for (OsqpInt k = 0; k < n; ++k)
    pinv_[perm_[k]] = k;
}

int LdlSolver::factor(const Csc& a)
{
  n_ = a.n;
  order(a);
  // symbolic (ldl_symbolic)
  const OsqpInt n = n_;
  parent_.assign(static_cast<std::size_t>(n), -1);
  lnz_.assign(static_cast<std::size_t>(n), 0);
  std::vector<OsqpInt> flag(static_cast<std::size_t>(n), 0);
  for (OsqpInt k = 0; k < n; ++k)
  {
    parent_[k] = -1;
    flag[k] = k;
    lnz_[k] = 0;
    const OsqpInt kk = perm_[k];
    for (OsqpInt p = a.p[kk]; p < a.p[kk + 1]; ++p)
    {
      OsqpInt i = pinv_[a.i[p]];
      if (i < k)
      {
        for (; flag[i] != k; i = parent_[i])
        {
          if (parent_[i] == -1)
            parent_[i] = k;
          lnz_[i]++;
          flag[i] = k;
        }
      }
    }
  }
  lp_.assign(static_cast<std::size_t>(n + 1), 0);
  for (OsqpInt k = 0; k < n; ++k)
    lp_[k + 1] = lp_[k] + lnz_[k];
  li_.assign(static_cast<std::size_t>(lp_[n]), 0);
  lx_.assign(static_cast<std::size_t>(lp_[n]), 0.0);
  d_.assign(static_cast<std::size_t>(n), 0.0);
  work_.assign(static_cast<std::size_t>(n), 0.0);
  return numeric(a);
}

int LdlSolver::refactor(const Csc& a) { return numeric(a); }

int LdlSolver::numeric(const Csc& a)
{
  const OsqpInt n = n_;
  std::vector<double> y(static_cast<std::size_t>(n), 0.0);
  std::vector<OsqpInt> pattern(static_cast<std::size_t>(n), 0), flag(static_cast<std::size_t>(n), 0);
  std::vector<OsqpInt> lnz(static_cast<std::size_t>(n), 0);
  int npos = 0;
  for (OsqpInt k = 0; k < n; ++k)
  {
    y[k] = 0.0;
    OsqpInt top = n;
    flag[k] = k;
    lnz[k] = 0;
    const OsqpInt kk = perm_[k];
    for (OsqpInt p = a.p[kk]; p < a.p[kk + 1]; ++p)
    {
      OsqpInt i = pinv_[a.i[p]];
      if (i <= k)
      {
        y[i] += a.x[p];
        OsqpInt len = 0;
        for (; flag[i] != k; i = parent_[i])
        {
          pattern[len++] = i;
          flag[i] = k;
        }
        while (len > 0)
          pattern[--top] = pattern[--len];
      }
    }
    d_[k] = y[k];
    y[k] = 0.0;
    for (; top < n; top++)
    {
      const OsqpInt i = pattern[top];
      const double yi = y[i];
      y[i] = 0.0;
      const OsqpInt p2 = lp_[i] + lnz[i];
      OsqpInt p;
      for (p = lp_[i]; p < p2; p++)
        y[li_[p]] -= lx_[p] * yi;
      const double l_ki = yi / d_[i];
      d_[k] -= l_ki * yi;
      li_[p] = k;
      lx_[p] = l_ki;
      lnz[i]++;
    }
    if (d_[k] == 0.0)
      return -1;
    if (d_[k] > 0)
      ++npos;
  }
  return npos;
}

void LdlSolver::solve(double* b) const
{
  const OsqpInt n = n_;
  for (OsqpInt k = 0; k < n; ++k)
    work_[k] = b[perm_[k]];
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = lp_[j]; p < lp_[j + 1]; ++p)
      work_[li_[p]] -= lx_[p] * work_[j];
  for (OsqpInt j = 0; j < n; ++j)
    work_[j] /= d_[j];
  for (OsqpInt j = n - 1; j >= 0; --j)
    for (OsqpInt p = lp_[j]; p < lp_[j + 1]; ++p)
      work_[j] -= lx_[p] * work_[li_[p]];
  for (OsqpInt k = 0; k < n; ++k)
    b[perm_[k]] = work_[k];
}

// --------------------------------------------------------------- OSQP solver
static void limit_scaling(std::vector<double>& v)
{
  for (double& a : v)
  {
    a = a < OSQP_MIN_SCALING ? 1.0 : a;
    a = a > OSQP_MAX_SCALING ? OSQP_MAX_SCALING : a;
  }
}
static double limit_scaling(double a)
{
  a = a < OSQP_MIN_SCALING ? 1.0 : a;
  a = a > OSQP_MAX_SCALING ? OSQP_MAX_SCALING : a;
  return a;
}

// inf-norm of the columns of the full symmetric matrix stored upper-triangular
static void sym_triu_col_norm_inf(const Csc& P, std::vector<double>& out)
{
  std::fill(out.begin(), out.end(), 0.0);
  for (OsqpInt j = 0; j < P.n; ++j)
    for (OsqpInt p = P.p[j]; p < P.p[j + 1]; ++p)
    {
      const OsqpInt i = P.i[p];
      const double a = std::fabs(P.x[p]);
      out[j] = std::max(out[j], a);
      if (i != j)
        out[i] = std::max(out[i], a);
    }
}

void OsqpSolver::scale_data()
{
  const auto n = static_cast<std::size_t>(n_), m = static_cast<std::size_t>(m_);
  c_ = 1.0;
  D_.assign(n, 1.0);
  E_.assign(m, 1.0);
  std::vector<double> Dt(n), DtA(n), Et(m);
  for (int it = 0; it < settings_.scaling; ++it)
  {
    // compute_inf_norm_cols_KKT
    sym_triu_col_norm_inf(P_, Dt);
    std::fill(DtA.begin(), DtA.end(), 0.0);
    std::fill(Et.begin(), Et.end(), 0.0);
    for (OsqpInt j = 0; j < A_.n; ++j)
      for (OsqpInt p = A_.p[j]; p < A_.p[j + 1]; ++p)
      {
        const double a = std::fabs(A_.x[p]);
        DtA[j] = std::max(DtA[j], a);
        Et[A_.i[p]] = std::max(Et[A_.i[p]], a);
      }
    for (std::size_t j = 0; j < n; ++j)
      Dt[j] = std::max(Dt[j], DtA[j]);
    limit_scaling(Dt);
    limit_scaling(Et);
    for (auto& a : Dt)
      a = 1.0 / std::sqrt(a);
    for (auto& a : Et)
      a = 1.0 / std::sqrt(a);
    // P <- D P D
    for (OsqpInt j = 0; j < P_.n; ++j)
      for (OsqpInt p = P_.p[j]; p < P_.p[j + 1]; ++p)
        P_.x[p] = (P_.x[p] * Dt[P_.i[p]]) * Dt[j];
    // A <- E A D
    for (OsqpInt j = 0; j < A_.n; ++j)
      for (OsqpInt p = A_.p[j]; p < A_.p[j + 1]; ++p)
        A_.x[p] = (A_.x[p] * Et[A_.i[p]]) * Dt[j];
    for (std::size_t j = 0; j < n; ++j)
      q_[j] *= Dt[j];
    for (std::size_t j = 0; j < n; ++j)
      D_[j] *= Dt[j];
    for (std::size_t r = 0; r < m; ++r)
      E_[r] *= Et[r];
    // cost normalisation
    sym_triu_col_norm_inf(P_, Dt);
    double c_temp = 0;
    for (double a : Dt)
      c_temp += a;
    c_temp = (n > 0) ? c_temp / static_cast<double>(n) : 0.0;
    double inf_norm_q = limit_scaling(norm_inf(q_));
    c_temp = std::max(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1.0 / c_temp;
    for (auto& a : P_.x)
      a *= c_temp;
    for (auto& a : q_)
      a *= c_temp;
    c_ *= c_temp;
  }
  cinv_ = 1.0 / c_;
  Dinv_.resize(n);
  Einv_.resize(m);
  for (std::size_t j = 0; j < n; ++j)
    Dinv_[j] = 1.0 / D_[j];
  for (std::size_t r = 0; r < m; ++r)
    Einv_[r] = 1.0 / E_[r];
  for (std::size_t r = 0; r < m; ++r)
  {
    l_[r] *= E_[r];
    u_[r] *= E_[r];
  }
}

// OSQP 1.0 unscale_data: P <- cinv Dinv P Dinv, q <- Dinv (cinv q), A <- Einv A Dinv,
// l <- Einv l, u <- Einv u
void OsqpSolver::unscale_data()
{
  for (OsqpInt j = 0; j < P_.n; ++j)
    for (OsqpInt p = P_.p[j]; p < P_.p[j + 1]; ++p)
      P_.x[p] = ((P_.x[p] * cinv_) * Dinv_[P_.i[p]]) * Dinv_[j];
  for (OsqpInt j = 0; j < n_; ++j)
    q_[j] = (q_[j] * cinv_) * Dinv_[j];
  for (OsqpInt j = 0; j < A_.n; ++j)
    for (OsqpInt p = A_.p[j]; p < A_.p[j + 1]; ++p)
      A_.x[p] = (A_.x[p] * Einv_[A_.i[p]]) * Dinv_[j];
  for (OsqpInt r = 0; r < m_; ++r)
  {
    l_[r] = l_[r] * Einv_[r];
    u_[r] = u_[r] * Einv_[r];
  }
}

// OSQP 1.0 update_rho_vec: the rows whose constraint type changed get the rho
// of their new type; refactor only if one did
int OsqpSolver::update_rho_vec()
{
  bool changed = false;
  for (OsqpInt i = 0; i < m_; ++i)
  {
    int ct;
    double rv;
    if (l_[i] < -OSQP_INFTY * OSQP_MIN_SCALING && u_[i] > OSQP_INFTY * OSQP_MIN_SCALING)
    {
      ct = -1;
      rv = OSQP_RHO_MIN;
    }
    else if (u_[i] - l_[i] < OSQP_RHO_TOL)
    {
      ct = 1;
      rv = OSQP_RHO_EQ_OVER_RHO_INEQ * settings_.rho;
    }
    else
    {
      ct = 0;
      rv = settings_.rho;
    }
    if (constr_type_[i] != ct)
    {
      constr_type_[i] = ct;
      rho_vec_[i] = rv;
      rho_inv_vec_[i] = 1.0 / rv;
      kkt_.x[kkt_rho_diag_[i]] = -rho_inv_vec_[i];
      changed = true;
    }
  }
  if (!changed)
    return 0;
  const int npos = ldl_.refactor(kkt_);
  if (npos < 0)
    return 4;
  return (npos < n_) ? 5 : 0;
}

int OsqpSolver::update_data_vec(const double* q, const double* l, const double* u)
{
  if (l && u)
    for (OsqpInt i = 0; i < m_; ++i)
      if (l[i] > u[i])
        return 1;  // OSQP_DATA_VALIDATION_ERROR, data unchanged
  const bool sc = settings_.scaling > 0;
  if (q)
    for (OsqpInt j = 0; j < n_; ++j)
      q_[j] = sc ? (D_[j] * q[j]) * c_ : q[j];
  if (l && u)
  {
    for (OsqpInt i = 0; i < m_; ++i)
    {
      l_[i] = sc ? E_[i] * l[i] : l[i];
      u_[i] = sc ? E_[i] * u[i] : u[i];
    }
    return update_rho_vec();
  }
  return 0;
}

int OsqpSolver::update_data_mat(const double* Px, const double* Ax)
{
  const bool sc = settings_.scaling > 0;
  if (sc)
    unscale_data();
  if (Px)
    std::copy(Px, Px + P_.nnz(), P_.x.begin());
  if (Ax)
    std::copy(Ax, Ax + A_.nnz(), A_.x.begin());
  if (sc)
    scale_data();
  At_ = csc_transpose(A_);
  // linsys update_matrices: the KKT values with the current rho vector
  const int e = build_and_factor_kkt();
  if (e == 1)
    return 4;
  if (e == 2)
    return 5;
  return 0;
}

void OsqpSolver::set_rho_vec()
{
  settings_.rho = std::min(std::max(settings_.rho, OSQP_RHO_MIN), OSQP_RHO_MAX);
  const auto m = static_cast<std::size_t>(m_);
  constr_type_.assign(m, 0);
  rho_vec_.assign(m, 0.0);
  rho_inv_vec_.assign(m, 0.0);
  for (std::size_t i = 0; i < m; ++i)
  {
    if (l_[i] < -OSQP_INFTY * OSQP_MIN_SCALING && u_[i] > OSQP_INFTY * OSQP_MIN_SCALING)
    {
      constr_type_[i] = -1;
      rho_vec_[i] = OSQP_RHO_MIN;
    }
    else if (u_[i] - l_[i] < OSQP_RHO_TOL)
    {
      constr_type_[i] = 1;
      rho_vec_[i] = OSQP_RHO_EQ_OVER_RHO_INEQ * settings_.rho;
    }
    else
    {
      constr_type_[i] = 0;
      rho_vec_[i] = settings_.rho;
    }
    rho_inv_vec_[i] = 1.0 / rho_vec_[i];
  }
}

// KKT = [P + sigma I, A'; A, -diag(1/rho)] as a full symmetric CSC
int OsqpSolver::build_and_factor_kkt()
{
  const OsqpInt n = n_, m = m_, N = n_ + m_;
  Csc K;
  K.m = K.n = N;
  K.p.assign(static_cast<std::size_t>(N + 1), 0);
  // columns 0..n-1: full P column j (both triangles) + sigma on diag, then A column j (rows n+r)
  // build P full columns
  std::vector<std::vector<std::pair<OsqpInt, double>>> cols(static_cast<std::size_t>(N));
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = P_.p[j]; p < P_.p[j + 1]; ++p)
    {
      const OsqpInt i = P_.i[p];
      cols[j].push_back({ i, P_.x[p] });
      if (i != j)
        cols[i].push_back({ j, P_.x[p] });
    }
  for (OsqpInt j = 0; j < n; ++j)
    cols[j].push_back({ j, settings_.sigma });
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = A_.p[j]; p < A_.p[j + 1]; ++p)
    {
      cols[j].push_back({ n + A_.i[p], A_.x[p] });
      cols[n + A_.i[p]].push_back({ j, A_.x[p] });
    }
  for (OsqpInt r = 0; r < m; ++r)
    cols[n + r].push_back({ n + r, -rho_inv_vec_[r] });
  kkt_rho_diag_.assign(static_cast<std::size_t>(m), 0);
  for (OsqpInt j = 0; j < N; ++j)
  {
    auto& c = cols[j];
    std::stable_sort(c.begin(), c.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    // sum duplicates
    OsqpInt last = -1;
    for (const auto& e : c)
    {
      if (e.first == last)
        K.x.back() += e.second;
      else
      {
        K.i.push_back(e.first);
        K.x.push_back(e.second);
        last = e.first;
      }
    }
    K.p[j + 1] = static_cast<OsqpInt>(K.i.size());
  }
  for (OsqpInt r = 0; r < m; ++r)
  {
    const OsqpInt j = n + r;
    for (OsqpInt p = K.p[j]; p < K.p[j + 1]; ++p)
      if (K.i[p] == j)
        kkt_rho_diag_[r] = p;
  }
  kkt_ = std::move(K);
  const int npos = ldl_.factor(kkt_);
  if (npos < 0)
    return 1;  // zero pivot
  if (npos < n_)
    return 2;  // not quasi-definite: non-convex
  return 0;
}

int OsqpSolver::setup(const Csc& P, const double* q, const Csc& A, const double* l, const double* u, OsqpInt m,
                      OsqpInt n, const OsqpSettings& settings)
{
  // validate_data
  if (P.n != n || P.m != n || A.n != n || A.m != m)
    return 1;
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = P.p[j]; p < P.p[j + 1]; ++p)
      if (P.i[p] > j)
        return 1;  // P not upper triangular
  for (OsqpInt i = 0; i < m; ++i)
    if (l[i] > u[i])
      return 1;
  settings_ = settings;
  if (settings_.adaptive_rho == 1 && settings_.adaptive_rho_interval == 0)
    settings_.adaptive_rho_interval = (settings_.check_termination != 0) ?
                                          OSQP_ADAPTIVE_RHO_MULTIPLE_TERMINATION * settings_.check_termination :
                                          OSQP_ADAPTIVE_RHO_FIXED;
  n_ = n;
  m_ = m;
  P_ = P;
  A_ = A;
  q_.assign(q, q + n);
  l_.assign(l, l + m);
  u_.assign(u, u + m);
  const auto nn = static_cast<std::size_t>(n), mm = static_cast<std::size_t>(m);
  if (settings_.scaling > 0)
    scale_data();
  else
  {
    c_ = cinv_ = 1;
    D_.assign(nn, 1);
    Dinv_.assign(nn, 1);
    E_.assign(mm, 1);
    Einv_.assign(mm, 1);
  }
  At_ = csc_transpose(A_);
  set_rho_vec();
  x_.assign(nn, 0.0);
  x_prev_.assign(nn, 0.0);
  delta_x_.assign(nn, 0.0);
  Px_.assign(nn, 0.0);
  Aty_.assign(nn, 0.0);
  Atdelta_y_.assign(nn, 0.0);
  Pdelta_x_.assign(nn, 0.0);
  z_.assign(mm, 0.0);
  y_.assign(mm, 0.0);
  z_prev_.assign(mm, 0.0);
  delta_y_.assign(mm, 0.0);
  Ax_.assign(mm, 0.0);
  Adelta_x_.assign(mm, 0.0);
  xz_tilde_.assign(nn + mm, 0.0);
  sol_.assign(nn + mm, 0.0);
  status_val = OSQP_UNSOLVED;
  status_polish = 0;
  iter = 0;
  rho_updates = 0;
  const int e = build_and_factor_kkt();
  if (e == 1)
    return 4;  // OSQP_LINSYS_SOLVER_INIT_ERROR
  if (e == 2)
    return 5;  // OSQP_NONCVX_ERROR
  return 0;
}

int OsqpSolver::warm_start(const double* x, const double* y)
{
  settings_.warm_starting = 1;
  const auto n = static_cast<std::size_t>(n_), m = static_cast<std::size_t>(m_);
  if (x)
    x_.assign(x, x + n);
  if (y)
    y_.assign(y, y + m);
  if (settings_.scaling > 0)
  {
    if (x)
      for (std::size_t j = 0; j < n; ++j)
        x_[j] *= Dinv_[j];
    if (y)
      for (std::size_t r = 0; r < m; ++r)
      {
        y_[r] *= Einv_[r];
        y_[r] *= c_;
      }
  }
  if (x)
    csc_axpy(A_, x_.data(), z_.data(), 1.0, 0.0);
  return 0;
}

void OsqpSolver::cold_start()
{
  std::fill(x_.begin(), x_.end(), 0.0);
  std::fill(z_.begin(), z_.end(), 0.0);
  std::fill(y_.begin(), y_.end(), 0.0);
}

void OsqpSolver::update_xz_tilde()
{
  const OsqpInt n = n_, m = m_;
  for (OsqpInt j = 0; j < n; ++j)
    xz_tilde_[j] = settings_.sigma * x_prev_[j] - q_[j];
  for (OsqpInt r = 0; r < m; ++r)
    xz_tilde_[n + r] = z_prev_[r] - rho_inv_vec_[r] * y_[r];
  // direct KKT solve, stores the solution in sol_
  std::copy(xz_tilde_.begin(), xz_tilde_.end(), sol_.begin());
  ldl_.solve(sol_.data());
  if (g_jitter.kkt_rel > 0)  // parity-gate rounding jitter (jitter.hpp)
    for (auto& v : sol_)
      v *= 1.0 + g_jitter.kkt_rel * jitterU();
  for (OsqpInt j = 0; j < n; ++j)
    xz_tilde_[j] = sol_[j];
  for (OsqpInt r = 0; r < m; ++r)
    xz_tilde_[n + r] += rho_inv_vec_[r] * sol_[n + r];
}

void OsqpSolver::update_x()
{
  const double a = settings_.alpha;
  for (OsqpInt j = 0; j < n_; ++j)
  {
    x_[j] = a * xz_tilde_[j] + (1.0 - a) * x_prev_[j];
    delta_x_[j] = x_[j] - x_prev_[j];
  }
}

void OsqpSolver::update_z()
{
  const double a = settings_.alpha;
  for (OsqpInt r = 0; r < m_; ++r)
  {
    double zr = rho_inv_vec_[r] * y_[r];
    zr = zr + a * xz_tilde_[n_ + r];
    zr = zr + (1.0 - a) * z_prev_[r];
    z_[r] = std::min(std::max(zr, l_[r]), u_[r]);
  }
}

void OsqpSolver::update_y()
{
  const double a = settings_.alpha;
  for (OsqpInt r = 0; r < m_; ++r)
  {
    delta_y_[r] = rho_vec_[r] * (a * xz_tilde_[n_ + r] + (1.0 - a) * z_prev_[r] - z_[r]);
    y_[r] += delta_y_[r];
  }
}

// Ax - z, stored in z_prev_ (workspace reuse as in OSQP); Ax kept in Ax_
double OsqpSolver::compute_prim_res(const std::vector<double>& x, const std::vector<double>& z)
{
  csc_axpy(A_, x.data(), Ax_.data(), 1.0, 0.0);
  for (OsqpInt r = 0; r < m_; ++r)
    z_prev_[r] = Ax_[r] - z[r];
  if (settings_.scaling > 0 && !settings_.scaled_termination)
    return scaled_norm_inf(Einv_, z_prev_);
  return norm_inf(z_prev_);
}

// q + P x + A' y, stored in x_prev_; Px_, Aty_ kept
double OsqpSolver::compute_dual_res(const std::vector<double>& x, const std::vector<double>& y)
{
  csc_sym_triu_axpy(P_, x.data(), Px_.data(), 1.0, 0.0);
  for (OsqpInt j = 0; j < n_; ++j)
    x_prev_[j] = q_[j] + Px_[j];
  if (m_ > 0)
  {
    csc_atxpy(A_, y.data(), Aty_.data(), 1.0, 0.0);
    for (OsqpInt j = 0; j < n_; ++j)
      x_prev_[j] += Aty_[j];
  }
  if (settings_.scaling > 0 && !settings_.scaled_termination)
    return cinv_ * scaled_norm_inf(Dinv_, x_prev_);
  return norm_inf(x_prev_);
}

double OsqpSolver::compute_prim_tol(double eps_abs, double eps_rel) const
{
  double max_rel;
  if (settings_.scaling > 0 && !settings_.scaled_termination)
    max_rel = std::max(scaled_norm_inf(Einv_, z_), scaled_norm_inf(Einv_, Ax_));
  else
    max_rel = std::max(norm_inf(z_), norm_inf(Ax_));
  return eps_abs + eps_rel * max_rel;
}

double OsqpSolver::compute_dual_tol(double eps_abs, double eps_rel) const
{
  double max_rel;
  if (settings_.scaling > 0 && !settings_.scaled_termination)
  {
    max_rel = scaled_norm_inf(Dinv_, q_);
    max_rel = std::max(max_rel, scaled_norm_inf(Dinv_, Aty_));
    max_rel = std::max(max_rel, scaled_norm_inf(Dinv_, Px_));
    max_rel *= cinv_;
  }
  else
    max_rel = std::max(std::max(norm_inf(q_), norm_inf(Aty_)), norm_inf(Px_));
  return eps_abs + eps_rel * max_rel;
}

bool OsqpSolver::is_primal_infeasible(double eps)
{
  for (OsqpInt r = 0; r < m_; ++r)
  {
    if (u_[r] > OSQP_INFTY * OSQP_MIN_SCALING)
    {
      if (l_[r] < -OSQP_INFTY * OSQP_MIN_SCALING)
        delta_y_[r] = 0.0;
      else
        delta_y_[r] = std::min(delta_y_[r], 0.0);
    }
    else if (l_[r] < -OSQP_INFTY * OSQP_MIN_SCALING)
      delta_y_[r] = std::max(delta_y_[r], 0.0);
  }
  double norm_dy;
  if (settings_.scaling > 0 && !settings_.scaled_termination)
    norm_dy = scaled_norm_inf(E_, delta_y_);
  else
    norm_dy = norm_inf(delta_y_);
  if (norm_dy > OSQP_DIVISION_TOL)
  {
    double ineq_lhs = 0;
    for (OsqpInt r = 0; r < m_; ++r)
      ineq_lhs += u_[r] * std::max(delta_y_[r], 0.0) + l_[r] * std::min(delta_y_[r], 0.0);
    if (ineq_lhs < eps * norm_dy)
    {
      csc_atxpy(A_, delta_y_.data(), Atdelta_y_.data(), 1.0, 0.0);
      if (settings_.scaling > 0 && !settings_.scaled_termination)
        for (OsqpInt j = 0; j < n_; ++j)
          Atdelta_y_[j] *= Dinv_[j];
      return norm_inf(Atdelta_y_) < eps * norm_dy;
    }
  }
  return false;
}

bool OsqpSolver::is_dual_infeasible(double eps)
{
  double norm_dx, cost_scaling;
  if (settings_.scaling > 0 && !settings_.scaled_termination)
  {
    norm_dx = scaled_norm_inf(D_, delta_x_);
    cost_scaling = c_;
  }
  else
  {
    norm_dx = norm_inf(delta_x_);
    cost_scaling = 1.0;
  }
  if (norm_dx > OSQP_DIVISION_TOL)
  {
    double qdx = 0;
    for (OsqpInt j = 0; j < n_; ++j)
      qdx += q_[j] * delta_x_[j];
    if (qdx < cost_scaling * eps * norm_dx)
    {
      csc_sym_triu_axpy(P_, delta_x_.data(), Pdelta_x_.data(), 1.0, 0.0);
      if (settings_.scaling > 0 && !settings_.scaled_termination)
        for (OsqpInt j = 0; j < n_; ++j)
          Pdelta_x_[j] *= Dinv_[j];
      if (norm_inf(Pdelta_x_) < cost_scaling * eps * norm_dx)
      {
        csc_axpy(A_, delta_x_.data(), Adelta_x_.data(), 1.0, 0.0);
        if (settings_.scaling > 0 && !settings_.scaled_termination)
          for (OsqpInt r = 0; r < m_; ++r)
            Adelta_x_[r] *= Einv_[r];
        for (OsqpInt r = 0; r < m_; ++r)
          if (((u_[r] < OSQP_INFTY * OSQP_MIN_SCALING) && (Adelta_x_[r] > eps * norm_dx)) ||
              ((l_[r] > -OSQP_INFTY * OSQP_MIN_SCALING) && (Adelta_x_[r] < -eps * norm_dx)))
            return false;
        return true;
      }
    }
  }
  return false;
}

bool OsqpSolver::check_termination(bool approximate)
{
  double eps_abs = settings_.eps_abs, eps_rel = settings_.eps_rel;
  double eps_prim_inf = settings_.eps_prim_inf, eps_dual_inf = settings_.eps_dual_inf;
  if (approximate)
  {
    eps_abs *= 10;
    eps_rel *= 10;
    eps_prim_inf *= 10;
    eps_dual_inf *= 10;
  }
  bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
  if (m_ == 0)
    prim_ok = true;
  else
  {
    const double eps_prim = compute_prim_tol(eps_abs, eps_rel);
    if (prim_res < eps_prim)
      prim_ok = true;
    else
      prim_inf = is_primal_infeasible(eps_prim_inf);
  }
  const double eps_dual = compute_dual_tol(eps_abs, eps_rel);
  if (dual_res < eps_dual)
    dual_ok = true;
  else
    dual_inf = is_dual_infeasible(eps_dual_inf);

  if (prim_ok && dual_ok)
  {
    status_val = approximate ? OSQP_SOLVED_INACCURATE : OSQP_SOLVED;
    return true;
  }
  if (prim_inf)
  {
    status_val = approximate ? OSQP_PRIMAL_INFEASIBLE_INACCURATE : OSQP_PRIMAL_INFEASIBLE;
    return true;
  }
  if (dual_inf)
  {
    status_val = approximate ? OSQP_DUAL_INFEASIBLE_INACCURATE : OSQP_DUAL_INFEASIBLE;
    return true;
  }
  return false;
}

double OsqpSolver::compute_rho_estimate() const
{
  double pr = norm_inf(z_prev_);
  double dr = norm_inf(x_prev_);
  double prn = std::max(norm_inf(z_), norm_inf(Ax_));
  pr /= (prn + OSQP_DIVISION_TOL);
  double drn = std::max(norm_inf(q_), norm_inf(Aty_));
  drn = std::max(drn, norm_inf(Px_));
  dr /= (drn + OSQP_DIVISION_TOL);
  double est = settings_.rho * std::sqrt(pr / (dr + OSQP_DIVISION_TOL));
  return std::min(std::max(est, OSQP_RHO_MIN), OSQP_RHO_MAX);
}

int OsqpSolver::update_rho(double rho_new)
{
  if (rho_new <= 0)
    return 1;
  settings_.rho = std::min(std::max(rho_new, OSQP_RHO_MIN), OSQP_RHO_MAX);
  for (OsqpInt r = 0; r < m_; ++r)
  {
    if (constr_type_[r] == 0)
    {
      rho_vec_[r] = settings_.rho;
      rho_inv_vec_[r] = 1.0 / settings_.rho;
    }
    else if (constr_type_[r] == 1)
    {
      rho_vec_[r] = OSQP_RHO_EQ_OVER_RHO_INEQ * settings_.rho;
      rho_inv_vec_[r] = 1.0 / rho_vec_[r];
    }
    kkt_.x[kkt_rho_diag_[r]] = -rho_inv_vec_[r];
  }
  const int npos = ldl_.refactor(kkt_);
  return (npos < n_) ? 1 : 0;
}

int OsqpSolver::adapt_rho()
{
  const double rho_new = compute_rho_estimate();
  if (rho_new > settings_.rho * settings_.adaptive_rho_tolerance ||
      rho_new < settings_.rho / settings_.adaptive_rho_tolerance)
  {
    ++rho_updates;
    return update_rho(rho_new);
  }
  return 0;
}

int OsqpSolver::solve()
{
  if (!settings_.warm_starting)
    cold_start();
  status_val = OSQP_UNSOLVED;
  status_polish = 0;
  polish_margin = 1e300;
  bool can_check = false;
  OsqpInt it;
  for (it = 1; it <= settings_.max_iter; ++it)
  {
    std::swap(x_, x_prev_);
    std::swap(z_, z_prev_);
    update_xz_tilde();
    update_x();
    update_z();
    update_y();
    can_check = settings_.check_termination && (it % settings_.check_termination == 0);
    if (can_check)
    {
      iter = it;
      prim_res = (m_ > 0) ? compute_prim_res(x_, z_) : 0.0;
      dual_res = compute_dual_res(x_, y_);
      if (check_termination(false))
        break;
    }
    if (settings_.adaptive_rho && settings_.adaptive_rho_interval && (it % settings_.adaptive_rho_interval == 0))
    {
      if (!can_check)
      {
        iter = it;
        prim_res = (m_ > 0) ? compute_prim_res(x_, z_) : 0.0;
        dual_res = compute_dual_res(x_, y_);
      }
      if (adapt_rho() != 0)
      {
        status_val = OSQP_NON_CVX;
        store_solution();
        return 1;
      }
    }
  }
  if (!can_check)
  {
    iter = it - 1;
    prim_res = (m_ > 0) ? compute_prim_res(x_, z_) : 0.0;
    dual_res = compute_dual_res(x_, y_);
    check_termination(false);
  }
  if (status_val == OSQP_UNSOLVED)
  {
    if (!check_termination(true))
      status_val = OSQP_MAX_ITER_REACHED;
  }
  if (settings_.polishing && status_val == OSQP_SOLVED)
    polish();
  store_solution();
  return 0;
}

void OsqpSolver::polish()
{
  const OsqpInt n = n_, m = m_;
  // form_Ared: active set guess, rows kept in original order
  std::vector<int> flag(static_cast<std::size_t>(m), 0);  // -1 lower, +1 upper, 0 inactive
  std::vector<OsqpInt> act;
  polish_margin = 1e300;
  for (OsqpInt r = 0; r < m; ++r)
  {
    if (l_[r] > -OSQP_INFTY * OSQP_MIN_SCALING)
      polish_margin = std::min(polish_margin, std::fabs((z_[r] - l_[r]) + y_[r]));
    if (u_[r] < OSQP_INFTY * OSQP_MIN_SCALING)
      polish_margin = std::min(polish_margin, std::fabs((u_[r] - z_[r]) - y_[r]));
    if (z_[r] - l_[r] < -y_[r])
      flag[r] = -1;
    else if (u_[r] - z_[r] < y_[r])
      flag[r] = 1;
    if (flag[r] != 0)
      act.push_back(r);
  }
  const auto mred = static_cast<OsqpInt>(act.size());
  std::vector<OsqpInt> row_map(static_cast<std::size_t>(m), -1);
  for (OsqpInt k = 0; k < mred; ++k)
    row_map[act[k]] = k;
  // Ared as CSC (mred x n)
  Csc Ared;
  Ared.m = mred;
  Ared.n = n;
  Ared.p.assign(static_cast<std::size_t>(n + 1), 0);
  for (OsqpInt j = 0; j < n; ++j)
  {
    for (OsqpInt p = A_.p[j]; p < A_.p[j + 1]; ++p)
      if (row_map[A_.i[p]] >= 0)
      {
        Ared.i.push_back(row_map[A_.i[p]]);
        Ared.x.push_back(A_.x[p]);
      }
    Ared.p[j + 1] = static_cast<OsqpInt>(Ared.i.size());
  }
  // reduced KKT [P + delta I, Ared'; Ared, -delta I]
  const OsqpInt N = n + mred;
  std::vector<std::vector<std::pair<OsqpInt, double>>> cols(static_cast<std::size_t>(N));
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = P_.p[j]; p < P_.p[j + 1]; ++p)
    {
      const OsqpInt i = P_.i[p];
      cols[j].push_back({ i, P_.x[p] });
      if (i != j)
        cols[i].push_back({ j, P_.x[p] });
    }
  for (OsqpInt j = 0; j < n; ++j)
    cols[j].push_back({ j, settings_.delta });
  for (OsqpInt j = 0; j < n; ++j)
    for (OsqpInt p = Ared.p[j]; p < Ared.p[j + 1]; ++p)
    {
      cols[j].push_back({ n + Ared.i[p], Ared.x[p] });
      cols[n + Ared.i[p]].push_back({ j, Ared.x[p] });
    }
  for (OsqpInt k = 0; k < mred; ++k)
    cols[n + k].push_back({ n + k, -settings_.delta });
  Csc K;
  K.m = K.n = N;
  K.p.assign(static_cast<std::size_t>(N + 1), 0);
  for (OsqpInt j = 0; j < N; ++j)
  {
    auto& c = cols[j];
    std::stable_sort(c.begin(), c.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    OsqpInt last = -1;
    for (const auto& e : c)
    {
      if (e.first == last)
        K.x.back() += e.second;
      else
      {
        K.i.push_back(e.first);
        K.x.push_back(e.second);
        last = e.first;
      }
    }
    K.p[j + 1] = static_cast<OsqpInt>(K.i.size());
  }
  LdlSolver plsh;
  const int npos = plsh.factor(K);
  if (npos < n)
  {
    status_polish = -1;
    return;
  }
  // rhs_red = [-q; l_low / u_upp]
  std::vector<double> rhs(static_cast<std::size_t>(N)), sol(static_cast<std::size_t>(N)), tmp(static_cast<std::size_t>(N));
  for (OsqpInt j = 0; j < n; ++j)
    rhs[j] = -q_[j];
  for (OsqpInt k = 0; k < mred; ++k)
    rhs[n + k] = (flag[act[k]] < 0) ? l_[act[k]] : u_[act[k]];
  sol = rhs;
  plsh.solve(sol.data());
  if (g_jitter.kkt_rel > 0)
    for (auto& v : sol)
      v *= 1.0 + g_jitter.kkt_rel * jitterU();
  // iterative refinement on the unregularised KKT
  for (int itr = 0; itr < settings_.polish_refine_iter; ++itr)
  {
    tmp = rhs;
    std::vector<double> t1(static_cast<std::size_t>(n)), t2(static_cast<std::size_t>(n)),
        t3(static_cast<std::size_t>(mred));
    csc_sym_triu_axpy(P_, sol.data(), t1.data(), 1.0, 0.0);
    csc_atxpy(Ared, sol.data() + n, t2.data(), 1.0, 0.0);
    csc_axpy(Ared, sol.data(), t3.data(), 1.0, 0.0);
    for (OsqpInt j = 0; j < n; ++j)
      tmp[j] = tmp[j] - t1[j] - t2[j];
    for (OsqpInt k = 0; k < mred; ++k)
      tmp[n + k] -= t3[k];
    plsh.solve(tmp.data());
    for (OsqpInt k = 0; k < N; ++k)
      sol[k] += tmp[k];
  }
  std::vector<double> px(sol.begin(), sol.begin() + n);
  std::vector<double> pz(static_cast<std::size_t>(m)), py(static_cast<std::size_t>(m), 0.0);
  csc_axpy(A_, px.data(), pz.data(), 1.0, 0.0);
  for (OsqpInt r = 0; r < m; ++r)
    py[r] = (row_map[r] >= 0) ? sol[n + row_map[r]] : 0.0;
  // project_normalcone
  for (OsqpInt r = 0; r < m; ++r)
  {
    const double t = pz[r] + py[r];
    pz[r] = std::min(std::max(t, l_[r]), u_[r]);
    py[r] = t - pz[r];
  }
  // residuals at the polished point (update_info(.., polish = 1))
  const double pol_prim = (m > 0) ? compute_prim_res(px, pz) : 0.0;
  const double pol_dual = compute_dual_res(px, py);
  const bool ok = (pol_prim < prim_res && pol_dual < dual_res) || (pol_prim < prim_res && dual_res < 1e-10) ||
                  (pol_dual < dual_res && prim_res < 1e-10);
  if (ok)
  {
    prim_res = pol_prim;
    dual_res = pol_dual;
    status_polish = 1;
    x_ = px;
    z_ = pz;
    y_ = py;
  }
  else
    status_polish = -1;
}

void OsqpSolver::store_solution()
{
  const auto n = static_cast<std::size_t>(n_), m = static_cast<std::size_t>(m_);
  sol_x.assign(n, 0.0);
  sol_y.assign(m, 0.0);
  if (status_val != OSQP_PRIMAL_INFEASIBLE && status_val != OSQP_PRIMAL_INFEASIBLE_INACCURATE &&
      status_val != OSQP_DUAL_INFEASIBLE && status_val != OSQP_DUAL_INFEASIBLE_INACCURATE)
  {
    for (std::size_t j = 0; j < n; ++j)
      sol_x[j] = (settings_.scaling > 0) ? D_[j] * x_[j] : x_[j];
    if (g_jitter.sol_rel > 0)  // parity-gate rounding jitter (jitter.hpp)
      for (std::size_t j = 0; j < n; ++j)
        sol_x[j] *= 1.0 + g_jitter.sol_rel * jitterU();
    for (std::size_t r = 0; r < m; ++r)
      sol_y[r] = (settings_.scaling > 0) ? cinv_ * (E_[r] * y_[r]) : y_[r];
  }
  else
  {
    std::fill(sol_x.begin(), sol_x.end(), NAN);
    std::fill(sol_y.begin(), sol_y.end(), NAN);
    cold_start();
  }
}

}  // namespace orc
