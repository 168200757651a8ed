// CPU replay of qp_csc.hip's level-scheduled sparse LDL^T (kkt_factor /
// kkt_solve) over kkt_symbolic's analysis: the numeric steps run level by level
// with the work inside a level in reversed and shuffled order (the device runs
// it in parallel), L starts as NaN so a read of an entry the schedule has not
// produced yet poisons the result, and the solve is checked against the KKT
// matrix itself.  Cases: random sparse QPs, a trajectory-shaped QP with
// hinge / contact rows, a dense P, m = 0, the polish variant (decoupled rows).
// Exit status 0 = every case passed.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../csrc/kkt_symbolic.hpp"

namespace
{
struct Qp
{
  int n = 0, m = 0;
  std::vector<int> Pp, Pi, Ap, Ai;
  std::vector<double> Px, Ax, rhoinv;
  std::vector<int> active;  // polish: rows kept (others decoupled with diagonal -1)
};

void add_col(std::vector<int>& p, std::vector<int>& idx, std::vector<double>& x, std::vector<std::pair<int, double>> c)
{
  std::sort(c.begin(), c.end());
  c.erase(std::unique(c.begin(), c.end(), [](auto& a, auto& b) { return a.first == b.first; }), c.end());
  for (auto& e : c)
  {
    idx.push_back(e.first);
    x.push_back(e.second);
  }
  p.push_back(static_cast<int>(idx.size()));
}

// dense KKT of the QP (ADMM: sigma, -1/rho; polish: delta, active rows)
std::vector<double> dense(const Qp& q, bool pol, double sigma)
{
  const int N = q.n + q.m;
  std::vector<double> K(static_cast<size_t>(N) * N, 0.0);
  for (int j = 0; j < q.n; ++j)
  {
    for (int e = q.Pp[j]; e < q.Pp[j + 1]; ++e)
    {
      K[q.Pi[e] * N + j] += q.Px[e];
      if (q.Pi[e] != j)
        K[j * N + q.Pi[e]] += q.Px[e];
    }
    K[j * N + j] += sigma;
    for (int e = q.Ap[j]; e < q.Ap[j + 1]; ++e)
    {
      const int r = q.Ai[e];
      if (pol && !q.active[r])
        continue;
      K[(q.n + r) * N + j] = K[j * N + q.n + r] = q.Ax[e];
    }
  }
  for (int r = 0; r < q.m; ++r)
    K[(q.n + r) * N + q.n + r] = pol ? (q.active[r] ? -sigma : -1.0) : -q.rhoinv[r];
  return K;
}

bool check(const char* name, const Qp& q, bool pol, std::mt19937& rng)
{
  KktSymbolic S;
  const std::string why = kkt_symbolic(q.n, q.m, q.Pp.data(), q.Pi.data(), q.Ap.data(), q.Ai.data(), S);
  if (!why.empty())
  {
    std::printf("FAIL %s: %s\n", name, why.c_str());
    return false;
  }
  const int N = q.n + q.m, nlev = static_cast<int>(S.lvp.size()) - 1;
  const double sigma = pol ? 1e-6 : 0.5;  // polish: delta
  auto entry = [&](int code) {
    if (code < 0)
      return 0.0;
    const int e = code >> 1;
    if (!(code & 1))
      return q.Px[e];
    return (pol && !q.active[q.Ai[e]]) ? 0.0 : q.Ax[e];
  };
  auto diag = [&](int k) {
    const int o = S.perm[k];
    if (o < q.n)
      return (S.dpd[k] >= 0 ? q.Px[S.dpd[k]] : 0.0) + sigma;
    const int r = o - q.n;
    return pol ? (q.active[r] ? -sigma : -1.0) : -q.rhoinv[r];
  };
  std::vector<double> LX(S.lrj.size(), NAN), DG(static_cast<size_t>(N), NAN);
  for (int lev = 0; lev < nlev; ++lev)
  {
    std::vector<int> nodes(S.lvn.begin() + S.lvp[lev], S.lvn.begin() + S.lvp[lev + 1]);
    std::shuffle(nodes.begin(), nodes.end(), rng);
    for (int k : nodes)
    {
      double d = diag(k);
      for (int e = S.lrp[k]; e < S.lrp[k + 1]; ++e)
        d -= (LX[e] * DG[S.lrj[e]]) * LX[e];
      DG[k] = d;
    }
    std::vector<int> items;
    for (int t = S.fip[lev]; t < S.fip[lev + 1]; ++t)
      items.push_back(t);
    std::reverse(items.begin(), items.end());
    std::shuffle(items.begin(), items.end(), rng);
    for (int t : items)
    {
      const int k = S.fik[t], c = S.fic[t], i = S.lci[c];
      if (S.lcpos[c] < S.lrp[i] || S.lcpos[c] >= S.lrp[i + 1] || S.lrj[S.lcpos[c]] != k)
      {
        std::printf("FAIL %s: column entry %d does not point at L(%d, %d)\n", name, c, i, k);
        return false;
      }
      double s = entry(S.lksrc[c]);
      int a = S.lrp[i], b = S.lrp[k];
      while (a < S.lrp[i + 1] && b < S.lrp[k + 1])
      {
        const int ja = S.lrj[a], jb = S.lrj[b];
        if (ja == jb)
        {
          s -= (LX[a] * DG[ja]) * LX[b];
          ++a;
          ++b;
        }
        else if (ja < jb)
          ++a;
        else
          ++b;
      }
      LX[S.lcpos[c]] = s / DG[k];
    }
  }
  // solve K x = b for a random b
  std::uniform_real_distribution<double> U(-1, 1);
  std::vector<double> b(static_cast<size_t>(N)), w(static_cast<size_t>(N)), x(static_cast<size_t>(N));
  for (auto& v : b)
    v = U(rng);
  if (pol)
    for (int r = 0; r < q.m; ++r)
      if (!q.active[r])
        b[q.n + r] = 0;
  for (int k = 0; k < N; ++k)
    w[k] = b[S.perm[k]];
  // the forward solve as the device runs it: passes of row segments
  // (S.fwp..fwb), the segments of a pass shuffled; every column a segment
  // reads must be final (all of its row's segments done) before the pass, and
  // each row's segments must tile its entries in order -- then the result is
  // bitwise the level-by-level forward solve below
  std::vector<double> wp = w;
  {
    std::vector<int> left(static_cast<size_t>(N)), next(static_cast<size_t>(N));
    for (int k = 0; k < N; ++k)
    {
      left[k] = S.lrp[k + 1] - S.lrp[k];
      next[k] = S.lrp[k];
    }
    bool sched_ok = true;
    const int npass = static_cast<int>(S.fwp.size()) - 1;
    for (int ps = 0; ps < npass; ++ps)
    {
      std::vector<int> items;
      for (int t = S.fwp[ps]; t < S.fwp[ps + 1]; ++t)
        items.push_back(t);
      std::shuffle(items.begin(), items.end(), rng);
      std::vector<int> done_before = left;  // finality as of the pass's start
      for (int t : items)
      {
        const int k = S.fwk[t];
        if (S.fwa[t] != next[k] || S.fwb[t] <= S.fwa[t])
          sched_ok = false;
        double s = wp[k];
        for (int e = S.fwa[t]; e < S.fwb[t]; ++e)
        {
          if (done_before[S.lrj[e]] != 0)
            sched_ok = false;
          s -= LX[e] * wp[S.lrj[e]];
        }
        wp[k] = s;
        next[k] = S.fwb[t];
        left[k] -= S.fwb[t] - S.fwa[t];
      }
    }
    for (int k = 0; k < N; ++k)
      if (left[k] != 0)
        sched_ok = false;
    if (!sched_ok)
    {
      std::printf("FAIL %s: forward pass schedule\n", name);
      return false;
    }
  }
  for (int lev = 0; lev < nlev; ++lev)
    for (int t = S.lvp[lev + 1] - 1; t >= S.lvp[lev]; --t)
    {
      const int k = S.lvn[t];
      double s = w[k];
      for (int e = S.lrp[k]; e < S.lrp[k + 1]; ++e)
        s -= LX[e] * w[S.lrj[e]];
      w[k] = s;
    }
  if (std::memcmp(wp.data(), w.data(), sizeof(double) * static_cast<size_t>(N)) != 0)
  {
    std::printf("FAIL %s: forward pass schedule not bitwise the level schedule\n", name);
    return false;
  }
  for (int k = 0; k < N; ++k)
    w[k] /= DG[k];
  for (int lev = nlev - 1; lev >= 0; --lev)
    for (int t = S.lvp[lev]; t < S.lvp[lev + 1]; ++t)
    {
      const int k = S.lvn[t];
      double s = w[k];
      for (int c = S.lcp[k]; c < S.lcp[k + 1]; ++c)
        s -= LX[S.lcpos[c]] * w[S.lci[c]];
      w[k] = s;
    }
  for (int k = 0; k < N; ++k)
    x[S.perm[k]] = w[k];
  const std::vector<double> K = dense(q, pol, sigma);
  // backward-stable residual: |Kx - b| <= tol (|K| |x| + |b|)
  double res = 0, scale = 0;
  for (int i = 0; i < N; ++i)
  {
    double s = 0, a = 0;
    for (int j = 0; j < N; ++j)
    {
      s += K[i * N + j] * x[j];
      a += std::fabs(K[i * N + j] * x[j]);
    }
    res = std::max(res, std::fabs(s - b[i]));
    scale = std::max(scale, a + std::fabs(b[i]));
  }
  res /= scale;
  // (delta = 1e-6 pivots: growth without pivoting, which polish refines away)
  const bool ok = std::isfinite(res) && res <= (pol ? 1e-9 : 1e-12);
  std::printf("%s %s: N %d nnzL %zu levels %d forward passes %zu (%zu segments) residual %.3e\n", ok ? "ok" : "FAIL",
              name, N, S.lrj.size(), nlev, S.fwp.size() - 1, S.fwk.size(), res);
  return ok;
}

Qp random_qp(std::mt19937& rng, int n, int m, double dp, double da)
{
  std::uniform_real_distribution<double> U(-1, 1), P01(0, 1);
  Qp q;
  q.n = n;
  q.m = m;
  q.Pp = { 0 };
  q.Ap = { 0 };
  for (int j = 0; j < n; ++j)
  {
    std::vector<std::pair<int, double>> pc, ac;
    for (int i = 0; i < j; ++i)
      if (P01(rng) < dp)
        pc.push_back({ i, 0.1 * U(rng) });
    if (P01(rng) < 0.8)
      pc.push_back({ j, 2.0 + P01(rng) });
    for (int r = 0; r < m; ++r)
      if (P01(rng) < da)
        ac.push_back({ r, U(rng) });
    add_col(q.Pp, q.Pi, q.Px, pc);
    add_col(q.Ap, q.Ai, q.Ax, ac);
  }
  for (int r = 0; r < m; ++r)
    q.rhoinv.push_back(r % 3 == 0 ? 1e-3 : 10.0);
  for (int r = 0; r < m; ++r)
    q.active.push_back(P01(rng) < 0.5);
  return q;
}

// trajectory-shaped: T steps x D joints, velocity cost couples neighbours,
// contact rows touch two steps' joints plus a hinge variable, bounds rows
Qp trajectory_qp(std::mt19937& rng, int T, int D, int contacts)
{
  std::uniform_real_distribution<double> U(-1, 1), P01(0, 1);
  const int nx = T * D, n = nx + contacts;
  Qp q;
  q.n = n;
  q.Pp = { 0 };
  q.Ap = { 0 };
  // rows: [contacts hinge rows][contacts hinge bounds][n variable bounds]
  const int m = 2 * contacts + n;
  q.m = m;
  std::vector<std::vector<std::pair<int, double>>> acol(static_cast<size_t>(n));
  for (int c = 0; c < contacts; ++c)
  {
    const int t = static_cast<int>(P01(rng) * (T - 1));
    for (int d = 0; d < D; ++d)
    {
      acol[t * D + d].push_back({ c, U(rng) });
      acol[(t + 1) * D + d].push_back({ c, U(rng) });
    }
    acol[nx + c].push_back({ c, -1.0 });
    acol[nx + c].push_back({ contacts + c, 1.0 });
  }
  for (int j = 0; j < n; ++j)
    acol[j].push_back({ 2 * contacts + j, 1.0 });
  for (int j = 0; j < n; ++j)
  {
    std::vector<std::pair<int, double>> pc;
    if (j < nx)
    {
      const int t = j / D;
      if (t > 0)
        pc.push_back({ j - D, -1.0 });
      pc.push_back({ j, (t > 0 && t < T - 1) ? 4.0 : 2.0 });
    }
    add_col(q.Pp, q.Pi, q.Px, pc);
    add_col(q.Ap, q.Ai, q.Ax, acol[j]);
  }
  for (int r = 0; r < m; ++r)
    q.rhoinv.push_back(r % 5 == 0 ? 1e-3 : 10.0);
  for (int r = 0; r < m; ++r)
    q.active.push_back(P01(rng) < 0.3);
  return q;
}
}  // namespace

int main()
{
  std::mt19937 rng(7);
  bool ok = true;
  for (int rep = 0; rep < 6; ++rep)
  {
    const Qp q = random_qp(rng, 10 + 7 * rep, 5 + 9 * rep, 0.15, 0.2);
    ok &= check("random", q, false, rng);
    ok &= check("random polish", q, true, rng);
  }
  {
    const Qp q = random_qp(rng, 40, 0, 0.1, 0.0);
    ok &= check("m = 0", q, false, rng);
  }
  {
    const Qp q = random_qp(rng, 30, 20, 1.0, 0.3);
    ok &= check("dense P", q, false, rng);
  }
  {
    const Qp q = trajectory_qp(rng, 20, 7, 120);
    ok &= check("trajectory", q, false, rng);
    ok &= check("trajectory polish", q, true, rng);
  }
  {
    // duplicate entries are refused
    KktSymbolic S;
    std::vector<int> Pp = { 0, 2, 2, 2, 2, 2 }, Pi = { 0, 0 }, Ap = { 0, 0, 0, 0, 0, 0 }, Ai;
    const std::string why = kkt_symbolic(5, 0, Pp.data(), Pi.data(), Ap.data(), Ai.data(), S);
    const bool refused = why.find("repeats") != std::string::npos;
    std::printf("%s duplicate entry refused: %s\n", refused ? "ok" : "FAIL", why.c_str());
    ok &= refused;
  }
  return ok ? 0 : 1;
}
