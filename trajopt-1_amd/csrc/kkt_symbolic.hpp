// Symbolic LDL^T of an OSQP KKT pattern for qp_csc.hip's level-scheduled
// sparse factor (host code; also compiled by tests/test_kkt_symbolic.py's
// checker, which replays the level schedule on the CPU).
#pragma once
#include <algorithm>
#include <iterator>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

// Symbolic LDL^T of the KKT pattern, once per thip_qp (the host side of
// kkt_factor / kkt_solve).  Nodes: x_j = j, constraint row r = n + r.
struct KktSymbolic
{
  std::vector<int> perm, lrp, lrj, lcp, lci, lcpos, lksrc, dpd, lvp, lvn, fip, fik, fic;
  // the forward solve as passes of row segments: entry e of row k is ready
  // once every column up to it is final, i.e. after level pm(e) - 1, with pm
  // the prefix maximum of level(j) + 1 along the row; a row's entries of equal
  // pm form one segment (k, fwa, fwb) of pass pm, and pass p runs after pass
  // p - 1 (empty passes dropped): each row is still summed in its order, but
  // the entries of a row near the root are taken as soon as they are ready
  // instead of all at its own level
  std::vector<int> fwp, fwk, fwa, fwb;
};

// Returns "" or the reason the pattern is refused.
inline std::string kkt_symbolic(int n, int m, const int* Pp, const int* Pi, const int* Ap, const int* Ai,
                                KktSymbolic& S)
{
  const int N = n + m;
  // off-diagonal entries (upper: lo < hi) and their value source
  std::vector<std::vector<int>> adj(static_cast<size_t>(N));
  std::unordered_map<long long, int> src;
  std::vector<int> pdiag(static_cast<size_t>(n), -1);
  auto key = [N](int lo, int hi) { return static_cast<long long>(lo) * N + hi; };
  for (int j = 0; j < n; ++j)
  {
    for (int e = Pp[j]; e < Pp[j + 1]; ++e)
    {
      const int i = Pi[e];
      if (i == j)
      {
        if (pdiag[j] >= 0)
          return "P repeats entry (" + std::to_string(i) + ", " + std::to_string(j) + ")";
        pdiag[j] = e;
        continue;
      }
      if (!src.emplace(key(i, j), 2 * e).second)
        return "P repeats entry (" + std::to_string(i) + ", " + std::to_string(j) + ")";
      adj[i].push_back(j);
      adj[j].push_back(i);
    }
    for (int e = Ap[j]; e < Ap[j + 1]; ++e)
    {
      const int r = n + Ai[e];
      if (!src.emplace(key(j, r), 2 * e + 1).second)
        return "A repeats entry (" + std::to_string(Ai[e]) + ", " + std::to_string(j) + ")";
      adj[j].push_back(r);
      adj[r].push_back(j);
    }
  }
  for (auto& v : adj)
    std::sort(v.begin(), v.end());
  const std::vector<std::vector<int>> nbr = adj;  // the KKT pattern (the ordering consumes adj)
  // minimum degree on the elimination graph (exact external degree, smallest
  // index breaks ties) -- the oracle's LdlSolver::order, where OSQP runs AMD
  S.perm.clear();
  S.perm.reserve(static_cast<size_t>(N));
  {
    std::set<std::pair<size_t, int>> pq;
    for (int j = 0; j < N; ++j)
      pq.insert({ adj[j].size(), j });
    std::vector<char> done(static_cast<size_t>(N), 0);
    std::vector<int> merged;
    while (!pq.empty())
    {
      const int v = pq.begin()->second;
      pq.erase(pq.begin());
      done[v] = 1;
      S.perm.push_back(v);
      const std::vector<int> nv = adj[v];
      for (int u : nv)
      {
        if (done[u])
          continue;
        pq.erase({ adj[u].size(), u });
        merged.clear();
        std::set_union(adj[u].begin(), adj[u].end(), nv.begin(), nv.end(), std::back_inserter(merged));
        adj[u].clear();
        for (int w : merged)
          if (w != u && w != v && !done[w])
            adj[u].push_back(w);
        pq.insert({ adj[u].size(), u });
      }
      adj[v].clear();
      adj[v].shrink_to_fit();
    }
  }
  std::vector<int> pinv(static_cast<size_t>(N));
  for (int k = 0; k < N; ++k)
    pinv[S.perm[k]] = k;
  // elimination tree and the rows of L (ldl_symbolic's walk up the tree)
  std::vector<int> parent(static_cast<size_t>(N), -1), flag(static_cast<size_t>(N), -1);
  std::vector<std::vector<int>> rows(static_cast<size_t>(N));
  long long nnzl = 0;
  for (int k = 0; k < N; ++k)
  {
    flag[k] = k;
    for (int o : nbr[S.perm[k]])
    {
      for (int i = pinv[o]; i < k && flag[i] != k; i = parent[i])
      {
        if (parent[i] == -1)
          parent[i] = k;
        rows[k].push_back(i);
        flag[i] = k;
      }
    }
    std::sort(rows[k].begin(), rows[k].end());
    nnzl += static_cast<long long>(rows[k].size());
    if (nnzl > (1LL << 28))
      return "the KKT factor has more than 2^28 entries";
  }
  S.lrp.assign(static_cast<size_t>(N) + 1, 0);
  S.lrj.clear();
  S.lrj.reserve(static_cast<size_t>(nnzl));
  for (int k = 0; k < N; ++k)
  {
    S.lrj.insert(S.lrj.end(), rows[k].begin(), rows[k].end());
    S.lrp[k + 1] = static_cast<int>(S.lrj.size());
  }
  // columns of L (rows ascending), their positions and KKT sources
  S.lcp.assign(static_cast<size_t>(N) + 1, 0);
  for (int j : S.lrj)
    S.lcp[j + 1]++;
  for (int k = 0; k < N; ++k)
    S.lcp[k + 1] += S.lcp[k];
  S.lci.assign(static_cast<size_t>(nnzl), 0);
  S.lcpos.assign(static_cast<size_t>(nnzl), 0);
  S.lksrc.assign(static_cast<size_t>(nnzl), -1);
  {
    std::vector<int> nx(S.lcp.begin(), S.lcp.end() - 1);
    for (int i = 0; i < N; ++i)
      for (int e = S.lrp[i]; e < S.lrp[i + 1]; ++e)
      {
        const int k = S.lrj[e], c = nx[k]++;
        S.lci[c] = i;
        S.lcpos[c] = e;
        const int a = S.perm[i], b = S.perm[k];
        const auto it = src.find(key(std::min(a, b), std::max(a, b)));
        if (it != src.end())
          S.lksrc[c] = it->second;
      }
  }
  S.dpd.assign(static_cast<size_t>(N), -1);
  for (int k = 0; k < N; ++k)
    if (S.perm[k] < n)
      S.dpd[k] = pdiag[S.perm[k]];
  // levels: a node after all of its descendants
  std::vector<int> level(static_cast<size_t>(N), 0);
  int nlev = 0;
  for (int k = 0; k < N; ++k)
  {
    nlev = std::max(nlev, level[k] + 1);
    if (parent[k] >= 0)
      level[parent[k]] = std::max(level[parent[k]], level[k] + 1);
  }
  S.lvp.assign(static_cast<size_t>(nlev) + 1, 0);
  for (int k = 0; k < N; ++k)
    S.lvp[level[k] + 1]++;
  for (int l = 0; l < nlev; ++l)
    S.lvp[l + 1] += S.lvp[l];
  S.lvn.assign(static_cast<size_t>(N), 0);
  {
    std::vector<int> nx(S.lvp.begin(), S.lvp.end() - 1);
    for (int k = 0; k < N; ++k)
      S.lvn[nx[level[k]]++] = k;
  }
  {
    std::vector<std::vector<int>> seg(static_cast<size_t>(nlev) + 1);  // per pass: (k, a, b) triples
    for (int k = 0; k < N; ++k)
    {
      int pm = 0, a = S.lrp[k];
      for (int e = S.lrp[k]; e < S.lrp[k + 1]; ++e)
      {
        const int r = std::max(pm, level[S.lrj[e]] + 1);
        if (r != pm && e > a)
        {
          seg[pm].insert(seg[pm].end(), { k, a, e });
          a = e;
        }
        pm = r;
      }
      if (S.lrp[k + 1] > a)
        seg[pm].insert(seg[pm].end(), { k, a, S.lrp[k + 1] });
    }
    S.fwp.assign(1, 0);
    S.fwk.clear();
    S.fwa.clear();
    S.fwb.clear();
    for (const auto& v : seg)
    {
      if (v.empty())
        continue;
      for (size_t i = 0; i < v.size(); i += 3)
      {
        S.fwk.push_back(v[i]);
        S.fwa.push_back(v[i + 1]);
        S.fwb.push_back(v[i + 2]);
      }
      S.fwp.push_back(static_cast<int>(S.fwk.size()));
    }
  }
  S.fip.assign(static_cast<size_t>(nlev) + 1, 0);
  S.fik.clear();
  S.fic.clear();
  for (int l = 0; l < nlev; ++l)
  {
    for (int t = S.lvp[l]; t < S.lvp[l + 1]; ++t)
    {
      const int k = S.lvn[t];
      for (int c = S.lcp[k]; c < S.lcp[k + 1]; ++c)
      {
        S.fik.push_back(k);
        S.fic.push_back(c);
      }
    }
    S.fip[l + 1] = static_cast<int>(S.fik.size());
  }
  return "";
}

