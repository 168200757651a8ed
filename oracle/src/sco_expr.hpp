// ORACLE — test infrastructure only. CPU restatement of trajopt_sco's
// expression algebra. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it; it is never part of the product path.
//
// Restates:
//   Var / VarRep / AffExpr / QuadExpr   trajopt_sco/include/trajopt_sco/solver_interface.hpp:113-219
//   AffExpr::value, QuadExpr::value     trajopt_sco/src/solver_interface.cpp:64-109
//   exprInc/exprDec/exprScale/exprMult  trajopt_sco/include/trajopt_sco/expr_ops.hpp:1-179
//   exprMult(Aff,Aff), exprSquare,
//   cleanupAff                          trajopt_sco/src/expr_ops.cpp:10-99
//   simplify2                           trajopt_sco/src/solver_interface.cpp:44-62
#pragma once
#include <cmath>
#include <cstddef>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace orc
{
using DblVec = std::vector<double>;
using IntVec = std::vector<int>;

struct VarRep
{
  using Ptr = std::shared_ptr<VarRep>;
  VarRep(std::size_t i, std::string n, void* c) : index(i), name(std::move(n)), creator(c) {}
  std::size_t index;
  std::string name;
  void* creator;
  bool removed = false;
};

struct Var
{
  VarRep::Ptr var_rep;
  Var() = default;
  explicit Var(VarRep::Ptr r) : var_rep(std::move(r)) {}
  double value(const double* x) const { return x[var_rep->index]; }
  double value(const DblVec& x) const { return x[var_rep->index]; }
};
using VarVector = std::vector<Var>;

struct CntRep
{
  using Ptr = std::shared_ptr<CntRep>;
  CntRep(std::size_t i, void* c) : index(i), creator(c) {}
  std::size_t index;
  void* creator;
  bool removed = false;
};
struct Cnt
{
  CntRep::Ptr cnt_rep;
  Cnt() = default;
  explicit Cnt(CntRep::Ptr r) : cnt_rep(std::move(r)) {}
};
using CntVector = std::vector<Cnt>;

struct AffExpr
{
  double constant = 0;
  DblVec coeffs;
  VarVector vars;
  AffExpr() = default;
  explicit AffExpr(double a) : constant(a) {}
  explicit AffExpr(const Var& v) : coeffs(1, 1.0), vars(1, v) {}
  std::size_t size() const { return coeffs.size(); }
  double value(const double* x) const
  {
    double out = constant;
    for (std::size_t i = 0; i < size(); ++i)
      out += coeffs[i] * vars[i].value(x);
    return out;
  }
  double value(const DblVec& x) const { return value(x.data()); }
};
using AffExprVector = std::vector<AffExpr>;

struct QuadExpr
{
  AffExpr affexpr;
  DblVec coeffs;
  VarVector vars1;
  VarVector vars2;
  QuadExpr() = default;
  explicit QuadExpr(double a) : affexpr(a) {}
  explicit QuadExpr(const Var& v) : affexpr(v) {}
  explicit QuadExpr(AffExpr a) : affexpr(std::move(a)) {}
  std::size_t size() const { return coeffs.size(); }
  double value(const double* x) const
  {
    double out = affexpr.value(x);
    for (std::size_t i = 0; i < size(); ++i)
      out += coeffs[i] * vars1[i].value(x) * vars2[i].value(x);
    return out;
  }
  double value(const DblVec& x) const { return value(x.data()); }
};

// ---- in-place ops (expr_ops.hpp) ----
inline void exprScale(AffExpr& v, double a)
{
  v.constant *= a;
  for (double& c : v.coeffs)
    c *= a;
}
inline void exprScale(QuadExpr& q, double a)
{
  exprScale(q.affexpr, a);
  for (double& c : q.coeffs)
    c *= a;
}
inline void exprInc(AffExpr& a, double b) { a.constant += b; }
inline void exprInc(AffExpr& a, const AffExpr& b)
{
  a.constant += b.constant;
  a.coeffs.insert(a.coeffs.end(), b.coeffs.begin(), b.coeffs.end());
  a.vars.insert(a.vars.end(), b.vars.begin(), b.vars.end());
}
inline void exprInc(AffExpr& a, const Var& b) { exprInc(a, AffExpr(b)); }
inline void exprInc(QuadExpr& a, double b) { exprInc(a.affexpr, b); }
inline void exprInc(QuadExpr& a, const Var& b) { exprInc(a.affexpr, AffExpr(b)); }
inline void exprInc(QuadExpr& a, const AffExpr& b) { exprInc(a.affexpr, b); }
inline void exprInc(QuadExpr& a, const QuadExpr& b)
{
  exprInc(a.affexpr, b.affexpr);
  a.coeffs.insert(a.coeffs.end(), b.coeffs.begin(), b.coeffs.end());
  a.vars1.insert(a.vars1.end(), b.vars1.begin(), b.vars1.end());
  a.vars2.insert(a.vars2.end(), b.vars2.begin(), b.vars2.end());
}
inline void exprDec(AffExpr& a, double b) { a.constant -= b; }
inline void exprDec(AffExpr& a, AffExpr b)
{
  exprScale(b, -1);
  exprInc(a, b);
}
inline void exprDec(AffExpr& a, const Var& b) { exprDec(a, AffExpr(b)); }
inline void exprDec(QuadExpr& a, double b) { exprDec(a.affexpr, b); }
inline void exprDec(QuadExpr& a, const AffExpr& b) { exprDec(a.affexpr, b); }
inline void exprDec(QuadExpr& a, QuadExpr b)
{
  exprScale(b, -1);
  exprInc(a, b);
}
inline AffExpr exprMult(const Var& a, double b)
{
  AffExpr c(a);
  exprScale(c, b);
  return c;
}
inline AffExpr exprMult(AffExpr a, double b)
{
  exprScale(a, b);
  return a;
}
inline QuadExpr exprMult(QuadExpr a, double b)
{
  exprScale(a, b);
  return a;
}
inline AffExpr exprAdd(AffExpr a, double b)
{
  exprInc(a, b);
  return a;
}
inline AffExpr exprSub(AffExpr a, double b)
{
  exprDec(a, b);
  return a;
}
inline AffExpr exprSub(AffExpr a, const AffExpr& b)
{
  exprDec(a, b);
  return a;
}

// ---- expr_ops.cpp ----
inline QuadExpr exprMult(const AffExpr& a1, const AffExpr& a2)
{
  QuadExpr out;
  const std::size_t n1 = a1.coeffs.size(), n2 = a2.coeffs.size();
  out.affexpr.constant = a1.constant * a2.constant;
  out.affexpr.vars.insert(out.affexpr.vars.end(), a1.vars.begin(), a1.vars.end());
  out.affexpr.vars.insert(out.affexpr.vars.end(), a2.vars.begin(), a2.vars.end());
  out.affexpr.coeffs.resize(n1 + n2);
  for (std::size_t i = 0; i < n1; ++i)
    out.affexpr.coeffs[i] = a2.constant * a1.coeffs[i];
  for (std::size_t i = 0; i < n2; ++i)
    out.affexpr.coeffs[i + n1] = a1.constant * a2.coeffs[i];
  for (std::size_t i = 0; i < n1; ++i)
    for (std::size_t j = 0; j < n2; ++j)
    {
      out.vars1.push_back(a1.vars[i]);
      out.vars2.push_back(a2.vars[j]);
      out.coeffs.push_back(a1.coeffs[i] * a2.coeffs[j]);
    }
  return out;
}

inline QuadExpr exprSquare(const Var& a)
{
  QuadExpr out;
  out.coeffs.push_back(1);
  out.vars1.push_back(a);
  out.vars2.push_back(a);
  return out;
}

inline QuadExpr exprSquare(const AffExpr& a)
{
  QuadExpr out;
  const std::size_t n = a.coeffs.size();
  out.affexpr.constant = a.constant * a.constant;
  out.affexpr.vars = a.vars;
  out.affexpr.coeffs.resize(n);
  for (std::size_t i = 0; i < n; ++i)
    out.affexpr.coeffs[i] = 2 * a.constant * a.coeffs[i];
  for (std::size_t i = 0; i < n; ++i)
  {
    out.vars1.push_back(a.vars[i]);
    out.vars2.push_back(a.vars[i]);
    out.coeffs.push_back(a.coeffs[i] * a.coeffs[i]);
    for (std::size_t j = i + 1; j < n; ++j)
    {
      out.vars1.push_back(a.vars[i]);
      out.vars2.push_back(a.vars[j]);
      out.coeffs.push_back(2 * a.coeffs[i] * a.coeffs[j]);
    }
  }
  return out;
}

// smallest | |c| - 1e-7 | cleanupAff has compared since the last reset: how close
// a linearisation's sparsity pattern (the warm-start test, quirk Q2) came to a
// tie (tests/parity.py's threshold-tie evidence; infinity after a reset)
inline thread_local double t_cleanup_margin = 1e300;

inline AffExpr cleanupAff(const AffExpr& a)
{
  AffExpr out;
  for (std::size_t i = 0; i < a.size(); ++i)
  {
    const double m = std::fabs(std::fabs(a.coeffs[i]) - 1e-7);
    if (m < t_cleanup_margin)
      t_cleanup_margin = m;
  }
  for (std::size_t i = 0; i < a.size(); ++i)
    if (std::fabs(a.coeffs[i]) > 1e-7)
    {
      out.coeffs.push_back(a.coeffs[i]);
      out.vars.push_back(a.vars[i]);
    }
  out.constant = a.constant;
  return out;
}

inline void simplify2(IntVec& inds, DblVec& vals)
{
  std::map<int, double> ind2val;
  for (std::size_t i = 0; i < inds.size(); ++i)
    if (vals[i] != 0.0)
      ind2val[inds[i]] += vals[i];
  inds.resize(ind2val.size());
  vals.resize(ind2val.size());
  std::size_t k = 0;
  for (const auto& iv : ind2val)
  {
    inds[k] = iv.first;
    vals[k] = iv.second;
    ++k;
  }
}

inline double vecSum(const DblVec& v)
{
  double s = 0;
  for (double x : v)
    s += x;
  return s;
}
inline double vecDot(const DblVec& a, const DblVec& b)
{
  double s = 0;
  for (std::size_t i = 0; i < a.size(); ++i)
    s += a[i] * b[i];
  return s;
}
inline double vecMax(const DblVec& v)
{
  double m = -INFINITY;
  for (double x : v)
    m = (x > m) ? x : m;
  return m;
}
inline double pospart(double x) { return x > 0 ? x : 0; }

}  // namespace orc
