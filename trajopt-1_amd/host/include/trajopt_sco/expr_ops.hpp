// Expression algebra (trajopt_sco/include/trajopt_sco/expr_ops.hpp,
// trajopt_sco/src/expr_ops.cpp:10-99, expr_vec_ops.cpp:34-41).
#pragma once
#include "trajopt_sco/solver_interface.hpp"

namespace sco
{
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
inline void exprDec(AffExpr& a, double b) { a.constant -= b; }
inline void exprDec(AffExpr& a, AffExpr b)
{
  exprScale(b, -1);
  exprInc(a, b);
}
inline void exprDec(AffExpr& a, const Var& b) { exprDec(a, AffExpr(b)); }
inline void exprDec(QuadExpr& a, double b) { exprDec(a.affexpr, b); }
inline void exprDec(QuadExpr& a, const Var& b) { exprDec(a.affexpr, b); }
inline void exprDec(QuadExpr& a, const AffExpr& b) { exprDec(a.affexpr, b); }
inline void exprDec(QuadExpr& a, QuadExpr b)
{
  exprScale(b, -1);
  exprInc(a, b);
}
inline AffExpr exprAdd(AffExpr a, double b)
{
  exprInc(a, b);
  return a;
}
inline AffExpr exprAdd(AffExpr a, const Var& b)
{
  exprInc(a, b);
  return a;
}
inline AffExpr exprAdd(AffExpr a, const AffExpr& b)
{
  exprInc(a, b);
  return a;
}
inline QuadExpr exprAdd(QuadExpr a, const QuadExpr& b)
{
  exprInc(a, b);
  return a;
}
inline AffExpr exprSub(AffExpr a, double b)
{
  exprDec(a, b);
  return a;
}
inline AffExpr exprSub(AffExpr a, const Var& b)
{
  exprDec(a, b);
  return a;
}
inline AffExpr exprSub(AffExpr a, const AffExpr& b)
{
  exprDec(a, b);
  return a;
}
inline QuadExpr exprSub(QuadExpr a, const QuadExpr& b)
{
  exprDec(a, b);
  return a;
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
QuadExpr exprMult(const AffExpr& a, const AffExpr& b);  // expr_ops.cpp:30-67
QuadExpr exprSquare(const Var& a);
QuadExpr exprSquare(const AffExpr& a);                  // expr_ops.cpp:10-28
AffExpr cleanupAff(const AffExpr& a);                   // drops |c| <= 1e-7 (expr_ops.cpp:86-99)
QuadExpr cleanupQuad(const QuadExpr& q);
AffExpr varDot(const DblVec& x, const VarVector& v);    // expr_vec_ops.cpp:34-41
}  // namespace sco
