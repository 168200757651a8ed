// ORACLE — test infrastructure only.  One driver, compiled twice by
// oracle/ref/Makefile:
//   -DREF: against the reference's own headers and its expr_ops.cpp
//          (/root/reference/trajopt_sco/src/expr_ops.cpp, compiled from where
//          it lies into oracle/_ref/; nothing of it is copied),
//   else:  against the oracle's restatement (oracle/src/sco_expr.hpp).
// Both print the same canonical text for the same seeded expressions; the test
// (tests/test_oracle.py::test_expr_ops_against_reference_build) compares them
// byte for byte.  Only entry points whose reference definitions compile here
// are exercised: exprMult(AffExpr, AffExpr), exprSquare(AffExpr / Var) and the
// inline exprInc / exprDec / exprScale of expr_ops.hpp.  (cleanupAff needs
// AffExpr::size() from solver_interface.cpp, which needs Eigen: it is dropped
// by --gc-sections and pinned by the oracle's own KATs instead.)
#include <cstdint>
#include <cstdio>
#include <memory>
#include <vector>

#ifdef REF
#include <trajopt_sco/expr_ops.hpp>
namespace ns = sco;
#else
#include "sco_expr.hpp"
namespace ns = orc;
#endif

namespace
{
std::uint64_t g_state = 20261015ULL;
std::uint64_t next_u64()
{
  std::uint64_t z = (g_state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
double uniform() { return static_cast<double>(next_u64() >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0; }

std::vector<ns::Var> g_vars;

ns::AffExpr random_aff(int n)
{
  ns::AffExpr a;  // fields set directly: the reference's AffExpr(double) / AffExpr(Var) are out of line
  a.constant = uniform();
  for (int i = 0; i < n; ++i)
  {
    a.coeffs.push_back(uniform() * ((next_u64() % 5 == 0) ? 1e-8 : 1.0));
    a.vars.push_back(g_vars[next_u64() % g_vars.size()]);
  }
  return a;
}

void print_aff(const char* tag, const ns::AffExpr& a)
{
  std::printf("%s %.17g", tag, a.constant);
  for (std::size_t i = 0; i < a.coeffs.size(); ++i)
    std::printf(" %zu:%.17g", a.vars[i].var_rep->index, a.coeffs[i]);
  std::printf("\n");
}

void print_quad(const char* tag, const ns::QuadExpr& q)
{
  print_aff(tag, q.affexpr);
  std::printf("%s.q", tag);
  for (std::size_t i = 0; i < q.coeffs.size(); ++i)
    std::printf(" %zu,%zu:%.17g", q.vars1[i].var_rep->index, q.vars2[i].var_rep->index, q.coeffs[i]);
  std::printf("\n");
}
}  // namespace

int main()
{
  for (std::size_t i = 0; i < 12; ++i)
    g_vars.emplace_back(std::make_shared<ns::VarRep>(i, "x" + std::to_string(i), nullptr));
  for (int trial = 0; trial < 200; ++trial)
  {
    const int n1 = static_cast<int>(next_u64() % 6), n2 = static_cast<int>(next_u64() % 6);
    const ns::AffExpr a = random_aff(n1), b = random_aff(n2);
    print_quad("mult", ns::exprMult(a, b));
    print_quad("square", ns::exprSquare(a));
    print_quad("squarevar", ns::exprSquare(g_vars[static_cast<std::size_t>(trial) % g_vars.size()]));
    ns::AffExpr c = a;
    ns::exprInc(c, b);
    ns::exprInc(c, 0.25 * uniform());
    print_aff("inc", c);
    ns::AffExpr d = a;
    ns::exprDec(d, b);
    ns::exprDec(d, uniform());
    print_aff("dec", d);
    ns::AffExpr e = b;
    ns::exprScale(e, uniform() * 3.0);
    print_aff("scale", e);
    ns::QuadExpr q = ns::exprSquare(a);
    ns::exprInc(q, ns::exprMult(a, b));
    ns::exprScale(q, -0.5);
    print_quad("quadinc", q);
  }
  return 0;
}
