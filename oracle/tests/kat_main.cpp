// ORACLE KATs — test infrastructure only.
//
// Known-answer tests ported from the reference's own unit tests, run against
// the CPU restatement to pin it before it is trusted as the parity oracle:
//   trajopt_sco/test/solver-utils-unit.cpp:19-244   (exprToEigen / eigenToCSC arrays)
//   trajopt_sco/test/modeling-unit.cpp:26-91         (getClosestFeasiblePoint)
//   trajopt_sco/test/solver-interface-unit.cpp:21-231 (simplify2, QP objective values)
//   trajopt_sco/test/small-problems-unit.cpp:48-172  (SQP on separable/nonseparable
//                                                      quadratics and Hock-Schittkowski TP1/3/6/7)
//   trajopt/test/joint_costs_unit.cpp:883-937       (finite-difference stencils on t^3)
//   trajopt/test/kinematic_costs_unit.cpp:62-254    (FD-consistency of the CartPose jacobian,
//                                                      calcTransformError sign convention)
// Prints one line per check and exits with the number of failures.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "../src/kin.hpp"
#include "../src/sco.hpp"
#include "../src/terms.hpp"

using namespace orc;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond, msg)                                     \
  do                                                         \
  {                                                          \
    if (cond)                                                \
      ++g_pass;                                              \
    else                                                     \
    {                                                        \
      ++g_fail;                                              \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
    }                                                        \
  } while (0)
#define NEAR(a, b, tol, msg) CHECK(std::fabs((a) - (b)) <= (tol), msg)

static VarVector makeVars(int n, std::vector<VarRep::Ptr>& keep)
{
  VarVector x;
  for (int i = 0; i < n; ++i)
  {
    keep.push_back(std::make_shared<VarRep>(static_cast<std::size_t>(i), "x_" + std::to_string(i), nullptr));
    x.emplace_back(keep.back());
  }
  return x;
}

static Csc denseToCsc(const std::vector<std::vector<double>>& M)
{
  std::vector<Triplet> t;
  const int m = static_cast<int>(M.size()), n = static_cast<int>(M[0].size());
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i)
      if (M[i][j] != 0)
        t.push_back({ i, j, M[i][j] });
  return cscFromTriplets(m, n, t);
}

static void kat_solver_utils()
{
  std::vector<VarRep::Ptr> keep;
  VarVector x = makeVars(2, keep);
  AffExpr aff;
  aff.vars = x;
  aff.coeffs = { 3, 2 };
  aff.constant = 1;
  DblVec v;
  exprToDense(aff, v, 2);
  CHECK(v[0] == 3 && v[1] == 2, "exprToEigen(AffExpr) = [3, 2]");
  Csc A;
  DblVec u;
  affVecToCsc(AffExprVector(1, aff), A, u, 2);
  CHECK(u.size() == 1 && u[0] == -1, "exprToEigen(AffExprVector) rhs = -constant");
  CHECK(A.nnz() == 2, "m_A.nonZeros() == 2");
  QuadExpr sq = exprSquare(aff);
  Csc Q;
  DblVec q;
  quadToCscFull(sq, Q, q, 2, false);
  CHECK(q[0] == 6 && q[1] == 4, "q = [6, 4]");
  CHECK(Q.nnz() == 4 && Q.x[0] == 9 && Q.x[1] == 6 && Q.x[2] == 6 && Q.x[3] == 4, "Q = [[9,6],[6,4]]");
  quadToCscFull(sq, Q, q, 2, true);
  CHECK(Q.nnz() == 4 && Q.x[0] == 18 && Q.x[1] == 12 && Q.x[3] == 8, "halved: Q = 2 * [[9,6],[6,4]]");
  aff.coeffs = { 0, 2 };
  sq = exprSquare(aff);
  quadToCscFull(sq, Q, q, 2, false, false);
  CHECK(Q.nnz() == 1 && Q.x[0] == 4, "Q = [[0,0],[0,4]] nnz 1");
  quadToCscFull(sq, Q, q, 2, true, false);
  CHECK(Q.nnz() == 1 && Q.x[0] == 8, "halved nnz 1");
  quadToCscFull(sq, Q, q, 2, false, true);
  CHECK(Q.nnz() == 2 && Q.x[0] == 0 && Q.x[1] == 4, "force_diagonal nnz 2");
  quadToCscFull(sq, Q, q, 2, true, true);
  CHECK(Q.nnz() == 2 && Q.x[1] == 8, "halved force_diagonal nnz 2");

  // eigenToCSC
  Csc M = denseToCsc({ { 1, 2, 3 }, { 1, 0, 9 }, { 1, 8, 0 } });
  CHECK((M.x == DblVec{ 1, 1, 1, 2, 8, 3, 9 }), "eigenToCSC P");
  CHECK((M.i == std::vector<OsqpInt>{ 0, 1, 2, 0, 2, 0, 1 }), "eigenToCSC rows_i");
  CHECK((M.p == std::vector<OsqpInt>{ 0, 3, 5, 7 }), "eigenToCSC cols_p");
  M = denseToCsc({ { 0, 2, 0 }, { 7, 0, 0 }, { 0, 0, 0 } });
  CHECK((M.x == DblVec{ 7, 2 }) && (M.i == std::vector<OsqpInt>{ 1, 0 }) && (M.p == std::vector<OsqpInt>{ 0, 1, 2, 2 }),
        "eigenToCSC 2");
  M = denseToCsc({ { 0, 0, 0 }, { 0, 0, 0 }, { 0, 6, 0 } });
  CHECK((M.x == DblVec{ 6 }) && (M.i == std::vector<OsqpInt>{ 2 }) && (M.p == std::vector<OsqpInt>{ 0, 0, 1, 1 }),
        "eigenToCSC 3");
  // upper triangular
  Csc F = denseToCsc({ { 1, 2, 0 }, { 2, 4, 0 }, { 0, 0, 9 } });
  std::vector<Triplet> tu;
  for (OsqpInt j = 0; j < F.n; ++j)
    for (OsqpInt p = F.p[j]; p < F.p[j + 1]; ++p)
      if (F.i[p] <= j)
        tu.push_back({ F.i[p], j, F.x[p] });
  Csc U = cscFromTriplets(3, 3, tu);
  CHECK((U.x == DblVec{ 1, 2, 4, 9 }) && (U.i == std::vector<OsqpInt>{ 0, 0, 1, 2 }) &&
            (U.p == std::vector<OsqpInt>{ 0, 1, 3, 4 }),
        "eigenToCSC upper triangular");
  // simplify2
  IntVec inds = { 0, 1, 3 };
  DblVec vals = { 1e-7, 1e3, 0., 0., 0. };
  simplify2(inds, vals);
  CHECK((inds == IntVec{ 0, 1 }) && (vals == DblVec{ 1e-7, 1e3 }), "simplify2");
}

static OptProb::Ptr problemWithBounds(const DblVec& lb, const DblVec& ub)
{
  auto prob = std::make_shared<OptProb>(OsqpSettings{});
  std::vector<std::string> names;
  for (std::size_t i = 0; i < lb.size(); ++i)
    names.push_back("x_" + std::to_string(i));
  prob->createVariables(names, lb, ub);
  return prob;
}

static void kat_modeling()
{
  const double delta = 1e-3;
  {
    auto prob = problemWithBounds({ -1, -1, -1, -1 }, { 1, 1, 1, 1 });
    const DblVec y = prob->getClosestFeasiblePoint({ 0.0, -2.0, 2.0, -1.0 }, delta);
    CHECK(y[0] == 0.0 && y[1] == -1.0 + delta && y[2] == 1.0 - delta && y[3] == -1.0 + delta, "clamps both bounds");
  }
  {
    auto prob = problemWithBounds({ -1, -1 }, { 1, 1 });
    const DblVec y = prob->getClosestFeasiblePoint({ -1.0 + delta / 2, 1.0 - delta / 2 }, delta);
    CHECK(y[0] == -1.0 + delta && y[1] == 1.0 - delta, "insets from both bounds");
  }
  {
    const DblVec lb{ 0.0, 0.5 }, ub{ delta, 0.5 };
    auto prob = problemWithBounds(lb, ub);
    bool ok = true;
    for (double x : { -1.0, 0.0, 0.25, 1.0 })
    {
      const DblVec y = prob->getClosestFeasiblePoint({ x, x }, delta);
      for (std::size_t i = 0; i < 2; ++i)
        ok = ok && y[i] >= lb[i] && y[i] <= ub[i] && y[i] == (lb[i] + ub[i]) / 2;
    }
    CHECK(ok, "respects narrow bounds");
  }
  {
    auto prob = problemWithBounds({ -INFINITY, -INFINITY }, { INFINITY, 1.0 });
    const DblVec y = prob->getClosestFeasiblePoint({ -1e9, -1e9 });
    CHECK(y[0] == -1e9 && y[1] == -1e9, "leaves unbounded vars alone");
  }
  {
    auto prob = problemWithBounds({ -1, -1, 0.0 }, { 1, 1, delta });
    const DblVec once = prob->getClosestFeasiblePoint({ -5.0, 5.0, 5.0 }, delta);
    const DblVec twice = prob->getClosestFeasiblePoint(once, delta);
    CHECK(once == twice, "idempotent");
  }
}

static OsqpSettings referenceOsqpSettings()
{
  OsqpSettings s;  // OSQP 1.0 defaults + OSQPModelConfig::setDefaultOSQPSettings
  s.eps_abs = 1e-4;
  s.eps_rel = 1e-6;
  s.max_iter = 8192;
  s.polishing = 1;
  s.adaptive_rho = 1;
  return s;
}

static void kat_solver_interface()
{
  {
    OSQPModel solver(referenceOsqpSettings());
    VarVector vars;
    for (int i = 0; i < 3; ++i)
      vars.push_back(solver.addVar("v" + std::to_string(i)));
    solver.update();
    AffExpr aff;
    for (std::size_t i = 0; i < 3; ++i)
    {
      exprInc(aff, vars[i]);
      solver.setVarBounds(vars[i], 0, 10);
    }
    aff.constant -= 3;
    solver.setObjective(exprSquare(aff));
    solver.update();
    solver.optimize();
    DblVec soln(3);
    for (std::size_t i = 0; i < 3; ++i)
      soln[i] = solver.getVarValue(vars[i]);
    NEAR(aff.value(soln), 0, 1e-6, "setup_problem: aff(soln) == 0");
    solver.removeVars(VarVector(1, vars[2]));
    solver.update();
    CHECK(solver.getVars().size() == 2, "removeVar");
  }
  auto exprMultTest = [](double v1_val, double v2_val, double c1, double c2, double k1, double k2, const char* msg) {
    OSQPModel solver(referenceOsqpSettings());
    VarVector vars;
    vars.push_back(solver.addVar("v1"));
    vars.push_back(solver.addVar("v2"));
    solver.update();
    AffExpr a1, a2;
    exprInc(a1, vars[0]);
    solver.setVarBounds(vars[0], v1_val, v1_val);
    a1.constant = k1;
    a1.coeffs[0] = c1;
    exprInc(a2, vars[1]);
    solver.setVarBounds(vars[1], v2_val, v2_val);
    a2.constant = k2;
    a2.coeffs[0] = c2;
    const QuadExpr a12 = exprMult(a1, a2);
    solver.setObjective(a12);
    solver.update();
    solver.optimize();
    DblVec soln(2);
    for (std::size_t i = 0; i < 2; ++i)
      soln[i] = solver.getVarValue(vars[i]);
    const double answer = (c1 * v1_val + k1) * (c2 * v2_val + k2);
    NEAR(a12.value(soln), answer, 1e-6, msg);
  };
  exprMultTest(10, 20, 2, 1, 0, 0, "ExprMult_test2: (2 v1)(v2) = 400");
  exprMultTest(10, 20, 3, 2, -3, -5, "ExprMult_test3: (3 v1 - 3)(2 v2 - 5) = 945");
}

static OptProb::Ptr setupProblem(std::size_t nvars)
{
  auto prob = std::make_shared<OptProb>(referenceOsqpSettings());
  std::vector<std::string> names;
  for (std::size_t i = 0; i < nvars; ++i)
    names.push_back("x_" + std::to_string(i));
  prob->createVariables(names);
  return prob;
}

static bool allNear(const DblVec& x, const DblVec& y, double tol)
{
  if (x.size() != y.size())
    return false;
  for (std::size_t i = 0; i < x.size(); ++i)
    if (std::fabs(x[i] - y[i]) > tol)
      return false;
  return true;
}

static double sqr(double a) { return a * a; }

static void kat_small_problems()
{
  {
    auto prob = setupProblem(3);
    prob->addCost(std::make_shared<CostFromFunc>(
        [](const DblVec& x) { return x[0] * x[0] + sqr(x[1] - 1) + sqr(x[2] - 2); }, prob->getVars(), "f"));
    BasicTrustRegionSQP solver(prob);
    solver.getParameters().trust_box_size = 100;
    solver.initialize({ 3, 4, 5 });
    const OptStatus st = solver.optimize();
    CHECK(st == OPT_CONVERGED, "QuadraticSeparable converged");
    CHECK(allNear(solver.x(), { 0, 1, 2 }, 1e-3), "QuadraticSeparable x = (0,1,2)");
  }
  {
    auto prob = setupProblem(3);
    prob->addCost(std::make_shared<CostFromFunc>(
        [](const DblVec& x) { return sqr(x[0] - x[1] + 3 * x[2]) + sqr(x[0] - 1) + sqr(x[2] - 2); }, prob->getVars(),
        "f", true));
    BasicTrustRegionSQP solver(prob);
    auto& p = solver.getParameters();
    p.trust_box_size = 100;
    p.min_trust_box_size = 1e-5;
    p.min_approx_improve = 1e-6;
    solver.initialize({ 3, 4, 5 });
    const OptStatus st = solver.optimize();
    CHECK(st == OPT_CONVERGED, "QuadraticNonseparable converged");
    CHECK(allNear(solver.x(), { 1, 7, 2 }, .01), "QuadraticNonseparable x = (1,7,2)");
  }
  auto testProblem = [](ScalarOfVector f, VectorOfVector g, ConstraintType type, const DblVec& init, const DblVec& sol,
                        const char* name) {
    auto prob = setupProblem(init.size());
    prob->addCost(std::make_shared<CostFromFunc>(f, prob->getVars(), "f", true));
    prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(g, MatrixOfVector(), prob->getVars(), DblVec(), type, "g"));
    BasicTrustRegionSQP solver(prob);
    auto& p = solver.getParameters();
    p.max_iter = 1000;
    p.min_trust_box_size = 1e-5;
    p.min_approx_improve = 1e-10;
    p.initial_merit_error_coeff = 1;
    solver.initialize(init);
    const OptStatus st = solver.optimize();
    std::string m1 = std::string(name) + " converged", m2 = std::string(name) + " solution";
    CHECK(st == OPT_CONVERGED, m1.c_str());
    CHECK(allNear(solver.x(), sol, .01), m2.c_str());
    if (!allNear(solver.x(), sol, .01))
      std::printf("  got (%g, %g)\n", solver.x()[0], solver.x()[1]);
  };
  testProblem([](const DblVec& x) { return 1 * sqr(x[1] - sqr(x[0])) + sqr(1 - x[0]); },
              [](const DblVec& x) { return DblVec{ -1.5 - x[1] }; }, INEQ, { -2, 1 }, { 1, 1 }, "TP1");
  testProblem([](const DblVec& x) { return x[1] + 1e-5 * sqr(x[1] - x[0]); },
              [](const DblVec& x) { return DblVec{ 0 - x[1] }; }, INEQ, { 10, 1 }, { 0, 0 }, "TP3");
  testProblem([](const DblVec& x) { return sqr(1 - x[0]); },
              [](const DblVec& x) { return DblVec{ 10 * (x[1] - sqr(x[0])) }; }, EQ, { 10, 1 }, { 1, 1 }, "TP6");
  testProblem([](const DblVec& x) { return std::log(1 + sqr(x[0])) - x[1]; },
              [](const DblVec& x) { return DblVec{ sqr(1 + sqr(x[0])) + sqr(x[1]) - 4 }; }, EQ, { 2, 2 },
              { 0., std::sqrt(3.) }, "TP7");
}

static void kat_joint_costs_stencil()
{
  // joint_costs_unit.cpp:883-937: forward-difference stencils on x = t^3, dt = 1
  auto x = [](double t) { return t * t * t; };
  const double t = 2;
  const double v = x(t + 1) - x(t);
  const double a = x(t + 2) - 2 * x(t + 1) + x(t);
  const double j = x(t + 3) - 3 * x(t + 2) + 3 * x(t + 1) - x(t);
  NEAR(v, 19, 1e-12, "velocity stencil");
  NEAR(a, 18, 1e-12, "acceleration stencil");
  NEAR(j, 6, 1e-12, "jerk stencil = 6");
}

static void kat_kinematics()
{
  // calcTransformError sign convention: err = target^-1 * source; source rotated by
  // AngleAxis(-0.1, x) relative to target gives err[3] = -0.1 (kinematic_costs_unit.cpp:250-254)
  Iso3 target = Iso3::identity();
  target.t[0] = 0.3;
  target.t[2] = 1.1;
  const double ax[3] = { 1, 0, 0 };
  Iso3 source = mul(target, axisAngle(ax, -0.1));
  double err[6];
  calcTransformError(target, source, err);
  NEAR(err[3], -0.1, 1e-12, "AngleAxis(-0.1, x) -> err[3] = -0.1");
  NEAR(err[4], 0, 1e-12, "err[4] = 0");
  NEAR(err[0], 0, 1e-12, "translation error 0");

  // FD consistency of the CartPose jacobian at q = (-1.1, 1.2, -3.3, -1.4, 5.5, -1.6, 7.7)
  // on a 7-dof chain (kinematic_costs_unit.cpp:62-77: isApprox(1e-5))
  thip_chain chain{};
  chain.n_links = 8;
  chain.n_dof = 7;
  Iso3::identity().to12(chain.base_pose);
  const double axes[7][3] = { { 0, 0, 1 }, { 0, 1, 0 }, { 1, 0, 0 }, { 0, 1, 0 }, { 1, 0, 0 }, { 0, 1, 0 }, { 1, 0, 0 } };
  const double offs[7][3] = { { 0, -0.188, 0 }, { 0.1, 0, 0 }, { 0, 0, 0 }, { 0.4, 0, 0 },
                              { 0, 0, 0 },      { 0.321, 0, 0 }, { 0, 0, 0 } };
  for (int k = 1; k <= 7; ++k)
  {
    Iso3 o = Iso3::identity();
    for (int i = 0; i < 3; ++i)
      o.t[i] = offs[k - 1][i];
    o.to12(chain.joint_origin[k]);
    chain.joint_type[k] = THIP_JOINT_REVOLUTE;
    chain.joint_dof[k] = k - 1;
    for (int i = 0; i < 3; ++i)
      chain.joint_axis[k][i] = axes[k - 1][i];
  }
  CartPoseCalc c;
  c.chain = &chain;
  c.source_link = 7;
  c.source_offset = Iso3::identity();
  c.source_offset.t[0] = 0.18;
  const DblVec q{ -1.1, 1.2, -3.3, -1.4, 5.5, -1.6, 7.7 };
  std::vector<Iso3> fk;
  chainFwdKin(chain, q.data(), fk);
  c.target_offset = mul(fk[7], c.source_offset);
  // perturb the target a little so the error is not zero
  const double ay[3] = { 0, 1, 0 };
  c.target_offset = mul(c.target_offset, axisAngle(ay, 0.2));
  c.target_offset.t[1] += 0.05;
  c.indices = { 0, 1, 2, 3, 4, 5 };
  const Mat J = c.jac(q);
  const Mat Jn = calcForwardNumJac([&](const DblVec& qq) { return c(qq); }, q, 1e-5);
  double num = 0, den = 0;
  for (std::size_t i = 0; i < J.a.size(); ++i)
  {
    num += sqr(J.a[i] - Jn.a[i]);
    den += sqr(Jn.a[i]);
  }
  CHECK(std::sqrt(num) <= 1e-5 * std::sqrt(den), "CartPose jacobian isApprox(numerical, 1e-5)");

  // Toleranced CartPose (kinematic_costs_unit.cpp:79-254): the pose error at the seed is a
  // rotation of rx0 about x, band [-0.52, 0.52] on rx and [0, 0] elsewhere.  The reference
  // tests put the active link in the target frame; here it is the source frame, which gives
  // the same error (err = static^-1 * active).
  const double axx[3] = { 1, 0, 0 };
  auto tol_calc = [&](double rx0) {
    CartPoseCalc t;
    t.chain = &chain;
    t.source_link = 7;
    t.source_offset = axisAngle(axx, rx0);
    t.target_offset = fk[7];
    t.indices = { 0, 1, 2, 3, 4, 5 };
    t.has_tol = true;
    for (int i = 0; i < 6; ++i)
      t.lower_tol[i] = t.upper_tol[i] = 0.0;
    t.lower_tol[3] = -0.52;
    t.upper_tol[3] = 0.52;
    return t;
  };
  auto fd_consistent = [&](const CartPoseCalc& t) {
    const Mat A = t.jac(q);
    const Mat Nm = calcForwardNumJac([&](const DblVec& qq) { return t(qq); }, q, 1e-5);
    double nu = 0, de = 0;
    for (std::size_t i = 0; i < A.a.size(); ++i)
    {
      nu += sqr(A.a[i] - Nm.a[i]);
      de += sqr(Nm.a[i]);
    }
    return std::sqrt(nu) <= 1e-5 * std::sqrt(de) || (de == 0 && nu == 0);
  };
  {
    // inside the band (0.1 rad): f = 0 at the seed, the rx row of J is zero, FD-consistent
    const CartPoseCalc t = tol_calc(0.1);
    const DblVec e = t(q);
    double emax = 0;
    for (double v : e)
      emax = std::fmax(emax, std::fabs(v));
    CHECK(emax <= 1e-9, "toleranced error inside the band is zero at the seed");
    const Mat A = t.jac(q);
    double rmax = 0;
    for (int j = 0; j < 7; ++j)
      rmax = std::fmax(rmax, std::fabs(A(3, j)));
    CHECK(rmax <= 1e-6, "rx row of the toleranced jacobian is zero inside the band");
    CHECK(fd_consistent(t), "toleranced jacobian isApprox(numerical, 1e-5) inside the band");
  }
  {
    // outside the band (0.8 rad): f = (true_err - upper) on rx, FD-consistent
    const CartPoseCalc t = tol_calc(0.8);
    const DblVec e = t(q);
    NEAR(e[3], 0.8 - 0.52, 1e-9, "toleranced error outside the band = true_err - upper");
    CHECK(fd_consistent(t), "toleranced jacobian isApprox(numerical, 1e-5) outside the band");
    const CartPoseCalc tn = tol_calc(-0.8);
    NEAR(tn(q)[3], -0.8 + 0.52, 1e-9, "below the band: true_err - lower");
  }
}

int main()
{
  kat_solver_utils();
  kat_modeling();
  kat_solver_interface();
  kat_small_problems();
  kat_joint_costs_stencil();
  kat_kinematics();
  std::printf("KAT pass=%d fail=%d\n", g_pass, g_fail);
  return g_fail;
}
