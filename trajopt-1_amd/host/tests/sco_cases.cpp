// Test driver (not part of libtrajopt_host): the reference's trajopt_sco unit
// problems run through this build's sco surface -- GpuModel for the convex
// subproblems, BasicTrustRegionSQP's host loop -- for tests/test_gpu.py.
// Case ids and set-ups match oracle/src/sco_cases.cpp, which restates the same
// reference tests on the oracle's OSQPModel:
//   0      solver-interface-unit.cpp:33-72   setup_problem
//   1, 2   solver-interface-unit.cpp:130-231 ExprMult_test2 / ExprMult_test3
//   3, 4   small-problems-unit.cpp:49-83     QuadraticSeparable / QuadraticNonseparable
//   5..8   small-problems-unit.cpp:111-172   TP1, TP3, TP6, TP7
//   9      a QP beyond THIP_QP_MAX_KKT (CVX_FAILED, before touching the device)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <exception>
#include <string>

#include "trajopt_amd/batch_sqp.hpp"
#include "trajopt_sco/expr_ops.hpp"
#include "trajopt_sco/gpu_model.hpp"
#include "trajopt_sco/modeling_utils.hpp"
#include "trajopt_sco/optimizers.hpp"

namespace
{
using namespace sco;

double sq(double a) { return a * a; }

struct CaseOut
{
  DblVec x;
  int status = 0, n_qp = 0, n_sqp = 0, n_vars_after = 0;
  long long n_admm = 0;
};

GpuModelConfig::ConstPtr config(int device)
{
  auto c = std::make_shared<GpuModelConfig>();
  c->device = device;
  return c;
}

CaseOut qpCase(int id, int device)
{
  CaseOut o;
  GpuModel solver(*config(device));
  if (id == 9)
  {
    // beyond the KKT capacity: 32769 bounded variables (n + m = 65538 > THIP_QP_MAX_KKT)
    VarVector vars;
    for (int i = 0; i < THIP_QP_MAX_KKT / 2 + 1; ++i)
      vars.push_back(solver.addVar("v" + std::to_string(i), -1, 1));
    solver.update();
    QuadExpr obj;
    for (const Var& v : vars)
      exprInc(obj, exprSquare(AffExpr(v)));
    solver.setObjective(obj);
    solver.update();
    o.status = solver.optimize();  // CVX_FAILED: the reference's failure handling applies
    return o;
  }
  if (id == 0)
  {
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
    o.status = solver.optimize();
    o.x = solver.getVarValues(vars);
    solver.removeVars(VarVector(1, vars[2]));
    solver.update();
    o.n_vars_after = static_cast<int>(solver.getVars().size());
  }
  else
  {
    const double v1 = 10, v2 = 20;
    const double c1 = id == 1 ? 2 : 3, c2 = id == 1 ? 1 : 2, k1 = id == 1 ? 0 : -3, k2 = id == 1 ? 0 : -5;
    VarVector vars{ solver.addVar("v1"), solver.addVar("v2") };
    solver.update();
    AffExpr a1, a2;
    exprInc(a1, vars[0]);
    solver.setVarBounds(vars[0], v1, v1);
    a1.constant = k1;
    a1.coeffs[0] = c1;
    exprInc(a2, vars[1]);
    solver.setVarBounds(vars[1], v2, v2);
    a2.constant = k2;
    a2.coeffs[0] = c2;
    solver.setObjective(exprMult(a1, a2));
    solver.update();
    o.status = solver.optimize();
    o.x = solver.getVarValues(vars);
    o.n_vars_after = static_cast<int>(solver.getVars().size());
  }
  o.n_qp = 1;
  o.n_admm = solver.admmItersTotal();
  return o;
}

OptProb::Ptr makeProblem(std::size_t n, int device)
{
  auto prob = std::make_shared<OptProb>(ModelType::OSQP, config(device));
  std::vector<std::string> names;
  for (std::size_t i = 0; i < n; ++i)
    names.push_back("x_" + std::to_string(i));
  prob->createVariables(names);
  return prob;
}

CaseOut sqpCase(int id, int device)
{
  DblVec init;
  OptProb::Ptr prob;
  BasicTrustRegionSQPParameters p;
  if (id == 3 || id == 4)
  {
    prob = makeProblem(3, device);
    if (id == 3)
      prob->addCost(std::make_shared<CostFromFunc>(
          ScalarOfVector::construct([](const DblVec& x) { return x[0] * x[0] + sq(x[1] - 1) + sq(x[2] - 2); }),
          prob->getVars(), "f"));
    else
      prob->addCost(std::make_shared<CostFromFunc>(
          ScalarOfVector::construct(
              [](const DblVec& x) { return sq(x[0] - x[1] + 3 * x[2]) + sq(x[0] - 1) + sq(x[2] - 2); }),
          prob->getVars(), "f", true));
    p.trust_box_size = 100;
    if (id == 4)
    {
      p.min_trust_box_size = 1e-5;
      p.min_approx_improve = 1e-6;
    }
    init = { 3, 4, 5 };
  }
  else
  {
    ScalarOfVector::func f;
    VectorOfVector::func g;
    ConstraintType t = INEQ;
    switch (id)
    {
      case 5:
        f = [](const DblVec& x) { return 1 * sq(x[1] - sq(x[0])) + sq(1 - x[0]); };
        g = [](const DblVec& x) { return DblVec{ -1.5 - x[1] }; };
        init = { -2, 1 };
        break;
      case 6:
        f = [](const DblVec& x) { return x[1] + 1e-5 * sq(x[1] - x[0]); };
        g = [](const DblVec& x) { return DblVec{ 0 - x[1] }; };
        init = { 10, 1 };
        break;
      case 7:
        f = [](const DblVec& x) { return sq(1 - x[0]); };
        g = [](const DblVec& x) { return DblVec{ 10 * (x[1] - sq(x[0])) }; };
        t = EQ;
        init = { 10, 1 };
        break;
      default:
        f = [](const DblVec& x) { return std::log(1 + sq(x[0])) - x[1]; };
        g = [](const DblVec& x) { return DblVec{ sq(1 + sq(x[0])) + sq(x[1]) - 4 }; };
        t = EQ;
        init = { 2, 2 };
        break;
    }
    prob = makeProblem(init.size(), device);
    prob->addCost(std::make_shared<CostFromFunc>(ScalarOfVector::construct(f), prob->getVars(), "f", true));
    prob->addConstraint(
        std::make_shared<ConstraintFromErrFunc>(VectorOfVector::construct(g), prob->getVars(), DblVec(), t, "g"));
    p.max_iter = 1000;
    p.min_trust_box_size = 1e-5;
    p.min_approx_improve = 1e-10;
    p.initial_merit_error_coeff = 1;
  }
  BasicTrustRegionSQP solver(prob);
  solver.setParameters(p);
  solver.initialize(init);
  CaseOut o;
  o.status = solver.optimize();
  o.x = solver.x();
  o.n_qp = solver.results().n_qp_solves;
  o.n_sqp = solver.results().n_sqp_iters;
  o.n_admm = solver.results().n_admm_iters;
  return o;
}

// TP1 (case 5) with the optimizer's logs, a time limit, or a QP that cannot be
// solved: the reference's diagnostics on the generic path.
//   mode 0: log_results into log_dir (optimizers.cpp:533-647 formats)
//   mode 1: max_time = 0 (optimizers.cpp:739-753: the limit is checked before
//           the first convexification)
//   mode 2: an infeasible linear constraint pair (x0 >= 1 and x0 <= 0): every
//           QP fails, /tmp/fail.lp is written (optimizers.cpp:817-842) and the
//           run ends OPT_FAILED after max_qp_solver_failures
CaseOut diagCase(int mode, int device, const char* log_dir)
{
  auto prob = makeProblem(2, device);
  prob->addCost(std::make_shared<CostFromFunc>(
      ScalarOfVector::construct([](const DblVec& x) { return 1 * sq(x[1] - sq(x[0])) + sq(1 - x[0]); }),
      prob->getVars(), "f", true));
  prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(
      VectorOfVector::construct([](const DblVec& x) { return DblVec{ -1.5 - x[1] }; }), prob->getVars(), DblVec(),
      INEQ, "g"));
  if (mode == 2)
  {
    const Var x0 = prob->getVars()[0];
    AffExpr ge;  // 1 - x0 <= 0
    ge.constant = 1;
    ge.coeffs = { -1 };
    ge.vars = { x0 };
    prob->addLinearConstraint(ge, INEQ);
    prob->addLinearConstraint(AffExpr(x0), INEQ);  // x0 <= 0
  }
  BasicTrustRegionSQP solver(prob);
  BasicTrustRegionSQPParameters p;
  p.max_iter = 1000;
  p.min_trust_box_size = 1e-5;
  p.min_approx_improve = 1e-10;
  p.initial_merit_error_coeff = 1;
  if (mode == 0)
  {
    p.log_results = true;
    p.log_dir = log_dir;
  }
  if (mode == 1)
    p.max_time = 0.0;
  solver.setParameters(p);
  solver.initialize({ -2, 1 });
  CaseOut o;
  o.status = solver.optimize();
  o.x = solver.x();
  o.n_qp = solver.results().n_qp_solves;
  o.n_sqp = solver.results().n_sqp_iters;
  return o;
}
}  // namespace

namespace
{
void setErr(char* err, int err_len, const char* what)
{
  if (err && err_len > 0)
  {
    const std::size_t n = std::min<std::size_t>(std::strlen(what), static_cast<std::size_t>(err_len - 1));
    std::memcpy(err, what, n);
    err[n] = '\0';
  }
}
}  // namespace

namespace
{
// the user term of the drop-in test (the same function as oracle/src/capi.cpp userCost)
double userCost(const DblVec& q) { return 2.0 * (std::sin(q[0]) - 0.25) * (std::sin(q[0]) - 0.25) + 0.5 * (q[1] + q[2] - 0.1) * (q[1] + q[2] - 0.1); }
}  // namespace

extern "C" {
// A JSON problem (ConstructProblem on its built-in environment) plus a user
// sco::CostFromFunc over waypoint n_steps / 2, joints 0..2, appended after the
// hatched terms -- a caller's custom term next to the built-in CartPose /
// collision terms -- solved by trajopt::BasicTrustRegionSQP (the host loop,
// kinematic terms evaluated on the device).  x: [n_steps][n_dof].
int sco_case_user_cost(const char* json, int device, double* x, thip_result* res, char* err, int err_len)
{
  try
  {
    const Json::Value root = Json::parse(json);
    std::string manip;
    json_marshal::childFromJson(root["basic_info"], manip, "manip");
    auto prob = trajopt::ConstructProblem(root, trajopt::Environment::builtin(manip));
    const int t = prob->GetNumSteps() / 2;
    prob->addCost(std::make_shared<CostFromFunc>(ScalarOfVector::construct(userCost), prob->GetVarRow(t, 0, 3),
                                                 "user_cost", false));
    trajopt::BasicTrustRegionSQP opt(prob, device);
    opt.initialize(trajopt::trajToDblVec(prob->GetInitTraj()));
    opt.optimize();
    const OptResults& r = opt.results();
    std::memcpy(x, r.x.data(), r.x.size() * sizeof(double));
    std::memset(res, 0, sizeof(*res));
    res->status = static_cast<int>(r.status);
    res->n_sqp_iters = r.n_sqp_iters;
    res->n_qp_solves = r.n_qp_solves;
    res->n_func_evals = r.n_func_evals;
    res->total_cost = r.total_cost;
    res->max_cnt_viol = r.max_cnt_viol;
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

// counts[3] = {status, n_qp_solves, n_sqp_iters}; x: [2]
int sco_case_diag(int mode, int device, const char* log_dir, double* x, int* counts, char* err, int err_len)
{
  try
  {
    const CaseOut o = diagCase(mode, device, log_dir ? log_dir : "/tmp");
    x[0] = o.x[0];
    x[1] = o.x[1];
    counts[0] = o.status;
    counts[1] = o.n_qp;
    counts[2] = o.n_sqp;
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

// x: [cap]; counts[5] = {n_x, status, n_qp_solves, n_sqp_iters, n_vars_after}
int sco_case_run(int id, int device, double* x, int cap, int* counts, long long* n_admm, char* err, int err_len)
{
  try
  {
    if (id < 0 || id > 9)
      throw std::runtime_error("unknown case");
    const CaseOut o = (id <= 2 || id == 9) ? qpCase(id, device) : sqpCase(id, device);
    if (static_cast<int>(o.x.size()) > cap)
      throw std::runtime_error("x capacity");
    std::memcpy(x, o.x.data(), o.x.size() * sizeof(double));
    counts[0] = static_cast<int>(o.x.size());
    counts[1] = o.status;
    counts[2] = o.n_qp;
    counts[3] = o.n_sqp;
    counts[4] = o.n_vars_after;
    if (n_admm)
      *n_admm = o.n_admm;
    return 0;
  }
  catch (const std::exception& e)
  {
    if (err && err_len > 0)
    {
      const std::size_t n = std::min<std::size_t>(std::strlen(e.what()), static_cast<std::size_t>(err_len - 1));
      std::memcpy(err, e.what(), n);
      err[n] = '\0';
    }
    return -1;
  }
}
}
