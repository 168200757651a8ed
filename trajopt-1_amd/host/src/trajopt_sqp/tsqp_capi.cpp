// C entry points of the trajopt_sqp front end (include/trajopt_host.h, tsqp_*):
// a tsqp_spec becomes NodesVariables + trajopt_ifopt joint constraint sets in a
// TrajOptQPProblem, solved by TrustRegionSQPSolver with a GpuQPSolver -- the
// setup of the reference's trajopt_sqp joint optimisation tests
// (trajopt_optimizers/trajopt_sqp/test/joint_*_optimization_unit.cpp).
#include <cstdio>
#include <cstring>
#include <exception>
#include <limits>
#include <memory>
#include <string>

#include "trajopt_host.h"
#include "trajopt_ifopt/constraints/joint_constraints.h"
#include "trajopt_sqp/gpu_qp_solver.h"
#include "trajopt_sqp/trajopt_qp_problem.h"
#include "trajopt_sqp/trust_region_sqp_solver.h"

namespace
{
void setErr(char* err, int len, const std::string& msg)
{
  if (err && len > 0)
    std::snprintf(err, static_cast<std::size_t>(len), "%s", msg.c_str());
}
}  // namespace

extern "C" {

void thost_tsqp_defaults(tsqp_spec* s)
{
  if (!s)
    return;
  const trajopt_sqp::SQPParameters p;
  s->improve_ratio_threshold = p.improve_ratio_threshold;
  s->min_trust_box_size = p.min_trust_box_size;
  s->min_approx_improve = p.min_approx_improve;
  s->min_approx_improve_frac = p.min_approx_improve_frac;
  s->max_iterations = p.max_iterations;
  s->trust_shrink_ratio = p.trust_shrink_ratio;
  s->trust_expand_ratio = p.trust_expand_ratio;
  s->cnt_tolerance = p.cnt_tolerance;
  s->max_merit_coeff_increases = p.max_merit_coeff_increases;
  s->max_qp_solver_failures = p.max_qp_solver_failures;
  s->merit_coeff_increase_ratio = p.merit_coeff_increase_ratio;
  s->max_time = p.max_time;
  s->initial_merit_error_coeff = p.initial_merit_error_coeff;
  s->inflate_constraints_individually = p.inflate_constraints_individually ? 1 : 0;
  s->initial_trust_box_size = p.initial_trust_box_size;
  trajopt_sqp::GpuQPSolver::setDefaultOSQPSettings(s->osqp);
}

int thost_tsqp_solve(const tsqp_spec* s, int device, double* x, tsqp_result* result, char* err, int err_len)
{
  try
  {
    using namespace trajopt_ifopt;
    if (!s || !x)
      throw std::runtime_error("thost_tsqp_solve: null argument");
    if (s->n_nodes < 1 || s->n_nodes > TSQP_MAX_NODES || s->n_dof < 1 || s->n_dof > THIP_MAX_DOF || s->n_terms < 0 ||
        s->n_terms > TSQP_MAX_TERMS)
      throw std::runtime_error("thost_tsqp_solve: spec out of range");
    const int D = s->n_dof;
    std::vector<std::unique_ptr<Node>> nodes;
    std::vector<std::shared_ptr<const Var>> vars;
    std::vector<Bounds> vb;
    for (int k = 0; k < D; ++k)
      vb.emplace_back(s->var_lower[k], s->var_upper[k]);
    for (int t = 0; t < s->n_nodes; ++t)
    {
      auto node = std::make_unique<Node>("Joint_Position_" + std::to_string(t));
      vars.push_back(node->addVar("position", std::vector<std::string>(static_cast<std::size_t>(D), "name"),
                                  VectorXd(s->init + t * D, s->init + (t + 1) * D), vb));
      nodes.push_back(std::move(node));
    }
    auto variables = std::make_shared<NodesVariables>("joint_trajectory", std::move(nodes));
    auto problem = std::make_shared<trajopt_sqp::TrajOptQPProblem>(variables);
    for (int i = 0; i < s->n_terms; ++i)
    {
      const tsqp_term& t = s->terms[i];
      if (t.first < 0 || t.last < t.first || t.last >= s->n_nodes)
        throw std::runtime_error("thost_tsqp_solve: term nodes out of range");
      if (t.n_coeffs != 0 && t.n_coeffs != 1 && t.n_coeffs != D)
        throw std::runtime_error("thost_tsqp_solve: term " + std::to_string(i) + ": n_coeffs must be 0, 1 or n_dof");
      const VectorXd coeffs(t.coeffs, t.coeffs + t.n_coeffs);
      const VectorXd lower(t.lower, t.lower + D);
      std::shared_ptr<ConstraintSet> cs;
      const std::vector<std::shared_ptr<const Var>> span(vars.begin() + t.first, vars.begin() + t.last + 1);
      switch (t.kind)
      {
        case TSQP_JOINT_POS:
        {
          std::vector<Bounds> b;
          for (int k = 0; k < D; ++k)
            b.emplace_back(t.lower[k], t.upper[k]);
          cs = std::make_shared<JointPosConstraint>(b, vars[static_cast<std::size_t>(t.first)], coeffs, "JointPos");
          break;
        }
        case TSQP_JOINT_VEL:
          cs = std::make_shared<JointVelConstraint>(lower, span, coeffs, "JointVel");
          break;
        case TSQP_JOINT_ACC:
          cs = std::make_shared<JointAccelConstraint>(lower, span, coeffs, "JointAccel");
          break;
        case TSQP_JOINT_JERK:
          cs = std::make_shared<JointJerkConstraint>(lower, span, coeffs, "JointJerk");
          break;
        default:
          throw std::runtime_error("thost_tsqp_solve: unknown term kind");
      }
      switch (t.penalty)
      {
        case TSQP_CONSTRAINT:
          problem->addConstraintSet(cs);
          break;
        case TSQP_SQUARED:
          problem->addCostSet(cs, trajopt_sqp::CostPenaltyType::kSquared);
          break;
        case TSQP_ABSOLUTE:
          problem->addCostSet(cs, trajopt_sqp::CostPenaltyType::kAbsolute);
          break;
        case TSQP_HINGE:
          problem->addCostSet(cs, trajopt_sqp::CostPenaltyType::kHinge);
          break;
        default:
          throw std::runtime_error("thost_tsqp_solve: unknown penalty type");
      }
    }
    problem->setup();
    // the QP keeps one size for the whole solve: check the GPU solver's capacity up front
    if (problem->getNumQPVars() + problem->getNumQPConstraints() > THIP_QP_MAX_KKT)
      throw std::runtime_error("thost_tsqp_solve: the QP has " + std::to_string(problem->getNumQPVars()) +
                               " variables and " + std::to_string(problem->getNumQPConstraints()) +
                               " constraints; the GPU QP solver takes n + m <= THIP_QP_MAX_KKT (" +
                               std::to_string(THIP_QP_MAX_KKT) + ")");
    auto qp_solver = std::make_shared<trajopt_sqp::GpuQPSolver>(device);
    qp_solver->settings = s->osqp;
    trajopt_sqp::TrustRegionSQPSolver solver(qp_solver);
    trajopt_sqp::SQPParameters& p = solver.params;
    p.improve_ratio_threshold = s->improve_ratio_threshold;
    p.min_trust_box_size = s->min_trust_box_size;
    p.min_approx_improve = s->min_approx_improve;
    p.min_approx_improve_frac = s->min_approx_improve_frac;
    p.max_iterations = s->max_iterations;
    p.trust_shrink_ratio = s->trust_shrink_ratio;
    p.trust_expand_ratio = s->trust_expand_ratio;
    p.cnt_tolerance = s->cnt_tolerance;
    p.max_merit_coeff_increases = s->max_merit_coeff_increases;
    p.max_qp_solver_failures = s->max_qp_solver_failures;
    p.merit_coeff_increase_ratio = s->merit_coeff_increase_ratio;
    p.max_time = s->max_time;
    p.initial_merit_error_coeff = s->initial_merit_error_coeff;
    p.inflate_constraints_individually = s->inflate_constraints_individually != 0;
    p.initial_trust_box_size = s->initial_trust_box_size;
    solver.solve(problem);
    const VectorXd xv = problem->getVariableValues();
    std::memcpy(x, xv.data(), sizeof(double) * xv.size());
    if (result)
    {
      std::memset(result, 0, sizeof(*result));
      result->status = static_cast<int>(solver.getStatus());
      const trajopt_sqp::SQPResults& r = solver.getResults();
      result->overall_iteration = r.overall_iteration;
      result->penalty_iteration = r.penalty_iteration;
      result->qp_setups = qp_solver->n_setups;
      result->qp_updates = qp_solver->n_updates;
      result->qp_solves = qp_solver->n_solves;
      result->admm_iters = qp_solver->admm_iters;
      result->best_exact_merit = r.best_exact_merit;
    }
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

int thost_tsqp_sizeof_spec(void) { return static_cast<int>(sizeof(tsqp_spec)); }
int thost_tsqp_sizeof_result(void) { return static_cast<int>(sizeof(tsqp_result)); }
}  // extern "C"
