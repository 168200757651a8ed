// trajopt_sqp types (trajopt_optimizers/trajopt_sqp/include/trajopt_sqp/types.h):
// the penalty kinds of a cost set, the SQP parameters with the reference's
// defaults, the per-solve results and the status.
#pragma once
#include <limits>
#include <string>
#include <vector>

#include "trajopt_ifopt/core/eigen_types.h"

namespace trajopt_sqp
{
using trajopt_ifopt::VectorXd;

enum class CostPenaltyType
{
  kSquared,
  kAbsolute,
  kHinge
};

struct SQPParameters
{
  double improve_ratio_threshold = 0.25;
  double min_trust_box_size = 1e-4;
  double min_approx_improve = 1e-4;
  double min_approx_improve_frac = std::numeric_limits<double>::lowest();
  int max_iterations = 50;
  double trust_shrink_ratio = 0.1;
  double trust_expand_ratio = 1.5;
  double cnt_tolerance = 1e-4;
  double max_merit_coeff_increases = 5;
  int max_qp_solver_failures = 3;
  double merit_coeff_increase_ratio = 10;
  double max_time = std::numeric_limits<double>::max();
  double initial_merit_error_coeff = 10;
  bool inflate_constraints_individually = true;
  double initial_trust_box_size = 1e-1;
  bool log_results = false;
  std::string log_dir = "/tmp";
};

struct SQPResults
{
  SQPResults() = default;
  SQPResults(long num_vars, long num_cnts, long num_costs);
  double best_exact_merit = std::numeric_limits<double>::max();
  double new_exact_merit = std::numeric_limits<double>::max();
  double best_approx_merit = std::numeric_limits<double>::max();
  double new_approx_merit = std::numeric_limits<double>::max();
  VectorXd best_var_vals, new_var_vals;
  double approx_merit_improve = 0, exact_merit_improve = 0, merit_improve_ratio = 0;
  VectorXd box_size, merit_error_coeffs;
  VectorXd best_constraint_violations, new_constraint_violations;
  VectorXd best_approx_constraint_violations, new_approx_constraint_violations;
  VectorXd best_costs, new_costs, best_approx_costs, new_approx_costs;
  std::vector<std::string> constraint_names, cost_names;
  int penalty_iteration = 0, convexify_iteration = 0, trust_region_iteration = 0, overall_iteration = 0;
};

enum class SQPStatus
{
  kRunning,
  kConverged,
  kIterationLimit,
  kPenaltyIterationLimit,
  kTimeLimit,
  kQPSolveFailed,
  kStoppedByCallback
};
std::string toString(SQPStatus status);
}  // namespace trajopt_sqp
