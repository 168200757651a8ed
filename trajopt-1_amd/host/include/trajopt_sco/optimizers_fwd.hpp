// OptStatus / OptResults / BasicTrustRegionSQPParameters
// (trajopt_sco/include/trajopt_sco/optimizers.hpp:25-135), split out so that
// modeling.hpp can name them.
#pragma once
#include <string>

#include "trajopt_sco/sco_common.hpp"

namespace sco
{
// optimizers.hpp:25-33
enum OptStatus : int
{
  OPT_CONVERGED,
  OPT_SCO_ITERATION_LIMIT,
  OPT_PENALTY_ITERATION_LIMIT,
  OPT_TIME_LIMIT,
  OPT_FAILED,
  INVALID
};
std::string toString(OptStatus status);

// optimizers.hpp:40-59 (+ the counters the MI355X build reports)
struct OptResults
{
  DblVec x;
  OptStatus status{ INVALID };
  double total_cost{ 0 };
  DblVec cost_vals;  // the batched kernel reports totals only (empty there)
  DblVec cnt_viols;
  int n_func_evals{ 0 }, n_qp_solves{ 0 };
  int n_sqp_iters{ 0 };
  long long n_admm_iters{ 0 };
  double max_cnt_viol{ 0 };
  int flags{ 0 };
  void clear()
  {
    x.clear();
    status = INVALID;
    total_cost = 0;
    cost_vals.clear();
    cnt_viols.clear();
    n_func_evals = n_qp_solves = n_sqp_iters = 0;
    n_admm_iters = 0;
    max_cnt_viol = 0;
    flags = 0;
  }
};

// optimizers.hpp:92-135
struct BasicTrustRegionSQPParameters
{
  double improve_ratio_threshold = 0.25;
  double min_trust_box_size = 1e-4;
  double min_approx_improve = 1e-4;
  double min_approx_improve_frac = -1.7976931348623157e308;
  int max_iter = 50;
  double trust_shrink_ratio = 0.1;
  double trust_expand_ratio = 1.5;
  double cnt_tolerance = 1e-4;
  double max_merit_coeff_increases = 5;
  int max_qp_solver_failures = 3;
  double merit_coeff_increase_ratio = 10;
  double max_time = 1.7976931348623157e308;
  double initial_merit_error_coeff = 10;
  bool inflate_constraints_individually = true;
  double trust_box_size = 1e-1;
  // optimizers.hpp:127-129: log_dir/trajopt_{solver,vars,costs,constraints}.log
  bool log_results = false;
  std::string log_dir = "/tmp";
  int num_threads = 0;  // BasicTrustRegionSQPMultiThreaded (the device runs the terms in parallel anyway)
};
}  // namespace sco
