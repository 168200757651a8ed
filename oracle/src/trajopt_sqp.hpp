// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of trajopt's second SQP front end, trajopt_sqp (the ifopt
// stack), for SURVEY.md §8f rank 3: the fixed-sparsity, update-in-place QP path
//   TrustRegionSQPSolver            trajopt_optimizers/trajopt_sqp/src/trust_region_sqp_solver.cpp:44-383
//   TrajOptQPProblem                trajopt_optimizers/trajopt_sqp/src/trajopt_qp_problem.cpp:131-245,405-1123
//   AffExprs / QuadExprs            trajopt_optimizers/trajopt_sqp/src/expressions.cpp:6-223
//   OSQPEigenSolver (+ OsqpEigen)   trajopt_optimizers/trajopt_sqp/src/osqp_eigen_solver.cpp:38-326
//   joint terms                     trajopt_ifopt/src/constraints/joint_{position,velocity,acceleration,jerk}_constraint.cpp
//   Bounds, calcBoundsViolations    trajopt_ifopt/src/core/bounds.cpp:24-84, src/utils/ifopt_utils.cpp:122-145
// on the oracle's OSQP 1.0 restatement with its update-in-place calls
// (osqp_restated.hpp).  OsqpEigen 0.11.2 (a git dependency, absent from
// /root/reference) is restated from its published behaviour: the solver is set
// up on the first solve, matrices with an unchanged pattern are updated in place
// (osqp_update_data_mat), vectors with osqp_update_data_vec.
#pragma once
#include <string>
#include <vector>

#include "../../include/trajopt_host.h"
#include "osqp_restated.hpp"

namespace orc
{
namespace tsqp
{
enum class BoundsType
{
  kEquality,
  kRangeBound,
  kLowerBound,
  kUpperBound,
  kUnbounded
};

// trajopt_ifopt::Bounds (bounds.cpp:24-84)
struct Bound
{
  double lo = 0, up = 0;
  BoundsType type = BoundsType::kUnbounded;
  Bound() = default;
  Bound(double l, double u);
};

// row-major sparse matrix (trajopt_ifopt::Jacobian is Eigen RowMajor)
struct Rm
{
  int rows = 0, cols = 0;
  std::vector<int> outer{ 0 };
  std::vector<int> inner;
  std::vector<double> val;
  void push(int c, double v)
  {
    inner.push_back(c);
    val.push_back(v);
  }
  void endRow() { outer.push_back(static_cast<int>(inner.size())); }
};

// one constraint set over the flat variable vector (NodesVariables)
struct Term
{
  std::string name;
  int rows = 0;
  std::vector<Bound> bounds;
  std::vector<double> coeffs;
  // value / jacobian of a joint term: rows of sum_k w_k x[col_k]
  std::vector<std::vector<int>> cols;
  std::vector<std::vector<double>> w;
  std::vector<double> values(const std::vector<double>& x) const;
  Rm jacobian(int n_vars) const;
};

struct Result
{
  std::vector<double> x;
  int status = 0;  // TSQP_STATUS_*
  int overall_iteration = 0, penalty_iteration = 0, qp_solves = 0, qp_setups = 0, qp_updates = 0;
  long long admm_iters = 0;
  double best_exact_merit = 0;
};

// builds the terms of a tsqp_spec, then TrustRegionSQPSolver::solve
Result solve(const tsqp_spec& spec);

}  // namespace tsqp
}  // namespace orc
