// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of the OSQP 1.0.0 solver the reference links
// (trajopt_ext/osqp/CMakeLists.txt:7,30-33; not vendored under the reference
// tree). Restated from OSQP's published algorithm (Stellato et al., "OSQP: an
// operator splitting solver for quadratic programs", 2020) and the call sites /
// settings of trajopt_sco/src/osqp_interface.cpp:78-90,283-370,440-615:
//   * modified Ruiz equilibration (settings.scaling passes) + cost scaling
//   * vector rho (equality rows x1e3, loose rows rho_min)
//   * direct quasi-definite KKT solve, LDL^T with a minimum-degree ordering
//   * ADMM with over-relaxation alpha, termination every check_termination
//     iterations on unscaled inf-norm residuals, infeasibility certificates
//   * iteration-based adaptive rho (interval 4 * check_termination)
//   * solution polishing: active-set reduced KKT + iterative refinement
//   * warm start of (x, y)
// Parity against the real OSQP binary is unpinned (OSQP is absent from this
// image); the reference's own small-problem KATs pin it at their tolerances.
#pragma once
#include <cstdint>
#include <vector>

namespace orc
{
using OsqpInt = long long;  // OSQPInt with OSQP_USE_LONG (OSQP 1.0 default)

struct Csc
{
  OsqpInt m = 0, n = 0;
  std::vector<OsqpInt> p;  // n+1
  std::vector<OsqpInt> i;  // nnz
  std::vector<double> x;   // nnz
  OsqpInt nnz() const { return p.empty() ? 0 : p[static_cast<std::size_t>(n)]; }
};

// OSQP 1.0 status values (osqp_api_constants.h)
enum OsqpStatus : int
{
  OSQP_SOLVED = 1,
  OSQP_SOLVED_INACCURATE = 2,
  OSQP_PRIMAL_INFEASIBLE = 3,
  OSQP_PRIMAL_INFEASIBLE_INACCURATE = 4,
  OSQP_DUAL_INFEASIBLE = 5,
  OSQP_DUAL_INFEASIBLE_INACCURATE = 6,
  OSQP_MAX_ITER_REACHED = 7,
  OSQP_TIME_LIMIT_REACHED = 8,
  OSQP_NON_CVX = 9,
  OSQP_SIGINT = 10,
  OSQP_UNSOLVED = 11
};

constexpr double OSQP_INFTY = 1e30;
constexpr double OSQP_RHO_MIN = 1e-6;
constexpr double OSQP_RHO_MAX = 1e6;
constexpr double OSQP_RHO_TOL = 1e-4;
constexpr double OSQP_RHO_EQ_OVER_RHO_INEQ = 1e3;
constexpr double OSQP_MIN_SCALING = 1e-4;
constexpr double OSQP_MAX_SCALING = 1e4;
constexpr double OSQP_DIVISION_TOL = 1.0 / OSQP_INFTY;
constexpr int OSQP_ADAPTIVE_RHO_MULTIPLE_TERMINATION = 4;
constexpr int OSQP_ADAPTIVE_RHO_FIXED = 100;

struct OsqpSettings
{
  double rho = 0.1;
  double sigma = 1e-6;
  double alpha = 1.6;
  int scaling = 10;
  int adaptive_rho = 1;
  int adaptive_rho_interval = 0;
  double adaptive_rho_tolerance = 5;
  int max_iter = 4000;
  double eps_abs = 1e-3;
  double eps_rel = 1e-3;
  double eps_prim_inf = 1e-4;
  double eps_dual_inf = 1e-4;
  int scaled_termination = 0;
  int check_termination = 25;
  int warm_starting = 1;
  int polishing = 0;
  double delta = 1e-6;
  int polish_refine_iter = 3;
};

// Sparse symmetric LDL^T (elimination-tree up-looking factorisation, the
// algorithm QDLDL implements) of a full-pattern symmetric CSC matrix under a
// fill-reducing permutation.
class LdlSolver
{
public:
  // Factor; returns number of positive pivots, or -1 on a zero pivot.
  int factor(const Csc& full_sym);
  // Refactor numerically with the same pattern (values changed).
  int refactor(const Csc& full_sym);
  void solve(double* b) const;  // in place
  OsqpInt dim() const { return n_; }

private:
  void order(const Csc& a);
  int numeric(const Csc& a);
  OsqpInt n_ = 0;
  std::vector<OsqpInt> perm_, pinv_, parent_, lnz_, lp_, li_;
  std::vector<double> lx_, d_;
  mutable std::vector<double> work_;
};

class OsqpSolver
{
public:
  // osqp_setup: P is upper-triangular CSC (n x n), A is m x n. Returns 0 or an
  // OSQP error code (>0).
  int setup(const Csc& P, const double* q, const Csc& A, const double* l, const double* u, OsqpInt m, OsqpInt n,
            const OsqpSettings& settings);
  int warm_start(const double* x, const double* y);
  int solve();
  // OSQP 1.0 update-in-place API (the resident solver object OsqpEigen keeps for
  // trajopt_sqp::OSQPEigenSolver): osqp_update_data_vec (q and / or l, u; NULL =
  // unchanged; the rho vector follows the constraint types, refactored only
  // when one changed) and osqp_update_data_mat (all P / A values, same pattern:
  // unscale_data, replace, scale_data, refactor).  0 or an OSQP error code.
  int update_data_vec(const double* q, const double* l, const double* u);
  int update_data_mat(const double* Px, const double* Ax);

  // unscaled solution
  std::vector<double> sol_x, sol_y;
  int status_val = OSQP_UNSOLVED;
  int status_polish = 0;
  OsqpInt iter = 0;
  double prim_res = 0, dual_res = 0;
  int rho_updates = 0;
  double polish_margin = 0;  // smallest margin of the last polish's active-set comparisons
  const OsqpSettings& settings() const { return settings_; }

private:
  // ---- data (scaled) ----
  OsqpInt n_ = 0, m_ = 0;
  Csc P_, A_, At_;  // P upper-tri (scaled), A (scaled), A^T
  std::vector<double> q_, l_, u_;
  // scaling
  std::vector<double> D_, Dinv_, E_, Einv_;
  double c_ = 1, cinv_ = 1;
  // rho
  std::vector<double> rho_vec_, rho_inv_vec_;
  std::vector<int> constr_type_;
  // iterates
  std::vector<double> x_, y_, z_, xz_tilde_, x_prev_, z_prev_, delta_x_, delta_y_;
  std::vector<double> Ax_, Px_, Aty_, Atdelta_y_, Adelta_x_, Pdelta_x_;
  // linear system
  Csc kkt_;
  std::vector<OsqpInt> kkt_rho_diag_;  // index into kkt_.x of the -1/rho diagonal entries
  LdlSolver ldl_;
  std::vector<double> sol_;
  OsqpSettings settings_;

  void scale_data();
  void unscale_data();
  int update_rho_vec();
  void set_rho_vec();
  int build_and_factor_kkt();
  int update_rho(double rho_new);
  void update_xz_tilde();
  void update_x();
  void update_z();
  void update_y();
  double compute_prim_res(const std::vector<double>& x, const std::vector<double>& z);
  double compute_dual_res(const std::vector<double>& x, const std::vector<double>& y);
  double compute_prim_tol(double eps_abs, double eps_rel) const;
  double compute_dual_tol(double eps_abs, double eps_rel) const;
  bool is_primal_infeasible(double eps);
  bool is_dual_infeasible(double eps);
  bool check_termination(bool approximate);
  double compute_rho_estimate() const;
  int adapt_rho();
  void polish();
  void store_solution();
  void cold_start();
};

// ---- small CSC helpers shared by the model restatement ----
// A x (A is m x n)
void csc_axpy(const Csc& A, const double* x, double* y, double alpha, double beta);
// A^T x
void csc_atxpy(const Csc& A, const double* x, double* y, double alpha, double beta);
// full symmetric product of an upper-triangular stored matrix
void csc_sym_triu_axpy(const Csc& P, const double* x, double* y, double alpha, double beta);
Csc csc_transpose(const Csc& A);

}  // namespace orc
