// trajopt_sqp::GpuQPSolver: the QPSolver of the trajopt_sqp front end on the GPU,
// in place of OSQPEigenSolver (src/osqp_eigen_solver.cpp:38-326, over OsqpEigen's
// Solver).  The OSQP 1.0 solver object lives in a thip_qp resident workspace
// (include/trajopt_hip.h): the first solve sets it up (scaling, rho vector, KKT
// factor) and warm starts it from setWarmStart's point; later convexifications
// with the same sparsity pattern only send the new values
// (thip_qp_update_mat / thip_qp_update_vec, osqp_update_data_mat / _vec), and
// trust-region steps only the new bounds.  A pattern change rebuilds the
// workspace warm started from the last solution, as OsqpEigen does.
#pragma once
#include <vector>

#include "trajopt_hip.h"
#include "trajopt_sqp/qp_solver.h"

namespace trajopt_sqp
{
class GpuQPSolver : public QPSolver
{
public:
  explicit GpuQPSolver(int device = 0);
  ~GpuQPSolver() override;
  GpuQPSolver(const GpuQPSolver&) = delete;
  GpuQPSolver& operator=(const GpuQPSolver&) = delete;
  // OSQPEigenSolver::setDefaultOSQPSettings: OSQP defaults with warm start, polish,
  // adaptive rho, 8192 iterations, eps_abs 1e-4, eps_rel 1e-6
  static void setDefaultOSQPSettings(thip_osqp_settings& settings);
  bool init(long num_vars, long num_cnts) override;
  bool clear() override;
  bool solve() override;
  trajopt_ifopt::VectorXd getSolution() override;
  bool updateHessianMatrix(const trajopt_ifopt::Jacobian& hessian) override;
  bool updateGradient(const trajopt_ifopt::VectorXd& gradient) override;
  bool updateLowerBound(const trajopt_ifopt::VectorXd& lowerBound) override;
  bool updateUpperBound(const trajopt_ifopt::VectorXd& upperBound) override;
  bool updateBounds(const trajopt_ifopt::VectorXd& lowerBound, const trajopt_ifopt::VectorXd& upperBound) override;
  bool updateLinearConstraintsMatrix(const trajopt_ifopt::Jacobian& linearConstraintsMatrix) override;
  bool setWarmStart(const QPProblem& qp_problem) override;
  QPSolverStatus getSolverStatus() const override { return status_; }

  thip_osqp_settings settings;  // applied at the next setup
  // counters: full setups, in-place updates of a convexification, solves, ADMM iterations
  int n_setups = 0, n_updates = 0, n_solves = 0;
  long long admm_iters = 0;
  const thip_qp_info& lastInfo() const { return info_; }

private:
  struct Csc
  {
    std::vector<int> p, i;
    std::vector<double> x;
  };
  bool setupNow();
  bool reinitKeepingSolution();
  void fail(const char* what);
  int device_;
  QPSolverStatus status_ = QPSolverStatus::kUninitialized;
  long nv_ = 0, nc_ = 0;
  thip_qp* qp_ = nullptr;
  bool resident_ = false;  // the device workspace exists (OsqpEigen::Solver::isInitialized)
  Csc P_, A_;
  std::vector<double> q_, lo_, up_, x0_, y0_, x_, y_;
  thip_qp_info info_{};
  bool have_solution_ = false;
};
}  // namespace trajopt_sqp
