// trajopt_sqp::QPSolver (include/trajopt_sqp/qp_solver.h): the QP backend
// interface, minimise 1/2 x'Px + q'x s.t. l <= A x <= u, with update-in-place
// calls between solves.  trajopt_sqp::GpuQPSolver (gpu_qp_solver.h) implements it
// on the GPU in place of OSQPEigenSolver.
#pragma once
#include <memory>

#include "trajopt_ifopt/core/eigen_types.h"

namespace trajopt_sqp
{
class QPProblem;

enum class QPSolverStatus
{
  kUninitialized,
  kInitialized,
  kFailed
};

class QPSolver
{
public:
  using Ptr = std::shared_ptr<QPSolver>;
  virtual ~QPSolver() = default;
  virtual bool init(long num_vars, long num_cnts) = 0;
  virtual bool clear() = 0;
  virtual bool solve() = 0;
  virtual trajopt_ifopt::VectorXd getSolution() = 0;
  virtual bool updateHessianMatrix(const trajopt_ifopt::Jacobian& hessian) = 0;
  virtual bool updateGradient(const trajopt_ifopt::VectorXd& gradient) = 0;
  virtual bool updateLowerBound(const trajopt_ifopt::VectorXd& lowerBound) = 0;
  virtual bool updateUpperBound(const trajopt_ifopt::VectorXd& upperBound) = 0;
  virtual bool updateBounds(const trajopt_ifopt::VectorXd& lowerBound, const trajopt_ifopt::VectorXd& upperBound) = 0;
  virtual bool updateLinearConstraintsMatrix(const trajopt_ifopt::Jacobian& linearConstraintsMatrix) = 0;
  virtual bool setWarmStart(const QPProblem& qp_problem) = 0;
  virtual QPSolverStatus getSolverStatus() const = 0;
  int verbosity = 0;
};
}  // namespace trajopt_sqp
