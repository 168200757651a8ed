// trajopt_sqp::GpuQPSolver (gpu_qp_solver.h): OSQPEigenSolver's behaviour
// (trajopt_optimizers/trajopt_sqp/src/osqp_eigen_solver.cpp:38-326) with the
// OSQP solver object in a thip_qp resident workspace on the GPU.  OsqpEigen
// 0.11.2 (absent from /root/reference) is restated from its published
// behaviour: the data is collected until the first solve sets the solver up; a
// matrix with the stored pattern is updated in place, another pattern rebuilds
// the solver warm started from its last primal / dual solution.
#include "trajopt_sqp/gpu_qp_solver.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

#include "trajopt_sqp/qp_problem.h"

namespace trajopt_sqp
{
namespace
{
constexpr double kOsqpInfty = 1e30;  // OSQP_INFTY

// CSC of a row-major matrix (all stored entries, zeros included), optionally the
// upper triangle only, scaled
void toCsc(const trajopt_ifopt::Jacobian& J, bool upper, double scale, std::vector<int>& p, std::vector<int>& idx,
           std::vector<double>& x)
{
  const long n = J.cols();
  std::vector<std::vector<std::pair<int, double>>> col(static_cast<std::size_t>(n));
  for (long r = 0; r < J.rows(); ++r)
    for (long e = J.rowBegin(r); e < J.rowEnd(r); ++e)
      if (!upper || r <= J.col(e))
        col[static_cast<std::size_t>(J.col(e))].emplace_back(static_cast<int>(r), J.value(e) * scale);
  p.assign(static_cast<std::size_t>(n) + 1, 0);
  idx.clear();
  x.clear();
  for (long j = 0; j < n; ++j)
  {
    for (const auto& e : col[static_cast<std::size_t>(j)])  // rows ascending: row-major scan order
    {
      idx.push_back(e.first);
      x.push_back(e.second);
    }
    p[static_cast<std::size_t>(j) + 1] = static_cast<int>(idx.size());
  }
}
}  // namespace

void GpuQPSolver::setDefaultOSQPSettings(thip_osqp_settings& s)
{
  thip_default_osqp_settings(&s);  // OSQP 1.0 defaults with trajopt's overrides (same values)
  s.warm_starting = 1;
  s.polishing = 1;
  s.adaptive_rho = 1;
  s.max_iter = 8192;
  s.eps_abs = 1e-4;
  s.eps_rel = 1e-6;
}

GpuQPSolver::GpuQPSolver(int device) : device_(device) { setDefaultOSQPSettings(settings); }

GpuQPSolver::~GpuQPSolver() { thip_qp_destroy(qp_); }

void GpuQPSolver::fail(const char* what)
{
  throw std::runtime_error(std::string("GpuQPSolver: ") + what + ": " + (qp_ ? thip_qp_last_error(qp_) : thip_qp_last_error(nullptr)));
}

bool GpuQPSolver::init(long num_vars, long num_cnts)
{
  nv_ = num_vars;
  nc_ = num_cnts;
  x0_.assign(static_cast<std::size_t>(nv_), 0.0);
  y0_.assign(static_cast<std::size_t>(nc_), 0.0);
  status_ = QPSolverStatus::kInitialized;
  return true;
}

bool GpuQPSolver::clear()
{
  thip_qp_destroy(qp_);
  qp_ = nullptr;
  resident_ = false;
  have_solution_ = false;
  nv_ = nc_ = 0;
  P_ = Csc{};
  A_ = Csc{};
  q_.clear();
  lo_.clear();
  up_.clear();
  x0_.clear();
  y0_.clear();
  status_ = QPSolverStatus::kUninitialized;
  return true;
}

// osqp_setup on the device (a new thip_qp when the pattern is new)
bool GpuQPSolver::setupNow()
{
  thip_qp_destroy(qp_);
  qp_ = nullptr;
  resident_ = false;
  if (nv_ + nc_ > THIP_QP_MAX_KKT)  // the KKT capacity bounds the problem size: a limit, not a QP failure
    throw std::runtime_error("GpuQPSolver: the QP has " + std::to_string(nv_) + " variables and " +
                             std::to_string(nc_) + " constraints; the GPU QP solver takes n + m <= THIP_QP_MAX_KKT (" +
                             std::to_string(THIP_QP_MAX_KKT) + ")");
  if (thip_qp_create(device_, static_cast<int>(nv_), static_cast<int>(nc_), P_.p.data(), P_.i.data(), A_.p.data(),
                     A_.i.data(), 1, &qp_) != THIP_OK)
    fail("thip_qp_create");
  ++n_setups;
  if (thip_qp_setup(qp_, P_.x.data(), q_.data(), A_.x.data(), lo_.data(), up_.data(), &settings, &info_) != THIP_OK)
    fail("thip_qp_setup");
  resident_ = info_.status != -1;
  return resident_;
}

// the pattern changed under a live solver: a new one warm started from the last solution
bool GpuQPSolver::reinitKeepingSolution()
{
  const std::vector<double> xs = x_, ys = y_;
  const bool had = have_solution_;
  if (!setupNow())
    return false;
  if (had && static_cast<long>(xs.size()) == nv_ && static_cast<long>(ys.size()) == nc_)
    if (thip_qp_warm_start(qp_, xs.data(), ys.data()) != THIP_OK)
      fail("thip_qp_warm_start");
  return true;
}

bool GpuQPSolver::updateHessianMatrix(const trajopt_ifopt::Jacobian& hessian)
{
  Csc n;
  toCsc(hessian, true, 2.0, n.p, n.i, n.x);  // OSQP halves the quadratic term
  const bool same = n.p == P_.p && n.i == P_.i;
  P_ = std::move(n);
  if (!resident_)
    return true;  // collected for the setup
  if (!same)
    return reinitKeepingSolution();
  if (thip_qp_update_mat(qp_, P_.x.data(), nullptr, &info_) != THIP_OK)
    fail("thip_qp_update_mat");
  if (info_.status == -1)
    resident_ = false;
  return info_.status != -1;
}

bool GpuQPSolver::updateGradient(const trajopt_ifopt::VectorXd& gradient)
{
  q_.resize(gradient.size());
  for (std::size_t j = 0; j < gradient.size(); ++j)
    q_[j] = (std::abs(gradient[j]) < 1e-7) ? 0.0 : gradient[j];
  if (!resident_)
    return true;
  if (thip_qp_update_vec(qp_, q_.data(), nullptr, nullptr, &info_) != THIP_OK)
    fail("thip_qp_update_vec");
  return info_.status != -1;
}

bool GpuQPSolver::updateLowerBound(const trajopt_ifopt::VectorXd& lowerBound)
{
  return updateBounds(lowerBound, up_.size() == lowerBound.size() ? up_ : trajopt_ifopt::VectorXd(lowerBound.size(), kOsqpInfty));
}

bool GpuQPSolver::updateUpperBound(const trajopt_ifopt::VectorXd& upperBound)
{
  return updateBounds(lo_.size() == upperBound.size() ? lo_ : trajopt_ifopt::VectorXd(upperBound.size(), -kOsqpInfty), upperBound);
}

bool GpuQPSolver::updateBounds(const trajopt_ifopt::VectorXd& lowerBound, const trajopt_ifopt::VectorXd& upperBound)
{
  lo_.resize(lowerBound.size());
  up_.resize(upperBound.size());
  for (std::size_t r = 0; r < lowerBound.size(); ++r)
    lo_[r] = std::max(lowerBound[r], -kOsqpInfty);
  for (std::size_t r = 0; r < upperBound.size(); ++r)
    up_[r] = std::min(upperBound[r], kOsqpInfty);
  if (!resident_)
    return true;
  if (thip_qp_update_vec(qp_, nullptr, lo_.data(), up_.data(), &info_) != THIP_OK)
    fail("thip_qp_update_vec");
  if (info_.status == -1 && info_.setup_error != 1)
    resident_ = false;  // the refactorisation failed
  return info_.status != -1;
}

bool GpuQPSolver::updateLinearConstraintsMatrix(const trajopt_ifopt::Jacobian& linearConstraintsMatrix)
{
  if (linearConstraintsMatrix.rows() != nc_ || linearConstraintsMatrix.cols() != nv_)
    throw std::runtime_error("GpuQPSolver::updateLinearConstraintsMatrix: size mismatch");
  Csc n;
  toCsc(linearConstraintsMatrix, false, 1.0, n.p, n.i, n.x);
  const bool same = n.p == A_.p && n.i == A_.i;
  A_ = std::move(n);
  if (!resident_)
    return true;
  if (!same)
    return reinitKeepingSolution();
  ++n_updates;  // one per convexification applied in place
  if (thip_qp_update_mat(qp_, nullptr, A_.x.data(), &info_) != THIP_OK)
    fail("thip_qp_update_mat");
  if (info_.status == -1)
    resident_ = false;
  return info_.status != -1;
}

// osqp_eigen_solver.cpp:267-324: primal start = [NLP values; slacks], the slack
// of constraint-matrix row k from convex violation k (the reference pairs the
// k-th merit violation with the k-th matrix row), dual start 0
bool GpuQPSolver::setWarmStart(const QPProblem& qp_problem)
{
  if (settings.warm_starting != 1)
    return true;
  const long nn = qp_problem.getNumNLPVars();
  x0_.assign(static_cast<std::size_t>(nv_), 0.0);
  const trajopt_ifopt::VectorXd vars = qp_problem.getVariableValues();
  std::copy(vars.begin(), vars.begin() + nn, x0_.begin());
  if (nv_ > nn)
  {
    const trajopt_ifopt::VectorXd viol = qp_problem.evaluateConvexConstraintViolations(vars);
    const trajopt_ifopt::Jacobian& A = qp_problem.getConstraintMatrix();
    for (long k = 0; k < static_cast<long>(viol.size()) && k < A.rows(); ++k)
      for (long e = A.rowBegin(k); e < A.rowEnd(k); ++e)
        if (A.col(e) >= nn && std::abs(A.value(e)) > 1e-14)
          x0_[static_cast<std::size_t>(A.col(e))] = std::max(0.0, viol[static_cast<std::size_t>(k)] / A.value(e));
  }
  y0_.assign(static_cast<std::size_t>(nc_), 0.0);
  return true;
}

bool GpuQPSolver::solve()
{
  if (!resident_)
  {
    // OsqpEigen initSolver right before the first solve, then the stored warm start
    if (!setupNow())
    {
      status_ = QPSolverStatus::kFailed;
      return false;
    }
    if (settings.warm_starting == 1 && thip_qp_warm_start(qp_, x0_.data(), y0_.data()) != THIP_OK)
      fail("thip_qp_warm_start");
  }
  x_.assign(static_cast<std::size_t>(nv_), 0.0);
  y_.assign(static_cast<std::size_t>(std::max<long>(nc_, 1)), 0.0);
  if (thip_qp_solve_resident(qp_, x_.data(), y_.data(), &info_) != THIP_OK)
    fail("thip_qp_solve_resident");
  y_.resize(static_cast<std::size_t>(nc_));
  ++n_solves;
  admm_iters += info_.iter;
  have_solution_ = true;
  if (info_.status == 1 || info_.status == 2)
    return true;
  if (info_.status == -1)
    resident_ = false;
  status_ = QPSolverStatus::kFailed;
  return false;
}

trajopt_ifopt::VectorXd GpuQPSolver::getSolution() { return x_; }
}  // namespace trajopt_sqp
