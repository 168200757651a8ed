// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of trajopt_sco's modelling layer and SQP driver:
//   Model / OSQPModel                 trajopt_sco/include/trajopt_sco/solver_interface.hpp:54-104,
//                                     trajopt_sco/src/osqp_interface.cpp:92-640
//   exprToEigen / eigenToCSC          trajopt_sco/src/solver_utils.cpp:12-144,
//                                     trajopt_sco/include/trajopt_sco/solver_utils.hpp:104-153
//   ConvexObjective / ConvexConstraints / Cost / Constraint / OptProb
//                                     trajopt_sco/src/modeling.cpp:16-295
//   CostFromFunc / CostFromErrFunc / ConstraintFromErrFunc, affFromValGrad
//                                     trajopt_sco/src/modeling_utils.cpp:31-269
//   numerical differentiation         trajopt_sco/src/num_diff.cpp:41-131
//   BasicTrustRegionSQP               trajopt_sco/src/optimizers.cpp:59-991
#pragma once
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "osqp_restated.hpp"
#include "sco_expr.hpp"

namespace orc
{
enum ConstraintType
{
  EQ,
  INEQ
};
enum CvxOptStatus
{
  CVX_SOLVED,
  CVX_INFEASIBLE,
  CVX_FAILED
};
enum PenaltyType
{
  SQUARED,
  ABS,
  HINGE
};
enum OptStatus
{
  OPT_CONVERGED,
  OPT_SCO_ITERATION_LIMIT,
  OPT_PENALTY_ITERATION_LIMIT,
  OPT_TIME_LIMIT,
  OPT_FAILED,
  INVALID
};

// ------------------------------------------------------------ sparse helpers
struct Triplet
{
  OsqpInt r, c;
  double v;
};
// Eigen::SparseMatrix::setFromTriplets semantics: sorted, duplicates summed,
// summed-to-zero entries kept.
Csc cscFromTriplets(OsqpInt m, OsqpInt n, const std::vector<Triplet>& t);
// exprToEigen(AffExpr, SparseVector) -> dense result of the sparse vector
void exprToDense(const AffExpr& expr, std::vector<double>& v, OsqpInt n_vars);
// exprToEigen(QuadExpr, ...) -> upper-triangular CSC of P, dense q
void quadToCsc(const QuadExpr& expr, Csc& P_upper, std::vector<double>& q, OsqpInt n_vars, bool matrix_is_halved,
               bool force_diagonal = false);
// the full symmetric (sm + sm^T [, * 0.5]) matrix as CSC, for KAT tests
void quadToCscFull(const QuadExpr& expr, Csc& P_full, std::vector<double>& q, OsqpInt n_vars, bool matrix_is_halved,
                   bool force_diagonal = false);
// exprToEigen(AffExprVector, ...)
void affVecToCsc(const AffExprVector& exprs, Csc& A, std::vector<double>& rhs, OsqpInt n_vars);

// ---------------------------------------------------------------- model
class Model
{
public:
  using Ptr = std::shared_ptr<Model>;
  virtual ~Model() = default;
  virtual Var addVar(const std::string& name) = 0;
  virtual Var addVar(const std::string& name, double lb, double ub);
  virtual Cnt addEqCnt(const AffExpr&, const std::string& name) = 0;
  virtual Cnt addIneqCnt(const AffExpr&, const std::string& name) = 0;
  virtual void removeVars(const VarVector& vars) = 0;
  virtual void removeCnts(const CntVector& cnts) = 0;
  virtual void update() = 0;
  virtual void setVarBounds(const Var& var, double lower, double upper);
  virtual void setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper) = 0;
  virtual double getVarValue(const Var& var) const;
  virtual DblVec getVarValues(const VarVector& vars) const = 0;
  virtual CvxOptStatus optimize() = 0;
  virtual void setObjective(const AffExpr&) = 0;
  virtual void setObjective(const QuadExpr&) = 0;
  virtual VarVector getVars() const = 0;
};

class OSQPModel : public Model
{
public:
  explicit OSQPModel(const OsqpSettings& settings);
  ~OSQPModel() override;
  Var addVar(const std::string& name) override;
  using Model::addVar;
  Cnt addEqCnt(const AffExpr&, const std::string& name) override;
  Cnt addIneqCnt(const AffExpr&, const std::string& name) override;
  void removeVars(const VarVector& vars) override;
  void removeCnts(const CntVector& cnts) override;
  void update() override;
  using Model::setVarBounds;
  void setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper) override;
  DblVec getVarValues(const VarVector& vars) const override;
  CvxOptStatus optimize() override;
  void setObjective(const AffExpr&) override;
  void setObjective(const QuadExpr&) override;
  VarVector getVars() const override { return vars_; }

  // counters the build adds (not in the reference)
  struct Trace
  {
    double warm, rho0, iters, status, polish, rho1, prim, dual, xsum, trust;
    double tie_cleanup;  // smallest | |J| - 1e-7 | of the linearisation this QP solves (cleanupAff)
    double tie_polish;   // smallest margin of polish's active-set comparisons (1e300 if no polish)
  };
  std::vector<Trace>* trace = nullptr;
  double trace_trust = 0;
  double trace_tie_cleanup = 1e300;
  long long admm_iters_total = 0;
  int last_osqp_status = 0;
  int last_polish_status = 0;
  bool last_warm_started = false;

  OsqpSettings settings_;
  bool update_workspace = false;

private:
  bool updateObjective(bool check_sparsity);
  bool updateConstraints(bool check_sparsity);
  void createOrUpdateSolver();

  std::mutex mutex_;
  VarVector vars_;
  DblVec lbs_, ubs_;
  CntVector cnts_;
  AffExprVector cnt_exprs_;
  std::vector<ConstraintType> cnt_types_;
  QuadExpr objective_;
  DblVec solution_;

  OsqpInt n_ = 0, m_ = 0;
  Csc P_, A_;
  bool has_P_ = false, has_A_ = false;
  DblVec q_, l_, u_;
  std::unique_ptr<OsqpSolver> ws_;
};

// ---------------------------------------------------------------- modelling
class ConvexObjective
{
public:
  using Ptr = std::shared_ptr<ConvexObjective>;
  explicit ConvexObjective(Model* model) : model_(model) {}
  ~ConvexObjective();
  ConvexObjective(const ConvexObjective&) = delete;
  ConvexObjective& operator=(const ConvexObjective&) = delete;
  void addAffExpr(const AffExpr&);
  void addQuadExpr(const QuadExpr&);
  void addHinge(const AffExpr&, double coeff);
  void addAbs(const AffExpr&, double coeff);
  void addHinges(const AffExprVector&);
  void addL1Norm(const AffExprVector&);
  void addL2Norm(const AffExprVector&);
  void addMax(const AffExprVector&);
  bool inModel() const { return model_ != nullptr; }
  void addConstraintsToModel();
  void removeFromModel();
  double value(const DblVec& x) const;

  Model* model_;
  QuadExpr quad_;
  VarVector vars_;
  AffExprVector eqs_;
  AffExprVector ineqs_;
  CntVector cnts_;
};

class ConvexConstraints
{
public:
  using Ptr = std::shared_ptr<ConvexConstraints>;
  explicit ConvexConstraints(Model* model) : model_(model) {}
  ~ConvexConstraints();
  ConvexConstraints(const ConvexConstraints&) = delete;
  ConvexConstraints& operator=(const ConvexConstraints&) = delete;
  void addEqCnt(const AffExpr&);
  void addIneqCnt(const AffExpr&);
  void setModel(Model* model) { model_ = model; }
  DblVec violations(const DblVec& x);
  double violation(const DblVec& x);
  bool inModel() const { return model_ != nullptr; }
  void addConstraintsToModel();
  void removeFromModel();

  AffExprVector eqs_;
  AffExprVector ineqs_;

private:
  Model* model_;
  CntVector cnts_;
};

class Cost
{
public:
  using Ptr = std::shared_ptr<Cost>;
  explicit Cost(std::string name = "unnamed") : name_(std::move(name)) {}
  virtual ~Cost() = default;
  virtual double value(const DblVec&) = 0;
  virtual ConvexObjective::Ptr convex(const DblVec& x, Model* model) = 0;
  virtual VarVector getVars() = 0;
  const std::string& name() const { return name_; }
  void setName(const std::string& n) { name_ = n; }

protected:
  std::string name_;
};

class Constraint
{
public:
  using Ptr = std::shared_ptr<Constraint>;
  explicit Constraint(std::string name = "unnamed") : name_(std::move(name)) {}
  virtual ~Constraint() = default;
  virtual ConstraintType type() = 0;
  virtual DblVec value(const DblVec& x) = 0;
  virtual ConvexConstraints::Ptr convex(const DblVec& x, Model* model) = 0;
  DblVec violations(const DblVec& x);
  double violation(const DblVec& x);
  virtual VarVector getVars() = 0;
  const std::string& name() const { return name_; }
  void setName(const std::string& n) { name_ = n; }

protected:
  std::string name_;
};

class OptProb
{
public:
  using Ptr = std::shared_ptr<OptProb>;
  explicit OptProb(const OsqpSettings& s);
  virtual ~OptProb() = default;
  VarVector createVariables(const std::vector<std::string>& names);
  VarVector createVariables(const std::vector<std::string>& names, const DblVec& lb, const DblVec& ub);
  void setLowerBounds(const DblVec& lb) { lower_bounds_ = lb; }
  void setUpperBounds(const DblVec& ub) { upper_bounds_ = ub; }
  void addCost(Cost::Ptr c) { costs_.push_back(std::move(c)); }
  void addConstraint(Constraint::Ptr c);
  void addLinearConstraint(const AffExpr&, ConstraintType type);
  std::vector<Constraint::Ptr> getConstraints() const;
  std::vector<Cost::Ptr>& getCosts() { return costs_; }
  DblVec getClosestFeasiblePoint(const DblVec& x, const double& delta = 1e-3);
  const VarVector& getVars() const { return vars_; }
  Model::Ptr getModel() { return model_; }
  const DblVec& getLowerBounds() const { return lower_bounds_; }
  const DblVec& getUpperBounds() const { return upper_bounds_; }
  std::size_t getNumVars() const { return vars_.size(); }

protected:
  Model::Ptr model_;
  VarVector vars_;
  DblVec lower_bounds_, upper_bounds_;
  std::vector<Cost::Ptr> costs_;
  std::vector<Constraint::Ptr> eqcnts_, ineqcnts_;
};

// ---- num_diff / modeling_utils
using ScalarOfVector = std::function<double(const DblVec&)>;
using VectorOfVector = std::function<DblVec(const DblVec&)>;
// column-major Jacobian: jac[i * cols... ] -> stored as rows x cols row-major
struct Mat
{
  int rows = 0, cols = 0;
  DblVec a;
  Mat() = default;
  Mat(int r, int c) : rows(r), cols(c), a(static_cast<std::size_t>(r * c), 0.0) {}
  double& operator()(int r, int c) { return a[static_cast<std::size_t>(r * cols + c)]; }
  double operator()(int r, int c) const { return a[static_cast<std::size_t>(r * cols + c)]; }
};
using MatrixOfVector = std::function<Mat(const DblVec&)>;

Mat calcForwardNumJac(const VectorOfVector& f, const DblVec& x, double epsilon);
DblVec calcForwardNumGrad(const ScalarOfVector& f, const DblVec& x, double epsilon);
void calcGradAndDiagHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad,
                         DblVec& hess);
void calcGradHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad, Mat& hess);
AffExpr affFromValGrad(double y, const DblVec& x, const DblVec& dydx, const VarVector& vars);
DblVec getDblVec(const DblVec& x, const VarVector& vars);

class CostFromFunc : public Cost
{
public:
  CostFromFunc(ScalarOfVector f, VarVector vars, const std::string& name, bool full_hessian = false);
  double value(const DblVec& x) override;
  ConvexObjective::Ptr convex(const DblVec& x, Model* model) override;
  VarVector getVars() override { return vars_; }

private:
  ScalarOfVector f_;
  VarVector vars_;
  bool full_hessian_;
  double epsilon_;
};

class CostFromErrFunc : public Cost
{
public:
  CostFromErrFunc(VectorOfVector f, MatrixOfVector dfdx, VarVector vars, DblVec coeffs, PenaltyType pen_type,
                  const std::string& name);
  double value(const DblVec& x) override;
  ConvexObjective::Ptr convex(const DblVec& x, Model* model) override;
  VarVector getVars() override { return vars_; }

private:
  VectorOfVector f_;
  MatrixOfVector dfdx_;
  VarVector vars_;
  DblVec coeffs_;
  PenaltyType pen_type_;
  double epsilon_;
};

class ConstraintFromErrFunc : public Constraint
{
public:
  ConstraintFromErrFunc(VectorOfVector f, MatrixOfVector dfdx, VarVector vars, DblVec coeffs, ConstraintType type,
                        const std::string& name);
  DblVec value(const DblVec& x) override;
  ConvexConstraints::Ptr convex(const DblVec& x, Model* model) override;
  ConstraintType type() override { return type_; }
  VarVector getVars() override { return vars_; }

private:
  VectorOfVector f_;
  MatrixOfVector dfdx_;
  VarVector vars_;
  DblVec coeffs_;
  ConstraintType type_;
  double epsilon_;
};

// ---------------------------------------------------------------- optimizer
struct OptResults
{
  DblVec x;
  OptStatus status = INVALID;
  double total_cost = 0;
  DblVec cost_vals;
  DblVec cnt_viols;
  int n_func_evals = 0, n_qp_solves = 0;
  // build counters
  int n_sqp_iters = 0;
  int n_merit_increases = 0;
  long long n_admm_iters = 0;
  void clear()
  {
    x.clear();
    status = INVALID;
    total_cost = 0;
    cost_vals.clear();
    cnt_viols.clear();
    n_func_evals = n_qp_solves = n_sqp_iters = n_merit_increases = 0;
    n_admm_iters = 0;
  }
};

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
  double initial_merit_error_coeff = 10;
  bool inflate_constraints_individually = true;
  double trust_box_size = 1e-1;
  double max_time = 1.7976931348623157e308;  // optimizers.hpp:117
};

class BasicTrustRegionSQP
{
public:
  explicit BasicTrustRegionSQP(OptProb::Ptr prob) : prob_(std::move(prob)), model_(prob_->getModel()) {}
  void initialize(const DblVec& x)
  {
    results_.clear();
    results_.x = x;
  }
  OptStatus optimize();
  BasicTrustRegionSQPParameters& getParameters() { return param_; }
  OptResults& results() { return results_; }
  DblVec& x() { return results_.x; }

private:
  void setTrustBoxConstraints(const DblVec& x);
  OptProb::Ptr prob_;
  Model::Ptr model_;
  BasicTrustRegionSQPParameters param_;
  OptResults results_;
};

}  // namespace orc
