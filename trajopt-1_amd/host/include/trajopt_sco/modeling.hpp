// Convex modelling and the non-convex problem (trajopt_sco/include/trajopt_sco/
// modeling.hpp:27-267): ConvexObjective / ConvexConstraints (the aux variables
// and rows a convexified term adds to the Model, removed again when the object
// is destroyed), Cost / Constraint (the plugin types TermInfo::hatch pushes),
// OptProb (variables, bounds, costs, constraints, the Model).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_sco/optimizers_fwd.hpp"
#include "trajopt_sco/solver_interface.hpp"

namespace sco
{
class ConvexObjective
{
public:
  using Ptr = std::shared_ptr<ConvexObjective>;
  explicit ConvexObjective(Model* model) : model_(model) {}
  virtual ~ConvexObjective();
  ConvexObjective(const ConvexObjective&) = delete;
  ConvexObjective& operator=(const ConvexObjective&) = delete;

  void addAffExpr(const AffExpr&);
  void addQuadExpr(const QuadExpr&);
  void addHinge(const AffExpr&, double coeff);  // aux h >= 0, row aff - h <= 0, objective coeff h
  void addAbs(const AffExpr&, double coeff);    // aux n, p >= 0, row aff + n - p = 0, objective coeff (n + p)
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
  virtual ~ConvexConstraints();
  ConvexConstraints(const ConvexConstraints&) = delete;
  ConvexConstraints& operator=(const ConvexConstraints&) = delete;

  void addEqCnt(const AffExpr&);    // == 0
  void addIneqCnt(const AffExpr&);  // <= 0
  void setModel(Model* model) { model_ = model; }
  bool inModel() { return model_ != nullptr; }
  void addConstraintsToModel();
  void removeFromModel();
  DblVec violations(const DblVec& x);
  double violation(const DblVec& x);

  AffExprVector eqs_;
  AffExprVector ineqs_;

private:
  Model* model_{ nullptr };
  CntVector cnts_;
};

class Cost
{
public:
  using Ptr = std::shared_ptr<Cost>;
  virtual double value(const DblVec&) = 0;
  virtual ConvexObjective::Ptr convex(const DblVec& x, Model* model) = 0;
  virtual VarVector getVars() = 0;
  std::string name() { return name_; }
  void setName(const std::string& name) { name_ = name; }
  Cost() = default;
  explicit Cost(std::string name) : name_(std::move(name)) {}
  virtual ~Cost() = default;

protected:
  std::string name_{ "unnamed" };
};

class Constraint
{
public:
  using Ptr = std::shared_ptr<Constraint>;
  virtual ConstraintType type() = 0;
  virtual DblVec value(const DblVec& x) = 0;
  virtual ConvexConstraints::Ptr convex(const DblVec& x, Model* model) = 0;
  // |value| for equality constraints, pospart(value) for inequality constraints
  DblVec violations(const DblVec& x);
  double violation(const DblVec& x);
  virtual VarVector getVars() = 0;
  std::string name() { return name_; }
  void setName(const std::string& name) { name_ = name; }
  Constraint() = default;
  explicit Constraint(std::string name) : name_(std::move(name)) {}
  virtual ~Constraint() = default;

protected:
  std::string name_{ "unnamed" };
};

class EqConstraint : public Constraint
{
public:
  using Ptr = std::shared_ptr<EqConstraint>;
  ConstraintType type() override { return EQ; }
  EqConstraint() = default;
  explicit EqConstraint(std::string name) : Constraint(std::move(name)) {}
};

class IneqConstraint : public Constraint
{
public:
  using Ptr = std::shared_ptr<IneqConstraint>;
  ConstraintType type() override { return INEQ; }
  IneqConstraint() = default;
  explicit IneqConstraint(std::string name) : Constraint(std::move(name)) {}
};

// modeling.hpp:194-267
class OptProb
{
public:
  using Ptr = std::shared_ptr<OptProb>;
  explicit OptProb(ModelType convex_solver = ModelType::AUTO_SOLVER,
                   const ModelConfig::ConstPtr& convex_solver_config = nullptr);
  virtual ~OptProb() = default;
  OptProb(const OptProb&) = delete;
  OptProb& operator=(const OptProb&) = delete;

  VarVector createVariables(const std::vector<std::string>& names);
  VarVector createVariables(const std::vector<std::string>& names, const DblVec& lb, const DblVec& ub);
  void setLowerBounds(const DblVec& lb);
  void setUpperBounds(const DblVec& ub);
  void setLowerBounds(const DblVec& lb, const VarVector& vars);
  void setUpperBounds(const DblVec& ub, const VarVector& vars);
  // persistent model-level constraint (added to the Model directly)
  void addLinearConstraint(const AffExpr&, ConstraintType type);
  void addCost(Cost::Ptr);
  void addConstraint(Constraint::Ptr);
  void addEqConstraint(Constraint::Ptr);
  void addIneqConstraint(Constraint::Ptr);
  // modeling.cpp:261-273: x pushed >= delta inside the bounds (the midpoint of narrower bounds)
  DblVec getClosestFeasiblePoint(const DblVec& x, const double& delta = 1e-3);

  std::vector<Constraint::Ptr> getConstraints() const;  // equality constraints first
  const std::vector<Cost::Ptr>& getCosts() { return costs_; }
  const std::vector<Constraint::Ptr>& getIneqConstraints() { return ineqcnts_; }
  const std::vector<Constraint::Ptr>& getEqConstraints() { return eqcnts_; }
  const DblVec& getLowerBounds() { return lower_bounds_; }
  const DblVec& getUpperBounds() { return upper_bounds_; }
  Model::Ptr getModel() { return model_; }
  const VarVector& getVars() { return vars_; }
  int getNumCosts() { return static_cast<int>(costs_.size()); }
  int getNumConstraints() { return static_cast<int>(eqcnts_.size() + ineqcnts_.size()); }
  int getNumVars() { return static_cast<int>(vars_.size()); }

  // MI355X build: a problem that knows a native batched path (TrajOptProb: the
  // fused sqp_kernel when every term lowered) solves itself there and returns
  // true; BasicTrustRegionSQP::optimize otherwise runs the reference's loop
  // over getCosts() / getConstraints() with the GpuModel.
  virtual bool solveNative(const BasicTrustRegionSQPParameters& param, const DblVec& x0, OptResults& results);
  // MI355X build: called by BasicTrustRegionSQP before it evaluates or
  // convexifies the costs and constraints at x, so that a problem whose terms
  // run on the device can evaluate them all in one launch (TrajOptProb: every
  // CartPose term at once) instead of one launch per term.  No effect on values.
  virtual void prefetch(const DblVec& /*x*/) {}

protected:
  Model::Ptr model_;
  VarVector vars_;
  DblVec lower_bounds_;
  DblVec upper_bounds_;
  std::vector<Cost::Ptr> costs_;
  std::vector<Constraint::Ptr> eqcnts_;
  std::vector<Constraint::Ptr> ineqcnts_;
};

template <typename VecType>
inline void setVec(DblVec& x, const VarVector& vars, const VecType& vals)
{
  for (std::size_t i = 0; i < vars.size(); ++i)
    x[vars[i].var_rep->index] = vals[i];
}
inline DblVec getDblVec(const DblVec& x, const VarVector& vars)
{
  DblVec out(vars.size());
  for (std::size_t i = 0; i < vars.size(); ++i)
    out[i] = x[vars[i].var_rep->index];
  return out;
}
}  // namespace sco
