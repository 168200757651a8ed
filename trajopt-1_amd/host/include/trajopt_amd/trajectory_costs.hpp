// Joint-space trajectory terms as sco::Cost / sco::Constraint objects
// (trajopt/include/trajopt/trajectory_costs.hpp, trajopt/src/trajectory_costs.cpp):
// position (order 0), velocity (1), acceleration (2) and jerk (3) of the
// waypoint sequence, each as Eq cost (quadratic), Ineq cost (hinges outside a
// tolerance band), Eq constraint and Ineq constraint.  The d-th forward
// difference at step i is the stencil over x_i .. x_{i+d} ([1], [-1 1],
// [1 -2 1], [-1 3 -3 1]) minus the target.  The hatch() of JointPos / JointVel
// terms lowers them into the batched kernel as well (they then run on the GPU
// inside sqp_kernel); JointAcc / JointJerk and JointVel equality constraints run
// only through these objects (sco::BasicTrustRegionSQP's host loop, every QP on
// the GPU through the GpuModel).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_sco/modeling.hpp"
#include "trajopt_sco/modeling_utils.hpp"

namespace trajopt
{
using sco::DblVec;

// rows x cols of sco::Var, row-major (trajopt_common/basic_array.hpp VarArray)
struct VarArray
{
  int n_rows = 0, n_cols = 0;
  std::vector<sco::Var> data;
  int rows() const { return n_rows; }
  int cols() const { return n_cols; }
  sco::Var& operator()(int i, int j) { return data[static_cast<std::size_t>(i) * n_cols + j]; }
  const sco::Var& operator()(int i, int j) const { return data[static_cast<std::size_t>(i) * n_cols + j]; }
  sco::Var& at(int i, int j) { return (*this)(i, j); }
  sco::VarVector row(int i) const { return rblock(i, 0, n_cols); }
  sco::VarVector rblock(int i, int start, int n) const
  {
    return sco::VarVector(data.begin() + static_cast<long>(i) * n_cols + start,
                          data.begin() + static_cast<long>(i) * n_cols + start + n);
  }
  sco::VarVector flatten() const { return data; }
};

// One joint-difference term of order 0..3 over steps [first, last].
struct JointDiffSpec
{
  VarArray vars;
  DblVec coeffs, targets, upper_tols, lower_tols;
  int order = 1, first_step = 0, last_step = 0;
};

class JointDiffEqCost : public sco::Cost
{
public:
  JointDiffEqCost(JointDiffSpec s, const std::string& name);
  double value(const DblVec& x) override;
  sco::ConvexObjective::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return s_.vars.flatten(); }

private:
  JointDiffSpec s_;
  sco::QuadExpr expr_;
};

class JointDiffIneqCost : public sco::Cost
{
public:
  JointDiffIneqCost(JointDiffSpec s, const std::string& name);
  double value(const DblVec& x) override;
  sco::ConvexObjective::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return s_.vars.flatten(); }
  const sco::AffExprVector& exprs() const { return exprs_; }
  DblVec blockValues(const DblVec& x) const;  // [upper block | lower block] column-major, not clamped

private:
  JointDiffSpec s_;
  sco::AffExprVector exprs_;
};

class JointDiffEqConstraint : public sco::EqConstraint
{
public:
  JointDiffEqConstraint(JointDiffSpec s, const std::string& name);
  DblVec value(const DblVec& x) override;  // coeff * diff^2 (the reference's value, quirk Q3)
  sco::ConvexConstraints::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return s_.vars.flatten(); }

private:
  JointDiffSpec s_;
  sco::AffExprVector exprs_;
};

class JointDiffIneqConstraint : public sco::IneqConstraint
{
public:
  JointDiffIneqConstraint(JointDiffSpec s, const std::string& name);
  DblVec value(const DblVec& x) override;
  sco::ConvexConstraints::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return rows_.getVars(); }

private:
  JointDiffIneqCost rows_;
  bool clamp_;  // JointPosIneqConstraint returns the raw block, the others pospart
};

// JointVelErrCalculator / JointVelJacCalculator (kinematic_terms.cpp:434-475):
// over v = (x_first..x_last, dt_first..dt_last), vel_i = (x_{i+1} - x_i) dt_{i+1},
// error [-(upper - (vel - target)); lower - (vel - target)] and its jacobian
sco::VectorOfVector::Ptr jointVelTimeErr(double target, double upper_tol, double lower_tol);
sco::MatrixOfVector::Ptr jointVelTimeJac();
// TimeCostCalculator / TimeCostJacCalculator (kinematic_terms.cpp:579-591):
// sum(1/v) - limit and its row -1/v^2
sco::VectorOfVector::Ptr totalTimeErr(double limit);
sco::MatrixOfVector::Ptr totalTimeJac();

}  // namespace trajopt
