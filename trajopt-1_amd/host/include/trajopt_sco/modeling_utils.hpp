// Costs and constraints from user functions (trajopt_sco/include/trajopt_sco/
// modeling_utils.hpp, num_diff.hpp), restated without Eigen: vectors are
// sco::DblVec and a Jacobian is a row-major sco::Mat.  A user TermInfo::hatch
// builds these (or its own Cost / Constraint) and calls prob.addCost(...); the
// problem then runs the host SQP loop with the GpuModel (optimizers.hpp).
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "trajopt_sco/modeling.hpp"

namespace sco
{
constexpr double DEFAULT_EPSILON = 1e-5;  // kinematic_terms.hpp:15 / modeling_utils.cpp

struct Mat  // row-major rows x cols
{
  int rows = 0, cols = 0;
  DblVec data;
  Mat() = default;
  Mat(int r, int c) : rows(r), cols(c), data(static_cast<std::size_t>(r) * c, 0.0) {}
  double& operator()(int i, int j) { return data[static_cast<std::size_t>(i) * cols + j]; }
  double operator()(int i, int j) const { return data[static_cast<std::size_t>(i) * cols + j]; }
  DblVec row(int i) const { return DblVec(data.begin() + static_cast<long>(i) * cols, data.begin() + static_cast<long>(i + 1) * cols); }
};

class ScalarOfVector
{
public:
  using Ptr = std::shared_ptr<ScalarOfVector>;
  virtual ~ScalarOfVector() = default;
  virtual double operator()(const DblVec& x) const = 0;
  double call(const DblVec& x) const { return operator()(x); }
  using func = std::function<double(const DblVec&)>;
  static ScalarOfVector::Ptr construct(func f);
};

class VectorOfVector
{
public:
  using Ptr = std::shared_ptr<VectorOfVector>;
  virtual ~VectorOfVector() = default;
  virtual DblVec operator()(const DblVec& x) const = 0;
  DblVec call(const DblVec& x) const { return operator()(x); }
  using func = std::function<DblVec(const DblVec&)>;
  static VectorOfVector::Ptr construct(func f);
};

class MatrixOfVector
{
public:
  using Ptr = std::shared_ptr<MatrixOfVector>;
  virtual ~MatrixOfVector() = default;
  virtual Mat operator()(const DblVec& x) const = 0;
  Mat call(const DblVec& x) const { return operator()(x); }
  using func = std::function<Mat(const DblVec&)>;
  static MatrixOfVector::Ptr construct(func f);
};

// num_diff.cpp: forward differences (f(x + eps e_i) - f(x)) / eps
Mat calcForwardNumJac(const VectorOfVector& f, const DblVec& x, double epsilon);
DblVec calcForwardNumGrad(const ScalarOfVector& f, const DblVec& x, double epsilon);
// num_diff.cpp:70-105: central gradient + diagonal Hessian; forward gradient + symmetrised
// forward Jacobian of it
void calcGradAndDiagHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad,
                         DblVec& hess);
void calcGradHess(const ScalarOfVector& f, const DblVec& x, double epsilon, double& y, DblVec& grad, Mat& hess);

enum PenaltyType : std::uint8_t
{
  SQUARED,
  ABS,
  HINGE
};

// modeling_utils.cpp:31-39: constant = y - dydx . x, cleanupAff
AffExpr affFromValGrad(double y, const DblVec& x, const DblVec& dydx, const VarVector& vars);

// modeling_utils.cpp:41-117: a scalar cost, convexified by its numerical
// gradient and the positive part of its (diagonal or full) numerical Hessian
class CostFromFunc : public Cost
{
public:
  CostFromFunc(ScalarOfVector::Ptr f, VarVector vars, const std::string& name, bool full_hessian = false);
  double value(const DblVec& x) override;
  ConvexObjective::Ptr convex(const DblVec& x, Model* model) override;
  VarVector getVars() override { return vars_; }

protected:
  ScalarOfVector::Ptr f_;
  VarVector vars_;
  bool full_hessian_;
  double epsilon_{ DEFAULT_EPSILON };
};

class CostFromErrFunc : public Cost
{
public:
  CostFromErrFunc(VectorOfVector::Ptr f, VarVector vars, DblVec coeffs, PenaltyType pen_type, const std::string& name);
  CostFromErrFunc(VectorOfVector::Ptr f, MatrixOfVector::Ptr dfdx, VarVector vars, DblVec coeffs,
                  PenaltyType pen_type, const std::string& name);
  double value(const DblVec& x) override;
  ConvexObjective::Ptr convex(const DblVec& x, Model* model) override;
  VarVector getVars() override { return vars_; }

protected:
  VectorOfVector::Ptr f_;
  MatrixOfVector::Ptr dfdx_;
  VarVector vars_;
  DblVec coeffs_;
  PenaltyType pen_type_;
  double epsilon_{ DEFAULT_EPSILON };
};

class ConstraintFromErrFunc : public Constraint
{
public:
  ConstraintFromErrFunc(VectorOfVector::Ptr f, VarVector vars, DblVec coeffs, ConstraintType type,
                        const std::string& name);
  ConstraintFromErrFunc(VectorOfVector::Ptr f, MatrixOfVector::Ptr dfdx, VarVector vars, DblVec coeffs,
                        ConstraintType type, const std::string& name);
  DblVec value(const DblVec& x) override;
  ConvexConstraints::Ptr convex(const DblVec& x, Model* model) override;
  ConstraintType type() override { return type_; }
  VarVector getVars() override { return vars_; }

protected:
  VectorOfVector::Ptr f_;
  MatrixOfVector::Ptr dfdx_;
  VarVector vars_;
  DblVec coeffs_;
  ConstraintType type_;
  double epsilon_{ DEFAULT_EPSILON };
};
}  // namespace sco
