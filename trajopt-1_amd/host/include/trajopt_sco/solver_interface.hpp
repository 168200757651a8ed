// The trajopt_sco::Model plugin surface (trajopt_sco/include/trajopt_sco/
// solver_interface.hpp:54-260): variables, constraints, affine and quadratic
// expressions, the convex-solver interface and its factory -- same names,
// signatures and semantics, restated for the MI355X build.  createModel()
// returns a GpuModel (gpu_model.hpp): OSQP 1.0 on the GPU through the C-ABI of
// include/trajopt_hip.h (thip_qp_*), standing in for the reference's OSQPModel.
// Errors are std::runtime_error; Model::optimize() reports by status code.
#pragma once
#include <cstdint>
#include <iosfwd>
#include <memory>
#include <string>
#include <vector>

#include "trajopt_sco/sco_common.hpp"

namespace sco
{
enum ConstraintType : std::uint8_t
{
  EQ,
  INEQ
};
using ConstraintTypeVector = std::vector<ConstraintType>;

enum CvxOptStatus : std::uint8_t
{
  CVX_SOLVED,
  CVX_INFEASIBLE,
  CVX_FAILED
};

struct VarRep
{
  using Ptr = std::shared_ptr<VarRep>;
  VarRep(std::size_t _index, std::string _name, void* _creator)
    : index(_index), name(std::move(_name)), creator(_creator)
  {
  }
  std::size_t index;
  std::string name;
  bool removed{ false };
  void* creator;
};

struct Var
{
  using Ptr = std::shared_ptr<Var>;
  VarRep::Ptr var_rep{ nullptr };
  Var() = default;
  Var(VarRep::Ptr rep) : var_rep(std::move(rep)) {}
  double value(const double* x) const { return x[var_rep->index]; }
  double value(const DblVec& x) const { return x[var_rep->index]; }
};

struct CntRep
{
  using Ptr = std::shared_ptr<CntRep>;
  CntRep(std::size_t _index, void* _creator) : index(_index), creator(_creator) {}
  std::size_t index;
  bool removed{ false };
  void* creator;
  ConstraintType type{ ConstraintType::EQ };
  std::string expr;
};

struct Cnt
{
  using Ptr = std::shared_ptr<Cnt>;
  CntRep::Ptr cnt_rep{ nullptr };
  Cnt() = default;
  Cnt(CntRep::Ptr rep) : cnt_rep(std::move(rep)) {}
};

using VarVector = std::vector<Var>;
using CntVector = std::vector<Cnt>;

struct AffExpr
{
  using Ptr = std::shared_ptr<AffExpr>;
  double constant{ 0 };
  DblVec coeffs;
  VarVector vars;
  AffExpr() = default;
  explicit AffExpr(double a);
  explicit AffExpr(const Var& v);
  std::size_t size() const;
  double value(const double* x) const;
  double value(const DblVec& x) const;
};

struct QuadExpr
{
  using Ptr = std::shared_ptr<QuadExpr>;
  AffExpr affexpr;
  DblVec coeffs;
  VarVector vars1;
  VarVector vars2;
  QuadExpr() = default;
  explicit QuadExpr(double a);
  explicit QuadExpr(const Var& v);
  explicit QuadExpr(AffExpr aff);
  std::size_t size() const;
  double value(const double* x) const;
  double value(const DblVec& x) const;
};

using AffExprVector = std::vector<AffExpr>;
using QuadExprVector = std::vector<QuadExpr>;

// solver_interface.hpp:54-104
class Model
{
public:
  using Ptr = std::shared_ptr<Model>;
  using ConstPtr = std::shared_ptr<const Model>;
  Model() = default;
  virtual ~Model() = default;
  Model(const Model&) = default;
  Model& operator=(const Model&) = default;

  // add / remove: threadsafe (the reference's convexify may run them concurrently)
  virtual Var addVar(const std::string& name) = 0;
  virtual Var addVar(const std::string& name, double lb, double ub);
  virtual Cnt addEqCnt(const AffExpr&, const std::string& name) = 0;     // expr == 0
  virtual Cnt addIneqCnt(const AffExpr&, const std::string& name) = 0;   // expr <= 0
  virtual Cnt addIneqCnt(const QuadExpr&, const std::string& name) = 0;  // expr <= 0
  virtual void removeVar(const Var& var);
  virtual void removeCnt(const Cnt& cnt);
  virtual void removeVars(const VarVector& vars) = 0;
  virtual void removeCnts(const CntVector& cnts) = 0;

  virtual void update() = 0;  // call after adding / deleting
  virtual void setVarBounds(const Var& var, double lower, double upper);
  virtual void setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper) = 0;
  virtual double getVarValue(const Var& var) const;
  virtual DblVec getVarValues(const VarVector& vars) const = 0;
  virtual CvxOptStatus optimize() = 0;

  virtual void setObjective(const AffExpr&) = 0;
  virtual void setObjective(const QuadExpr&) = 0;
  virtual void writeToFile(const std::string& fname) const = 0;

  virtual VarVector getVars() const = 0;
};

struct ModelConfig
{
  using Ptr = std::shared_ptr<ModelConfig>;
  using ConstPtr = std::shared_ptr<const ModelConfig>;
  virtual ~ModelConfig() = default;
};

// solver_interface.hpp:226-256.  MODEL_NAMES_ keeps the reference's order
// {GUROBI, BPMPD, OSQP, QPOASES} (quirk Q1: it differs from the enum order, so
// the string constructor maps "OSQP" to QPOASES exactly as the reference does)
class ModelType
{
public:
  enum Value : std::uint8_t
  {
    GUROBI,
    OSQP,
    QPOASES,
    BPMPD,
    AUTO_SOLVER
  };
  static const std::vector<std::string> MODEL_NAMES_;
  ModelType();
  ModelType(const ModelType::Value& v);
  ModelType(const int& v);
  ModelType(const std::string& s);
  operator int() const;
  bool operator==(const ModelType::Value& a) const;
  bool operator==(const ModelType& a) const;
  bool operator!=(const ModelType& a) const;
  friend std::ostream& operator<<(std::ostream& os, const ModelType& cs);

private:
  Value value_{ Value::AUTO_SOLVER };
};

// The backends of this build: OSQP (OSQP 1.0 on the GPU, GpuModel).  Gurobi,
// BPMPD and qpOASES are out of scope.
std::vector<ModelType> availableSolvers();
std::ostream& operator<<(std::ostream& os, const ModelType& cs);

// AUTO_SOLVER resolves through $TRAJOPT_CONVEX_SOLVER, else the first available
// solver (solver_interface.cpp:289-365); OSQP -> GpuModel; others throw.
Model::Ptr createModel(ModelType model_type = ModelType::AUTO_SOLVER,
                       const ModelConfig::ConstPtr& model_config = nullptr);

void vars2inds(const VarVector& vars, SizeTVec& inds);
void vars2inds(const VarVector& vars, IntVec& inds);
void cnts2inds(const CntVector& cnts, SizeTVec& inds);
void cnts2inds(const CntVector& cnts, IntVec& inds);

std::ostream& operator<<(std::ostream&, const Var&);
std::ostream& operator<<(std::ostream&, const Cnt&);
std::ostream& operator<<(std::ostream&, const AffExpr&);
std::ostream& operator<<(std::ostream&, const QuadExpr&);
}  // namespace sco
