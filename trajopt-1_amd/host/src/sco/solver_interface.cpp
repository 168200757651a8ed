// trajopt_sco::Model surface: expressions, ModelType, createModel
// (restating trajopt_sco/src/solver_interface.cpp:14-365 and expr_ops.cpp:10-99).
#include "trajopt_sco/solver_interface.hpp"

#include <algorithm>
#include <cstdlib>
#include <ostream>
#include <sstream>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"
#include "trajopt_sco/gpu_model.hpp"

namespace sco
{
// ------------------------------------------------------------------ expressions
AffExpr::AffExpr(double a) : constant(a) {}
AffExpr::AffExpr(const Var& v) : coeffs(1, 1.0), vars(1, v) {}
std::size_t AffExpr::size() const { return coeffs.size(); }
double AffExpr::value(const double* x) const
{
  double acc = constant;
  for (std::size_t k = 0; k < coeffs.size(); ++k)
    acc += coeffs[k] * vars[k].value(x);
  return acc;
}
double AffExpr::value(const DblVec& x) const { return value(x.data()); }

QuadExpr::QuadExpr(double a) : affexpr(a) {}
QuadExpr::QuadExpr(const Var& v) : affexpr(v) {}
QuadExpr::QuadExpr(AffExpr aff) : affexpr(std::move(aff)) {}
std::size_t QuadExpr::size() const { return coeffs.size(); }
double QuadExpr::value(const double* x) const
{
  double acc = affexpr.value(x);
  for (std::size_t k = 0; k < coeffs.size(); ++k)
    acc += coeffs[k] * vars1[k].value(x) * vars2[k].value(x);
  return acc;
}
double QuadExpr::value(const DblVec& x) const { return value(x.data()); }

QuadExpr exprMult(const AffExpr& a, const AffExpr& b)
{
  // (ca + sum ai xi)(cb + sum bj xj): constant, the cross terms with the other
  // constant (a's variables first), then every pair ai bj xi xj in a-major order
  QuadExpr out;
  out.affexpr.constant = a.constant * b.constant;
  out.affexpr.vars = a.vars;
  out.affexpr.vars.insert(out.affexpr.vars.end(), b.vars.begin(), b.vars.end());
  out.affexpr.coeffs.reserve(a.size() + b.size());
  for (double ai : a.coeffs)
    out.affexpr.coeffs.push_back(b.constant * ai);
  for (double bj : b.coeffs)
    out.affexpr.coeffs.push_back(a.constant * bj);
  for (std::size_t i = 0; i < a.size(); ++i)
    for (std::size_t j = 0; j < b.size(); ++j)
    {
      out.vars1.push_back(a.vars[i]);
      out.vars2.push_back(b.vars[j]);
      out.coeffs.push_back(a.coeffs[i] * b.coeffs[j]);
    }
  return out;
}

QuadExpr exprSquare(const Var& a)
{
  QuadExpr out;
  out.coeffs.assign(1, 1.0);
  out.vars1.assign(1, a);
  out.vars2.assign(1, a);
  return out;
}

QuadExpr exprSquare(const AffExpr& a)
{
  // (c + sum ai xi)^2 = c^2 + sum 2 c ai xi + sum ai^2 xi^2 + sum_{i<j} 2 ai aj xi xj
  QuadExpr out;
  out.affexpr.constant = sq(a.constant);
  out.affexpr.vars = a.vars;
  for (double ai : a.coeffs)
    out.affexpr.coeffs.push_back(2 * a.constant * ai);
  const std::size_t n = a.size();
  for (std::size_t i = 0; i < n; ++i)
  {
    out.vars1.push_back(a.vars[i]);
    out.vars2.push_back(a.vars[i]);
    out.coeffs.push_back(sq(a.coeffs[i]));
    for (std::size_t j = i + 1; j < n; ++j)
    {
      out.vars1.push_back(a.vars[i]);
      out.vars2.push_back(a.vars[j]);
      out.coeffs.push_back(2 * a.coeffs[i] * a.coeffs[j]);
    }
  }
  return out;
}

AffExpr cleanupAff(const AffExpr& a)
{
  AffExpr out(a.constant);
  for (std::size_t k = 0; k < a.size(); ++k)
    if (std::fabs(a.coeffs[k]) > 1e-7)
    {
      out.coeffs.push_back(a.coeffs[k]);
      out.vars.push_back(a.vars[k]);
    }
  return out;
}

QuadExpr cleanupQuad(const QuadExpr& q)
{
  QuadExpr out;
  out.affexpr = cleanupAff(q.affexpr);
  for (std::size_t k = 0; k < q.size(); ++k)
    if (std::fabs(q.coeffs[k]) > 1e-8)
    {
      out.coeffs.push_back(q.coeffs[k]);
      out.vars1.push_back(q.vars1[k]);
      out.vars2.push_back(q.vars2[k]);
    }
  return out;
}

AffExpr varDot(const DblVec& x, const VarVector& v)
{
  AffExpr out;
  out.coeffs = x;
  out.vars = v;
  return out;
}

// ------------------------------------------------------------------ model defaults
Var Model::addVar(const std::string& name, double lb, double ub)
{
  Var v = addVar(name);
  setVarBounds(v, lb, ub);
  return v;
}
void Model::removeVar(const Var& var) { removeVars(VarVector(1, var)); }
void Model::removeCnt(const Cnt& cnt) { removeCnts(CntVector(1, cnt)); }
void Model::setVarBounds(const Var& var, double lower, double upper)
{
  setVarBounds(VarVector(1, var), DblVec(1, lower), DblVec(1, upper));
}
double Model::getVarValue(const Var& var) const { return getVarValues(VarVector(1, var))[0]; }

void vars2inds(const VarVector& vars, SizeTVec& inds)
{
  inds.resize(vars.size());
  for (std::size_t k = 0; k < vars.size(); ++k)
    inds[k] = vars[k].var_rep->index;
}
void vars2inds(const VarVector& vars, IntVec& inds)
{
  inds.resize(vars.size());
  for (std::size_t k = 0; k < vars.size(); ++k)
    inds[k] = static_cast<int>(vars[k].var_rep->index);
}
void cnts2inds(const CntVector& cnts, SizeTVec& inds)
{
  inds.resize(cnts.size());
  for (std::size_t k = 0; k < cnts.size(); ++k)
    inds[k] = cnts[k].cnt_rep->index;
}
void cnts2inds(const CntVector& cnts, IntVec& inds)
{
  inds.resize(cnts.size());
  for (std::size_t k = 0; k < cnts.size(); ++k)
    inds[k] = static_cast<int>(cnts[k].cnt_rep->index);
}

// ------------------------------------------------------------------ printing (LP-ish, solver_interface.cpp:142-212)
std::ostream& operator<<(std::ostream& o, const Var& v)
{
  return o << (v.var_rep ? v.var_rep->name : std::string("nullvar"));
}
std::ostream& operator<<(std::ostream& o, const Cnt& c)
{
  return o << c.cnt_rep->expr << ((c.cnt_rep->type == EQ) ? " == 0" : " <= 0");
}
std::ostream& operator<<(std::ostream& o, const AffExpr& e)
{
  const char* sep = "";
  if (e.constant != 0)
  {
    o << e.constant;
    sep = " + ";
  }
  for (std::size_t k = 0; k < e.size(); ++k)
  {
    if (e.coeffs[k] == 0)
      continue;
    o << sep;
    if (e.coeffs[k] != 1)
      o << e.coeffs[k] << " ";
    o << e.vars[k];
    sep = " + ";
  }
  return o;
}
std::ostream& operator<<(std::ostream& o, const QuadExpr& e)
{
  o << e.affexpr << " + [ ";
  const char* sep = "";
  for (std::size_t k = 0; k < e.size(); ++k)
  {
    if (e.coeffs[k] == 0)
      continue;
    o << sep;
    if (e.coeffs[k] != 1)
      o << e.coeffs[k] << " ";
    if (e.vars1[k].var_rep->name == e.vars2[k].var_rep->name)
      o << e.vars1[k] << " ^ 2";
    else
      o << e.vars1[k] << " * " << e.vars2[k];
    sep = " + ";
  }
  return o << " ] /2\n";
}

// ------------------------------------------------------------------ ModelType / factory
const std::vector<std::string> ModelType::MODEL_NAMES_ = { "GUROBI", "BPMPD", "OSQP", "QPOASES", "AUTO_SOLVER" };

ModelType::ModelType() = default;
ModelType::ModelType(const ModelType::Value& v) : value_(v) {}
ModelType::ModelType(const int& v) : value_(static_cast<Value>(v)) {}
ModelType::ModelType(const std::string& s)
{
  for (std::size_t k = 0; k < MODEL_NAMES_.size(); ++k)
    if (s == MODEL_NAMES_[k])
    {
      value_ = static_cast<Value>(k);  // Q1: the reference indexes the enum by the names' order
      return;
    }
  throw std::runtime_error("invalid solver name:\"" + s + "\"");
}
ModelType::operator int() const { return static_cast<int>(value_); }
bool ModelType::operator==(const ModelType::Value& a) const { return value_ == a; }
bool ModelType::operator==(const ModelType& a) const { return value_ == a.value_; }
bool ModelType::operator!=(const ModelType& a) const { return value_ != a.value_; }
std::ostream& operator<<(std::ostream& os, const ModelType& cs)
{
  const auto k = static_cast<std::size_t>(cs.value_);
  if (k >= ModelType::MODEL_NAMES_.size())
    throw std::runtime_error("Error converting ModelType to string - enum value is " + std::to_string(k));
  return os << ModelType::MODEL_NAMES_[k];
}

std::vector<ModelType> availableSolvers() { return { ModelType::OSQP }; }

Model::Ptr createModel(ModelType model_type, const ModelConfig::ConstPtr& model_config)
{
  if (model_type == ModelType::AUTO_SOLVER)
  {
    if (const char* env = std::getenv("TRAJOPT_CONVEX_SOLVER"))
    {
      const ModelType t{ std::string(env) };
      const auto avail = availableSolvers();
      if (std::find(avail.begin(), avail.end(), t) == avail.end())
        throw std::runtime_error("Failed to create solver: environment variable TRAJOPT_CONVEX_SOLVER is set to '" +
                                 std::string(env) + "' but that solver is not available.");
      model_type = t;
    }
    else
      model_type = availableSolvers()[0];
  }
  if (model_type == ModelType::OSQP)
  {
    auto cfg = std::dynamic_pointer_cast<const GpuModelConfig>(model_config);
    return std::make_shared<GpuModel>(cfg ? *cfg : GpuModelConfig());
  }
  std::ostringstream os;
  os << "Failed to create solver: " << model_type << " is not available in this build (OSQP runs on the GPU)";
  throw std::runtime_error(os.str());
}
}  // namespace sco
