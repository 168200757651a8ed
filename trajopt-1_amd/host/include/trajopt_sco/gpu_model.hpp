// GpuModel: the sco::Model backend of the MI355X build (SURVEY.md §8b tier i).
// The model bookkeeping is OSQPModel's (trajopt_sco/src/osqp_interface.cpp:
// 73-640): variables and constraints in creation order, update() compacts
// removed ones, the objective QuadExpr becomes an upper-triangular CSC P
// (duplicates summed, P_ii = 2c), the constraint rows and an identity block of
// variable bounds become A with l / u, and the previous solution warm-starts
// the next solve when the last status was solved and the sparsity "matches"
// (the reference compares n + 1 / nnz BYTES, quirk Q2).  optimize() runs the
// QP on the GPU: thip_qp_solve, OSQP 1.0 with OSQPModelConfig's settings.
#pragma once
#include <memory>
#include <array>
#include <mutex>
#include <vector>

#include "trajopt_hip.h"
#include "trajopt_sco/gpu_qp_batcher.hpp"
#include "trajopt_sco/solver_interface.hpp"

namespace sco
{
struct GpuModelConfig : public ModelConfig
{
  using Ptr = std::shared_ptr<GpuModelConfig>;
  using ConstPtr = std::shared_ptr<const GpuModelConfig>;
  GpuModelConfig();
  thip_osqp_settings settings{};  // OSQPModelConfig::setDefaultOSQPSettings (osqp_interface.cpp:78-90)
  bool update_workspace{ false };  // (the reference's default: rebuild every solve)
  int device{ 0 };
};

class GpuModel : public Model
{
public:
  explicit GpuModel(const GpuModelConfig& config = GpuModelConfig());
  ~GpuModel() override;
  GpuModel(const GpuModel&) = delete;
  GpuModel& operator=(const GpuModel&) = delete;

  Var addVar(const std::string& name) override;
  using Model::addVar;
  Cnt addEqCnt(const AffExpr&, const std::string& name) override;
  Cnt addIneqCnt(const AffExpr&, const std::string& name) override;
  Cnt addIneqCnt(const QuadExpr&, const std::string& name) override;  // throws, as OSQPModel
  void removeVars(const VarVector& vars) override;
  void removeCnts(const CntVector& cnts) override;
  void update() override;
  using Model::setVarBounds;
  void setVarBounds(const VarVector& vars, const DblVec& lower, const DblVec& upper) override;
  DblVec getVarValues(const VarVector& vars) const override;
  CvxOptStatus optimize() override;
  void setObjective(const AffExpr&) override;
  void setObjective(const QuadExpr&) override;
  void writeToFile(const std::string& fname) const override;  // osqp_interface.cpp:621-640
  VarVector getVars() const override;

  // HIP device of the following solves
  void setDevice(int device);
  int device() const { return config_.device; }
  // solve through a batcher shared with other models (one launch per pattern for
  // the QPs of many problems' host loops); null: one launch per QP
  void setBatcher(GpuQPBatcher::Ptr b) { batcher_ = std::move(b); }

  // diagnostics of the last solve
  const thip_qp_info& lastInfo() const { return info_; }
  // diagnostics: one record per solve appended to *trace (null: off) -- warm
  // start, rho in, ADMM iterations, OSQP status, polish status, rho out, primal /
  // dual residual, sum |x*| (the oracle's OSQPModel trace fields 0-8)
  void setTrace(std::vector<std::array<double, 9>>* trace) { trace_ = trace; }
  long long admmItersTotal() const { return admm_total_; }

private:
  struct Csc
  {
    int n = 0, m = 0;
    std::vector<int> p, i;
    std::vector<double> x;
  };
  void buildObjective(Csc& P, DblVec& q) const;
  void buildConstraints(Csc& A, DblVec& l, DblVec& u) const;
  static bool bytesEqual(const Csc& a, const Csc& b);
  void solveDirect(const Csc& P, const Csc& A, const DblVec& q, const DblVec& l, const DblVec& u,
                   const thip_osqp_settings& s, bool ws, DblVec& x, DblVec& y);
  CvxOptStatus finishSolve(Csc&& P, Csc&& A, const DblVec& x, const DblVec& y);

  GpuModelConfig config_;
  std::mutex mutex_;
  VarVector vars_;
  DblVec lbs_, ubs_;
  CntVector cnts_;
  AffExprVector cnt_exprs_;
  ConstraintTypeVector cnt_types_;
  QuadExpr objective_;
  DblVec solution_;
  // previous solve: pattern (for the warm-start test), solution, rho, status
  Csc prev_P_, prev_A_;
  bool have_prev_{ false };
  DblVec prev_x_, prev_y_;
  double prev_rho_{ 0 };
  int prev_status_{ 0 };
  thip_qp* qp_{ nullptr };  // device pattern of the last solve (reused while it matches)
  std::vector<int> qp_Pp_, qp_Pi_, qp_Ap_, qp_Ai_;
  thip_qp_info info_{};
  long long admm_total_{ 0 };
  GpuQPBatcher::Ptr batcher_;
  std::vector<std::array<double, 9>>* trace_{ nullptr };
};
}  // namespace sco
