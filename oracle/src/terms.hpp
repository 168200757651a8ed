// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of the trajopt-level terms on the hot path and of problem
// construction from the lowered descriptor:
//   JointVelEqCost                  trajopt/src/trajectory_costs.cpp:257-301
//   JointVelTermInfo::hatch         trajopt/src/problem_description.cpp:1216-1391 (step clamping)
//   JointPos{Eq,Ineq}{Cost,Constraint} trajopt/src/trajectory_costs.cpp:28-254
//   JointPosTermInfo::hatch         trajopt/src/problem_description.cpp:1097-1196
//   CartPoseErrCalculator           trajopt/src/kinematic_terms.cpp:189-266
//   CartPoseJacCalculator           trajopt/src/kinematic_terms.cpp:289-370
//   CartPoseTermInfo::hatch         trajopt/src/problem_description.cpp:919-1005
//   ConstructProblem / TrajOptProb  trajopt/src/problem_description.cpp:414-598
#pragma once
#include <memory>
#include <vector>

#include "kin.hpp"
#include "sco.hpp"

namespace orc
{
struct TrajProblem
{
  OptProb::Ptr prob;
  std::vector<Var> traj_vars;  // [n_steps * (n_dof + use_time)]: per step the joints, then dt (use_time)
  int n_steps = 0, n_dof = 0, n_cols = 0;
  DblVec init;
};

OsqpSettings toOsqpSettings(const thip_osqp_settings& s);
BasicTrustRegionSQPParameters toSqpParams(const thip_sqp_params& p);

// The CartPose error / FD jacobian of one term at joint values q (reduced to
// the rows with |coeff| > 1e-5, in CartPoseTermInfo::hatch order).
struct CartPoseCalc
{
  const thip_chain* chain;
  int source_link;
  Iso3 source_offset;
  Iso3 target_offset;  // target frame = chain root (static)
  std::vector<int> indices;
  bool has_tol = false;  // tolerance band (kinematic_terms.cpp:209-247, 319-339)
  int target_link = 0;   // > 0: DynamicCartPose, the target is this active link (kinematic_terms.cpp:58-187)
  double lower_tol[6] = {}, upper_tol[6] = {};
  DblVec operator()(const DblVec& q) const;  // error
  Mat jac(const DblVec& q) const;            // forward-difference jacobian, eps = 1e-5
};
void cartPoseIndices(const thip_problem_desc& d, int term, std::vector<int>& indices, DblVec& coeffs);
void setCartPoseTolerances(const thip_problem_desc& d, int term, CartPoseCalc& c);

// Build the TrajOptProb of problem b of a batch (ConstructProblem restated).
// jpos_targets [n_jpos][D] (null: the descriptor's targets)
TrajProblem constructProblem(const thip_problem_desc& d, const double* init_traj, const double* cart_targets,
                             const double* scene, const double* jpos_targets = nullptr);

}  // namespace orc
