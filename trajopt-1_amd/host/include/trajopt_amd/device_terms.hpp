// The kinematic terms of a TrajOptProb as sco::Cost / sco::Constraint objects
// whose values and convexifications come from the device (include/trajopt_hip.h
// thip_eval_*), so that sco::BasicTrustRegionSQP's host loop can run them next
// to terms the batched kernel does not lower (JointAcc / JointJerk, time terms,
// user sco::Costs), on single-waypoint problems and with several collision
// terms.  The same objects describe the problem to the batched kernel: a
// lowerable problem never evaluates them on the host.
//
//   CartPoseDeviceErr / CartPoseDeviceJac   CartPoseErrCalculator /
//       CartPoseJacCalculator (trajopt/src/kinematic_terms.cpp:189-370) as the
//       sco::VectorOfVector / MatrixOfVector of the TrajOptCostFromErrFunc /
//       TrajOptConstraintFromErrFunc that CartPoseTermInfo::hatch builds
//       (problem_description.cpp:919-1005)
//   DeviceCollisionCost / DeviceCollisionConstraint   CollisionCost /
//       CollisionConstraint (collision_terms.cpp:1267-1386), one per unit (a free
//       waypoint for DISCRETE, a step pair otherwise) as
//       CollisionTermInfo::hatch adds them (problem_description.cpp:1735-1858)
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_hip.h"
#include "trajopt_sco/modeling.hpp"
#include "trajopt_sco/modeling_utils.hpp"

namespace trajopt
{
class TrajOptProb;
using sco::DblVec;

// One TrajOptProb's thip_eval, created at the first evaluation (after every
// term has hatched) on the problem's device.  Collision records are cached per
// term for the last joint trajectory they were computed at (the reference's
// evaluators cache contacts by x the same way, collision_terms.cpp:737-800).
class DeviceTermEvaluator
{
public:
  explicit DeviceTermEvaluator(const TrajOptProb* prob) : prob_(prob) {}
  ~DeviceTermEvaluator();
  DeviceTermEvaluator(const DeviceTermEvaluator&) = delete;
  DeviceTermEvaluator& operator=(const DeviceTermEvaluator&) = delete;

  // CartPose term k (descriptor order) at its waypoint's joint values q:
  // err[6], jac[6][n_dof] (row-major; may be null)
  void cartPose(int k, const DblVec& q, double* err, double* jac);
  // every CartPose term at its waypoint of the full variable vector x in one
  // launch (thip_eval_cart_pose_all); cartPose(k, q) then answers from it while
  // q is bitwise term k's waypoint of that x
  void prefetchCart(const DblVec& x);

  // the contact records of one collision term (0 = the descriptor's coll_*,
  // then coll_extra[]) at the full variable vector x; W = 8 + 2 n_dof + 1
  struct Contacts
  {
    int W = 0;
    std::vector<double> rec;   // [n][W] in unit order, then ContactResultMap order
    std::vector<int> t;        // per record: the unit's (first) waypoint
    // per record: its link pair's margin and coefficient (the term's dist_pen /
    // coeffs unless the term's "pairs" override them: CollisionMarginData /
    // CollisionCoeffData lookups, collision_terms.cpp:243-386)
    std::vector<double> margin, coeff;
  };
  const Contacts& collision(int term, const DblVec& x);

private:
  void ensure();
  const TrajOptProb* prob_;
  thip_eval* ev_ = nullptr;
  int device_ = -1;
  struct Cache
  {
    DblVec q;  // the joint trajectory the contacts belong to
    Contacts c;
    bool valid = false;
  };
  std::vector<Cache> cache_;
  struct CartCache
  {
    DblVec q;                 // the joint trajectory [n_steps][n_dof] of the prefetch
    std::vector<double> err;  // [n_cart][6]
    std::vector<double> jac;  // [n_cart][6][n_dof]
    bool valid = false;
  } cart_;
  DblVec jointTrajectory(const DblVec& x) const;
  std::vector<std::vector<double>> pair_tab_;  // per term: pair_data.hpp table, empty = the term's own
};

class CartPoseDeviceErr : public sco::VectorOfVector
{
public:
  CartPoseDeviceErr(std::shared_ptr<DeviceTermEvaluator> ev, int term, std::vector<int> indices)
    : ev_(std::move(ev)), term_(term), indices_(std::move(indices))
  {
  }
  DblVec operator()(const DblVec& q) const override;

private:
  std::shared_ptr<DeviceTermEvaluator> ev_;
  int term_;
  std::vector<int> indices_;
};

class CartPoseDeviceJac : public sco::MatrixOfVector
{
public:
  CartPoseDeviceJac(std::shared_ptr<DeviceTermEvaluator> ev, int term, std::vector<int> indices)
    : ev_(std::move(ev)), term_(term), indices_(std::move(indices))
  {
  }
  sco::Mat operator()(const DblVec& q) const override;

private:
  std::shared_ptr<DeviceTermEvaluator> ev_;
  int term_;
  std::vector<int> indices_;
};

// TrajOptCostFromErrFunc / TrajOptConstraintFromErrFunc of a CartPose term
// (problem_description.cpp:961-1000): sco's error-function term over the
// device calculators above (named types, so callers can tell them apart)
class DeviceCartPoseCost : public sco::CostFromErrFunc
{
public:
  using sco::CostFromErrFunc::CostFromErrFunc;
};
class DeviceCartPoseConstraint : public sco::ConstraintFromErrFunc
{
public:
  using sco::ConstraintFromErrFunc::ConstraintFromErrFunc;
};

// the distance expressions of one unit: dist + sum scale g (x - x0) over its free ends
struct DeviceCollisionUnit
{
  std::shared_ptr<DeviceTermEvaluator> ev;
  int term = 0;              // thip_eval collision term index
  int t = 0;                 // the unit's (first) waypoint
  sco::VarVector vars0, vars1;  // waypoint t, t + 1 (empty for DISCRETE)
  // the unit's records at x: [first, first + n) of the term's contacts
  void records(const DblVec& x, const DeviceTermEvaluator::Contacts*& c, int& first, int& n) const;
  // the distance expressions of the unit's contacts, with each contact's margin and coefficient
  sco::AffExprVector exprs(const DblVec& x, DblVec* margins = nullptr, DblVec* coeffs = nullptr) const;
  sco::VarVector vars() const;
};

class DeviceCollisionCost : public sco::Cost
{
public:
  DeviceCollisionCost(DeviceCollisionUnit u, const std::string& name) : sco::Cost(name), u_(std::move(u)) {}
  double value(const DblVec& x) override;  // sum coeff * max(margin - d, 0) (no buffer)
  sco::ConvexObjective::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return u_.vars(); }

private:
  DeviceCollisionUnit u_;
};

class DeviceCollisionConstraint : public sco::IneqConstraint
{
public:
  DeviceCollisionConstraint(DeviceCollisionUnit u, const std::string& name)
    : sco::IneqConstraint(name), u_(std::move(u))
  {
  }
  DblVec value(const DblVec& x) override;  // per contact coeff * max(margin - d, 0)
  sco::ConvexConstraints::Ptr convex(const DblVec& x, sco::Model* model) override;
  sco::VarVector getVars() override { return u_.vars(); }

private:
  DeviceCollisionUnit u_;
};
}  // namespace trajopt
