// Host front door of the batched HIP SQP: trajopt's problem-construction
// surface (ProblemConstructionInfo / TermInfo registry / fromJson / hatch /
// ConstructProblem, trajopt/include/trajopt/problem_description.hpp:30-260)
// restated in C++ over the C-ABI of include/trajopt_hip.h.
//
// Differences from the reference, all forced by what the HIP path lowers:
//  * hatch() lowers a term into the batch-shared structure (thip_problem_desc)
//    and the problem's own data (targets, initial trajectory) of a
//    TrajOptProb, instead of pushing sco::Cost objects; BatchTrustRegionSQP
//    (batch_sqp.hpp) then solves many TrajOptProbs that share one structure.
//  * The registered term types are the ones on the HIP path: joint_pos,
//    joint_vel, cart_pose, dynamic_cart_pose, collision.  The reference's other
//    makers (cart_vel, joint_acc, joint_jerk, total_time,
//    problem_description.cpp:57-70) are registered too, and their hatch()
//    throws "not supported on the HIP path" so a JSON that uses them fails
//    loudly rather than silently dropping a term.
//  * Environment / KinematicGroup stand in for tesseract's Environment and
//    JointGroup (which are out of scope): a serial chain with link and joint
//    names, joint limits, the current state, the collision spheres of the
//    robot links and the scene primitives (THIP_PRIM_* records).
// Errors are std::runtime_error, as PRINT_AND_THROW (trajopt_common/macros.h:90-103).
#pragma once
#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "trajopt_amd/json.hpp"
#include "trajopt_hip.h"

namespace sco
{
// trajopt_sco/include/trajopt_sco/optimizers.hpp:25-33
enum OptStatus : int
{
  OPT_CONVERGED,
  OPT_SCO_ITERATION_LIMIT,
  OPT_PENALTY_ITERATION_LIMIT,
  OPT_TIME_LIMIT,
  OPT_FAILED,
  INVALID
};
std::string toString(OptStatus status);

using DblVec = std::vector<double>;
using IntVec = std::vector<int>;

// optimizers.hpp:40-59 (+ the counters the HIP path reports)
struct OptResults
{
  DblVec x;
  OptStatus status{ INVALID };
  double total_cost{ 0 };
  DblVec cost_vals;  // not reported per term by the batch kernel (empty)
  DblVec cnt_viols;  // idem
  int n_func_evals{ 0 }, n_qp_solves{ 0 };
  int n_sqp_iters{ 0 };
  long long n_admm_iters{ 0 };
  double max_cnt_viol{ 0 };
  int flags{ 0 };
};

// optimizers.hpp:92-135 (numeric members; max_time is checked on the device at
// the top of every SQP iteration against the problem's own clock)
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
  double max_time = 1.7976931348623157e308;
  double initial_merit_error_coeff = 10;
  bool inflate_constraints_individually = true;
  double trust_box_size = 1e-1;
  // optimizers.hpp:127-129: with log_results, log_dir/trajopt_solver.log gets one
  // writeSolver line per trust-region step (the vars / costs / constraints logs are not
  // written: the device loop keeps no per-iteration copies of x and the term values)
  bool log_results = false;
  std::string log_dir = "/tmp";
};
}  // namespace sco

namespace trajopt
{
using sco::DblVec;
using sco::IntVec;

// problem_description.hpp:30-60
enum class TermType : char
{
  TT_INVALID = 0,
  TT_COST = 0x1,
  TT_CNT = 0x2,
  TT_USE_TIME = 0x4,
};
inline TermType operator|(TermType a, TermType b) { return TermType(static_cast<char>(a) | static_cast<char>(b)); }
inline TermType operator&(TermType a, TermType b) { return TermType(static_cast<char>(a) & static_cast<char>(b)); }
inline bool any(TermType t) { return static_cast<char>(t) != 0; }

// tesseract JointGroup, restated for a kinematic tree (thip_chain::parent)
struct KinematicGroup
{
  using ConstPtr = std::shared_ptr<const KinematicGroup>;
  std::string name;
  thip_chain chain{};
  std::vector<std::string> link_names;   // chain link k (link 0 = static chain root)
  std::vector<std::string> joint_names;  // per dof
  // static frames outside the chain (e.g. base_footprint) with their world poses
  std::map<std::string, std::array<double, 12>> static_frames;

  int numJoints() const { return chain.n_dof; }
  int linkIndex(const std::string& link) const;  // -1 if not a chain link
  bool hasLinkId(const std::string& link) const { return linkIndex(link) >= 0 || static_frames.count(link) > 0; }
  bool isActiveLinkId(const std::string& link) const;  // moved by one of the group's joints
  // world pose of a static frame (chain root or static_frames entry)
  std::array<double, 12> staticWorldPose(const std::string& link) const;
};

struct CollisionSphere
{
  std::string link;   // robot link name
  double center[3];   // in the link frame
  double radius;
};

// tesseract Environment, restated: kinematic groups, the current state, the
// robot's collision spheres and the scene.
class Environment
{
public:
  using Ptr = std::shared_ptr<Environment>;
  using ConstPtr = std::shared_ptr<const Environment>;

  void addJointGroup(KinematicGroup g);
  KinematicGroup::ConstPtr getJointGroup(const std::string& name) const;  // null if absent
  DblVec getCurrentJointValues(const std::string& group) const;
  void setState(const std::string& group, const DblVec& q);

  std::vector<CollisionSphere> collision_spheres;      // robot collision model
  std::vector<std::array<double, 16>> scene;           // THIP_PRIM_* records

  // PR2 arms (groups "right_arm", "left_arm": torso_lift_link ->
  // *_gripper_tool_frame, and "both_arms", joint data of
  // trajopt_common/data/arm_around_table.urdf), zero state, the 14-sphere
  // per-arm collision model of trajopt_amd/scene.py, empty scene.
  static Ptr makePR2();

private:
  std::map<std::string, KinematicGroup::ConstPtr> groups_;
  std::map<std::string, DblVec> state_;
};

// problem_description.hpp:122-160
struct BasicInfo
{
  int n_steps{ -1 };
  std::string manip;
  IntVec fixed_timesteps;
  IntVec fixed_dofs;
  std::string convex_solver{ "OSQP" };
  bool use_time = false;
  double dt_upper_lim = 1.0;
  double dt_lower_lim = 1.0;
};

// problem_description.hpp:165-190
struct InitInfo
{
  enum Type
  {
    STATIONARY,
    JOINT_INTERPOLATED,
    GIVEN_TRAJ,
  };
  Type type{ STATIONARY };
  std::vector<DblVec> data;  // GIVEN_TRAJ: n_steps rows; JOINT_INTERPOLATED: one row (endpoint)
  double dt{ 1.0 };
};

class TrajOptProb;
struct ProblemConstructionInfo;

// problem_description.hpp:200-231
struct TermInfo
{
  using Ptr = std::shared_ptr<TermInfo>;
  using MakerFunc = std::shared_ptr<TermInfo> (*)();

  std::string name;
  TermType term_type{ TermType::TT_INVALID };
  TermType getSupportedTypes() const { return supported_term_types_; }
  virtual void fromJson(ProblemConstructionInfo& pci, const Json::Value& v) = 0;
  virtual void hatch(TrajOptProb& prob) = 0;

  static TermInfo::Ptr fromName(const std::string& type);
  static void RegisterMaker(const std::string& type, MakerFunc);

  virtual ~TermInfo() = default;

protected:
  explicit TermInfo(TermType supported) : supported_term_types_(supported) {}

private:
  TermType supported_term_types_;
};

// problem_description.hpp:1061-1095 (JointPosTermInfo)
struct JointPosTermInfo : public TermInfo
{
  DblVec coeffs, targets, upper_tols, lower_tols;
  int first_step = 0, last_step = -1;
  JointPosTermInfo() : TermInfo(TermType::TT_COST | TermType::TT_CNT) {}
  void fromJson(ProblemConstructionInfo& pci, const Json::Value& v) override;
  void hatch(TrajOptProb& prob) override;
  static TermInfo::Ptr create() { return std::make_shared<JointPosTermInfo>(); }
};

// JointVelTermInfo
struct JointVelTermInfo : public TermInfo
{
  DblVec coeffs, targets, upper_tols, lower_tols;
  int first_step = 0, last_step = -1;
  JointVelTermInfo() : TermInfo(TermType::TT_COST | TermType::TT_CNT | TermType::TT_USE_TIME) {}
  void fromJson(ProblemConstructionInfo& pci, const Json::Value& v) override;
  void hatch(TrajOptProb& prob) override;
  static TermInfo::Ptr create() { return std::make_shared<JointVelTermInfo>(); }
};

// CartPoseTermInfo (problem_description.hpp:353-387); poses are 3x4 row-major
struct CartPoseTermInfo : public TermInfo
{
  int timestep = 0;
  std::array<double, 3> pos_coeffs{ { 1, 1, 1 } }, rot_coeffs{ { 1, 1, 1 } };
  std::string source_frame, target_frame;
  std::array<double, 12> source_frame_offset{ { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 } };
  std::array<double, 12> target_frame_offset{ { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 } };
  DblVec lower_tolerance, upper_tolerance;
  CartPoseTermInfo() : TermInfo(TermType::TT_COST | TermType::TT_CNT) {}
  void fromJson(ProblemConstructionInfo& pci, const Json::Value& v) override;
  void hatch(TrajOptProb& prob) override;
  static TermInfo::Ptr create() { return std::make_shared<CartPoseTermInfo>(); }

protected:
  bool dynamic_ = false;  // DynamicCartPoseTermInfo: both frames active
};

// problem_description.cpp:683-842: source and target both active links at one timestep
// (DynamicCartPoseErrCalculator / DynamicCartPoseJacCalculator, kinematic_terms.cpp:58-187)
struct DynamicCartPoseTermInfo : public CartPoseTermInfo
{
  DynamicCartPoseTermInfo() { dynamic_ = true; }
  static TermInfo::Ptr create() { return std::make_shared<DynamicCartPoseTermInfo>(); }
};

// CollisionTermInfo (problem_description.cpp:1636-1858) with the
// TrajOptCollisionConfig fields the HIP path lowers
struct CollisionTermInfo : public TermInfo
{
  int first_step = 0, last_step = -1;
  IntVec fixed_steps;
  int evaluator_type = 1;        // tesseract CollisionEvaluatorType {NONE, DISCRETE, LVS_DISCRETE, ...}
  int contact_test_type = 2;     // FIRST, CLOSEST, ALL
  double longest_valid_segment_length = 0.5;
  double collision_margin_buffer = 0.5;
  double coeff = 20;             // CollisionCoeffData default
  double dist_pen = 0;           // collision margin
  bool has_pairs = false;        // a "pairs" override differing from coeff / dist_pen
  CollisionTermInfo() : TermInfo(TermType::TT_COST | TermType::TT_CNT) {}
  void fromJson(ProblemConstructionInfo& pci, const Json::Value& v) override;
  void hatch(TrajOptProb& prob) override;
  static TermInfo::Ptr create() { return std::make_shared<CollisionTermInfo>(); }
};

// problem_description.hpp:236-260
struct ProblemConstructionInfo
{
  BasicInfo basic_info;
  sco::BasicTrustRegionSQPParameters opt_info;
  thip_osqp_settings osqp{};  // OSQPModelConfig (osqp_interface.cpp:78-90 defaults)
  std::vector<TermInfo::Ptr> cost_infos;
  std::vector<TermInfo::Ptr> cnt_infos;
  InitInfo init_info;
  Environment::ConstPtr env;
  KinematicGroup::ConstPtr kin;

  explicit ProblemConstructionInfo(Environment::ConstPtr e);
  void fromJson(const Json::Value& v);

private:
  void readBasicInfo(const Json::Value& v);
  void readOptInfo(const Json::Value& v);
  void readCosts(const Json::Value& v);
  void readConstraints(const Json::Value& v);
  void readInitInfo(const Json::Value& v);
};

// The lowered problem: batch-shared structure + this problem's data.
class TrajOptProb
{
public:
  using Ptr = std::shared_ptr<TrajOptProb>;

  int GetNumSteps() const { return desc_.n_steps; }
  int GetNumDOF() const { return desc_.chain.n_dof; }
  KinematicGroup::ConstPtr GetKin() const { return kin_; }
  Environment::ConstPtr GetEnv() const { return env_; }
  const std::vector<DblVec>& GetInitTraj() const { return init_; }
  void SetInitTraj(const std::vector<DblVec>& x) { init_ = x; }

  // lowered form (C-ABI)
  const thip_problem_desc& desc() const { return desc_; }
  thip_problem_desc& desc() { return desc_; }
  std::vector<double> cart_targets;  // [n_cart][12] target-frame offsets in the chain root
  std::vector<double> jpos_targets;  // [n_jpos][D]
  std::vector<double> scene;         // [n_prims][16]

  friend TrajOptProb::Ptr ConstructProblem(const ProblemConstructionInfo& pci);

private:
  thip_problem_desc desc_{};
  std::vector<DblVec> init_;
  KinematicGroup::ConstPtr kin_;
  Environment::ConstPtr env_;
};

TrajOptProb::Ptr ConstructProblem(const ProblemConstructionInfo& pci);
TrajOptProb::Ptr ConstructProblem(const Json::Value& root, const Environment::ConstPtr& env);
}  // namespace trajopt
