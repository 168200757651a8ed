// Host front door: ProblemConstructionInfo::fromJson, the TermInfo registry,
// hatch() lowering and ConstructProblem, restating
// trajopt/src/problem_description.cpp:36-598 (+ the term infos at
// :843-1005, :1078-1391, :1636-1858) over the C-ABI descriptor.
#include "trajopt_amd/problem_description.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <iostream>
#include <stdexcept>

#include "trajopt_sco/expr_ops.hpp"

namespace
{
bool gRegisteredMakers = false;
std::map<std::string, trajopt::TermInfo::MakerFunc>& name2maker()
{
  static std::map<std::string, trajopt::TermInfo::MakerFunc> m;
  return m;
}

// problem_description.cpp:36-54
void ensure_only_members(const Json::Value& v, const char** fields, int nvalid)
{
  for (const auto& name : v.getMemberNames())
  {
    bool valid = false;
    for (int j = 0; j < nvalid; ++j)
      if (name == fields[j])
      {
        valid = true;
        break;
      }
    if (!valid)
      throw std::runtime_error("invalid field found: " + name);
  }
}

// problem_description.cpp:80-95
void checkParameterSize(trajopt::DblVec& parameter, unsigned expected_size, const std::string& name,
                        bool apply_first = true)
{
  if (apply_first && parameter.size() == 1)
    parameter = trajopt::DblVec(expected_size, parameter[0]);
  else if (parameter.size() != expected_size)
    throw std::runtime_error("wrong number of " + name + ". expected " + std::to_string(expected_size) + " got " +
                             std::to_string(parameter.size()));
}

bool doubleEquals(double a, double b) { return std::fabs(a - b) < 1e-5; }  // trajopt_common::doubleEquals

[[noreturn]] void unsupported(const std::string& what)
{
  throw std::runtime_error(what + " is not supported on the HIP path");
}

// A registered maker whose lowering does not exist on the HIP path.
struct UnsupportedTermInfo : public trajopt::TermInfo
{
  std::string type;
  explicit UnsupportedTermInfo(std::string t)
    : TermInfo(trajopt::TermType::TT_COST | trajopt::TermType::TT_CNT | trajopt::TermType::TT_USE_TIME)
    , type(std::move(t))
  {
  }
  void fromJson(trajopt::ProblemConstructionInfo&, const Json::Value&) override {}
  void hatch(trajopt::TrajOptProb&) override { unsupported("term type '" + type + "'"); }
};
template <const char* kName>
trajopt::TermInfo::Ptr makeUnsupported()
{
  return std::make_shared<UnsupportedTermInfo>(kName);
}
constexpr char kCartVel[] = "cart_vel";

// problem_description.cpp:57-70
void RegisterMakers()
{
  gRegisteredMakers = true;  // first: RegisterMaker() below checks it
  trajopt::TermInfo::RegisterMaker("dynamic_cart_pose", &trajopt::DynamicCartPoseTermInfo::create);
  trajopt::TermInfo::RegisterMaker("cart_pose", &trajopt::CartPoseTermInfo::create);
  trajopt::TermInfo::RegisterMaker("cart_vel", &makeUnsupported<kCartVel>);
  trajopt::TermInfo::RegisterMaker("joint_pos", &trajopt::JointPosTermInfo::create);
  trajopt::TermInfo::RegisterMaker("joint_vel", &trajopt::JointVelTermInfo::create);
  trajopt::TermInfo::RegisterMaker("joint_acc", &trajopt::JointAccTermInfo::create);
  trajopt::TermInfo::RegisterMaker("joint_jerk", &trajopt::JointJerkTermInfo::create);
  trajopt::TermInfo::RegisterMaker("collision", &trajopt::CollisionTermInfo::create);
  trajopt::TermInfo::RegisterMaker("total_time", &trajopt::TotalTimeTermInfo::create);
}

bool iequals(const std::string& a, const std::string& b)
{
  if (a.size() != b.size())
    return false;
  for (std::size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
      return false;
  return true;
}

using Pose12 = std::array<double, 12>;
Pose12 poseMul(const Pose12& a, const Pose12& b)
{
  Pose12 o{};
  for (int r = 0; r < 3; ++r)
  {
    for (int c = 0; c < 3; ++c)
      o[r * 4 + c] = a[r * 4 + 0] * b[0 * 4 + c] + a[r * 4 + 1] * b[1 * 4 + c] + a[r * 4 + 2] * b[2 * 4 + c];
    o[r * 4 + 3] = a[r * 4 + 0] * b[3] + a[r * 4 + 1] * b[7] + a[r * 4 + 2] * b[11] + a[r * 4 + 3];
  }
  return o;
}
Pose12 poseInv(const Pose12& a)
{
  Pose12 o{};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      o[r * 4 + c] = a[c * 4 + r];
  for (int r = 0; r < 3; ++r)
    o[r * 4 + 3] = -(o[r * 4 + 0] * a[3] + o[r * 4 + 1] * a[7] + o[r * 4 + 2] * a[11]);
  return o;
}

// Eigen::Quaterniond(w, x, y, z).matrix() (Eigen/src/Geometry/Quaternion.h toRotationMatrix)
Pose12 poseFromXyzWxyz(const std::array<double, 3>& p, const std::array<double, 4>& q)
{
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  return Pose12{ { 1.0 - (tyy + tzz), txy - twz, txz + twy, p[0],  //
                   txy + twz, 1.0 - (txx + tzz), tyz - twx, p[1],  //
                   txz - twy, tyz + twx, 1.0 - (txx + tyy), p[2] } };
}

void readVec3(const Json::Value& params, const char* name, std::array<double, 3>& out, std::array<double, 3> df)
{
  if (!params.isMember(name))
  {
    out = df;
    return;
  }
  std::vector<double> v;
  json_marshal::fromJsonArray(params[name], v, 3);
  std::copy(v.begin(), v.end(), out.begin());
}
void readVec4(const Json::Value& params, const char* name, std::array<double, 4>& out, std::array<double, 4> df)
{
  if (!params.isMember(name))
  {
    out = df;
    return;
  }
  std::vector<double> v;
  json_marshal::fromJsonArray(params[name], v, 4);
  std::copy(v.begin(), v.end(), out.begin());
}

// Eigen 3.4 LinSpaced(size, low, high)(i), as in collision_device.hpp
double linspaced(int size, double low, double high, int i)
{
  if (size == 1)
    return high;
  const int size1 = size - 1;
  const double step = (high - low) / size1;
  if (std::fabs(high) < std::fabs(low))
    return (i == 0) ? low : high - double(size1 - i) * step;
  return (i == size1) ? high : low + double(i) * step;
}

bool allZero(const trajopt::DblVec& v)
{
  return std::all_of(v.begin(), v.end(), [](double a) { return doubleEquals(a, 0.); });
}

// the JointVel / JointAcc / JointJerk step clamping of the reference's hatch()
// (problem_description.cpp:1227-1243, 1423-1440, 1545-1562): `span` steps are needed
// for one difference
void clampSteps(int n_steps, int order, int& first, int& last)
{
  if (last <= -1)
    last = n_steps - 1;
  if ((n_steps - (order + 1)) <= first)
    first = n_steps - (order + 1);
  if ((n_steps - 1) <= last)
    last = n_steps - 1;
  if (last == first)
    last += (order == 1) ? 1 : (order == 2) ? 2 : 4;
  if (last < first)
    std::swap(first, last);
}

trajopt::JointDiffSpec diffSpec(trajopt::TrajOptProb& prob, int order, const trajopt::DblVec& coeffs,
                                const trajopt::DblVec& targets, const trajopt::DblVec& upper,
                                const trajopt::DblVec& lower, int first, int last)
{
  trajopt::JointDiffSpec s;
  s.vars = prob.GetJointVars();
  s.coeffs = coeffs;
  s.targets = targets;
  s.upper_tols = upper;
  s.lower_tols = lower;
  s.order = order;
  s.first_step = first;
  s.last_step = last;
  return s;
}

// the host cost / constraint object of a joint-difference term (trajectory_costs.hpp)
void addJointDiffObjects(trajopt::TrajOptProb& prob, const trajopt::JointDiffSpec& s, bool is_cost, bool zero_tols,
                         const std::string& name, bool lowered)
{
  if (is_cost)
  {
    sco::Cost::Ptr c = zero_tols ? sco::Cost::Ptr(std::make_shared<trajopt::JointDiffEqCost>(s, name))
                                 : sco::Cost::Ptr(std::make_shared<trajopt::JointDiffIneqCost>(s, name));
    if (lowered)
      prob.addLoweredCost(c);
    else
      prob.addCost(c);
  }
  else
  {
    sco::Constraint::Ptr c = zero_tols
                                 ? sco::Constraint::Ptr(std::make_shared<trajopt::JointDiffEqConstraint>(s, name))
                                 : sco::Constraint::Ptr(std::make_shared<trajopt::JointDiffIneqConstraint>(s, name));
    if (lowered)
      prob.addLoweredConstraint(c);
    else
      prob.addConstraint(c);
  }
}

// a JointVel equality constraint / JointAcc / JointJerk term: the descriptor's jdt
// table (the oracle's input; the batched kernel takes JointAccEqCost only,
// thip_jdt_fused) and the host object
void addJointDiffTerm(trajopt::TrajOptProb& prob, int order, bool is_cost, const trajopt::DblVec& coeffs,
                      const trajopt::DblVec& targets, const trajopt::DblVec& upper, const trajopt::DblVec& lower,
                      int first, int last, const std::string& name)
{
  thip_problem_desc& d = prob.desc();
  if (d.n_jdt >= THIP_MAX_JDT)
    unsupported("more than " + std::to_string(THIP_MAX_JDT) + " JointVel-constraint / JointAcc / JointJerk terms");
  if (first < 0 || last > prob.GetNumSteps() - 1)
    throw std::runtime_error(name + ": the trajectory is too short for a difference of order " +
                             std::to_string(order) + " over steps " + std::to_string(first) + ".." +
                             std::to_string(last));
  const int k = d.n_jdt++;
  d.jdt_order[k] = order;
  d.jdt_is_cnt[k] = is_cost ? 0 : 1;
  d.jdt_first_step[k] = first;
  d.jdt_last_step[k] = last;
  for (std::size_t j = 0; j < coeffs.size(); ++j)
  {
    d.jdt_coeffs[k][j] = coeffs[j];
    d.jdt_targets[k][j] = targets[j];
    d.jdt_upper_tols[k][j] = upper[j];
    d.jdt_lower_tols[k][j] = lower[j];
  }
  // JointAccEqCost runs in the fused kernel (waypoint-pair blocks) when the whole
  // problem qualifies (TrajOptProb::lowerable, thip_jdt_fused); every other form
  // only on the generic path
  const bool zero_tols = allZero(upper) && allZero(lower);
  addJointDiffObjects(prob, diffSpec(prob, order, coeffs, targets, upper, lower, first, last), is_cost, zero_tols,
                      name, order == 2 && is_cost && zero_tols);
}

sco::ModelConfig::ConstPtr modelConfig(const trajopt::ProblemConstructionInfo& pci)
{
  auto c = std::make_shared<sco::GpuModelConfig>();
  c->settings = pci.osqp;
  return c;
}
}  // namespace

namespace trajopt
{
// ------------------------------------------------------------ kinematics / environment
int KinematicGroup::linkIndex(const std::string& link) const
{
  for (std::size_t k = 0; k < link_names.size(); ++k)
    if (link_names[k] == link)
      return static_cast<int>(k);
  return -1;
}

bool KinematicGroup::isActiveLinkId(const std::string& link) const
{
  // moved by a joint on its path from the root
  for (int i = linkIndex(link); i > 0; i = chain.is_tree ? chain.parent[i] : i - 1)
    if (chain.joint_type[i] != THIP_JOINT_FIXED)
      return true;
  return false;
}

std::array<double, 12> KinematicGroup::staticWorldPose(const std::string& link) const
{
  const int k = linkIndex(link);
  if (k >= 0)
  {
    if (isActiveLinkId(link))
      throw std::runtime_error("staticWorldPose: link " + link + " is active");
    std::vector<int> path;  // root -> link
    for (int i = k; i > 0; i = chain.is_tree ? chain.parent[i] : i - 1)
      path.insert(path.begin(), i);
    Pose12 T;
    std::copy(chain.base_pose, chain.base_pose + 12, T.begin());
    for (const int i : path)
    {
      Pose12 O;
      std::copy(chain.joint_origin[i], chain.joint_origin[i] + 12, O.begin());
      T = poseMul(T, O);
    }
    return T;
  }
  auto it = static_frames.find(link);
  if (it == static_frames.end())
    throw std::runtime_error("unknown link " + link);
  return it->second;
}

void Environment::addJointGroup(KinematicGroup g)
{
  const std::string name = g.name;
  state_[name] = DblVec(static_cast<std::size_t>(g.chain.n_dof), 0.0);
  groups_[name] = std::make_shared<const KinematicGroup>(std::move(g));
}

KinematicGroup::ConstPtr Environment::getJointGroup(const std::string& name) const
{
  auto it = groups_.find(name);
  return it == groups_.end() ? nullptr : it->second;
}

DblVec Environment::getCurrentJointValues(const std::string& group) const
{
  auto it = state_.find(group);
  if (it == state_.end())
    throw std::runtime_error("unknown joint group " + group);
  return it->second;
}

void Environment::setState(const std::string& group, const DblVec& q)
{
  auto g = getJointGroup(group);
  if (!g || static_cast<int>(q.size()) != g->numJoints())
    throw std::runtime_error("setState: bad group or joint count");
  state_[group] = q;
}

// ------------------------------------------------------------ registry
void TermInfo::RegisterMaker(const std::string& type, MakerFunc f)
{
  if (!gRegisteredMakers)
    RegisterMakers();
  name2maker()[type] = f;
}

TermInfo::Ptr TermInfo::fromName(const std::string& type)
{
  if (!gRegisteredMakers)
    RegisterMakers();
  auto it = name2maker().find(type);
  if (it != name2maker().end())
    return (*it->second)();
  return {};
}

// ------------------------------------------------------------ ProblemConstructionInfo
ProblemConstructionInfo::ProblemConstructionInfo(Environment::ConstPtr e) : env(std::move(e))
{
  thip_default_osqp_settings(&osqp);
}

void ProblemConstructionInfo::readBasicInfo(const Json::Value& v)
{
  json_marshal::childFromJson(v, basic_info.n_steps, "n_steps");
  json_marshal::childFromJson(v, basic_info.manip, "manip");
  json_marshal::childFromJson(v, basic_info.fixed_timesteps, "fixed_timesteps", IntVec());
  json_marshal::childFromJson(v, basic_info.fixed_dofs, "fixed_dofs", IntVec());
  json_marshal::childFromJson(v, basic_info.convex_solver, "convex_solver", std::string("OSQP"));
  json_marshal::childFromJson(v, basic_info.dt_lower_lim, "dt_lower_lim", 1.0);
  json_marshal::childFromJson(v, basic_info.dt_upper_lim, "dt_upper_lim", 1.0);
  json_marshal::childFromJson(v, basic_info.use_time, "use_time", false);
  if (basic_info.dt_lower_lim <= 0 || basic_info.dt_upper_lim < basic_info.dt_lower_lim)
    throw std::runtime_error("dt limits (Basic Info) invalid. The lower limit must be positive, "
                             "and the minimum upper limit is equal to the lower limit.");
}

void ProblemConstructionInfo::readOptInfo(const Json::Value& v)
{
  auto& o = opt_info;
  json_marshal::childFromJson(v, o.improve_ratio_threshold, "improve_ratio_threshold", o.improve_ratio_threshold);
  json_marshal::childFromJson(v, o.min_trust_box_size, "min_trust_box_size", o.min_trust_box_size);
  json_marshal::childFromJson(v, o.min_approx_improve, "min_approx_improve", o.min_approx_improve);
  json_marshal::childFromJson(v, o.min_approx_improve_frac, "min_approx_improve_frac", o.min_approx_improve_frac);
  json_marshal::childFromJson(v, o.max_iter, "max_iter", o.max_iter);
  json_marshal::childFromJson(v, o.trust_shrink_ratio, "trust_shrink_ratio", o.trust_shrink_ratio);
  json_marshal::childFromJson(v, o.trust_expand_ratio, "trust_expand_ratio", o.trust_expand_ratio);
  json_marshal::childFromJson(v, o.cnt_tolerance, "cnt_tolerance", o.cnt_tolerance);
  json_marshal::childFromJson(v, o.max_merit_coeff_increases, "max_merit_coeff_increases",
                              o.max_merit_coeff_increases);
  json_marshal::childFromJson(v, o.merit_coeff_increase_ratio, "merit_coeff_increase_ratio",
                              o.merit_coeff_increase_ratio);
  json_marshal::childFromJson(v, o.max_time, "max_time", o.max_time);
  json_marshal::childFromJson(v, o.initial_merit_error_coeff, "initial_merit_error_coeff",
                              o.initial_merit_error_coeff);
  json_marshal::childFromJson(v, o.inflate_constraints_individually, "inflate_constraints_individually",
                              o.inflate_constraints_individually);
  json_marshal::childFromJson(v, o.trust_box_size, "trust_box_size", o.trust_box_size);
}

void ProblemConstructionInfo::readCosts(const Json::Value& v)
{
  cost_infos.clear();
  for (const auto& it : v)
  {
    std::string type;
    bool use_time = false;
    json_marshal::childFromJson(it, type, "type");
    json_marshal::childFromJson(it, use_time, "use_time", false);
    const TermInfo::Ptr term = TermInfo::fromName(type);
    if (!term)
      throw std::runtime_error("failed to construct cost named " + type);
    if (use_time)
    {
      term->term_type = TermType::TT_COST | TermType::TT_USE_TIME;
      basic_info.use_time = true;
    }
    else
      term->term_type = TermType::TT_COST;
    term->fromJson(*this, it);
    json_marshal::childFromJson(it, term->name, "name", type);
    cost_infos.push_back(term);
  }
}

void ProblemConstructionInfo::readConstraints(const Json::Value& v)
{
  cnt_infos.clear();
  for (const auto& it : v)
  {
    std::string type;
    bool use_time = false;
    json_marshal::childFromJson(it, type, "type");
    json_marshal::childFromJson(it, use_time, "use_time", false);
    const TermInfo::Ptr term = TermInfo::fromName(type);
    if (!term)
      throw std::runtime_error("failed to construct constraint named " + type);
    if (use_time)
    {
      term->term_type = TermType::TT_CNT | TermType::TT_USE_TIME;
      basic_info.use_time = true;
    }
    else
      term->term_type = TermType::TT_CNT;
    term->fromJson(*this, it);
    json_marshal::childFromJson(it, term->name, "name", type);
    cnt_infos.push_back(term);
  }
}

void ProblemConstructionInfo::readInitInfo(const Json::Value& v)
{
  std::string type_str;
  json_marshal::childFromJson(v, type_str, "type");
  json_marshal::childFromJson(v, init_info.dt, "dt", 1.0);
  const int n_steps = basic_info.n_steps;
  const int n_dof = kin->numJoints();
  if (iequals(type_str, "stationary"))
    init_info.type = InitInfo::STATIONARY;
  else if (iequals(type_str, "given_traj"))
  {
    init_info.type = InitInfo::GIVEN_TRAJ;
    if (!v.isMember("data"))
      throw std::runtime_error("init_info given_traj: missing data");
    const Json::Value& vdata = v["data"];
    if (static_cast<int>(vdata.size()) != n_steps)
      throw std::runtime_error("given initialization traj has wrong length");
    init_info.data.assign(static_cast<std::size_t>(n_steps), DblVec());
    for (int i = 0; i < n_steps; ++i)
      json_marshal::fromJsonArray(vdata[i], init_info.data[static_cast<std::size_t>(i)], n_dof);
  }
  else if (iequals(type_str, "joint_interpolated"))
  {
    init_info.type = InitInfo::JOINT_INTERPOLATED;
    if (!v.isMember("endpoint"))
      throw std::runtime_error("init_info joint_interpolated: missing endpoint");
    DblVec endpoint;
    json_marshal::childFromJson(v, endpoint, "endpoint");
    if (static_cast<int>(endpoint.size()) != n_dof)
      throw std::runtime_error("wrong number of dof values in initialization. expected " + std::to_string(n_dof) +
                               " got " + std::to_string(endpoint.size()));
    init_info.data = { endpoint };
  }
  else
    throw std::runtime_error("init_info did not have a valid type from Json. Valid types are "
                             "stationary, joint_interpolated, or given_traj");
}

void ProblemConstructionInfo::fromJson(const Json::Value& v)
{
  if (v.isMember("basic_info"))
    readBasicInfo(v["basic_info"]);
  else
    throw std::runtime_error("Json missing required section basic_info!");
  if (v.isMember("opt_info"))
    readOptInfo(v["opt_info"]);
  kin = env ? env->getJointGroup(basic_info.manip) : nullptr;
  if (!kin)
    throw std::runtime_error("Manipulator does not exist: " + basic_info.manip);
  if (v.isMember("costs"))
    readCosts(v["costs"]);
  if (v.isMember("constraints"))
    readConstraints(v["constraints"]);
  if (v.isMember("init_info"))
    readInitInfo(v["init_info"]);
  else
    throw std::runtime_error("Json missing required section init_info!");
}

// ------------------------------------------------------------ JointPos
void JointPosTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  if (!v.isMember("params"))
    throw std::runtime_error("JointPosTermInfo: missing params");
  const Json::Value& params = v["params"];
  const auto n_dof = static_cast<std::size_t>(pci.kin->numJoints());
  json_marshal::childFromJson(params, targets, "targets");
  json_marshal::childFromJson(params, coeffs, "coeffs", DblVec(n_dof, 1));
  json_marshal::childFromJson(params, upper_tols, "upper_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, lower_tols, "lower_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, first_step, "first_step", 0);
  json_marshal::childFromJson(params, last_step, "last_step", pci.basic_info.n_steps - 1);
  const char* all_fields[] = { "coeffs", "first_step", "last_step", "targets", "lower_tols", "upper_tols" };
  ensure_only_members(params, all_fields, sizeof(all_fields) / sizeof(char*));
}

// problem_description.cpp:1097-1196
void JointPosTermInfo::hatch(TrajOptProb& prob)
{
  const auto n_dof = static_cast<unsigned>(prob.GetNumDOF());
  if (coeffs.empty())
    coeffs = DblVec(n_dof, 1);
  if (upper_tols.empty())
    upper_tols = DblVec(n_dof, 0);
  if (lower_tols.empty())
    lower_tols = DblVec(n_dof, 0);
  if (last_step <= -1)
    last_step = prob.GetNumSteps() - 1;
  if ((prob.GetNumSteps() - 1) <= first_step)
    first_step = prob.GetNumSteps() - 1;
  if ((prob.GetNumSteps() - 1) <= last_step)
    last_step = prob.GetNumSteps() - 1;
  if (last_step < first_step)
    std::swap(first_step, last_step);
  checkParameterSize(coeffs, n_dof, "JointPosTermInfo coeffs", true);
  checkParameterSize(targets, n_dof, "JointPosTermInfo targets", true);
  checkParameterSize(upper_tols, n_dof, "JointPosTermInfo upper_tols", true);
  checkParameterSize(lower_tols, n_dof, "JointPosTermInfo lower_tols", true);
  // zero tolerances -> JointPosEq*, otherwise JointPosIneq* (thip_create applies the same
  // doubleEquals(tol, 0.) rule to the lowered tolerances)
  thip_problem_desc& d = prob.desc();
  if (d.n_jpos >= THIP_MAX_JPOS)
    unsupported("more than " + std::to_string(THIP_MAX_JPOS) + " JointPos terms");
  const int k = d.n_jpos++;
  d.jpos_is_cnt[k] = any(term_type & TermType::TT_COST) ? 0 : 1;
  d.jpos_first_step[k] = first_step;
  d.jpos_last_step[k] = last_step;
  for (unsigned j = 0; j < n_dof; ++j)
  {
    d.jpos_coeffs[k][j] = coeffs[j];
    d.jpos_upper_tols[k][j] = upper_tols[j];
    d.jpos_lower_tols[k][j] = lower_tols[j];
    d.jpos_targets[k][j] = 0.0;  // per problem: TrajOptProb::jpos_targets
    prob.jpos_targets.push_back(targets[j]);
  }
  addJointDiffObjects(prob, diffSpec(prob, 0, coeffs, targets, upper_tols, lower_tols, first_step, last_step),
                      !d.jpos_is_cnt[k], allZero(upper_tols) && allZero(lower_tols), name, true);
}

// ------------------------------------------------------------ JointVel
void JointVelTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  if (!v.isMember("params"))
    throw std::runtime_error("JointVelTermInfo: missing params");
  const Json::Value& params = v["params"];
  const auto n_dof = static_cast<std::size_t>(pci.kin->numJoints());
  json_marshal::childFromJson(params, targets, "targets");
  json_marshal::childFromJson(params, coeffs, "coeffs", DblVec(n_dof, 1));
  json_marshal::childFromJson(params, upper_tols, "upper_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, lower_tols, "lower_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, first_step, "first_step", 0);
  json_marshal::childFromJson(params, last_step, "last_step", pci.basic_info.n_steps - 1);
  const char* all_fields[] = { "coeffs", "first_step", "last_step", "targets", "lower_tols", "upper_tols", "use_time" };
  ensure_only_members(params, all_fields, sizeof(all_fields) / sizeof(char*));
}

// problem_description.cpp:1216-1391.  The kernel lowers the costs and the
// tolerance constraint (thip_create clamps the raw steps as below); an equality
// constraint goes to the jdt table and runs on the generic path.
void JointVelTermInfo::hatch(TrajOptProb& prob)
{
  const auto n_dof = static_cast<unsigned>(prob.GetNumDOF());
  if (coeffs.empty())
    coeffs = DblVec(n_dof, 1);
  if (upper_tols.empty())
    upper_tols = DblVec(n_dof, 0);
  if (lower_tols.empty())
    lower_tols = DblVec(n_dof, 0);
  int first = first_step, last = last_step;
  clampSteps(prob.GetNumSteps(), 1, first, last);
  checkParameterSize(coeffs, n_dof, "JointVelTermInfo coeffs", true);
  checkParameterSize(targets, n_dof, "JointVelTermInfo targets", true);
  checkParameterSize(upper_tols, n_dof, "JointVelTermInfo upper_tols", true);
  checkParameterSize(lower_tols, n_dof, "JointVelTermInfo lower_tols", true);
  // doubleEquals(tol, 0) (problem_description.cpp:1254-1257): zero tolerances -> the Eq forms
  const bool zero_tols = allZero(upper_tols) && allZero(lower_tols);
  const bool is_cost = any(term_type & TermType::TT_COST);
  if (any(term_type & TermType::TT_USE_TIME))
  {
    // :1263-1344: per joint, the (x_j, dt) columns of steps [first, last]
    thip_problem_desc& d = prob.desc();
    if (!prob.GetHasTime())
      throw std::runtime_error("A term is using time and basic_info is not set correctly. Try basic_info.use_time = "
                               "true");
    if (d.n_jvt >= THIP_MAX_JVT)
      unsupported("more than " + std::to_string(THIP_MAX_JVT) + " time-parameterised JointVel terms");
    const int k = d.n_jvt++;
    d.jvt_is_cnt[k] = is_cost ? 0 : 1;
    d.jvt_first_step[k] = first;
    d.jvt_last_step[k] = last;
    const int nv = last - first, D = prob.GetNumDOF();
    for (unsigned j = 0; j < n_dof; ++j)
    {
      d.jvt_coeffs[k][j] = coeffs[j];
      d.jvt_targets[k][j] = targets[j];
      d.jvt_upper_tols[k][j] = upper_tols[j];
      d.jvt_lower_tols[k][j] = lower_tols[j];
      sco::VarVector vars;
      for (int i = first; i <= last; ++i)
        vars.push_back(prob.GetVar(i, static_cast<int>(j)));
      for (int i = first; i <= last; ++i)
        vars.push_back(prob.GetVar(i, D));
      const DblVec c(static_cast<std::size_t>(2 * nv), coeffs[j]);
      const std::string nm = name + "_j" + std::to_string(j);
      auto f = jointVelTimeErr(targets[j], upper_tols[j], lower_tols[j]);
      if (is_cost)
        prob.addCost(std::make_shared<sco::CostFromErrFunc>(f, jointVelTimeJac(), vars, c,
                                                            zero_tols ? sco::SQUARED : sco::HINGE, nm));
      else
        prob.addConstraint(std::make_shared<sco::ConstraintFromErrFunc>(f, jointVelTimeJac(), vars, c,
                                                                        zero_tols ? sco::EQ : sco::INEQ, nm));
    }
    return;
  }
  const JointDiffSpec spec = diffSpec(prob, 1, coeffs, targets, upper_tols, lower_tols, first, last);
  thip_problem_desc& d = prob.desc();
  if (!is_cost && zero_tols)
  {
    addJointDiffTerm(prob, 1, false, coeffs, targets, upper_tols, lower_tols, first, last, name);
    return;
  }
  if (!zero_tols && (!is_cost || d.jv_enabled))
  {
    // JointVelIneqConstraint, or a further JointVelIneqCost: two hinge rows per (step, joint)
    if (d.n_jvx >= THIP_MAX_JVX)
      unsupported("more than " + std::to_string(THIP_MAX_JVX + 1) + " JointVel tolerance terms");
    const int x = d.n_jvx++;
    d.jvx_is_cnt[x] = is_cost ? 0 : 1;
    d.jvx_first_step[x] = first_step;
    d.jvx_last_step[x] = last_step;
    for (unsigned j = 0; j < n_dof; ++j)
    {
      d.jvx_coeffs[x][j] = coeffs[j];
      d.jvx_targets[x][j] = targets[j];
      d.jvx_upper_tols[x][j] = upper_tols[j];
      d.jvx_lower_tols[x][j] = lower_tols[j];
    }
    addJointDiffObjects(prob, spec, is_cost, false, name, true);
    return;
  }
  if (d.jv_enabled)
  {
    // a second JointVelEqCost: the generic path runs it (a jdt term of order 1;
    // the fused kernel's JointVel band holds one term)
    addJointDiffTerm(prob, 1, true, coeffs, targets, upper_tols, lower_tols, first, last, name);
    return;
  }
  d.jv_enabled = 1;
  d.jv_first_step = first_step;
  d.jv_last_step = last_step;
  for (unsigned j = 0; j < n_dof; ++j)
  {
    d.jv_coeffs[j] = coeffs[j];
    d.jv_targets[j] = targets[j];
    d.jv_upper_tols[j] = upper_tols[j];  // nonzero: JointVelIneqCost
    d.jv_lower_tols[j] = lower_tols[j];
  }
  addJointDiffObjects(prob, spec, true, zero_tols, name, true);
}

// ------------------------------------------------------------ JointAcc / JointJerk
namespace
{
void readJointDiffParams(ProblemConstructionInfo& pci, const Json::Value& v, const char* what, bool allow_use_time,
                         DblVec& coeffs, DblVec& targets, DblVec& upper_tols, DblVec& lower_tols, int& first_step,
                         int& last_step)
{
  if (!v.isMember("params"))
    throw std::runtime_error(std::string(what) + ": missing params");
  const Json::Value& params = v["params"];
  const auto n_dof = static_cast<std::size_t>(pci.kin->numJoints());
  json_marshal::childFromJson(params, targets, "targets");
  json_marshal::childFromJson(params, coeffs, "coeffs", DblVec(n_dof, 1));
  json_marshal::childFromJson(params, upper_tols, "upper_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, lower_tols, "lower_tols", DblVec(n_dof, 0));
  json_marshal::childFromJson(params, first_step, "first_step", 0);
  json_marshal::childFromJson(params, last_step, "last_step", pci.basic_info.n_steps - 1);
  // (JointJerkTermInfo's list has no "use_time", problem_description.cpp:1530)
  const char* all_fields[] = { "coeffs", "first_step", "last_step", "targets", "lower_tols", "upper_tols", "use_time" };
  ensure_only_members(params, all_fields, allow_use_time ? 7 : 6);
}

// problem_description.cpp:1412-1512 / 1534-1634
void hatchJointDiff(TrajOptProb& prob, TermType term_type, int order, const char* what, const std::string& name,
                    DblVec& coeffs, DblVec& targets, DblVec& upper_tols, DblVec& lower_tols, int& first_step,
                    int& last_step)
{
  const auto n_dof = static_cast<unsigned>(prob.GetNumDOF());
  if (coeffs.empty())
    coeffs = DblVec(n_dof, 1);
  if (upper_tols.empty())
    upper_tols = DblVec(n_dof, 0);
  if (lower_tols.empty())
    lower_tols = DblVec(n_dof, 0);
  clampSteps(prob.GetNumSteps(), order, first_step, last_step);
  const std::string w(what);
  checkParameterSize(coeffs, n_dof, w + " coeffs", true);
  checkParameterSize(targets, n_dof, w + " targets", true);
  checkParameterSize(upper_tols, n_dof, w + " upper_tols", true);
  checkParameterSize(lower_tols, n_dof, w + " lower_tols", true);
  if (any(term_type & TermType::TT_USE_TIME))
  {
    // the reference logs and adds nothing
    std::cerr << w << ": Use time version of this term has not been defined.\n";
    return;
  }
  addJointDiffTerm(prob, order, any(term_type & TermType::TT_COST), coeffs, targets, upper_tols, lower_tols,
                   first_step, last_step, name);
}
}  // namespace

void JointAccTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  readJointDiffParams(pci, v, "JointAccTermInfo", true, coeffs, targets, upper_tols, lower_tols, first_step,
                      last_step);
}
void JointAccTermInfo::hatch(TrajOptProb& prob)
{
  hatchJointDiff(prob, term_type, 2, "JointAccTermInfo", name, coeffs, targets, upper_tols, lower_tols, first_step,
                 last_step);
}
void JointJerkTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  readJointDiffParams(pci, v, "JointJerkTermInfo", false, coeffs, targets, upper_tols, lower_tols, first_step,
                      last_step);
}
void JointJerkTermInfo::hatch(TrajOptProb& prob)
{
  hatchJointDiff(prob, term_type, 3, "JointJerkTermInfo", name, coeffs, targets, upper_tols, lower_tols, first_step,
                 last_step);
}

// ------------------------------------------------------------ TotalTime
// problem_description.cpp:1860-1870
void TotalTimeTermInfo::fromJson(ProblemConstructionInfo&, const Json::Value& v)
{
  if (!v.isMember("params"))
    throw std::runtime_error("TotalTimeTermInfo: missing params");
  const Json::Value& params = v["params"];
  json_marshal::childFromJson(params, coeff, "coeff", 1.0);
  json_marshal::childFromJson(params, limit, "limit", 1.0);
  const char* all_fields[] = { "coeff", "limit" };
  ensure_only_members(params, all_fields, sizeof(all_fields) / sizeof(char*));
}

// :1872-1913: the last variable column (dt with use_time) of steps 1..N-1
void TotalTimeTermInfo::hatch(TrajOptProb& prob)
{
  thip_problem_desc& d = prob.desc();
  if (d.n_ttt >= THIP_MAX_TTT)
    unsupported("more than " + std::to_string(THIP_MAX_TTT) + " TotalTime terms");
  const bool is_cost = any(term_type & TermType::TT_COST);
  if (!is_cost && !any(term_type & TermType::TT_CNT))
    throw std::runtime_error("A valid term type was not specified in TotalTimeTermInfo");
  const int k = d.n_ttt++;
  d.ttt_is_cnt[k] = is_cost ? 0 : 1;
  d.ttt_coeff[k] = coeff;
  d.ttt_limit[k] = limit;
  const VarArray& tv = prob.GetVars();
  sco::VarVector vars;
  for (int i = 1; i < prob.GetNumSteps(); ++i)
    vars.push_back(tv(i, tv.n_cols - 1));
  const bool zero = std::fabs(limit) < 1e-5;  // doubleEquals(limit, 0)
  if (is_cost)
    prob.addCost(std::make_shared<sco::CostFromErrFunc>(totalTimeErr(limit), totalTimeJac(), vars, DblVec{ coeff },
                                                        zero ? sco::SQUARED : sco::HINGE, name));
  else
    prob.addConstraint(std::make_shared<sco::ConstraintFromErrFunc>(totalTimeErr(limit), totalTimeJac(), vars,
                                                                    DblVec{ coeff }, zero ? sco::EQ : sco::INEQ, name));
}

// ------------------------------------------------------------ CartPose
void CartPoseTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  if (!v.isMember("params"))
    throw std::runtime_error("CartPoseTermInfo: missing params");
  const Json::Value& params = v["params"];
  json_marshal::childFromJson(params, timestep, "timestep", pci.basic_info.n_steps - 1);
  readVec3(params, "pos_coeffs", pos_coeffs, { 1, 1, 1 });
  readVec3(params, "rot_coeffs", rot_coeffs, { 1, 1, 1 });
  json_marshal::childFromJson(params, source_frame, "source_frame");
  json_marshal::childFromJson(params, target_frame, "target_frame");
  std::array<double, 3> sxyz, txyz;
  std::array<double, 4> swxyz, twxyz;
  readVec3(params, "source_frame_offset_xyz", sxyz, { 0, 0, 0 });
  readVec4(params, "source_frame_offset_wxyz", swxyz, { 1, 0, 0, 0 });
  readVec3(params, "target_frame_offset_xyz", txyz, { 0, 0, 0 });
  readVec4(params, "target_frame_offset_wxyz", twxyz, { 1, 0, 0, 0 });
  source_frame_offset = poseFromXyzWxyz(sxyz, swxyz);
  target_frame_offset = poseFromXyzWxyz(txyz, twxyz);
  if (!pci.kin->hasLinkId(source_frame))
    throw std::runtime_error("invalid source frame: " + source_frame);
  if (!pci.kin->hasLinkId(target_frame))
    throw std::runtime_error("invalid target frame: " + target_frame);
  const bool source_active = pci.kin->isActiveLinkId(source_frame);
  const bool target_active = pci.kin->isActiveLinkId(target_frame);
  if (dynamic_)
  {
    if (!(source_active && target_active))
      throw std::runtime_error("source '" + source_frame + "' and target '" + target_frame +
                               "' are not both active links");
  }
  else if (source_active && target_active)
    throw std::runtime_error("source '" + source_frame + "' and target '" + target_frame + "' are both active");
  else if (!source_active && !target_active)
    throw std::runtime_error("source '" + source_frame + "' and target '" + target_frame + "' are both static");
  const char* all_fields[] = { "timestep",
                               "pos_coeffs",
                               "rot_coeffs",
                               "source_frame",
                               "target_frame",
                               "source_frame_offset_xyz",
                               "source_frame_offset_wxyz",
                               "target_frame_offset_xyz",
                               "target_frame_offset_wxyz" };
  ensure_only_members(params, all_fields, sizeof(all_fields) / sizeof(char*));
}

// problem_description.cpp:919-1005
void CartPoseTermInfo::hatch(TrajOptProb& prob)
{
  if (any(term_type & TermType::TT_USE_TIME))
  {
    // the reference logs and adds nothing (problem_description.cpp:948-955)
    std::cerr << "CartPoseTermInfo: Use time version of this term has not been defined.\n";
    return;
  }
  const auto kin = prob.GetKin();
  // is_target_active_ (kinematic_terms.cpp:206, 213-247, 313-339): the error is
  // calcTransformError(static, active) and the jacobian perturbs the active frame either way,
  // so an active target lowers as the kernel's active frame with the source as the static one
  const bool target_active = kin->isActiveLinkId(target_frame) && !dynamic_;
  if (!dynamic_ && target_active == kin->isActiveLinkId(source_frame))
    throw std::runtime_error("CartPoseTermInfo: source and target frames are both " +
                             std::string(target_active ? "active" : "static"));
  const std::string& active_frame = target_active ? target_frame : source_frame;
  const std::string& static_frame = target_active ? source_frame : target_frame;
  const Pose12& active_offset = target_active ? target_frame_offset : source_frame_offset;
  const Pose12& static_offset = target_active ? source_frame_offset : target_frame_offset;
  // validateTolerances (kinematic_terms.cpp:41-56), then the band is used unless both
  // bounds are empty or almost equal (:209-212)
  bool has_tol = false;
  if (!lower_tolerance.empty() || !upper_tolerance.empty())
  {
    if (lower_tolerance.size() != upper_tolerance.size())
      throw std::runtime_error("CartPoseErrCalculator: Mismatched tolerance sizes. lower: " +
                               std::to_string(lower_tolerance.size()) +
                               ", upper: " + std::to_string(upper_tolerance.size()));
    bool equal = true;
    for (std::size_t i = 0; i < lower_tolerance.size(); ++i)
    {
      if (lower_tolerance[i] > upper_tolerance[i])
        throw std::runtime_error("CartPoseErrCalculator: Inverted tolerance band - lower > upper at one or more "
                                 "indices");
      equal = equal && doubleEquals(lower_tolerance[i], upper_tolerance[i]);
    }
    if (!equal && lower_tolerance.size() != 6)
      throw std::runtime_error("CartPoseTermInfo: tolerances must have 6 entries (x, y, z, rx, ry, rz)");
    has_tol = !equal;
  }
  if (timestep < 0 || timestep >= prob.GetNumSteps())
    throw std::runtime_error("CartPoseTermInfo: timestep " + std::to_string(timestep) + " out of range");
  thip_problem_desc& d = prob.desc();
  if (d.n_cart >= THIP_MAX_CART)
    unsupported("more than " + std::to_string(THIP_MAX_CART) + " CartPose terms");
  const int k = d.n_cart++;
  d.cart_step[k] = timestep;
  d.cart_has_tol[k] = has_tol ? 1 : 0;
  for (int i = 0; has_tol && i < 6; ++i)
  {
    d.cart_lower_tol[k][i] = lower_tolerance[static_cast<std::size_t>(i)];
    d.cart_upper_tol[k][i] = upper_tolerance[static_cast<std::size_t>(i)];
  }
  d.cart_is_cnt[k] = any(term_type & TermType::TT_COST) ? 0 : 1;
  d.cart_source_link[k] = kin->linkIndex(active_frame);
  // DynamicCartPose: the target is an active link and its offset stays in that link's frame
  d.cart_target_link[k] = dynamic_ ? kin->linkIndex(target_frame) : 0;
  for (int i = 0; i < 12; ++i)
    d.cart_source_offset[k][i] = active_offset[static_cast<std::size_t>(i)];
  for (int i = 0; i < 3; ++i)
  {
    d.cart_pos_coeffs[k][i] = pos_coeffs[static_cast<std::size_t>(i)];
    d.cart_rot_coeffs[k][i] = rot_coeffs[static_cast<std::size_t>(i)];
  }
  // per-problem static frame pose: the offset in the chain root frame (the kernel forms
  // base_pose * offset)
  Pose12 off = static_offset;
  if (!dynamic_ && kin->linkIndex(static_frame) != 0)
  {
    Pose12 base;
    std::copy(kin->chain.base_pose, kin->chain.base_pose + 12, base.begin());
    off = poseMul(poseInv(base), poseMul(kin->staticWorldPose(static_frame), static_offset));
  }
  prob.cart_targets.insert(prob.cart_targets.end(), off.begin(), off.end());
  // the reference's TrajOptCostFromErrFunc / TrajOptConstraintFromErrFunc over the
  // waypoint's joints with the nonzero coefficients (problem_description.cpp:924-1005),
  // the error and its jacobian evaluated on the device (thip_eval_cart_pose)
  std::vector<int> indices;
  DblVec coeffs;
  for (int i = 0; i < 6; ++i)
  {
    const double cf = (i < 3) ? pos_coeffs[static_cast<std::size_t>(i)] : rot_coeffs[static_cast<std::size_t>(i - 3)];
    if (std::fabs(cf) > 1e-5)
    {
      indices.push_back(i);
      coeffs.push_back(cf);
    }
  }
  auto f = std::make_shared<CartPoseDeviceErr>(prob.deviceTerms(), k, indices);
  auto dfdx = std::make_shared<CartPoseDeviceJac>(prob.deviceTerms(), k, indices);
  const sco::VarVector vars = prob.GetVarRow(timestep, 0, prob.GetNumDOF());
  if (d.cart_is_cnt[k])
    prob.addLoweredConstraint(std::make_shared<DeviceCartPoseConstraint>(f, dfdx, vars, coeffs, sco::EQ, name));
  else
    prob.addLoweredCost(std::make_shared<DeviceCartPoseCost>(f, dfdx, vars, coeffs, sco::ABS, name));
}

// ------------------------------------------------------------ Collision
void CollisionTermInfo::fromJson(ProblemConstructionInfo& pci, const Json::Value& v)
{
  if (!v.isMember("params"))
    throw std::runtime_error("CollisionTermInfo: missing params");
  const Json::Value& params = v["params"];
  const int n_steps = pci.basic_info.n_steps;
  json_marshal::childFromJson(params, evaluator_type, "evaluator_type", 1);
  json_marshal::childFromJson(params, first_step, "first_step", 0);
  json_marshal::childFromJson(params, last_step, "last_step", n_steps - 1);
  json_marshal::childFromJson(params, longest_valid_segment_length, "longest_valid_segment_length", 0.5);
  // read, but not in all_fields below: a JSON that sets it is rejected (reference quirk,
  // problem_description.cpp:1649,1722-1732), so JSON problems always get 0.5
  json_marshal::childFromJson(params, collision_margin_buffer, "safety_margin_buffer", 0.5);
  if (!(longest_valid_segment_length >= 0) || !(first_step >= 0 && first_step < n_steps) ||
      !(last_step >= first_step && last_step < n_steps) || !(evaluator_type <= 4) || !(collision_margin_buffer >= 0))
    throw std::runtime_error("CollisionTermInfo: invalid params");
  json_marshal::childFromJson(params, fixed_steps, "fixed_steps", IntVec());
  for (int fs : fixed_steps)
    if (fs < first_step || fs > last_step)
      throw std::runtime_error("Fixed step " + std::to_string(fs) + " is not between first step " +
                               std::to_string(first_step) + " and last step " + std::to_string(last_step));
  json_marshal::childFromJson(params, contact_test_type, "contact_test_type", 2);
  if (contact_test_type < 0 || contact_test_type >= 3)
    throw std::runtime_error("CollisionTermInfo: invalid contact_test_type");
  json_marshal::childFromJson(params, coeff, "coeffs");
  json_marshal::childFromJson(params, dist_pen, "dist_pen");
  // problem_description.cpp:1686-1719: per link-pair margin / coefficient overrides,
  // validated as the reference does; lowered in hatch() (coll_pairs)
  pairs.clear();
  if (params.isMember("pairs"))
  {
    for (const Json::Value& it : params["pairs"])
    {
      if (!it.isMember("link"))
        throw std::runtime_error("expected true: it->isMember(\"link\")");
      std::string link;
      json_marshal::childFromJson(it, link, "link");
      if (!it.isMember("pair"))
        throw std::runtime_error("expected true: it->isMember(\"pair\")");
      std::vector<std::string> pair;
      json_marshal::childFromJson(it, pair, "pair");
      if (pair.empty())
        throw std::runtime_error("wrong size: pair. expected > 0 got " + std::to_string(pair.size()));
      double pair_coeffs = 20, pair_dist_pen = 0;
      json_marshal::childFromJson(it, pair_coeffs, "coeffs");
      json_marshal::childFromJson(it, pair_dist_pen, "dist_pen");
      for (const std::string& p : pair)
        pairs.push_back({ link, p, pair_coeffs, pair_dist_pen });
    }
  }
  const char* all_fields[] = { "type",           "first_step",        "last_step",
                               "evaluator_type", "fixed_steps",       "contact_test_type",
                               "longest_valid_segment_length", "coeffs", "dist_pen", "pairs" };
  ensure_only_members(params, all_fields, sizeof(all_fields) / sizeof(char*));
}

// problem_description.cpp:1735-1858: DISCRETE (single-timestep terms on the free waypoints),
// LVS_DISCRETE, CONTINUOUS and LVS_CONTINUOUS (step-pair terms)
void CollisionTermInfo::hatch(TrajOptProb& prob)
{
  // tesseract CollisionEvaluatorType {NONE, DISCRETE, LVS_DISCRETE, CONTINUOUS, LVS_CONTINUOUS}
  if (evaluator_type < 1 || evaluator_type > 4)
    unsupported("collision evaluator_type " + std::to_string(evaluator_type) +
                " (DISCRETE = 1, LVS_DISCRETE = 2, CONTINUOUS = 3, LVS_CONTINUOUS = 4 are)");
  const auto env = prob.GetEnv();
  thip_problem_desc& d = prob.desc();
  // the first collision term lowers into the descriptor's coll_* fields (the batched
  // kernel runs it), further ones into coll_extra (the generic path runs the problem)
  const bool extra = d.coll_enabled != 0;
  if (extra && d.n_coll_extra >= THIP_MAX_COLL_EXTRA)
    unsupported("more than " + std::to_string(THIP_MAX_COLL_EXTRA + 1) + " collision terms");
  const int n_steps = prob.GetNumSteps();
  for (int i = first_step; evaluator_type != 1 && i < last_step; ++i)
  {
    const bool a = std::find(fixed_steps.begin(), fixed_steps.end(), i) != fixed_steps.end();
    const bool b = std::find(fixed_steps.begin(), fixed_steps.end(), i + 1) != fixed_steps.end();
    if (a && b)
      throw std::runtime_error("Currently two adjacent fixed steps are not supported in collision term.");
  }
  // the robot spheres on the group's links (the other robot links are outside the joint group)
  std::vector<const CollisionSphere*> spheres;
  for (const auto& cs : env->collision_spheres)
    if (prob.GetKin()->linkIndex(cs.link) > 0)
      spheres.push_back(&cs);
  if (spheres.empty() || static_cast<int>(spheres.size()) > THIP_MAX_SPHERES)
    unsupported("a collision model with " + std::to_string(spheres.size()) + " spheres");
  // (a scene beyond THIP_MAX_PRIMS runs the generic path, TrajOptProb::lowerable)
  if (static_cast<int>(env->scene.size()) > THIP_EVAL_MAX_PRIMS)
    unsupported("a scene of more than " + std::to_string(THIP_EVAL_MAX_PRIMS) + " primitives");
  if (static_cast<int>(fixed_steps.size()) > THIP_MAX_STEPS)
    throw std::runtime_error("CollisionTermInfo: too many fixed steps");
  const bool is_cnt = !any(term_type & TermType::TT_COST);
  const int last = std::min(last_step, n_steps - 1);
  // CONTINUOUS casts each step pair once (lvs = max(), problem_description.cpp:1742-1744)
  // DISCRETE: SingleTimestepCollisionEvaluator per free waypoint (:1782-1796, :1842-1856)
  const int continuous = (evaluator_type == 1) ? 2 : (evaluator_type >= 3) ? 1 : 0;
  const double lvs = (evaluator_type == 3) ? 1.7976931348623157e308 : longest_valid_segment_length;
  const int term = extra ? 1 + d.n_coll_extra : 0;  // thip_eval's collision term index
  // tesseract ContactTestType {FIRST = 0, CLOSEST = 1, ALL = 2} -> THIP_CONTACT_* (ALL = 0)
  const int ctest = contact_test_type == 0 ? THIP_CONTACT_FIRST
                                           : (contact_test_type == 1 ? THIP_CONTACT_CLOSEST : THIP_CONTACT_ALL);
  if (extra)
  {
    thip_coll_term& x = d.coll_extra[d.n_coll_extra++];
    x.is_cnt = is_cnt ? 1 : 0;
    x.first_step = first_step;
    x.last_step = last;
    x.n_fixed = static_cast<int>(fixed_steps.size());
    for (std::size_t k = 0; k < fixed_steps.size(); ++k)
      x.fixed_steps[k] = fixed_steps[k];
    x.margin = dist_pen;
    x.coeff = coeff;
    x.buffer = collision_margin_buffer;
    x.lvs = lvs;
    x.continuous = continuous;
    x.contact_test = ctest;
  }
  else
  {
    d.coll_enabled = 1;
    d.coll_is_cnt = is_cnt ? 1 : 0;
    d.coll_first_step = first_step;
    d.coll_last_step = last;
    d.coll_n_fixed = static_cast<int>(fixed_steps.size());
    for (std::size_t k = 0; k < fixed_steps.size(); ++k)
      d.coll_fixed_steps[k] = fixed_steps[k];
    d.coll_margin = dist_pen;
    d.coll_coeff = coeff;
    d.coll_buffer = collision_margin_buffer;
    d.coll_continuous = continuous;
    d.coll_contact_test = ctest;
    d.coll_lvs = lvs;
  }
  // one CollisionCost / CollisionConstraint per unit, named <name>_<i> (:1735-1858)
  const int n_dof = prob.GetNumDOF();
  auto addUnit = [&](int i, bool single) {
    DeviceCollisionUnit u;
    u.ev = prob.deviceTerms();
    u.term = term;
    u.t = i;
    u.vars0 = prob.GetVarRow(i, 0, n_dof);
    if (!single)
      u.vars1 = prob.GetVarRow(i + 1, 0, n_dof);
    const std::string nm = name + "_" + std::to_string(i);
    if (is_cnt)
    {
      auto c = std::make_shared<DeviceCollisionConstraint>(std::move(u), nm);
      if (extra)
        prob.addConstraint(c);
      else
        prob.addLoweredConstraint(c);
    }
    else
    {
      auto c = std::make_shared<DeviceCollisionCost>(std::move(u), nm);
      if (extra)
        prob.addCost(c);
      else
        prob.addLoweredCost(c);
    }
  };
  auto fixedStep = [&](int i) { return std::find(fixed_steps.begin(), fixed_steps.end(), i) != fixed_steps.end(); };
  if (continuous == 2)
  {
    for (int i = first_step; i <= last; ++i)
      if (!fixedStep(i))
        addUnit(i, true);
  }
  else
    for (int i = first_step; i < last; ++i)
      addUnit(i, false);
  // "pairs": each named link pair's margin and coefficient for this term
  // (CollisionMarginData::setCollisionMargin / CollisionCoeffData::setCollisionCoeff,
  // problem_description.cpp:1707-1718), as (robot link, scene object) or (robot
  // link, robot link) entries of the descriptor; a name that is neither a link of
  // the group nor a scene object can be in no contact, so its entries do nothing
  auto lowerPairs = [&]() {
    const auto kin = prob.GetKin();
    for (const PairData& pd : pairs)
    {
      const int ra = kin->linkIndex(pd.link), rb = kin->linkIndex(pd.other);
      const int sa = env->sceneIndex(pd.link), sb = env->sceneIndex(pd.other);
      thip_coll_pair e{};
      e.term = term;
      if (ra > 0 && sb >= 0)
      {
        e.link = ra;
        e.other = sb;
      }
      else if (sa >= 0 && rb > 0)
      {
        e.link = rb;
        e.other = sa;
      }
      else if (ra > 0 && rb > 0)
      {
        e.link = ra;
        e.other = -1 - rb;
      }
      else
        continue;
      e.margin = pd.dist_pen;
      e.coeff = pd.coeff;
      // insert_or_assign: the pair's earlier entry of this term goes
      for (int k = 0; k < d.n_coll_pairs; ++k)
      {
        thip_coll_pair& o = d.coll_pairs[k];
        const bool same = o.term == e.term &&
                          ((o.link == e.link && o.other == e.other) ||
                           (e.other < 0 && o.other < 0 && o.link == -1 - e.other && -1 - o.other == e.link));
        if (same)
        {
          for (int j = k + 1; j < d.n_coll_pairs; ++j)
            d.coll_pairs[j - 1] = d.coll_pairs[j];
          --d.n_coll_pairs;
          break;
        }
      }
      if (d.n_coll_pairs >= THIP_MAX_COLL_PAIRS)
        unsupported("more than " + std::to_string(THIP_MAX_COLL_PAIRS) + " collision link pairs with their own data");
      d.coll_pairs[d.n_coll_pairs++] = e;
    }
  };
  if (extra)
  {
    // the robot model and the scene are the environment's, shared with the first term
    if (d.n_spheres != static_cast<int>(spheres.size()) || d.n_prims != static_cast<int>(env->scene.size()))
      throw std::runtime_error("CollisionTermInfo: collision terms of one problem must share the robot model and scene");
    lowerPairs();
    return;
  }
  d.n_spheres = static_cast<int>(spheres.size());
  for (int s = 0; s < d.n_spheres; ++s)
  {
    const CollisionSphere& cs = *spheres[static_cast<std::size_t>(s)];
    d.sphere_link[s] = prob.GetKin()->linkIndex(cs.link);
    for (int i = 0; i < 3; ++i)
      d.sphere_center[s][i] = cs.center[i];
    d.sphere_radius[s] = cs.radius;
  }
  d.n_prims = static_cast<int>(env->scene.size());
  for (const auto& p : env->scene)
    prob.scene.insert(prob.scene.end(), p.begin(), p.end());
  // self-collision: every pair of the group's sphere links (ascending link index) the
  // allowed-collision matrix does not disable -- the contact manager tests all its
  // active links against each other (collision_terms.cpp:817-898 via contactTest)
  std::vector<std::pair<int, std::string>> slinks;
  for (const CollisionSphere* cs : spheres)
  {
    const int li = prob.GetKin()->linkIndex(cs->link);
    if (std::find_if(slinks.begin(), slinks.end(), [&](const auto& e) { return e.first == li; }) == slinks.end())
      slinks.push_back({ li, cs->link });
  }
  std::sort(slinks.begin(), slinks.end());
  d.n_self_pairs = 0;
  for (std::size_t a = 0; a < slinks.size(); ++a)
    for (std::size_t b = a + 1; b < slinks.size(); ++b)
    {
      if (env->isCollisionAllowed(slinks[a].second, slinks[b].second))
        continue;
      if (d.n_self_pairs >= THIP_MAX_SELF_PAIRS)
        unsupported("more than " + std::to_string(THIP_MAX_SELF_PAIRS) + " self-collision link pairs");
      d.self_pair[d.n_self_pairs][0] = slinks[a].first;
      d.self_pair[d.n_self_pairs][1] = slinks[b].first;
      ++d.n_self_pairs;
    }
  lowerPairs();
}

// ------------------------------------------------------------ ConstructProblem
// problem_description.cpp:414-546 + generateInitTraj (:314-360)
TrajOptProb::Ptr ConstructProblem(const ProblemConstructionInfo& pci)
{
  const BasicInfo& bi = pci.basic_info;
  const int n_steps = bi.n_steps;
  if (!pci.kin)
    throw std::runtime_error("ConstructProblem: pci.kin is null");
  // problem_description.cpp:419-453
  bool use_time = false;
  for (const auto& ci : pci.cost_infos)
  {
    if (!any(ci->getSupportedTypes() & TermType::TT_COST))
      throw std::runtime_error(ci->name + " is only a constraint, but you listed it as a cost");
    if (any(ci->term_type & TermType::TT_USE_TIME))
    {
      use_time = true;
      if (!any(ci->getSupportedTypes() & TermType::TT_USE_TIME))
        throw std::runtime_error(ci->name + " does not support time, but you listed it as a using time");
    }
  }
  for (const auto& ci : pci.cnt_infos)
  {
    if (!any(ci->getSupportedTypes() & TermType::TT_CNT))
      throw std::runtime_error(ci->name + " is only a cost, but you listed it as a constraint");
    if (any(ci->term_type & TermType::TT_USE_TIME))
    {
      use_time = true;
      if (!any(ci->getSupportedTypes() & TermType::TT_USE_TIME))
        throw std::runtime_error(ci->name + " does not support time, but you listed it as a using time");
    }
  }
  if (use_time && !bi.use_time)
    throw std::runtime_error("A term is using time and basic_info is not set correctly. Try basic_info.use_time = "
                             "true");
  if (!use_time && bi.use_time)
    throw std::runtime_error("No terms use time and basic_info is not set correctly. Try basic_info.use_time = false");
  if (!iequals(bi.convex_solver, "OSQP") && !iequals(bi.convex_solver, "AUTO_SOLVER"))
    unsupported("convex_solver " + bi.convex_solver);
  // (the fused kernel takes n_steps <= THIP_MAX_STEPS; longer problems run the
  // generic path, whose device evaluator takes THIP_EVAL_MAX_STEPS)
  if (n_steps < 1 || n_steps > THIP_EVAL_MAX_STEPS)
    throw std::runtime_error("n_steps must be in [1, " + std::to_string(THIP_EVAL_MAX_STEPS) + "]");

  auto prob = std::make_shared<TrajOptProb>(n_steps, pci);
  thip_problem_desc& d = prob->desc_;
  const int n_dof = pci.kin->numJoints();

  // initial trajectory
  const DblVec start = pci.env->getCurrentJointValues(pci.kin->name);
  std::vector<DblVec> init;
  if (pci.init_info.type == InitInfo::STATIONARY)
    init.assign(static_cast<std::size_t>(n_steps), start);
  else if (pci.init_info.type == InitInfo::JOINT_INTERPOLATED)
  {
    if (pci.init_info.data.size() != 1 || static_cast<int>(pci.init_info.data[0].size()) != n_dof)
      throw std::runtime_error("JOINT_INTERPOLATED selected, but init_info.data is the wrong size. It should be 1 x "
                               "pci.kin->numJoints()");
    const DblVec& end = pci.init_info.data[0];
    init.assign(static_cast<std::size_t>(n_steps), DblVec(static_cast<std::size_t>(n_dof)));
    for (int j = 0; j < n_dof; ++j)
      for (int i = 0; i < n_steps; ++i)
        init[static_cast<std::size_t>(i)][static_cast<std::size_t>(j)] =
            linspaced(n_steps, start[static_cast<std::size_t>(j)], end[static_cast<std::size_t>(j)], i);
  }
  else
    init = pci.init_info.data;
  if (static_cast<int>(init.size()) != n_steps)
    throw std::runtime_error("initial trajectory has " + std::to_string(init.size()) + " rows, expected " +
                             std::to_string(n_steps));
  for (const auto& row : init)
    if (static_cast<int>(row.size()) != n_dof)
      throw std::runtime_error("initial trajectory row has the wrong number of dofs");
  // with use_time, the constant init dt column (problem_description.cpp:372-379)
  if (bi.use_time)
    for (auto& row : init)
      row.push_back(pci.init_info.dt);
  prob->init_ = init;
  d.use_time = bi.use_time ? 1 : 0;
  if (bi.use_time)  // (zero otherwise: the descriptor of a problem without time is unchanged)
  {
    d.dt_lower = bi.dt_lower_lim;
    d.dt_upper = bi.dt_upper_lim;
    d.init_dt = pci.init_info.dt;
  }

  // fixed timesteps (problem_description.cpp:489-510)
  if (bi.fixed_timesteps.size() > THIP_MAX_STEPS)
    throw std::runtime_error("too many fixed timesteps");
  for (int t : bi.fixed_timesteps)
  {
    if (t < 0 || t >= n_steps)
      throw std::runtime_error("Fixed timestep index is outside the bounds of the initial trajectory.");
    d.fixed_steps[d.n_fixed++] = t;
    for (int j = 0; j < n_dof; ++j)
      prob->addLinearConstraint(
          sco::exprSub(sco::AffExpr(prob->GetVar(t, j)), init[static_cast<std::size_t>(t)][static_cast<std::size_t>(j)]),
          sco::EQ);
  }
  // fixed dofs (:528-546): the joint pinned to the initial trajectory at every
  // step that is not a fixed timestep
  if (bi.fixed_dofs.size() > THIP_MAX_DOF)
    throw std::runtime_error("too many fixed dofs");
  for (int dof : bi.fixed_dofs)
  {
    // (the reference tests n_dof < dof; a dof equal to n_dof would index past the joints)
    if (dof < 0 || dof >= n_dof)
      throw std::runtime_error("DOF(aka Joint) indice is greater than the number of DOF available.");
    d.fixed_dofs[d.n_fixed_dofs++] = dof;
    for (int i = 0; i < n_steps; ++i)
    {
      if (std::find(bi.fixed_timesteps.begin(), bi.fixed_timesteps.end(), i) != bi.fixed_timesteps.end())
        continue;
      prob->addLinearConstraint(sco::exprSub(sco::AffExpr(prob->GetVar(i, dof)),
                                             sco::AffExpr(init[static_cast<std::size_t>(i)][static_cast<std::size_t>(dof)])),
                                sco::EQ);
    }
  }

  // optimizer parameters: BasicTrustRegionSQP(prob) takes them from the caller
  // in the reference; here they travel with the problem (opt_info)
  const auto& o = pci.opt_info;
  d.sqp.improve_ratio_threshold = o.improve_ratio_threshold;
  d.sqp.min_trust_box_size = o.min_trust_box_size;
  d.sqp.min_approx_improve = o.min_approx_improve;
  d.sqp.min_approx_improve_frac = o.min_approx_improve_frac;
  d.sqp.max_iter = o.max_iter;
  d.sqp.trust_shrink_ratio = o.trust_shrink_ratio;
  d.sqp.trust_expand_ratio = o.trust_expand_ratio;
  d.sqp.cnt_tolerance = o.cnt_tolerance;
  d.sqp.max_merit_coeff_increases = o.max_merit_coeff_increases;
  d.sqp.max_qp_solver_failures = o.max_qp_solver_failures;
  d.sqp.merit_coeff_increase_ratio = o.merit_coeff_increase_ratio;
  d.sqp.initial_merit_error_coeff = o.initial_merit_error_coeff;
  d.sqp.inflate_constraints_individually = o.inflate_constraints_individually ? 1 : 0;
  d.sqp.trust_box_size = o.trust_box_size;
  d.sqp.max_time = o.max_time;
  d.osqp = pci.osqp;

  for (const auto& ci : pci.cost_infos)
    ci->hatch(*prob);
  for (const auto& ci : pci.cnt_infos)
    ci->hatch(*prob);
  return prob;
}

// ------------------------------------------------------------ TrajOptProb
// problem_description.cpp:557-598: the j_i_j variables with the joint limits as bounds
TrajOptProb::TrajOptProb(int n_steps, const ProblemConstructionInfo& pci)
  : sco::OptProb(sco::ModelType::OSQP, modelConfig(pci))
  , kin_(pci.kin)
  , env_(pci.env)
  , device_terms_(std::make_shared<DeviceTermEvaluator>(this))
{
  if (!kin_)
    throw std::runtime_error("TrajOptProb: pci.kin is null");
  const int n_dof = kin_->numJoints();
  std::memset(&desc_, 0, sizeof(desc_));
  desc_.abi_version = THIP_ABI_VERSION;
  desc_.n_steps = n_steps;
  desc_.chain = kin_->chain;
  desc_.use_time = pci.basic_info.use_time ? 1 : 0;
  const int W = n_dof + desc_.use_time;
  std::vector<std::string> names;
  DblVec lb, ub;
  for (int i = 0; i < n_steps; ++i)
  {
    for (int j = 0; j < n_dof; ++j)
    {
      names.push_back("j_" + std::to_string(i) + "_" + std::to_string(j));
      lb.push_back(kin_->chain.lower[j]);
      ub.push_back(kin_->chain.upper[j]);
    }
    if (desc_.use_time)
    {
      names.push_back("dt_" + std::to_string(i));
      lb.push_back(pci.basic_info.dt_lower_lim);
      ub.push_back(pci.basic_info.dt_upper_lim);
    }
  }
  traj_vars_.n_rows = n_steps;
  traj_vars_.n_cols = W;
  traj_vars_.data = createVariables(names, lb, ub);
  joint_vars_.n_rows = n_steps;
  joint_vars_.n_cols = n_dof;
  for (int i = 0; i < n_steps; ++i)
    for (int j = 0; j < n_dof; ++j)
      joint_vars_.data.push_back(traj_vars_(i, j));
}

void TrajOptProb::addLoweredCost(sco::Cost::Ptr c)
{
  lowered_.push_back(c.get());
  addCost(std::move(c));
}

void TrajOptProb::addLoweredConstraint(sco::Constraint::Ptr c)
{
  lowered_.push_back(c.get());
  addConstraint(std::move(c));
}

std::string TrajOptProb::unloweredTerms() const
{
  std::string out;
  auto note = [&](const std::string& n) { out += (out.empty() ? "" : ", ") + ("'" + n + "'"); };
  for (const auto& c : costs_)
    if (std::find(lowered_.begin(), lowered_.end(), c.get()) == lowered_.end())
      note(c->name());
  for (const auto& c : getConstraints())
    if (std::find(lowered_.begin(), lowered_.end(), c.get()) == lowered_.end())
      note(c->name());
  return out;
}

bool TrajOptProb::lowerable() const
{
  // the fused kernel's domain: at most THIP_MAX_STEPS waypoints and THIP_MAX_PRIMS
  // scene primitives, and no term it does not lower
  return desc_.n_steps >= 2 && desc_.n_steps <= THIP_MAX_STEPS && desc_.n_prims <= THIP_MAX_PRIMS &&
         thip_jdt_fused(&desc_) && desc_.n_jvt == 0 && desc_.n_ttt == 0 && !desc_.use_time && desc_.n_fixed_dofs == 0 &&
         desc_.n_coll_extra == 0 && unloweredTerms().empty();
}

LoweredProblem TrajOptProb::lowered() const
{
  LoweredProblem lp;
  lp.desc = desc_;
  for (const auto& row : init_)  // the joint columns
    lp.init.insert(lp.init.end(), row.begin(), row.begin() + GetNumDOF());
  lp.cart_targets = cart_targets;
  lp.jpos_targets = jpos_targets;
  lp.scene = scene;
  return lp;
}

TrajOptProb::Ptr ConstructProblem(const Json::Value& root, const Environment::ConstPtr& env)
{
  ProblemConstructionInfo pci(env);
  pci.fromJson(root);
  return ConstructProblem(pci);
}
}  // namespace trajopt
