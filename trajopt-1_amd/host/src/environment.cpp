// Built-in environment: the PR2 arms of the reference's test data
// (trajopt_common/data/arm_around_table.urdf joints; pr2.srdf groups
// "right_arm" / "left_arm": torso_lift_link -> *_gripper_tool_frame, and
// "both_arms", the two as one 14-joint tree), the same numbers as
// trajopt_amd/robots.py, and the 14-sphere-per-arm collision model of
// trajopt_amd/scene.py (PR2_ARM_SPHERES).
#include <cmath>
#include <string>
#include <vector>

#include "trajopt_amd/problem_description.hpp"

namespace trajopt
{
namespace
{
struct JointRow
{
  std::string joint;
  std::string child;
  int type;
  double xyz[3];
  double axis[3];
  double lower, upper;
};

// One arm's joints, torso_lift_link -> *_gripper_tool_frame (11 joints, 7 movable).
void armRows(bool left, std::vector<JointRow>& rows)
{
  const double kPi4 = 4 * M_PI;
  const double y = left ? 0.188 : -0.188;
  // l_shoulder_pan 2396-2402 / r 1479-1485; l_upper_arm_roll 2462-2468 / r 1545-1550
  const double pan_lo = left ? -0.714601836603 : -2.2853981634, pan_hi = left ? 2.2853981634 : 0.714601836603;
  const double roll_lo = left ? -0.8 : -3.9, roll_hi = left ? 3.9 : 0.8;
  const char* p = left ? "l_" : "r_";
  auto n = [&](const char* base) { return std::string(p) + base; };
  rows.push_back({ n("shoulder_pan_joint"), n("shoulder_pan_link"), THIP_JOINT_REVOLUTE, { 0.0, y, 0.0 }, { 0, 0, 1 },
                   pan_lo, pan_hi });
  rows.push_back({ n("shoulder_lift_joint"), n("shoulder_lift_link"), THIP_JOINT_REVOLUTE, { 0.1, 0.0, 0.0 },
                   { 0, 1, 0 }, -0.5236, 1.3963 });
  rows.push_back({ n("upper_arm_roll_joint"), n("upper_arm_roll_link"), THIP_JOINT_REVOLUTE, { 0, 0, 0 }, { 1, 0, 0 },
                   roll_lo, roll_hi });
  rows.push_back({ n("upper_arm_joint"), n("upper_arm_link"), THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 });
  rows.push_back({ n("elbow_flex_joint"), n("elbow_flex_link"), THIP_JOINT_REVOLUTE, { 0.4, 0.0, 0.0 }, { 0, 1, 0 },
                   -2.3213, 0.0 });
  rows.push_back({ n("forearm_roll_joint"), n("forearm_roll_link"), THIP_JOINT_CONTINUOUS, { 0, 0, 0 }, { 1, 0, 0 },
                   -kPi4, kPi4 });
  rows.push_back({ n("forearm_joint"), n("forearm_link"), THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 });
  rows.push_back({ n("wrist_flex_joint"), n("wrist_flex_link"), THIP_JOINT_REVOLUTE, { 0.321, 0.0, 0.0 }, { 0, 1, 0 },
                   -2.18, 0.0 });
  rows.push_back({ n("wrist_roll_joint"), n("wrist_roll_link"), THIP_JOINT_CONTINUOUS, { 0, 0, 0 }, { 1, 0, 0 },
                   -kPi4, kPi4 });
  rows.push_back({ n("gripper_palm_joint"), n("gripper_palm_link"), THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 });
  rows.push_back({ n("gripper_tool_joint"), n("gripper_tool_frame"), THIP_JOINT_FIXED, { 0.18, 0.0, 0.0 },
                   { 0, 0, 0 }, 0, 0 });
}

// A joint group of one or two arms off torso_lift_link (each arm a branch of
// the tree rooted at the group's link 0).
KinematicGroup makeGroup(const std::string& name, const std::vector<bool>& arms_left)
{
  KinematicGroup g;
  g.name = name;
  thip_chain& c = g.chain;
  const double eye[12] = { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 };
  // world pose of torso_lift_link: base_footprint -> base_link (0, 0, 0.051) -> torso (-0.05, 0, 0.739675)
  for (int i = 0; i < 12; ++i)
    c.base_pose[i] = eye[i];
  c.base_pose[3] = -0.05;
  c.base_pose[7] = 0.0;
  c.base_pose[11] = 0.051 + 0.739675;
  c.joint_dof[0] = -1;
  c.parent[0] = 0;
  c.is_tree = arms_left.size() > 1 ? 1 : 0;
  g.link_names.push_back("torso_lift_link");
  int dof = 0, k = 1;
  for (const bool left : arms_left)
  {
    std::vector<JointRow> rows;
    armRows(left, rows);
    int prev = 0;  // each arm hangs off the root
    for (const auto& r : rows)
    {
      c.joint_type[k] = r.type;
      c.parent[k] = prev;
      for (int i = 0; i < 12; ++i)
        c.joint_origin[k][i] = eye[i];
      c.joint_origin[k][3] = r.xyz[0];
      c.joint_origin[k][7] = r.xyz[1];
      c.joint_origin[k][11] = r.xyz[2];
      if (r.type == THIP_JOINT_FIXED)
        c.joint_dof[k] = -1;
      else
      {
        c.joint_dof[k] = dof;
        for (int i = 0; i < 3; ++i)
          c.joint_axis[k][i] = r.axis[i];
        c.lower[dof] = r.lower;
        c.upper[dof] = r.upper;
        g.joint_names.push_back(r.joint);
        ++dof;
      }
      g.link_names.push_back(r.child);
      prev = k;
      ++k;
    }
  }
  c.n_links = k;
  c.n_dof = dof;
  std::array<double, 12> bf{}, bl{};
  for (int i = 0; i < 12; ++i)
    bf[static_cast<std::size_t>(i)] = bl[static_cast<std::size_t>(i)] = eye[i];
  bl[11] = 0.051;
  g.static_frames["base_footprint"] = bf;
  g.static_frames["base_link"] = bl;
  return g;
}
}  // namespace

Environment::Ptr Environment::makePR2()
{
  auto env = std::make_shared<Environment>();
  // pr2.srdf:12-17 left_arm / right_arm; both_arms = the two chains as one
  // 14-joint group (left arm first), branching at torso_lift_link
  env->addJointGroup(makeGroup("right_arm", { false }));
  env->addJointGroup(makeGroup("left_arm", { true }));
  env->addJointGroup(makeGroup("both_arms", { true, false }));
  // 2 spheres per moving arm link (link, center in the link frame, radius),
  // trajopt_amd/scene.py PR2_ARM_SPHERES; the left arm mirrors the right
  const char* links[] = { "shoulder_pan_link", "shoulder_pan_link", "shoulder_lift_link", "shoulder_lift_link",
                          "upper_arm_roll_link", "upper_arm_roll_link", "elbow_flex_link", "elbow_flex_link",
                          "forearm_roll_link", "forearm_roll_link", "wrist_flex_link", "wrist_flex_link",
                          "wrist_roll_link", "wrist_roll_link" };
  const double cx[] = { 0.0, 0.1, 0.0, 0.1, 0.15, 0.3, 0.0, 0.08, 0.12, 0.24, 0.0, 0.08, 0.12, 0.18 };
  const double rad[] = { 0.09, 0.08, 0.08, 0.07, 0.07, 0.07, 0.07, 0.06, 0.06, 0.06, 0.06, 0.06, 0.06, 0.06 };
  for (const char* side : { "l_", "r_" })
    for (int s = 0; s < 14; ++s)
      env->collision_spheres.push_back({ std::string(side) + links[s], { cx[s], 0.0, 0.0 }, rad[s] });
  // pr2.srdf <disable_collisions> (trajopt_common/data/pr2.srdf:752-1036) between the
  // sphere-carrying arm links; the pairs it leaves enabled are the self-collision pairs
  // (each arm's shoulder_pan vs its wrist links, and most left-vs-right pairs)
  static const char* const acm[][2] = {
    { "l_elbow_flex_link", "l_forearm_roll_link" },      { "l_elbow_flex_link", "l_shoulder_lift_link" },
    { "l_elbow_flex_link", "l_shoulder_pan_link" },      { "l_elbow_flex_link", "l_upper_arm_roll_link" },
    { "l_elbow_flex_link", "l_wrist_flex_link" },        { "l_elbow_flex_link", "l_wrist_roll_link" },
    { "l_elbow_flex_link", "r_shoulder_lift_link" },     { "l_elbow_flex_link", "r_shoulder_pan_link" },
    { "l_elbow_flex_link", "r_upper_arm_roll_link" },    { "l_forearm_roll_link", "l_shoulder_lift_link" },
    { "l_forearm_roll_link", "l_shoulder_pan_link" },    { "l_forearm_roll_link", "l_upper_arm_roll_link" },
    { "l_forearm_roll_link", "l_wrist_flex_link" },      { "l_forearm_roll_link", "l_wrist_roll_link" },
    { "l_forearm_roll_link", "r_shoulder_lift_link" },   { "l_forearm_roll_link", "r_shoulder_pan_link" },
    { "l_forearm_roll_link", "r_upper_arm_roll_link" },  { "l_shoulder_lift_link", "l_shoulder_pan_link" },
    { "l_shoulder_lift_link", "l_upper_arm_roll_link" }, { "l_shoulder_lift_link", "l_wrist_flex_link" },
    { "l_shoulder_lift_link", "l_wrist_roll_link" },     { "l_shoulder_lift_link", "r_elbow_flex_link" },
    { "l_shoulder_lift_link", "r_forearm_roll_link" },   { "l_shoulder_lift_link", "r_shoulder_lift_link" },
    { "l_shoulder_lift_link", "r_upper_arm_roll_link" }, { "l_shoulder_pan_link", "l_upper_arm_roll_link" },
    { "l_shoulder_pan_link", "r_elbow_flex_link" },      { "l_shoulder_pan_link", "r_forearm_roll_link" },
    { "l_upper_arm_roll_link", "l_wrist_flex_link" },    { "l_upper_arm_roll_link", "l_wrist_roll_link" },
    { "l_upper_arm_roll_link", "r_elbow_flex_link" },    { "l_upper_arm_roll_link", "r_forearm_roll_link" },
    { "l_upper_arm_roll_link", "r_shoulder_lift_link" }, { "l_upper_arm_roll_link", "r_upper_arm_roll_link" },
    { "l_wrist_flex_link", "l_wrist_roll_link" },        { "r_elbow_flex_link", "r_forearm_roll_link" },
    { "r_elbow_flex_link", "r_shoulder_lift_link" },     { "r_elbow_flex_link", "r_shoulder_pan_link" },
    { "r_elbow_flex_link", "r_upper_arm_roll_link" },    { "r_elbow_flex_link", "r_wrist_flex_link" },
    { "r_elbow_flex_link", "r_wrist_roll_link" },        { "r_forearm_roll_link", "r_shoulder_lift_link" },
    { "r_forearm_roll_link", "r_shoulder_pan_link" },    { "r_forearm_roll_link", "r_upper_arm_roll_link" },
    { "r_forearm_roll_link", "r_wrist_flex_link" },      { "r_forearm_roll_link", "r_wrist_roll_link" },
    { "r_shoulder_lift_link", "r_shoulder_pan_link" },   { "r_shoulder_lift_link", "r_upper_arm_roll_link" },
    { "r_shoulder_lift_link", "r_wrist_flex_link" },     { "r_shoulder_lift_link", "r_wrist_roll_link" },
    { "r_shoulder_pan_link", "r_upper_arm_roll_link" },  { "r_upper_arm_roll_link", "r_wrist_flex_link" },
    { "r_upper_arm_roll_link", "r_wrist_roll_link" },    { "r_wrist_flex_link", "r_wrist_roll_link" },
  };
  for (const auto& pr : acm)
    env->allowCollision(pr[0], pr[1]);
  return env;
}

void Environment::addSceneObject(const std::string& name, const std::array<double, 16>& rec)
{
  scene_names.resize(scene.size());
  scene.push_back(rec);
  scene_names.push_back(name);
}

std::string Environment::sceneName(std::size_t k) const
{
  if (k < scene_names.size() && !scene_names[k].empty())
    return scene_names[k];
  return "scene_" + std::to_string(k);
}

int Environment::sceneIndex(const std::string& name) const
{
  for (std::size_t k = 0; k < scene.size(); ++k)
    if (sceneName(k) == name)
      return static_cast<int>(k);
  return -1;
}

void Environment::allowCollision(const std::string& a, const std::string& b)
{
  allowed_collisions.insert(a < b ? std::make_pair(a, b) : std::make_pair(b, a));
}

bool Environment::isCollisionAllowed(const std::string& a, const std::string& b) const
{
  return allowed_collisions.count(a < b ? std::make_pair(a, b) : std::make_pair(b, a)) != 0;
}

// trajopt_common/data/spherebot.urdf / spherebot.srdf: group "manipulator" =
// base_link -> spherebot_link over two prismatic joints (x, then y; limits
// +-20), a 0.5 m sphere on spherebot_link; the static test spheres (0.5 m) at
// the origin (test_sphere_link), (-0.75, 0, 0) and (0, 0.75, 0) off base_link.
Environment::Ptr Environment::makeSpherebot()
{
  auto env = std::make_shared<Environment>();
  KinematicGroup g;
  g.name = "manipulator";
  thip_chain& c = g.chain;
  const double eye[12] = { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 };
  for (int i = 0; i < 12; ++i)
    c.base_pose[i] = eye[i];
  c.is_tree = 0;
  c.joint_dof[0] = -1;
  g.link_names = { "base_link", "spherebot_linkX", "spherebot_linkY", "spherebot_link" };
  const int types[] = { 0, THIP_JOINT_PRISMATIC, THIP_JOINT_PRISMATIC, THIP_JOINT_FIXED };
  const double axes[][3] = { { 0, 0, 0 }, { 1, 0, 0 }, { 0, 1, 0 }, { 0, 0, 0 } };
  for (int k = 1; k < 4; ++k)
  {
    c.joint_type[k] = types[k];
    c.parent[k] = k - 1;
    for (int i = 0; i < 12; ++i)
      c.joint_origin[k][i] = eye[i];
    c.joint_dof[k] = types[k] == THIP_JOINT_FIXED ? -1 : k - 1;
    for (int i = 0; i < 3; ++i)
      c.joint_axis[k][i] = axes[k][i];
  }
  c.n_links = 4;
  c.n_dof = 2;
  for (int j = 0; j < 2; ++j)
  {
    c.lower[j] = -20.0;
    c.upper[j] = 20.0;
  }
  g.joint_names = { "spherebot_x_joint", "spherebot_y_joint" };
  env->addJointGroup(std::move(g));
  env->collision_spheres.push_back({ "spherebot_link", { 0.0, 0.0, 0.0 }, 0.5 });
  const double centers[][3] = { { 0.0, 0.0, 0.0 }, { -0.75, 0.0, 0.0 }, { 0.0, 0.75, 0.0 } };
  const char* names[] = { "test_sphere_link", "test_sphere_link2", "test_sphere_link3" };  // spherebot.urdf:42-105
  for (int k = 0; k < 3; ++k)
  {
    std::array<double, 16> rec{};
    rec[0] = THIP_PRIM_SPHERE;
    rec[1] = centers[k][0];
    rec[2] = centers[k][1];
    rec[3] = centers[k][2];
    rec[4] = 0.5;
    env->addSceneObject(names[k], rec);
  }
  return env;
}

Environment::Ptr Environment::builtin(const std::string& manip)
{
  return manip == "manipulator" ? makeSpherebot() : makePR2();
}
}  // namespace trajopt
