// Built-in environment: the PR2 right arm of the reference's test data
// (trajopt_common/data/arm_around_table.urdf joints, pr2.srdf group
// "right_arm": torso_lift_link -> r_gripper_tool_frame), the same numbers as
// trajopt_amd/robots.py and the 14-sphere collision model of
// trajopt_amd/scene.py (PR2_ARM_SPHERES).
#include <cmath>

#include "trajopt_amd/problem_description.hpp"

namespace trajopt
{
namespace
{
struct JointRow
{
  const char* joint;
  const char* child;
  int type;
  double xyz[3];
  double axis[3];
  double lower, upper;
};
}  // namespace

Environment::Ptr Environment::makePR2()
{
  const double kPi4 = 4 * M_PI;
  const JointRow rows[] = {
    { "r_shoulder_pan_joint", "r_shoulder_pan_link", THIP_JOINT_REVOLUTE, { 0.0, -0.188, 0.0 }, { 0, 0, 1 },
      -2.2853981634, 0.714601836603 },
    { "r_shoulder_lift_joint", "r_shoulder_lift_link", THIP_JOINT_REVOLUTE, { 0.1, 0.0, 0.0 }, { 0, 1, 0 }, -0.5236,
      1.3963 },
    { "r_upper_arm_roll_joint", "r_upper_arm_roll_link", THIP_JOINT_REVOLUTE, { 0, 0, 0 }, { 1, 0, 0 }, -3.9, 0.8 },
    { "r_upper_arm_joint", "r_upper_arm_link", THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 },
    { "r_elbow_flex_joint", "r_elbow_flex_link", THIP_JOINT_REVOLUTE, { 0.4, 0.0, 0.0 }, { 0, 1, 0 }, -2.3213, 0.0 },
    { "r_forearm_roll_joint", "r_forearm_roll_link", THIP_JOINT_CONTINUOUS, { 0, 0, 0 }, { 1, 0, 0 }, -kPi4, kPi4 },
    { "r_forearm_joint", "r_forearm_link", THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 },
    { "r_wrist_flex_joint", "r_wrist_flex_link", THIP_JOINT_REVOLUTE, { 0.321, 0.0, 0.0 }, { 0, 1, 0 }, -2.18, 0.0 },
    { "r_wrist_roll_joint", "r_wrist_roll_link", THIP_JOINT_CONTINUOUS, { 0, 0, 0 }, { 1, 0, 0 }, -kPi4, kPi4 },
    { "r_gripper_palm_joint", "r_gripper_palm_link", THIP_JOINT_FIXED, { 0, 0, 0 }, { 0, 0, 0 }, 0, 0 },
    { "r_gripper_tool_joint", "r_gripper_tool_frame", THIP_JOINT_FIXED, { 0.18, 0.0, 0.0 }, { 0, 0, 0 }, 0, 0 },
  };
  KinematicGroup g;
  g.name = "right_arm";
  thip_chain& c = g.chain;
  const double eye[12] = { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 };
  // world pose of torso_lift_link: base_footprint -> base_link (0, 0, 0.051) -> torso (-0.05, 0, 0.739675)
  for (int i = 0; i < 12; ++i)
    c.base_pose[i] = eye[i];
  c.base_pose[3] = -0.05;
  c.base_pose[7] = 0.0;
  c.base_pose[11] = 0.051 + 0.739675;
  c.joint_dof[0] = -1;
  g.link_names.push_back("torso_lift_link");
  int dof = 0, k = 1;
  for (const auto& r : rows)
  {
    c.joint_type[k] = r.type;
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
    ++k;
  }
  c.n_links = k;
  c.n_dof = dof;
  std::array<double, 12> bf{}, bl{};
  for (int i = 0; i < 12; ++i)
    bf[static_cast<std::size_t>(i)] = bl[static_cast<std::size_t>(i)] = eye[i];
  bl[11] = 0.051;
  g.static_frames["base_footprint"] = bf;
  g.static_frames["base_link"] = bl;

  auto env = std::make_shared<Environment>();
  env->addJointGroup(g);
  // (link, center in the link frame, radius)
  const CollisionSphere spheres[] = {
    { 1, { 0.0, 0.0, 0.0 }, 0.09 },  { 1, { 0.1, 0.0, 0.0 }, 0.08 },  { 2, { 0.0, 0.0, 0.0 }, 0.08 },
    { 2, { 0.1, 0.0, 0.0 }, 0.07 },  { 3, { 0.15, 0.0, 0.0 }, 0.07 }, { 3, { 0.3, 0.0, 0.0 }, 0.07 },
    { 5, { 0.0, 0.0, 0.0 }, 0.07 },  { 5, { 0.08, 0.0, 0.0 }, 0.06 }, { 6, { 0.12, 0.0, 0.0 }, 0.06 },
    { 6, { 0.24, 0.0, 0.0 }, 0.06 }, { 8, { 0.0, 0.0, 0.0 }, 0.06 },  { 8, { 0.08, 0.0, 0.0 }, 0.06 },
    { 9, { 0.12, 0.0, 0.0 }, 0.06 }, { 9, { 0.18, 0.0, 0.0 }, 0.06 },
  };
  env->collision_spheres.assign(std::begin(spheres), std::end(spheres));
  return env;
}
}  // namespace trajopt
