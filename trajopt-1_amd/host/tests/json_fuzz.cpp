// Fuzz driver for the problem front door (not part of libtrajopt_host), built
// with AddressSanitizer + UBSan by tests/test_sanitizers.py: seeded mutations
// of valid TrajOptRequest documents through Json::parse and ConstructProblem
// (fromJson, every TermInfo's fromJson / hatch, the sco objects).  Every input
// must either construct or throw std::exception; the sanitizers turn memory
// and undefined-behaviour errors into a non-zero exit.
//   json_fuzz <seed> <iterations>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <random>
#include <string>
#include <vector>

#include "trajopt_amd/problem_description.hpp"

namespace
{
const char* kSeeds[] = {
  R"({"basic_info": {"n_steps": 10, "manip": "right_arm", "fixed_timesteps": [0]},
      "costs": [{"type": "joint_vel", "params": {"coeffs": [1], "targets": [0]}},
                {"type": "cart_pose", "params": {"timestep": 9, "source_frame": "r_gripper_tool_frame",
                 "target_frame": "torso_lift_link", "target_frame_offset_xyz": [0.6, -0.2, 0.1],
                 "target_frame_offset_wxyz": [1, 0, 0, 0], "pos_coeffs": [10, 10, 10], "rot_coeffs": [1, 1, 1]}},
                {"type": "collision", "params": {"coeffs": 20, "dist_pen": 0.025, "evaluator_type": 2,
                 "first_step": 0, "last_step": 9, "longest_valid_segment_length": 0.05}}],
      "constraints": [{"type": "joint_pos", "params": {"targets": [0, 0, 0, -0.5, 0, -0.5, 0],
                       "first_step": 9, "last_step": 9, "lower_tols": [-0.1], "upper_tols": [0.1]}}],
      "init_info": {"type": "joint_interpolated", "endpoint": [0.1, 0.2, 0.0, -0.5, 0.0, -0.4, 0.0]}})",
  R"({"basic_info": {"n_steps": 8, "manip": "right_arm"},
      "opt_info": {"max_iter": 20, "trust_box_size": 0.1, "max_time": 5.0},
      "costs": [{"type": "joint_acc", "params": {"coeffs": [10], "targets": [0.1]}},
                {"type": "joint_jerk", "params": {"coeffs": [1], "targets": [0], "first_step": 2, "last_step": 2}}],
      "constraints": [{"type": "joint_vel", "params": {"coeffs": [10], "targets": [0], "first_step": 0,
                       "last_step": 0}},
                      {"type": "joint_acc", "params": {"targets": [0], "lower_tols": [-0.1], "upper_tols": [0.2]}}],
      "init_info": {"type": "stationary"}})",
  R"({"basic_info": {"n_steps": 6, "manip": "both_arms"},
      "costs": [{"type": "dynamic_cart_pose", "params": {"timestep": 5, "source_frame": "l_gripper_tool_frame",
                 "target_frame": "r_gripper_tool_frame", "target_frame_offset_xyz": [0, 0.2, 0]}},
                {"type": "collision", "params": {"coeffs": 20, "dist_pen": 0.025, "evaluator_type": 4,
                 "pairs": [{"link": "r_forearm_link", "pair": ["table"], "coeffs": 20, "dist_pen": 0.025}]}}],
      "init_info": {"type": "given_traj", "data": [[0,0,0,0,0,0,0,0,0,0,0,0,0,0],[0,0,0,0,0,0,0,0,0,0,0,0,0,0],
                    [0,0,0,0,0,0,0,0,0,0,0,0,0,0],[0,0,0,0,0,0,0,0,0,0,0,0,0,0],
                    [0,0,0,0,0,0,0,0,0,0,0,0,0,0],[0,0,0,0,0,0,0,0,0,0,0,0,0,0]]}})",
};
const char* kTokens[] = { "{", "}", "[", "]", ",", ":", "\"", "null", "true", "false", "-", "1e308", "-1e308",
                          "1e-320", "0", "-0", "2147483648", "-2147483649", "1.5", "NaN", "\"\\u0000\"",
                          "\"n_steps\"", "\"type\"", "\"params\"", "\"first_step\"", "\"last_step\"", "9999",
                          "-1", "\"joint_acc\"", "\"collision\"", "\"cart_pose\"", "[[[[", "]]]]" };

std::string mutate(std::string s, std::mt19937_64& g)
{
  std::uniform_int_distribution<int> op(0, 5);
  const int n = 1 + static_cast<int>(g() % 6);
  for (int k = 0; k < n && !s.empty(); ++k)
  {
    const std::size_t at = g() % s.size();
    switch (op(g))
    {
      case 0:  // flip a byte
        s[at] = static_cast<char>(g() & 0xff);
        break;
      case 1:  // delete a span
        s.erase(at, 1 + g() % 16);
        break;
      case 2:  // insert a token
        s.insert(at, kTokens[g() % (sizeof(kTokens) / sizeof(kTokens[0]))]);
        break;
      case 3:  // truncate
        s.resize(at);
        break;
      case 4:  // duplicate a span
        s.insert(at, s.substr(g() % s.size(), 1 + g() % 32));
        break;
      default:  // replace a digit run by an extreme number
      {
        std::size_t p = s.find_first_of("0123456789", at);
        if (p != std::string::npos)
        {
          std::size_t e = s.find_first_not_of("0123456789.eE+-", p);
          s.replace(p, (e == std::string::npos ? s.size() : e) - p, kTokens[11 + g() % 10]);
        }
      }
    }
  }
  return s;
}
}  // namespace

int main(int argc, char** argv)
{
  const unsigned long long seed = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  std::mt19937_64 g(seed);
  auto env = trajopt::Environment::makePR2();
  int built = 0, thrown = 0;
  for (const char* s : kSeeds)  // the seeds themselves construct
  {
    auto prob = trajopt::ConstructProblem(Json::parse(s), env);
    built += prob ? 1 : 0;
  }
  for (int it = 0; it < iters; ++it)
  {
    const std::string doc = mutate(kSeeds[g() % (sizeof(kSeeds) / sizeof(kSeeds[0]))], g);
    try
    {
      auto prob = trajopt::ConstructProblem(Json::parse(doc), env);
      if (prob)
      {
        // exercise the lowered form and the host objects' values
        const trajopt::LoweredProblem lp = prob->lowered();
        const sco::DblVec x(static_cast<std::size_t>(prob->getNumVars()), 0.01);
        // (CartPose and collision terms evaluate on the device: not in this CPU-only run)
        for (const auto& c : prob->getCosts())
          if (!dynamic_cast<trajopt::DeviceCartPoseCost*>(c.get()) &&
              !dynamic_cast<trajopt::DeviceCollisionCost*>(c.get()))
            (void)c->value(x);
        for (const auto& c : prob->getConstraints())
          if (!dynamic_cast<trajopt::DeviceCartPoseConstraint*>(c.get()) &&
              !dynamic_cast<trajopt::DeviceCollisionConstraint*>(c.get()))
            (void)c->violation(x);
        built += lp.init.empty() ? 0 : 1;
      }
    }
    catch (const std::exception&)
    {
      ++thrown;
    }
  }
  std::printf("json_fuzz seed %llu: %d constructed, %d rejected\n", seed, built, thrown);
  return 0;
}
