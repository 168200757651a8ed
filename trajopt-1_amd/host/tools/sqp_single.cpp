// The reference's per-problem optimizer usage on the HIP path (planning_unit.cpp:83-124):
//   ConstructProblem(pci) -> BasicTrustRegionSQP opt(prob); opt.initialize(...); opt.optimize()
// usage: sqp_single [--log DIR] [--callback] [--trace] problem.json
//   prints "status <s> iters <n> cost <c> fevals <f> callbacks <k>" and the trajectory;
//   --log: the reference's log_results CSV logs in DIR; --callback: a callback counting
//   its calls (optimizers.cpp:754, 978); --trace: one "qp" line per QP solve of the host
//   loop (GpuModel::setTrace fields).  Each observes the iterations, so the problem
//   runs the host loop (sco::BasicTrustRegionSQP::optimize).
#include <cstdio>
#include <array>
#include <stdexcept>
#include <string>
#include <vector>

#include "trajopt_amd/batch_sqp.hpp"
#include "trajopt_sco/gpu_model.hpp"

int main(int argc, char** argv)
{
  std::string log_dir, file;
  bool callback = false, trace = false;
  for (int a = 1; a < argc; ++a)
  {
    const std::string s = argv[a];
    if (s == "--log" && a + 1 < argc)
      log_dir = argv[++a];
    else if (s == "--callback")
      callback = true;
    else if (s == "--trace")
      trace = true;
    else if (file.empty() && s.rfind("--", 0) != 0)
      file = s;
    else
      file.clear(), a = argc;
  }
  if (file.empty())
  {
    std::fprintf(stderr, "usage: sqp_single [--log DIR] [--callback] [--trace] problem.json\n");
    return 2;
  }
  try
  {
    const Json::Value root = Json::parseFile(file.c_str());
    std::string manip;
    json_marshal::childFromJson(root["basic_info"], manip, "manip");
    trajopt::TrajOptProb::Ptr prob = trajopt::ConstructProblem(root, trajopt::Environment::builtin(manip));
    trajopt::BasicTrustRegionSQP opt(prob);
    if (!log_dir.empty())
    {
      opt.getParameters().log_results = true;
      opt.getParameters().log_dir = log_dir;
    }
    int calls = 0;
    if (callback)
      opt.addCallback([&calls](sco::OptProb*, sco::OptResults&) { ++calls; });
    std::vector<std::array<double, 9>> records;
    if (trace)
    {
      auto* gm = dynamic_cast<sco::GpuModel*>(prob->getModel().get());
      if (!gm)
        throw std::runtime_error("--trace: the problem has no GpuModel");
      gm->setTrace(&records);
      opt.addCallback([](sco::OptProb*, sco::OptResults&) {});  // observed: the host loop
    }
    opt.initialize(trajopt::trajToDblVec(prob->GetInitTraj()));
    const sco::OptStatus st = opt.optimize();
    for (const auto& r : records)
      std::fprintf(stderr, "qp %.0f %.17g %.0f %.0f %.0f %.17g %.17g %.17g %.17g\n", r[0], r[1], r[2], r[3], r[4], r[5],
                   r[6], r[7], r[8]);
    std::printf("status %s iters %d cost %.17g fevals %d callbacks %d\n", sco::toString(st).c_str(),
                opt.results().n_sqp_iters, opt.results().total_cost, opt.results().n_func_evals, calls);
    const int D = prob->GetNumDOF();
    for (std::size_t i = 0; i < opt.x().size(); ++i)
      std::printf("%.17g%c", opt.x()[i], (static_cast<int>(i) % D == D - 1) ? '\n' : ' ');
    return 0;
  }
  catch (const std::exception& e)
  {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
