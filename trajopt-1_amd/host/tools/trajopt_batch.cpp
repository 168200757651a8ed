// trajopt_batch: solve JSON problems (the reference's TrajOptRequest format)
// as one batch on one MI355X through the C++ front door.
//   trajopt_batch [--device D] [--repeat R] problem.json [problem.json ...]
// Every file is one problem (all must share one structure); --repeat R
// replicates the list R times.  Prints one line per problem.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "trajopt_amd/batch_sqp.hpp"

int main(int argc, char** argv)
{
  int device = 0, repeat = 1;
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i)
  {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc)
      device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--repeat") && i + 1 < argc)
      repeat = std::atoi(argv[++i]);
    else
      files.emplace_back(argv[i]);
  }
  if (files.empty() || repeat < 1)
  {
    std::fprintf(stderr, "usage: %s [--device D] [--repeat R] problem.json [...]\n", argv[0]);
    return 2;
  }
  try
  {
    auto env = trajopt::Environment::makePR2();
    std::vector<trajopt::TrajOptProb::Ptr> probs;
    for (int r = 0; r < repeat; ++r)
      for (const auto& f : files)
        probs.push_back(trajopt::ConstructProblem(Json::parseFile(f), env));
    trajopt::BatchTrustRegionSQP opt(probs, device);
    const auto res = opt.optimize();
    for (std::size_t b = 0; b < res.size(); ++b)
      std::printf("problem %zu: %s sqp_iters %d qp_solves %d cost %.9g max_viol %.3g\n", b,
                  sco::toString(res[b].status).c_str(), res[b].n_sqp_iters, res[b].n_qp_solves, res[b].total_cost,
                  res[b].max_cnt_viol);
    std::printf("kernel %.3f ms for %zu problems\n", opt.lastKernelMs(), res.size());
  }
  catch (const std::exception& e)
  {
    std::fprintf(stderr, "trajopt_batch: %s\n", e.what());
    return 1;
  }
  return 0;
}
