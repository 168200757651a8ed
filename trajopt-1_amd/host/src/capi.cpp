// C entry points of the host front door (include/trajopt_host.h).
#include "trajopt_host.h"

#include <algorithm>
#include <cstring>
#include <exception>
#include <memory>
#include <string>

#include "trajopt_amd/batch_sqp.hpp"

namespace
{
thread_local long long g_batch_qp_launches = 0, g_batch_qp_solves = 0;

void setErr(char* err, int err_len, const std::string& msg)
{
  if (!err || err_len <= 0)
    return;
  const std::size_t n = std::min<std::size_t>(msg.size(), static_cast<std::size_t>(err_len - 1));
  std::memcpy(err, msg.data(), n);
  err[n] = '\0';
}

trajopt::TrajOptProb::Ptr construct(const char* json_text, const double* scene, int n_prims)
{
  if (!json_text)
    throw std::runtime_error("null json text");
  if (n_prims < 0 || (n_prims > 0 && !scene))
    throw std::runtime_error("bad scene");
  const Json::Value root = Json::parse(json_text);
  std::string manip;
  if (root.isMember("basic_info") && root["basic_info"].isMember("manip"))
    json_marshal::childFromJson(root["basic_info"], manip, "manip");
  // the built-in environment of the group (the PR2, or spherebot for "manipulator"),
  // then the caller's primitives after the environment's own
  auto env = trajopt::Environment::builtin(manip);
  for (int p = 0; p < n_prims; ++p)
  {
    std::array<double, 16> rec{};
    std::copy(scene + 16 * p, scene + 16 * (p + 1), rec.begin());
    env->addSceneObject("scene_" + std::to_string(p), rec);  // the caller's primitive p
  }
  return trajopt::ConstructProblem(root, env);
}
}  // namespace

extern "C" {

int thost_lower_json(const char* json_text, const double* scene, int n_prims, thip_problem_desc* desc, double* init,
                     double* cart_targets, double* jpos_targets, double* scene_out, char* err, int err_len)
{
  try
  {
    auto prob = construct(json_text, scene, n_prims);
    if (desc)
      *desc = prob->desc();
    if (init)  // the joint columns
    {
      const trajopt::LoweredProblem lp = prob->lowered();
      std::copy(lp.init.begin(), lp.init.end(), init);
    }
    if (cart_targets)
      std::copy(prob->cart_targets.begin(), prob->cart_targets.end(), cart_targets);
    if (jpos_targets)
      std::copy(prob->jpos_targets.begin(), prob->jpos_targets.end(), jpos_targets);
    if (scene_out)
      std::copy(prob->scene.begin(), prob->scene.end(), scene_out);
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

int thost_solve_json(const char* json_text, const double* scene, int n_prims, int device, double* x,
                     thip_result* result, int* native, char* err, int err_len)
{
  try
  {
    if (!x)
      throw std::runtime_error("thost_solve_json: null x");
    auto prob = construct(json_text, scene, n_prims);
    const bool lowered = prob->lowerable();
    trajopt::BasicTrustRegionSQP opt(prob, device);
    opt.initialize(trajopt::trajToDblVec(prob->GetInitTraj()));
    opt.optimize();
    const sco::OptResults& r = opt.results();
    std::copy(r.x.begin(), r.x.end(), x);
    if (result)
    {
      std::memset(result, 0, sizeof(*result));
      result->status = static_cast<int>(r.status);
      result->n_sqp_iters = r.n_sqp_iters;
      result->n_qp_solves = r.n_qp_solves;
      result->n_func_evals = r.n_func_evals;
      result->n_admm_iters = r.n_admm_iters;
      result->total_cost = r.total_cost;
      result->max_cnt_viol = r.max_cnt_viol;
      result->flags = r.flags;
    }
    if (native)
      *native = lowered ? 1 : 0;
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

void thost_last_batch_qp_stats(long long* launches, long long* qps)
{
  if (launches)
    *launches = g_batch_qp_launches;
  if (qps)
    *qps = g_batch_qp_solves;
}

void thost_set_host_loop_workers(int n) { trajopt::BatchTrustRegionSQP::setDefaultHostLoopWorkers(n); }

int thost_solve_json_batch(const char* const* json_texts, int batch, const double* scenes, int n_prims, int device,
                           double* x, thip_result* results, char* err, int err_len)
{
  return thost_solve_json_batch_multi(json_texts, batch, scenes, n_prims, &device, 1, x, results, err, err_len);
}

namespace
{
void toResult(const sco::OptResults& r, thip_result& o)
{
  std::memset(&o, 0, sizeof(o));
  o.status = static_cast<int>(r.status);
  o.n_sqp_iters = r.n_sqp_iters;
  o.n_qp_solves = r.n_qp_solves;
  o.n_func_evals = r.n_func_evals;
  o.n_admm_iters = r.n_admm_iters;
  o.total_cost = r.total_cost;
  o.max_cnt_viol = r.max_cnt_viol;
  o.flags = r.flags;
}
}  // namespace

int thost_solve_json_stream(const char* const* json_texts, int n_batches, int batch, const double* scenes, int n_prims,
                            const int* devices, int n_devices, int inflight, double* x, thip_result* results, char* err,
                            int err_len)
{
  try
  {
    if (!json_texts || n_batches <= 0 || batch <= 0 || !x || !devices || n_devices <= 0)
      throw std::runtime_error("thost_solve_json_stream: bad arguments");
    std::vector<std::vector<trajopt::TrajOptProb::Ptr>> batches(static_cast<std::size_t>(n_batches));
    for (int j = 0; j < n_batches; ++j)
      for (int b = 0; b < batch; ++b)
      {
        const std::size_t i = static_cast<std::size_t>(j) * batch + b;
        batches[static_cast<std::size_t>(j)].push_back(
            construct(json_texts[i], scenes ? scenes + i * static_cast<std::size_t>(n_prims) * 16 : nullptr, n_prims));
      }
    const auto res = trajopt::MultiDeviceBatchSQP::optimizeStream(
        batches, std::vector<int>(devices, devices + n_devices), inflight);
    std::size_t i = 0;
    for (const auto& rb : res)
      for (const auto& r : rb)
      {
        std::copy(r.x.begin(), r.x.end(), x + i * r.x.size());
        if (results)
          toResult(r, results[i]);
        ++i;
      }
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

int thost_solve_json_batch_multi(const char* const* json_texts, int batch, const double* scenes, int n_prims,
                                 const int* devices, int n_devices, double* x, thip_result* results, char* err,
                                 int err_len)
{
  try
  {
    if (!json_texts || batch <= 0 || !x)
      throw std::runtime_error("thost_solve_json_batch: bad arguments");
    if (!devices || n_devices <= 0)
      throw std::runtime_error("thost_solve_json_batch_multi: no devices");
    std::vector<trajopt::TrajOptProb::Ptr> probs;
    for (int b = 0; b < batch; ++b)
      probs.push_back(construct(json_texts[b], scenes ? scenes + static_cast<std::size_t>(b) * n_prims * 16 : nullptr,
                                n_prims));
    trajopt::MultiDeviceBatchSQP opt(probs, std::vector<int>(devices, devices + n_devices));
    const auto res = opt.optimize();
    g_batch_qp_launches = opt.qpLaunches();
    g_batch_qp_solves = opt.qpSolves();
    for (int b = 0; b < batch; ++b)
    {
      const auto& r = res[static_cast<std::size_t>(b)];
      std::copy(r.x.begin(), r.x.end(), x + static_cast<std::size_t>(b) * r.x.size());
      if (results)
      {
        thip_result& o = results[b];
        std::memset(&o, 0, sizeof(o));
        o.status = static_cast<int>(r.status);
        o.n_sqp_iters = r.n_sqp_iters;
        o.n_qp_solves = r.n_qp_solves;
        o.n_func_evals = r.n_func_evals;
        o.n_admm_iters = r.n_admm_iters;
        o.total_cost = r.total_cost;
        o.max_cnt_viol = r.max_cnt_viol;
        o.flags = r.flags;
      }
    }
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

struct thost_batch
{
  std::unique_ptr<trajopt::BatchTrustRegionSQP> solver;
  bool solved = false;
};

int thost_batch_create(const char* const* json_texts, int batch, const double* scenes, int n_prims, int device,
                       thost_batch** out, char* err, int err_len)
{
  try
  {
    if (!json_texts || batch <= 0 || !out)
      throw std::runtime_error("thost_batch_create: bad arguments");
    std::vector<trajopt::TrajOptProb::Ptr> probs;
    for (int b = 0; b < batch; ++b)
      probs.push_back(construct(json_texts[b], scenes ? scenes + static_cast<std::size_t>(b) * n_prims * 16 : nullptr,
                                n_prims));
    auto h = std::make_unique<thost_batch>();
    h->solver = std::make_unique<trajopt::BatchTrustRegionSQP>(probs, device);
    h->solver->setHostLoopWorkers(batch);  // every problem's loop at once: each QP round is one launch per pattern
    *out = h.release();
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

int thost_batch_solve(thost_batch* h, double* x, thip_result* results, char* err, int err_len)
{
  try
  {
    if (!h || !x)
      throw std::runtime_error("thost_batch_solve: bad arguments");
    if (h->solved && h->solver->hostLoops())
      throw std::runtime_error("thost_batch_solve: a host-loop batch is solved once (its models keep their warm starts)");
    const auto res = h->solver->optimize();
    h->solved = true;
    for (std::size_t b = 0; b < res.size(); ++b)
    {
      const auto& r = res[b];
      std::copy(r.x.begin(), r.x.end(), x + b * r.x.size());
      if (results)
        toResult(r, results[b]);
    }
    setErr(err, err_len, "");
    return 0;
  }
  catch (const std::exception& e)
  {
    setErr(err, err_len, e.what());
    return -1;
  }
}

int thost_batch_stats(const thost_batch* h, int* host_loops, long long* qp_launches, long long* qps, double* qp_bytes,
                      double* qp_seconds)
{
  if (!h)
    return -1;
  if (host_loops)
    *host_loops = h->solver->hostLoops() ? 1 : 0;
  if (qp_launches)
    *qp_launches = h->solver->qpLaunches();
  if (qps)
    *qps = h->solver->qpSolves();
  if (qp_bytes)
    *qp_bytes = h->solver->qpBytes();
  if (qp_seconds)
    *qp_seconds = h->solver->qpLaunchSeconds();
  return 0;
}

int thost_batch_qp_shape(const thost_batch* h, long long* out)
{
  if (!h || !h->solver || !out)
    return -1;
  out[0] = h->solver->qpAdmmIters();
  std::copy(h->solver->qpMaxShape(), h->solver->qpMaxShape() + 6, out + 1);
  return 0;
}

void thost_batch_destroy(thost_batch* h) { delete h; }
}
