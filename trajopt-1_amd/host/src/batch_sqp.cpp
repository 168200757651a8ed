#include "trajopt_amd/batch_sqp.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>

#include "trajopt_sco/gpu_qp_batcher.hpp"

namespace trajopt
{
namespace
{
// The structure of a lowered problem: its descriptor with the per-problem
// default targets cleared (they travel in LoweredProblem::jpos_targets).
thip_problem_desc structureOf(const LoweredProblem& p)
{
  thip_problem_desc d = p.desc;
  for (auto& row : d.jpos_targets)
    for (double& v : row)
      v = 0.0;
  return d;
}

std::vector<LoweredProblem> lowerAll(const std::vector<TrajOptProb::Ptr>& probs)
{
  std::vector<LoweredProblem> out;
  out.reserve(probs.size());
  for (const auto& p : probs)
  {
    if (!p)
      throw std::runtime_error("BatchTrustRegionSQP: null problem");
    if (!p->lowerable())
      throw std::runtime_error("BatchTrustRegionSQP: the batched kernel does not run " + p->unloweredTerms() +
                               "; solve such a problem with sco::BasicTrustRegionSQP (the generic path)");
    out.push_back(p->lowered());
  }
  return out;
}

void copyParams(const sco::BasicTrustRegionSQPParameters& p, thip_sqp_params& q)
{
  q.improve_ratio_threshold = p.improve_ratio_threshold;
  q.min_trust_box_size = p.min_trust_box_size;
  q.min_approx_improve = p.min_approx_improve;
  q.min_approx_improve_frac = p.min_approx_improve_frac;
  q.max_iter = p.max_iter;
  q.trust_shrink_ratio = p.trust_shrink_ratio;
  q.trust_expand_ratio = p.trust_expand_ratio;
  q.cnt_tolerance = p.cnt_tolerance;
  q.max_merit_coeff_increases = p.max_merit_coeff_increases;
  q.max_qp_solver_failures = p.max_qp_solver_failures;
  q.merit_coeff_increase_ratio = p.merit_coeff_increase_ratio;
  q.initial_merit_error_coeff = p.initial_merit_error_coeff;
  q.inflate_constraints_individually = p.inflate_constraints_individually ? 1 : 0;
  q.trust_box_size = p.trust_box_size;
  q.max_time = p.max_time;
}

void paramsFrom(const thip_sqp_params& q, sco::BasicTrustRegionSQPParameters& p)
{
  p.improve_ratio_threshold = q.improve_ratio_threshold;
  p.min_trust_box_size = q.min_trust_box_size;
  p.min_approx_improve = q.min_approx_improve;
  p.min_approx_improve_frac = q.min_approx_improve_frac;
  p.max_iter = q.max_iter;
  p.trust_shrink_ratio = q.trust_shrink_ratio;
  p.trust_expand_ratio = q.trust_expand_ratio;
  p.cnt_tolerance = q.cnt_tolerance;
  p.max_merit_coeff_increases = q.max_merit_coeff_increases;
  p.max_qp_solver_failures = q.max_qp_solver_failures;
  p.merit_coeff_increase_ratio = q.merit_coeff_increase_ratio;
  p.initial_merit_error_coeff = q.initial_merit_error_coeff;
  p.inflate_constraints_individually = q.inflate_constraints_individually != 0;
  p.trust_box_size = q.trust_box_size;
  p.max_time = q.max_time;
}

// BasicTrustRegionSQPResults::writeSolver (optimizers.cpp:533-547), from the trace records
void writeSolverLog(const std::string& path, const std::vector<double>& rec)
{
  std::FILE* f = std::fopen(path.c_str(), "w");
  if (!f)
    throw std::runtime_error("BasicTrustRegionSQP: cannot open " + path);
  bool header = true;
  for (std::size_t k = 0; k + THIP_TRACE_W <= rec.size(); k += THIP_TRACE_W)
  {
    const double* r = rec.data() + k;
    if (r[15] == 0)
      continue;  // a QP without a merit evaluation (solver failure)
    if (header)
      std::fprintf(f, "%s,%s,%s,%s,%s,%s\n", "DESCRIPTION", "oldexact", "new_exact", "dapprox", "dexact", "ratio");
    header = false;
    std::fprintf(f, "%s,%10.3e,%10.3e,%10.3e,%10.3e,%10.3e\n", "Solver", r[10], r[11], r[12], r[13], r[14]);
  }
  std::fclose(f);
}
}  // namespace

// ------------------------------------------------------------ BatchTrustRegionSQP
namespace
{
bool allLowerable(const std::vector<TrajOptProb::Ptr>& probs)
{
  for (const auto& p : probs)
  {
    if (!p)
      throw std::runtime_error("BatchTrustRegionSQP: null problem");
    if (!p->lowerable())
      return false;
  }
  return true;
}
}  // namespace

BatchTrustRegionSQP::BatchTrustRegionSQP(const std::vector<TrajOptProb::Ptr>& probs, int device) : device_(device)
{
  if (probs.empty())
    throw std::runtime_error("BatchTrustRegionSQP: empty batch");
  if (!allLowerable(probs))
  {
    generic_ = probs;
    return;
  }
  probs_ = lowerAll(probs);
  init(device);
}

namespace
{
std::atomic<int> g_default_workers{ 64 };
}

void BatchTrustRegionSQP::setDefaultHostLoopWorkers(int n) { g_default_workers = n > 0 ? n : 64; }

int BatchTrustRegionSQP::hostLoopWorkers() const
{
  const int want = workers_ > 0 ? workers_ : g_default_workers.load();
  return std::max(1, std::min(want, batch()));
}

std::vector<sco::OptResults> BatchTrustRegionSQP::optimizeHostLoops()
{
  const std::size_t B = generic_.size();
  const std::size_t W = static_cast<std::size_t>(hostLoopWorkers());
  auto batcher = std::make_shared<sco::GpuQPBatcher>();
  std::vector<sco::OptResults> out(B);
  std::vector<std::string> errs(B);
  // one batcher client per worker, all registered before any thread starts, so
  // the first rounds batch every worker's QPs; a worker leaves when the batch
  // has no unsolved problem left
  std::vector<std::unique_ptr<sco::GpuQPBatcherClient>> clients;
  for (std::size_t w = 0; w < W; ++w)
    clients.push_back(std::make_unique<sco::GpuQPBatcherClient>(batcher));
  std::atomic<std::size_t> next{ 0 };
  std::vector<std::thread> threads;
  threads.reserve(W);
  for (std::size_t w = 0; w < W; ++w)
    threads.emplace_back([&, w]() {
      for (std::size_t b = next++; b < B; b = next++)
      {
        try
        {
          const TrajOptProb::Ptr& prob = generic_[b];
          BasicTrustRegionSQP opt(prob, device_);
          auto* gm = dynamic_cast<sco::GpuModel*>(prob->getModel().get());
          if (!gm)
            throw std::runtime_error("BatchTrustRegionSQP: problem " + std::to_string(b) + " has no GpuModel");
          gm->setBatcher(batcher);
          opt.initialize(trajToDblVec(prob->GetInitTraj()));
          opt.optimizeHostLoop();
          out[b] = opt.results();
          gm->setBatcher(nullptr);
        }
        catch (const std::exception& e)
        {
          errs[b] = e.what();
        }
      }
      clients[w].reset();  // leave: the others' rounds no longer wait for this worker
    });
  for (auto& t : threads)
    t.join();
  qp_launches_ = batcher->launches();
  qp_solves_ = batcher->qps();
  qp_bytes_ = batcher->bytes();
  qp_launch_s_ = batcher->launchSeconds();
  qp_admm_ = batcher->admmIters();
  std::copy(batcher->maxShape(), batcher->maxShape() + 6, qp_shape_);
  for (std::size_t b = 0; b < B; ++b)
    if (!errs[b].empty())
      throw std::runtime_error("BatchTrustRegionSQP: problem " + std::to_string(b) + ": " + errs[b]);
  return out;
}

BatchTrustRegionSQP::BatchTrustRegionSQP(std::vector<LoweredProblem> probs, int device) : probs_(std::move(probs))
{
  init(device);
}

void BatchTrustRegionSQP::init(int device)
{
  if (probs_.empty())
    throw std::runtime_error("BatchTrustRegionSQP: empty batch");
  const thip_problem_desc d0 = structureOf(probs_[0]);
  for (std::size_t b = 1; b < probs_.size(); ++b)
  {
    const thip_problem_desc db = structureOf(probs_[b]);
    if (std::memcmp(&d0, &db, sizeof(d0)) != 0)
      throw std::runtime_error("BatchTrustRegionSQP: problem " + std::to_string(b) +
                               " does not share problem 0's structure (steps, chain, terms, parameters and scene "
                               "size must be equal across a batch)");
  }
  const int rc = thip_create(device, &d0, static_cast<int>(probs_.size()), &ctx_);
  if (rc != THIP_OK)
    throw std::runtime_error(std::string("thip_create: ") + thip_last_error(nullptr));
}

BatchTrustRegionSQP::~BatchTrustRegionSQP() { thip_destroy(ctx_); }

void BatchTrustRegionSQP::check(int rc, const char* what) const
{
  if (rc != THIP_OK)
    throw std::runtime_error(std::string(what) + ": " + thip_last_error(ctx_));
}

void BatchTrustRegionSQP::setStream(void* stream)
{
  if (!generic_.empty())
    return;  // (host loops: each problem's QPs run on the batcher's launches)
  check(thip_set_stream(ctx_, stream), "thip_set_stream");
}

std::vector<sco::OptResults> BatchTrustRegionSQP::optimize()
{
  submit();
  return collect();
}

void BatchTrustRegionSQP::submit()
{
  if (!generic_.empty())
  {
    generic_results_ = optimizeHostLoops();  // (host loops: synchronous)
    return;
  }
  const thip_problem_desc& d = probs_[0].desc;
  const int B = batch(), N = d.n_steps, D = d.chain.n_dof;
  std::vector<double> init, tgt, jpt, scene;
  init.reserve(static_cast<std::size_t>(B) * N * D);
  for (const auto& p : probs_)
  {
    init.insert(init.end(), p.init.begin(), p.init.end());
    tgt.insert(tgt.end(), p.cart_targets.begin(), p.cart_targets.end());
    jpt.insert(jpt.end(), p.jpos_targets.begin(), p.jpos_targets.end());
    scene.insert(scene.end(), p.scene.begin(), p.scene.end());
  }
  if (init.size() != static_cast<std::size_t>(B) * N * D ||
      tgt.size() != static_cast<std::size_t>(B) * d.n_cart * 12 ||
      jpt.size() != static_cast<std::size_t>(B) * d.n_jpos * D ||
      scene.size() != static_cast<std::size_t>(B) * (d.coll_enabled ? d.n_prims : 0) * 16)
    throw std::runtime_error("BatchTrustRegionSQP: per-problem data sizes do not match the structure");
  check(thip_upload(ctx_, init.data(), tgt.empty() ? nullptr : tgt.data(), scene.empty() ? nullptr : scene.data()),
        "thip_upload");
  if (d.n_jpos > 0)
    check(thip_upload_joint_targets(ctx_, jpt.data()), "thip_upload_joint_targets");
  check(thip_sqp_run(ctx_), "thip_sqp_run");
}

void BatchTrustRegionSQP::submit(std::vector<LoweredProblem> probs)
{
  if (!generic_.empty())
    throw std::runtime_error("BatchTrustRegionSQP::submit: a host-loop batch takes its problems at construction");
  if (probs.size() != probs_.size())
    throw std::runtime_error("BatchTrustRegionSQP::submit: a batch of " + std::to_string(probs.size()) +
                             " problems on a context of " + std::to_string(probs_.size()));
  const thip_problem_desc d0 = structureOf(probs_[0]);
  for (std::size_t b = 0; b < probs.size(); ++b)
  {
    const thip_problem_desc db = structureOf(probs[b]);
    if (std::memcmp(&d0, &db, sizeof(d0)) != 0)
      throw std::runtime_error("BatchTrustRegionSQP::submit: problem " + std::to_string(b) +
                               " does not share the context's structure");
  }
  probs_ = std::move(probs);
  submit();
}

std::vector<sco::OptResults> BatchTrustRegionSQP::collect()
{
  if (!generic_.empty())
    return std::move(generic_results_);
  const thip_problem_desc& d = probs_[0].desc;
  const int B = batch(), N = d.n_steps, D = d.chain.n_dof;
  std::vector<double> x(static_cast<std::size_t>(B) * N * D);
  std::vector<thip_result> res(static_cast<std::size_t>(B));
  check(thip_download(ctx_, x.data(), res.data()), "thip_download");
  std::vector<sco::OptResults> out(static_cast<std::size_t>(B));
  for (int b = 0; b < B; ++b)
  {
    sco::OptResults& o = out[static_cast<std::size_t>(b)];
    const thip_result& r = res[static_cast<std::size_t>(b)];
    o.x.assign(x.begin() + static_cast<long>(b) * N * D, x.begin() + static_cast<long>(b + 1) * N * D);
    o.status = static_cast<sco::OptStatus>(r.status);  // THIP_OPT_* == sco::OptStatus order
    o.total_cost = r.total_cost;
    o.n_func_evals = r.n_func_evals;
    o.n_qp_solves = r.n_qp_solves;
    o.n_sqp_iters = r.n_sqp_iters;
    o.n_admm_iters = r.n_admm_iters;
    o.max_cnt_viol = r.max_cnt_viol;
    o.flags = r.flags;
  }
  return out;
}

// ------------------------------------------------------------ MultiDeviceBatchSQP
MultiDeviceBatchSQP::MultiDeviceBatchSQP(const std::vector<TrajOptProb::Ptr>& probs, const std::vector<int>& devices)
{
  if (devices.empty())
    throw std::runtime_error("MultiDeviceBatchSQP: no devices");
  if (probs.empty())
    throw std::runtime_error("MultiDeviceBatchSQP: empty batch");
  const std::size_t W = devices.size();
  if (!allLowerable(probs))
  {
    // host-loop shards (BatchTrustRegionSQP's batched QPs), one per device entry
    const std::size_t B = probs.size();
    std::size_t lo = 0;
    for (std::size_t r = 0; r < W; ++r)
    {
      const std::size_t n = B / W + (r < B % W ? 1 : 0);
      sizes_.push_back(static_cast<int>(n));
      if (n == 0)
        continue;
      shards_.push_back(std::make_unique<BatchTrustRegionSQP>(
          std::vector<TrajOptProb::Ptr>(probs.begin() + static_cast<long>(lo), probs.begin() + static_cast<long>(lo + n)),
          devices[r]));
      lo += n;
    }
    return;
  }
  const std::vector<LoweredProblem> all = lowerAll(probs);
  const std::size_t B = all.size();
  std::size_t lo = 0;
  for (std::size_t r = 0; r < W; ++r)
  {
    const std::size_t n = B / W + (r < B % W ? 1 : 0);  // shard r: [lo, lo + n)
    sizes_.push_back(static_cast<int>(n));
    if (n == 0)
      continue;
    std::vector<LoweredProblem> part(all.begin() + static_cast<long>(lo), all.begin() + static_cast<long>(lo + n));
    shards_.push_back(std::make_unique<BatchTrustRegionSQP>(std::move(part), devices[r]));
    lo += n;
  }
}

std::vector<sco::OptResults> MultiDeviceBatchSQP::optimize()
{
  if (!shards_.empty() && shards_[0]->hostLoops())
  {
    // host-loop shards run concurrently, each from its own thread
    std::vector<std::vector<sco::OptResults>> part(shards_.size());
    std::vector<std::string> errs(shards_.size());
    std::vector<std::thread> th;
    for (std::size_t k = 0; k < shards_.size(); ++k)
      th.emplace_back([&, k]() {
        try
        {
          part[k] = shards_[k]->optimize();
        }
        catch (const std::exception& e)
        {
          errs[k] = e.what();
        }
      });
    for (auto& t : th)
      t.join();
    std::vector<sco::OptResults> out;
    for (std::size_t k = 0; k < shards_.size(); ++k)
    {
      if (!errs[k].empty())
        throw std::runtime_error(errs[k]);
      out.insert(out.end(), std::make_move_iterator(part[k].begin()), std::make_move_iterator(part[k].end()));
    }
    return out;
  }
  for (auto& s : shards_)
    s->submit();
  std::vector<sco::OptResults> out;
  for (auto& s : shards_)
  {
    std::vector<sco::OptResults> r = s->collect();
    out.insert(out.end(), std::make_move_iterator(r.begin()), std::make_move_iterator(r.end()));
  }
  return out;
}

std::vector<std::vector<sco::OptResults>> MultiDeviceBatchSQP::optimizeStream(
    const std::vector<std::vector<TrajOptProb::Ptr>>& batches, const std::vector<int>& devices, int inflight)
{
  if (devices.empty())
    throw std::runtime_error("MultiDeviceBatchSQP: no devices");
  if (inflight < 1)
    throw std::runtime_error("MultiDeviceBatchSQP: inflight must be >= 1");
  std::vector<std::vector<sco::OptResults>> out(batches.size());
  if (batches.empty())
    return out;
  const std::size_t B = batches[0].size(), W = devices.size(), K = static_cast<std::size_t>(inflight);
  if (B == 0)
    throw std::runtime_error("MultiDeviceBatchSQP: empty batch");
  // the shard bounds of every batch: contiguous, sizes differing by at most one
  std::vector<std::size_t> lo(W + 1, 0);
  for (std::size_t r = 0; r < W; ++r)
    lo[r + 1] = lo[r] + B / W + (r < B % W ? 1 : 0);
  // slots[k][r]: the context of device entry r in slot k (created with its first batch)
  std::vector<std::vector<std::unique_ptr<BatchTrustRegionSQP>>> slots(K);
  std::vector<long> owner(K, -1);  // the batch a slot holds, -1 = none
  auto collectSlot = [&](std::size_t k) {
    if (owner[k] < 0)
      return;
    std::vector<sco::OptResults>& res = out[static_cast<std::size_t>(owner[k])];
    for (auto& ctx : slots[k])
      if (ctx)
      {
        std::vector<sco::OptResults> r = ctx->collect();
        res.insert(res.end(), std::make_move_iterator(r.begin()), std::make_move_iterator(r.end()));
      }
    owner[k] = -1;
  };
  for (std::size_t j = 0; j < batches.size(); ++j)
  {
    if (batches[j].size() != B)
      throw std::runtime_error("MultiDeviceBatchSQP::optimizeStream: batch " + std::to_string(j) + " has " +
                               std::to_string(batches[j].size()) + " problems, batch 0 has " + std::to_string(B));
    const std::vector<LoweredProblem> all = lowerAll(batches[j]);
    const std::size_t k = j % K;
    collectSlot(k);
    if (slots[k].empty())
      slots[k].resize(W);
    for (std::size_t r = 0; r < W; ++r)
    {
      if (lo[r + 1] == lo[r])
        continue;
      std::vector<LoweredProblem> part(all.begin() + static_cast<long>(lo[r]), all.begin() + static_cast<long>(lo[r + 1]));
      if (!slots[k][r])
      {
        slots[k][r] = std::make_unique<BatchTrustRegionSQP>(std::move(part), devices[r]);
        slots[k][r]->submit();
      }
      else
        slots[k][r]->submit(std::move(part));
    }
    owner[k] = static_cast<long>(j);
  }
  // drain in submission order
  for (std::size_t n = 0; n < K; ++n)
  {
    std::size_t best = K;
    for (std::size_t k = 0; k < K; ++k)
      if (owner[k] >= 0 && (best == K || owner[k] < owner[best]))
        best = k;
    if (best == K)
      break;
    collectSlot(best);
  }
  return out;
}

long long MultiDeviceBatchSQP::qpLaunches() const
{
  long long n = 0;
  for (const auto& s : shards_)
    n += s->qpLaunches();
  return n;
}
long long MultiDeviceBatchSQP::qpSolves() const
{
  long long n = 0;
  for (const auto& s : shards_)
    n += s->qpSolves();
  return n;
}

double BatchTrustRegionSQP::lastKernelMs() const { return generic_.empty() ? thip_last_kernel_ms(ctx_) : 0.0; }

void BatchTrustRegionSQP::writeSolverLog(int b, const std::string& path) const
{
  if (trace_cap_ <= 0)
    throw std::runtime_error("BatchTrustRegionSQP::writeSolverLog: enableTrace() before optimize()");
  if (b < 0 || b >= batch())
    throw std::runtime_error("BatchTrustRegionSQP::writeSolverLog: problem out of range");
  trajopt::writeSolverLog(path, trace()[static_cast<std::size_t>(b)]);
}

void BatchTrustRegionSQP::enableTrace(int capacity)
{
  if (!generic_.empty())
    throw std::runtime_error("BatchTrustRegionSQP::enableTrace: the fused kernel's trace (a host-loop batch logs "
                             "through sco::BasicTrustRegionSQPParameters::log_results)");
  check(thip_debug_trace(ctx_, capacity), "thip_debug_trace");
  trace_cap_ = capacity;
}

std::vector<std::vector<double>> BatchTrustRegionSQP::trace() const
{
  const std::size_t B = static_cast<std::size_t>(batch()), W = THIP_TRACE_W;
  std::vector<double> rec(B * static_cast<std::size_t>(trace_cap_) * W);
  std::vector<int> cnt(B);
  check(thip_debug_get_trace(ctx_, rec.data(), cnt.data()), "thip_debug_get_trace");
  std::vector<std::vector<double>> out(B);
  for (std::size_t b = 0; b < B; ++b)
  {
    const auto* p = rec.data() + b * static_cast<std::size_t>(trace_cap_) * W;
    out[b].assign(p, p + static_cast<std::size_t>(std::min(cnt[b], trace_cap_)) * W);
    // the device counts every record, also those past the capacity
    if (cnt[b] > trace_cap_)
      std::fprintf(stderr, "BatchTrustRegionSQP: trace of problem %zu truncated: %d of %d QP records kept\n", b,
                   trace_cap_, cnt[b]);
  }
  return out;
}

// ------------------------------------------------------------ the native path of one problem
int traceCapacity(const sco::BasicTrustRegionSQPParameters& param)
{
  // one record per QP solve: at most (penalty rounds) x (SQP iterations) x
  // (trust-region tries per iteration); the box shrinks by trust_shrink_ratio
  // per rejected try from at most trust_box_size * expand^max_iter down to
  // min_trust_box_size
  const double grow = param.max_iter * std::log(std::max(param.trust_expand_ratio, 1.0));
  const double span = std::log(param.trust_box_size / param.min_trust_box_size) + grow;
  const double tries = 2.0 + std::max(0.0, span / std::log(1.0 / param.trust_shrink_ratio));
  const double bound = (param.max_merit_coeff_increases + 1.0) * param.max_iter * tries;
  // (a non-finite bound -- absurd parameters -- takes the fixed cap)
  return static_cast<int>(std::isfinite(bound) ? std::min(std::max(bound, 64.0), 1.0e6) : 1.0e6);
}

void TrajOptProb::prefetch(const DblVec& x)
{
  if (device_terms_)
    device_terms_->prefetchCart(x);
}

bool TrajOptProb::solveNative(const sco::BasicTrustRegionSQPParameters& param, const DblVec& x0,
                              sco::OptResults& results)
{
  if (!lowerable())
    return false;
  if (!(param.trust_shrink_ratio > 0 && param.trust_shrink_ratio < 1) || !(param.min_trust_box_size > 0) ||
      !(param.trust_box_size > 0) || !(param.trust_expand_ratio > 0))
    throw std::runtime_error("BasicTrustRegionSQP: need 0 < trust_shrink_ratio < 1, trust_expand_ratio > 0, "
                             "min_trust_box_size > 0 and trust_box_size > 0");
  const int N = GetNumSteps(), D = GetNumDOF();
  if (x0.size() != static_cast<std::size_t>(N) * static_cast<std::size_t>(D))
    throw std::runtime_error("BasicTrustRegionSQP: expected " + std::to_string(N * D) + " initial values, got " +
                             std::to_string(x0.size()));
  // fixed timesteps are linear equalities to ConstructProblem's initial trajectory
  // (problem_description.cpp:489-510); the kernel pins them to the uploaded start,
  // so a start that moves a fixed step would change the problem: refuse it
  for (int f = 0; f < desc_.n_fixed; ++f)
  {
    const int t = desc_.fixed_steps[f];
    for (int j = 0; j < D; ++j)
      if (x0[static_cast<std::size_t>(t * D + j)] != init_[static_cast<std::size_t>(t)][static_cast<std::size_t>(j)])
        throw std::runtime_error("BasicTrustRegionSQP::initialize: fixed timestep " + std::to_string(t) +
                                 " differs from the problem's initial trajectory");
  }
  LoweredProblem lp = lowered();
  lp.init = x0;
  copyParams(param, lp.desc.sqp);
  BatchTrustRegionSQP batch(std::vector<LoweredProblem>{ std::move(lp) }, device);
  results = batch.optimize()[0];
  return true;
}

// ------------------------------------------------------------ BasicTrustRegionSQP
BasicTrustRegionSQP::BasicTrustRegionSQP(const TrajOptProb::Ptr& prob, int device)
  : sco::BasicTrustRegionSQP(prob)
{
  prob->device = device;
  if (auto* gm = dynamic_cast<sco::GpuModel*>(prob->getModel().get()))
    gm->setDevice(device);
  // the problem's own parameters (ProblemConstructionInfo::opt_info) are the defaults
  paramsFrom(prob->desc().sqp, param_);
}

DblVec trajToDblVec(const std::vector<DblVec>& traj)
{
  DblVec out;
  for (const auto& row : traj)
    out.insert(out.end(), row.begin(), row.end());
  return out;
}
}  // namespace trajopt
