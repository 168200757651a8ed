// GpuQPBatcher (gpu_qp_batcher.hpp).
#include "trajopt_sco/gpu_qp_batcher.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace sco
{
namespace
{
void appendInts(std::string& k, const std::vector<int>& v)
{
  const std::size_t o = k.size();
  k.resize(o + v.size() * sizeof(int));
  if (!v.empty())
    std::memcpy(&k[o], v.data(), v.size() * sizeof(int));
}

// the group a QP launches with: device, sizes, patterns and every setting but
// rho (each QP's rho travels in warm_rho)
std::string groupKey(const GpuQPBatcher::Request& r)
{
  std::string k;
  const int head[3] = { r.device, r.n, r.m };
  k.append(reinterpret_cast<const char*>(head), sizeof(head));
  thip_osqp_settings s = r.settings;
  s.rho = 0;
  k.append(reinterpret_cast<const char*>(&s), sizeof(s));
  for (const std::vector<int>* v : { r.Pp, r.Pi, r.Ap, r.Ai })
  {
    const int len = static_cast<int>(v->size());
    k.append(reinterpret_cast<const char*>(&len), sizeof(len));
    appendInts(k, *v);
  }
  return k;
}
}  // namespace

GpuQPBatcher::~GpuQPBatcher()
{
  for (auto& kv : cache_)
    thip_qp_destroy(kv.second.qp);
}

void GpuQPBatcher::enter()
{
  std::lock_guard<std::mutex> lk(mu_);
  ++active_;
}

void GpuQPBatcher::leave()
{
  std::unique_lock<std::mutex> lk(mu_);
  --active_;
  // the clients still running may all be waiting now
  if (!pending_.empty() && static_cast<int>(pending_.size()) >= active_)
    flushLocked();
}

void GpuQPBatcher::solve(Request& r)
{
  std::unique_lock<std::mutex> lk(mu_);
  r.done = false;
  r.error.clear();
  pending_.push_back(&r);
  if (static_cast<int>(pending_.size()) >= active_)
    flushLocked();  // the last client of the round launches it
  else
    cv_.wait(lk, [&] { return r.done; });
  if (!r.error.empty())
    throw std::runtime_error(r.error);
}

// Called with the lock held by the thread that completed the round: every other
// running client is blocked in solve(), so the pending set cannot change.
void GpuQPBatcher::flushLocked()
{
  std::vector<Request*> reqs;
  reqs.swap(pending_);
  ++round_;
  std::map<std::string, std::vector<Request*>> groups;
  for (Request* r : reqs)
    groups[groupKey(*r)].push_back(r);
  // every pattern's QPs are staged (inputs copied on each QP object's own
  // stream), then the round is one launch per device (thip_qp_launch_staged:
  // the workgroups of all patterns in one grid), then collected: the round
  // takes its slowest QP, not the sum of its patterns' launches
  struct Launch
  {
    std::vector<Request*>* g = nullptr;
    Slot* slot = nullptr;
    int n = 0, m = 0;
    std::vector<double> P, A, q, l, u, wx, wy, wr, x, y;
    std::vector<int> mask;
    std::vector<thip_qp_info> info;
    bool submitted = false;
    int device = 0;
  };
  std::vector<Launch> launches;
  launches.reserve(groups.size());
  const auto t0 = std::chrono::steady_clock::now();
  for (auto& kv : groups)
  {
    std::vector<Request*>& g = kv.second;
    const Request& r0 = *g.front();
    const int count = static_cast<int>(g.size()), n = r0.n, m = r0.m;
    launches.emplace_back();
    Launch& L = launches.back();
    L.g = &g;
    L.n = n;
    L.m = m;
    try
    {
      Slot& slot = cache_[kv.first];
      if (!slot.qp || slot.capacity < count)
      {
        thip_qp_destroy(slot.qp);
        slot.qp = nullptr;
        if (thip_qp_create(r0.device, n, m, r0.Pp->data(), r0.Pi->data(), r0.Ap->data(), r0.Ai->data(), count,
                           &slot.qp) != THIP_OK)
          throw std::runtime_error(std::string("GpuQPBatcher: ") + thip_qp_last_error(nullptr));
        slot.capacity = count;
      }
      slot.last_round = round_;
      L.slot = &slot;
      const std::size_t np = r0.Px->size(), na = r0.Ax->size(), nn = static_cast<std::size_t>(n),
                        mm = static_cast<std::size_t>(m);
      L.P.resize(np * count);
      L.A.resize(na * count);
      L.q.resize(nn * count);
      L.l.resize(mm * count);
      L.u.resize(mm * count);
      L.wx.assign(nn * count, 0.0);
      L.wy.assign(mm * count, 0.0);
      L.wr.resize(static_cast<std::size_t>(count));
      L.x.resize(nn * count);
      L.y.resize(std::max<std::size_t>(mm, 1) * count);
      L.mask.assign(static_cast<std::size_t>(count), 0);
      L.info.resize(static_cast<std::size_t>(count));
      bool any_warm = false;
      for (int k = 0; k < count; ++k)
      {
        const Request& r = *g[static_cast<std::size_t>(k)];
        const std::size_t ku = static_cast<std::size_t>(k);
        std::copy(r.Px->begin(), r.Px->end(), L.P.begin() + static_cast<long>(ku * np));
        std::copy(r.Ax->begin(), r.Ax->end(), L.A.begin() + static_cast<long>(ku * na));
        std::copy(r.q->begin(), r.q->end(), L.q.begin() + static_cast<long>(ku * nn));
        std::copy(r.l->begin(), r.l->end(), L.l.begin() + static_cast<long>(ku * mm));
        std::copy(r.u->begin(), r.u->end(), L.u.begin() + static_cast<long>(ku * mm));
        L.wr[ku] = r.settings.rho;
        if (r.warm)
        {
          any_warm = true;
          L.mask[ku] = 1;
          std::copy(r.wx->begin(), r.wx->begin() + static_cast<long>(nn), L.wx.begin() + static_cast<long>(ku * nn));
          std::copy(r.wy->begin(), r.wy->begin() + static_cast<long>(mm), L.wy.begin() + static_cast<long>(ku * mm));
        }
      }
      {
        long long sh[6];
        if (thip_qp_shape(slot.qp, sh) == THIP_OK && sh[0] > shape_[0])
          std::copy(sh, sh + 6, shape_);
      }
      if (thip_qp_stage(slot.qp, count, L.P.data(), L.q.data(), L.A.data(), L.l.data(), L.u.data(), &r0.settings,
                        any_warm ? L.wx.data() : nullptr, any_warm ? L.wy.data() : nullptr,
                        any_warm ? L.mask.data() : nullptr, L.wr.data()) != THIP_OK)
        throw std::runtime_error(std::string("GpuQPBatcher: thip_qp_stage: ") + thip_qp_last_error(slot.qp));
      L.submitted = true;
      L.device = r0.device;
    }
    catch (const std::exception& e)
    {
      for (Request* r : g)
        r->error = e.what();
    }
  }
  // one launch per device for every pattern staged this round
  {
    std::map<int, std::vector<Launch*>> by_dev;
    for (Launch& L : launches)
      if (L.submitted)
        by_dev[L.device].push_back(&L);
    for (auto& kv : by_dev)
    {
      std::vector<thip_qp*> qps;
      for (Launch* L : kv.second)
        qps.push_back(L->slot->qp);
      if (thip_qp_launch_staged(qps.data(), static_cast<int>(qps.size())) != THIP_OK)
      {
        const std::string msg = std::string("GpuQPBatcher: thip_qp_launch_staged: ") + thip_qp_last_error(qps[0]);
        for (Launch* L : kv.second)
        {
          L->submitted = false;
          for (Request* r : *L->g)
            r->error = msg;
        }
      }
    }
  }
  for (Launch& L : launches)
  {
    if (!L.submitted)
      continue;
    std::vector<Request*>& g = *L.g;
    const Request& r0 = *g.front();
    const int count = static_cast<int>(g.size()), n = L.n, m = L.m;
    try
    {
      if (thip_qp_collect(L.slot->qp, L.x.data(), L.y.data(), L.info.data()) != THIP_OK)
        throw std::runtime_error(std::string("GpuQPBatcher: thip_qp_solve_some: ") +
                                 thip_qp_last_error(L.slot->qp));
      ++launches_;
      qps_ += count;
      const std::size_t np = r0.Px->size(), na = r0.Ax->size(), nn = static_cast<std::size_t>(n),
                        mm = static_cast<std::size_t>(m);
      {
        // the algorithmic-byte model (gpu_qp_batcher.hpp bytes())
        // a pattern staged in LDS (thip_qp_shape out[4]: factor, D and the
        // 16-bit indices LDS-resident for the whole launch) never streams L
        // from HBM, so its factor and solve terms count only the vectors
        long long sh[6] = { 0, 0, 0, 0, 0, 0 };
        const bool lds_pat = thip_qp_shape(L.slot->qp, sh) == THIP_OK && sh[4] != 0;
        const double nl = lds_pat ? 0.0 : static_cast<double>(thip_qp_factor_nnz(L.slot->qp)),
                     nP = static_cast<double>(np), nA = static_cast<double>(na), N = static_cast<double>(n + m);
        const double per_solve = 2 * 12 * nl + 8 * N;
        const double per_iter = per_solve + 2 * 12 * nA + 2 * 12 * nP + 8 * (6.0 * n + 8.0 * m);
        const double per_factor = 12 * (nP + nA) + 12 * nl;
        for (int k = 0; k < count; ++k)
        {
          const thip_qp_info& in = L.info[static_cast<std::size_t>(k)];
          admm_iters_ += in.iter;
          bytes_ += in.iter * per_iter + per_factor;
          if (in.polish_status != 0)
            bytes_ += per_factor + (1 + r0.settings.polish_refine_iter) * per_solve;
        }
      }
      for (int k = 0; k < count; ++k)
      {
        Request& r = *g[static_cast<std::size_t>(k)];
        const std::size_t ku = static_cast<std::size_t>(k);
        r.x->assign(L.x.begin() + static_cast<long>(ku * nn), L.x.begin() + static_cast<long>((ku + 1) * nn));
        r.y->assign(L.y.begin() + static_cast<long>(ku * mm), L.y.begin() + static_cast<long>((ku + 1) * mm));
        *r.info = L.info[ku];
      }
    }
    catch (const std::exception& e)
    {
      for (Request* r : g)
        r->error = e.what();
    }
  }
  launch_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  // patterns unused for kKeepRounds rounds go (collision QPs change pattern with
  // their contacts, and often return to an earlier one: a kept pattern skips
  // thip_qp_create's symbolic analysis and allocations), and at most kMaxSlots stay
  constexpr long long kKeepRounds = 8;
  constexpr std::size_t kMaxSlots = 256;
  for (auto it = cache_.begin(); it != cache_.end();)
    if (it->second.last_round + kKeepRounds <= round_)
    {
      thip_qp_destroy(it->second.qp);
      it = cache_.erase(it);
    }
    else
      ++it;
  while (cache_.size() > kMaxSlots)
  {
    auto oldest = cache_.begin();
    for (auto it = cache_.begin(); it != cache_.end(); ++it)
      if (it->second.last_round < oldest->second.last_round)
        oldest = it;
    thip_qp_destroy(oldest->second.qp);
    cache_.erase(oldest);
  }
  for (Request* r : reqs)
    r->done = true;
  cv_.notify_all();
}
}  // namespace sco
