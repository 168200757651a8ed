// Device-evaluated kinematic terms (device_terms.hpp) over thip_eval_*.
#include "trajopt_amd/device_terms.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "../../csrc/pair_data.hpp"
#include "trajopt_amd/problem_description.hpp"
#include "trajopt_sco/expr_ops.hpp"

namespace trajopt
{
DeviceTermEvaluator::~DeviceTermEvaluator() { thip_eval_destroy(ev_); }

void DeviceTermEvaluator::ensure()
{
  if (ev_ && device_ == prob_->device)
    return;
  thip_eval_destroy(ev_);
  ev_ = nullptr;
  const thip_problem_desc& d = prob_->desc();
  if (thip_eval_create(prob_->device, &d, 1, &ev_) != THIP_OK)
    throw std::runtime_error(std::string("thip_eval_create: ") + thip_eval_last_error(nullptr));
  device_ = prob_->device;
  const bool coll = d.coll_enabled || d.n_coll_extra > 0;
  if (static_cast<int>(prob_->cart_targets.size()) != d.n_cart * 12 ||
      (coll && static_cast<int>(prob_->scene.size()) != d.n_prims * 16))
    throw std::runtime_error("DeviceTermEvaluator: CartPose targets / scene do not match the problem's terms");
  if (thip_eval_upload(ev_, d.n_cart > 0 ? prob_->cart_targets.data() : nullptr,
                       coll && d.n_prims > 0 ? prob_->scene.data() : nullptr) != THIP_OK)
    throw std::runtime_error(std::string("thip_eval_upload: ") + thip_eval_last_error(ev_));
  cache_.assign(static_cast<std::size_t>((d.coll_enabled ? 1 : 0) + d.n_coll_extra), Cache());
  pair_tab_.assign(cache_.size(), {});
  for (std::size_t k = 0; k < pair_tab_.size(); ++k)
    thip::coll_pair_table(d, static_cast<int>(k), pair_tab_[k]);
}

DblVec DeviceTermEvaluator::jointTrajectory(const DblVec& x) const
{
  // the joint trajectory [n_steps][n_dof] (x also holds dt columns with use_time)
  auto* prob = const_cast<TrajOptProb*>(prob_);
  const VarArray& jv = prob->GetJointVars();
  DblVec q(jv.data.size());
  for (std::size_t i = 0; i < q.size(); ++i)
    q[i] = x[static_cast<std::size_t>(jv.data[i].var_rep->index)];
  return q;
}

void DeviceTermEvaluator::prefetchCart(const DblVec& x)
{
  const thip_problem_desc& d = prob_->desc();
  if (d.n_cart == 0)
    return;
  ensure();
  DblVec q = jointTrajectory(x);
  if (cart_.valid && cart_.q == q)
    return;
  const std::size_t D = static_cast<std::size_t>(prob_->GetNumDOF()), nc = static_cast<std::size_t>(d.n_cart);
  cart_.valid = false;
  cart_.err.resize(nc * 6);
  cart_.jac.resize(nc * 6 * D);
  if (thip_eval_cart_pose_all(ev_, q.data(), cart_.err.data(), cart_.jac.data()) != THIP_OK)
    throw std::runtime_error(std::string("thip_eval_cart_pose_all: ") + thip_eval_last_error(ev_));
  cart_.q = std::move(q);
  cart_.valid = true;
}

void DeviceTermEvaluator::cartPose(int k, const DblVec& q, double* err, double* jac)
{
  ensure();
  if (static_cast<int>(q.size()) != prob_->GetNumDOF())
    throw std::runtime_error("CartPose evaluation: expected " + std::to_string(prob_->GetNumDOF()) + " joint values");
  if (cart_.valid && k >= 0 && k < prob_->desc().n_cart)
  {
    // the prefetched values when q is this term's waypoint of the prefetched x
    const std::size_t D = q.size(), t = static_cast<std::size_t>(prob_->desc().cart_step[k]);
    if (std::equal(q.begin(), q.end(), cart_.q.begin() + static_cast<long>(t * D)))
    {
      const std::size_t ku = static_cast<std::size_t>(k);
      std::copy(cart_.err.begin() + static_cast<long>(ku * 6), cart_.err.begin() + static_cast<long>(ku * 6 + 6), err);
      if (jac)
        std::copy(cart_.jac.begin() + static_cast<long>(ku * 6 * D),
                  cart_.jac.begin() + static_cast<long>((ku + 1) * 6 * D), jac);
      return;
    }
  }
  if (thip_eval_cart_pose(ev_, k, q.data(), err, jac) != THIP_OK)
    throw std::runtime_error(std::string("thip_eval_cart_pose: ") + thip_eval_last_error(ev_));
}

const DeviceTermEvaluator::Contacts& DeviceTermEvaluator::collision(int term, const DblVec& x)
{
  ensure();
  if (term < 0 || term >= static_cast<int>(cache_.size()))
    throw std::runtime_error("collision evaluation: term out of range");
  const DblVec q = jointTrajectory(x);
  Cache& c = cache_[static_cast<std::size_t>(term)];
  if (c.valid && c.q == q)
    return c.c;
  const int D = prob_->GetNumDOF(), W = 8 + 2 * D + 1;
  int count = 0;
  int cap = static_cast<int>(c.c.rec.size() / static_cast<std::size_t>(W));
  for (int attempt = 0; attempt < 2; ++attempt)
  {
    c.c.rec.resize(static_cast<std::size_t>(std::max(cap, 1)) * W);
    if (thip_eval_collision(ev_, term, q.data(), c.c.rec.data(), cap, &count) != THIP_OK)
      throw std::runtime_error(std::string("thip_eval_collision: ") + thip_eval_last_error(ev_));
    if (count <= cap)
      break;
    cap = count;  // more contacts than room: once more with room for all
  }
  c.c.W = W;
  c.c.rec.resize(static_cast<std::size_t>(count) * W);
  c.c.t.resize(static_cast<std::size_t>(count));
  c.c.margin.resize(static_cast<std::size_t>(count));
  c.c.coeff.resize(static_cast<std::size_t>(count));
  const thip_problem_desc& d = prob_->desc();
  const std::vector<double>& tab = pair_tab_[static_cast<std::size_t>(term)];
  // the main term only when enabled (pair_data.hpp coll_pair_table)
  const bool main_term = d.coll_enabled && term == 0;
  const int extra = term - (d.coll_enabled ? 1 : 0);
  const double m0 = main_term ? d.coll_margin : d.coll_extra[extra].margin;
  const double c0 = main_term ? d.coll_coeff : d.coll_extra[extra].coeff;
  for (int r = 0; r < count; ++r)
  {
    const double* rec = c.c.rec.data() + static_cast<std::size_t>(r) * W;
    c.c.t[static_cast<std::size_t>(r)] = static_cast<int>(rec[0]);
    // record: [t, link, prim (or -1 - sphere b), sphere, ...]
    double m = m0, cf = c0;
    if (!tab.empty())
    {
      const int P = d.n_prims, s = static_cast<int>(rec[3]), p = static_cast<int>(rec[2]);
      const std::size_t e = (static_cast<std::size_t>(s) * (P + d.n_spheres) + (p >= 0 ? p : P + (-1 - p))) * 2;
      m = tab[e];
      cf = tab[e + 1];
    }
    c.c.margin[static_cast<std::size_t>(r)] = m;
    c.c.coeff[static_cast<std::size_t>(r)] = cf;
  }
  c.q = q;
  c.valid = true;
  return c.c;
}

DblVec CartPoseDeviceErr::operator()(const DblVec& q) const
{
  double err[6];
  ev_->cartPose(term_, q, err, nullptr);
  DblVec out;
  for (int i : indices_)
    out.push_back(err[i]);
  return out;
}

sco::Mat CartPoseDeviceJac::operator()(const DblVec& q) const
{
  const int D = static_cast<int>(q.size());
  double err[6];
  std::vector<double> jac(static_cast<std::size_t>(6 * D));
  ev_->cartPose(term_, q, err, jac.data());
  sco::Mat J(static_cast<int>(indices_.size()), D);
  for (int r = 0; r < J.rows; ++r)
    for (int j = 0; j < D; ++j)
      J(r, j) = jac[static_cast<std::size_t>(indices_[static_cast<std::size_t>(r)] * D + j)];
  return J;
}

void DeviceCollisionUnit::records(const DblVec& x, const DeviceTermEvaluator::Contacts*& c, int& first, int& n) const
{
  c = &ev->collision(term, x);
  first = 0;
  const int total = static_cast<int>(c->t.size());
  while (first < total && c->t[static_cast<std::size_t>(first)] < t)
    ++first;
  n = 0;
  while (first + n < total && c->t[static_cast<std::size_t>(first + n)] == t)
    ++n;
}

sco::VarVector DeviceCollisionUnit::vars() const
{
  sco::VarVector v = vars0;
  v.insert(v.end(), vars1.begin(), vars1.end());
  return v;
}

// CalcDistExpressions* (collision_terms.cpp:463-554): the record's kept coefficients
// over the unit's variables, vars0 first, and its constant
sco::AffExprVector DeviceCollisionUnit::exprs(const DblVec& x, DblVec* margins, DblVec* coeffs) const
{
  const DeviceTermEvaluator::Contacts* c;
  int first, n;
  records(x, c, first, n);
  const int D = static_cast<int>(vars0.size());
  sco::AffExprVector out;
  for (int r = first; r < first + n; ++r)
  {
    const double* rec = c->rec.data() + static_cast<std::size_t>(r) * c->W;
    sco::AffExpr e(rec[8 + 2 * D]);
    for (int j = 0; j < D; ++j)
      if (rec[8 + j] != 0.0)
      {
        e.coeffs.push_back(rec[8 + j]);
        e.vars.push_back(vars0[static_cast<std::size_t>(j)]);
      }
    for (int j = 0; j < D && !vars1.empty(); ++j)
      if (rec[8 + D + j] != 0.0)
      {
        e.coeffs.push_back(rec[8 + D + j]);
        e.vars.push_back(vars1[static_cast<std::size_t>(j)]);
      }
    out.push_back(e);
    if (margins)
      margins->push_back(c->margin[static_cast<std::size_t>(r)]);
    if (coeffs)
      coeffs->push_back(c->coeff[static_cast<std::size_t>(r)]);
  }
  return out;
}

double DeviceCollisionCost::value(const DblVec& x)
{
  const DeviceTermEvaluator::Contacts* c;
  int first, n;
  u_.records(x, c, first, n);
  double out = 0;
  for (int r = first; r < first + n; ++r)
    out += std::fmax(c->margin[static_cast<std::size_t>(r)] - c->rec[static_cast<std::size_t>(r) * c->W + 5], 0.0) *
           c->coeff[static_cast<std::size_t>(r)];
  return out;
}

sco::ConvexObjective::Ptr DeviceCollisionCost::convex(const DblVec& x, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexObjective>(model);
  DblVec margin, coeff;
  const sco::AffExprVector ex = u_.exprs(x, &margin, &coeff);
  for (std::size_t i = 0; i < ex.size(); ++i)
    out->addHinge(sco::exprSub(sco::AffExpr(margin[i]), ex[i]), coeff[i]);
  return out;
}

DblVec DeviceCollisionConstraint::value(const DblVec& x)
{
  const DeviceTermEvaluator::Contacts* c;
  int first, n;
  u_.records(x, c, first, n);
  DblVec out;
  for (int r = first; r < first + n; ++r)
    out.push_back(std::fmax(c->margin[static_cast<std::size_t>(r)] - c->rec[static_cast<std::size_t>(r) * c->W + 5],
                            0.0) *
                  c->coeff[static_cast<std::size_t>(r)]);
  return out;
}

sco::ConvexConstraints::Ptr DeviceCollisionConstraint::convex(const DblVec& x, sco::Model* model)
{
  auto out = std::make_shared<sco::ConvexConstraints>(model);
  DblVec margin, coeff;
  const sco::AffExprVector ex = u_.exprs(x, &margin, &coeff);
  for (std::size_t i = 0; i < ex.size(); ++i)
    out->addIneqCnt(sco::exprMult(sco::exprSub(sco::AffExpr(margin[i]), ex[i]), coeff[i]));
  return out;
}
}  // namespace trajopt
