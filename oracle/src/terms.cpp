// ORACLE — test infrastructure only (see sco_expr.hpp header).
#include "terms.hpp"

#include <cmath>
#include <stdexcept>
#include <string>

#include "collision.hpp"

namespace orc
{
OsqpSettings toOsqpSettings(const thip_osqp_settings& s)
{
  OsqpSettings o;
  o.rho = s.rho;
  o.sigma = s.sigma;
  o.alpha = s.alpha;
  o.scaling = s.scaling;
  o.adaptive_rho = s.adaptive_rho;
  o.adaptive_rho_interval = s.adaptive_rho_interval;
  o.adaptive_rho_tolerance = s.adaptive_rho_tolerance;
  o.max_iter = s.max_iter;
  o.eps_abs = s.eps_abs;
  o.eps_rel = s.eps_rel;
  o.eps_prim_inf = s.eps_prim_inf;
  o.eps_dual_inf = s.eps_dual_inf;
  o.check_termination = s.check_termination;
  o.warm_starting = s.warm_starting;
  o.polishing = s.polishing;
  o.delta = s.delta;
  o.polish_refine_iter = s.polish_refine_iter;
  return o;
}

BasicTrustRegionSQPParameters toSqpParams(const thip_sqp_params& p)
{
  BasicTrustRegionSQPParameters o;
  o.improve_ratio_threshold = p.improve_ratio_threshold;
  o.min_trust_box_size = p.min_trust_box_size;
  o.min_approx_improve = p.min_approx_improve;
  o.min_approx_improve_frac = p.min_approx_improve_frac;
  o.max_iter = p.max_iter;
  o.trust_shrink_ratio = p.trust_shrink_ratio;
  o.trust_expand_ratio = p.trust_expand_ratio;
  o.cnt_tolerance = p.cnt_tolerance;
  o.max_merit_coeff_increases = p.max_merit_coeff_increases;
  o.max_qp_solver_failures = p.max_qp_solver_failures;
  o.merit_coeff_increase_ratio = p.merit_coeff_increase_ratio;
  o.initial_merit_error_coeff = p.initial_merit_error_coeff;
  o.inflate_constraints_individually = p.inflate_constraints_individually != 0;
  o.trust_box_size = p.trust_box_size;
  return o;
}

// ------------------------------------------------------------ JointVelEqCost
namespace
{
class JointVelEqCost : public Cost
{
public:
  JointVelEqCost(std::vector<VarVector> rows, DblVec coeffs, DblVec targets, int first_step, int last_step)
    : Cost("JointVelEq")
    , rows_(std::move(rows))
    , coeffs_(std::move(coeffs))
    , targets_(std::move(targets))
    , first_(first_step)
    , last_(last_step)
  {
    if (((last_ - 1) - first_) < 0)
      throw std::runtime_error("JointVelEqCost, trajectory is too short!");
    for (int i = first_; i <= last_ - 1; ++i)
      for (std::size_t j = 0; j < coeffs_.size(); ++j)
      {
        AffExpr vel;
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i)][j], -1));
        exprInc(vel, exprMult(rows_[static_cast<std::size_t>(i + 1)][j], 1));
        exprDec(vel, targets_[j]);
        exprInc(expr_, exprMult(exprSquare(vel), coeffs_[j]));
      }
  }
  double value(const DblVec& x) override
  {
    // (diffAxis0(traj) - targets)^2 * diag(coeffs), summed column-major
    double s = 0;
    for (std::size_t j = 0; j < coeffs_.size(); ++j)
      for (int i = first_; i <= last_ - 1; ++i)
      {
        const double d = (rows_[static_cast<std::size_t>(i + 1)][j].value(x) - rows_[static_cast<std::size_t>(i)][j].value(x)) -
                         targets_[j];
        s += (d * d) * coeffs_[j];
      }
    return s;
  }
  ConvexObjective::Ptr convex(const DblVec&, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    out->addQuadExpr(expr_);
    return out;
  }
  VarVector getVars() override
  {
    VarVector v;
    for (auto& r : rows_)
      v.insert(v.end(), r.begin(), r.end());
    return v;
  }

private:
  std::vector<VarVector> rows_;
  DblVec coeffs_, targets_;
  int first_, last_;
  QuadExpr expr_;
};
}  // namespace

// ------------------------------------------------------------ CartPose
void cartPoseIndices(const thip_problem_desc& d, int term, std::vector<int>& indices, DblVec& coeffs)
{
  indices.clear();
  coeffs.clear();
  for (int i = 0; i < 3; ++i)
    if (std::fabs(d.cart_pos_coeffs[term][i]) > 1e-5)
    {
      indices.push_back(i);
      coeffs.push_back(d.cart_pos_coeffs[term][i]);
    }
  for (int i = 0; i < 3; ++i)
    if (std::fabs(d.cart_rot_coeffs[term][i]) > 1e-5)
    {
      indices.push_back(i + 3);
      coeffs.push_back(d.cart_rot_coeffs[term][i]);
    }
}

DblVec CartPoseCalc::operator()(const DblVec& q) const
{
  std::vector<Iso3> fk;
  chainFwdKin(*chain, q.data(), fk);
  const Iso3 source_tf = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
  const Iso3 target_tf = mul(fk[0], target_offset);
  double err[6];
  calcTransformError(target_tf, source_tf, err);
  DblVec out(indices.size());
  for (std::size_t i = 0; i < indices.size(); ++i)
    out[i] = err[indices[i]];
  return out;
}

Mat CartPoseCalc::jac(const DblVec& q) const
{
  const double eps = 1e-5;
  std::vector<Iso3> fk;
  chainFwdKin(*chain, q.data(), fk);
  const Iso3 source_tf = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
  const Iso3 target_tf = mul(fk[0], target_offset);
  Mat J(static_cast<int>(indices.size()), static_cast<int>(q.size()));
  DblVec qp = q;
  for (std::size_t i = 0; i < q.size(); ++i)
  {
    qp[i] = q[i] + eps;
    chainFwdKin(*chain, qp.data(), fk);
    const Iso3 sp = mul(fk[static_cast<std::size_t>(source_link)], source_offset);
    double diff[6];
    calcJacobianTransformErrorDiff(target_tf, source_tf, sp, diff);
    for (std::size_t r = 0; r < indices.size(); ++r)
      J(static_cast<int>(r), static_cast<int>(i)) = diff[indices[r]] / eps;
    qp[i] = q[i];
  }
  return J;
}

// ------------------------------------------------------------ construction
TrajProblem constructProblem(const thip_problem_desc& d, const double* init_traj, const double* cart_targets,
                             const double* scene)
{
  TrajProblem tp;
  const int N = d.n_steps, D = d.chain.n_dof;
  tp.n_steps = N;
  tp.n_dof = D;
  tp.prob = std::make_shared<OptProb>(toOsqpSettings(d.osqp));
  // TrajOptProb ctor: variables j_i_j with joint-limit bounds (problem_description.cpp:557-598)
  std::vector<std::string> names;
  DblVec lb, ub;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < D; ++j)
    {
      names.push_back("j_" + std::to_string(i) + "_" + std::to_string(j));
      lb.push_back(d.chain.lower[j]);
      ub.push_back(d.chain.upper[j]);
    }
  tp.traj_vars = tp.prob->createVariables(names, lb, ub);
  tp.init.assign(init_traj, init_traj + N * D);
  std::vector<VarVector> rows(static_cast<std::size_t>(N));
  for (int i = 0; i < N; ++i)
    rows[static_cast<std::size_t>(i)] =
        VarVector(tp.traj_vars.begin() + i * D, tp.traj_vars.begin() + (i + 1) * D);

  // fixed timesteps: persistent linear equalities (problem_description.cpp:489-510)
  for (int f = 0; f < d.n_fixed; ++f)
  {
    const int t = d.fixed_steps[f];
    for (int j = 0; j < D; ++j)
      tp.prob->addLinearConstraint(exprSub(AffExpr(rows[static_cast<std::size_t>(t)][static_cast<std::size_t>(j)]),
                                           init_traj[t * D + j]),
                                   EQ);
  }

  // cost_infos: JointVel, CartPose costs, collision cost
  if (d.jv_enabled)
  {
    int first = d.jv_first_step, last = d.jv_last_step;
    if (last <= -1)
      last = N - 1;
    if ((N - 2) <= first)
      first = N - 2;
    if ((N - 1) <= last)
      last = N - 1;
    if (last == first)
      last += 1;
    if (last < first)
      std::swap(first, last);
    tp.prob->addCost(std::make_shared<JointVelEqCost>(rows, DblVec(d.jv_coeffs, d.jv_coeffs + D),
                                                      DblVec(d.jv_targets, d.jv_targets + D), first, last));
  }
  auto makeCalc = [&](int k) {
    auto calc = std::make_shared<CartPoseCalc>();
    calc->chain = &d.chain;
    calc->source_link = d.cart_source_link[k];
    calc->source_offset = Iso3::from12(d.cart_source_offset[k]);
    calc->target_offset = Iso3::from12(cart_targets + 12 * k);
    DblVec coeffs;
    cartPoseIndices(d, k, calc->indices, coeffs);
    return std::make_pair(calc, coeffs);
  };
  for (int k = 0; k < d.n_cart; ++k)
  {
    if (d.cart_is_cnt[k])
      continue;
    auto [calc, coeffs] = makeCalc(k);
    tp.prob->addCost(std::make_shared<CostFromErrFunc>([calc](const DblVec& q) { return (*calc)(q); },
                                                       [calc](const DblVec& q) { return calc->jac(q); },
                                                       rows[static_cast<std::size_t>(d.cart_step[k])], coeffs, ABS,
                                                       "cart_pose_" + std::to_string(k)));
  }
  if (d.coll_enabled && !d.coll_is_cnt)
    addCollisionTerms(tp, rows, d, scene);
  // cnt_infos: CartPose constraints, collision constraint
  for (int k = 0; k < d.n_cart; ++k)
  {
    if (!d.cart_is_cnt[k])
      continue;
    auto [calc, coeffs] = makeCalc(k);
    tp.prob->addConstraint(std::make_shared<ConstraintFromErrFunc>(
        [calc](const DblVec& q) { return (*calc)(q); }, [calc](const DblVec& q) { return calc->jac(q); },
        rows[static_cast<std::size_t>(d.cart_step[k])], coeffs, EQ, "cart_pose_cnt_" + std::to_string(k)));
  }
  if (d.coll_enabled && d.coll_is_cnt)
    addCollisionTerms(tp, rows, d, scene);
  return tp;
}

}  // namespace orc
