// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of the LVS-discrete collision term on a primitive scene:
//   DiscreteCollisionEvaluator::CalcCollisions  trajopt/src/collision_terms.cpp:817-898
//   SingleTimestepCollisionEvaluator            trajopt/src/collision_terms.cpp:538-554,600-688 (DISCRETE)
//   CastCollisionEvaluator::CalcCollisions      trajopt/src/collision_terms.cpp:1065-1161 (LVS_CONTINUOUS)
//   CollisionEvaluator::GetGradient             trajopt/src/collision_terms.cpp:195-242
//   CollisionsToDistanceExpressions             trajopt/src/collision_terms.cpp:341-386
//   CalcDistExpressions{BothFree,..}            trajopt/src/collision_terms.cpp:463-536
//   CollisionCost::convex / value               trajopt/src/collision_terms.cpp:1267-1306
//   CollisionTermInfo::hatch (cost branch)      trajopt/src/problem_description.cpp:1735-1781
//   removeInvalidContactResults                 trajopt_common/src/collision_utils.cpp:73-114
// tesseract's ContactResultMap::addInterpolatedCollisionResults [ext] is
// restated as SURVEY.md §8c.1 item 7 (cc_time = i dt, Time0 / Between /
// Time1, cc_transform = transform for discrete results).  Bullet's
// contactTest is replaced by closed-form sphere-vs-primitive signed distance
// shared with the GPU path: contact values are "parity unpinned" against
// Bullet; the map order is (robot link, primitive) rather than tesseract's
// link-id hash order.
#pragma once
#include <memory>
#include <map>
#include <set>
#include <vector>

#include "terms.hpp"

namespace orc
{
struct CollisionModel
{
  const thip_chain* chain = nullptr;
  int n_spheres = 0;
  int sphere_link[THIP_MAX_SPHERES];
  double sphere_center[THIP_MAX_SPHERES][3];
  double sphere_radius[THIP_MAX_SPHERES];
  int n_prims = 0;
  std::vector<double> scene_store;
  const double* scene = nullptr;  // [n_prims][16]
  double margin = 0, coeff = 0, buffer = 0, lvs = 0;
  bool continuous = false;  // LVS_CONTINUOUS (CastCollisionEvaluator) instead of LVS_DISCRETE
  int contact_test = THIP_CONTACT_ALL;  // the request's test type (trajopt_hip.h THIP_CONTACT_*)
  // robot self-collision (desc.self_pair): sphere pairs (a, b) in key order --
  // link pairs in descriptor order, then the spheres of a, then those of b
  // (sphere index order) -- and the key of each
  std::vector<int> self_a, self_b, self_key;
  int n_self_keys = 0;
  // per link-pair data (CollisionTermInfo "pairs", problem_description.cpp:1686-1719):
  // the contact manager's pair margins (CollisionMarginData, override MODIFY) and
  // CollisionCoeffData's pair coefficients and zero-coefficient set
  // (trajopt_common/src/collision_types.cpp:40-72), keyed by the unordered link
  // pair -- a scene primitive p is the "link" kScenePair + p
  static constexpr int kScenePair = 1 << 20;
  std::map<std::pair<int, int>, double> pair_margin, pair_coeff;
  std::set<std::pair<int, int>> zero_coeff;
  static std::pair<int, int> key(int a, int b) { return a < b ? std::make_pair(a, b) : std::make_pair(b, a); }
  // CollisionMarginData::getCollisionMargin / CollisionCoeffData::getCollisionCoeff
  double marginOf(int a, int b) const
  {
    const auto it = pair_margin.find(key(a, b));
    return it == pair_margin.end() ? margin : it->second;
  }
  double coeffOf(int a, int b) const
  {
    const auto it = pair_coeff.find(key(a, b));
    return it == pair_coeff.end() ? coeff : it->second;
  }
  bool hasZeroCoeff(int a, int b) const { return zero_coeff.count(key(a, b)) != 0; }
};

// A contact between a robot link sphere (link_ids[0], active) and a scene
// primitive (link_ids[1], static), or -- a self contact -- another robot link
// sphere (link_ids[1], active: prim = -1 - sphere_b).
struct Contact
{
  int link = 0, prim = 0, sphere = 0, substate = 0;
  int link_b = -1, sphere_b = -1;  // self contact: the second body
  double distance = 0;
  double normal[3];    // from the robot sphere toward the primitive
  double p_robot[3];   // nearest points, world
  double p_prim[3];
  double p_local[3];   // nearest_points_local[0] (robot link frame at the sub-state)
  Iso3 transform;      // robot link pose at the sub-state (discrete) / at the cast's start state (continuous)
  Iso3 cc_transform;   // = transform (discrete) / link pose at the cast's end state (continuous)
  double cc_time = 0;  // interpolation time of the sub-state / of the closest point along the cast
  int cc_type = 0;     // 0 None (single-timestep contactTest), 1 Time0, 2 Time1, 3 Between
  // the second body of a self contact, as the first's fields
  double p_local_b[3] = { 0, 0, 0 };
  Iso3 transform_b, cc_transform_b;
  double cc_time_b = 0;
  int cc_type_b = 0;
  bool self() const { return sphere_b >= 0; }
  // the contact's link pair in CollisionModel's key space
  int other() const { return self() ? link_b : CollisionModel::kScenePair + prim; }
};

void spherePrimDistance(const double c[3], double r, const double* prim, double& dist, double n[3],
                        double p_robot[3], double p_prim[3]);
// Swept sphere (center a -> b, radius r: a capsule) vs primitive: the signed
// distance min_t d(a + t (b - a)) and its first minimiser t (see collision.cpp).
void sweptSpherePrimDistance(const double a[3], const double b[3], double r, const double* prim, double& dist,
                             double n[3], double p_robot[3], double p_prim[3], double& t_star);
// Robot sphere vs robot sphere (self-collision), see collision.cpp.
void selfSphereDistance(const double a0[3], const double a1[3], double ra, const double b0[3], const double b1[3],
                        double rb, bool cast, double& dist, double n[3], double pa[3], double pb[3], double& sa,
                        double& sb);
std::vector<Contact> calcCollisionsSingle(const CollisionModel& cm, const double* q);
std::vector<Contact> calcCollisions(const CollisionModel& cm, const double* q0, const double* q1, bool vars0_fixed,
                                    bool vars1_fixed);
// GetGradient of one side (0: link_ids[0], the robot sphere; 1: the second
// robot link of a self contact)
void contactGradient(const CollisionModel& cm, const double* dofvals, const Contact& ct, bool timestep1,
                     double* grad, double& scale, int side = 0);
// The linearised distance of a contact over the free ends of its unit
// (CollisionsToDistanceExpressions + CalcDistExpressions*, collision_terms.cpp:
// 341-386, 463-554) as dense coefficients a0 (x_t) / a1 (x_t+1) and constant:
// cleanupAff's 1e-7 per side term, a variable's side terms summed (the QP
// builder sums the duplicates); mask bit e*D+j = coefficient present.
// single: DISCRETE (0 + sum g.(x - q) + d over x_t, scale 1).
void contactExpression(const CollisionModel& cm, const Contact& ct, const double* q0, const double* q1, bool use0,
                       bool use1, bool single, double* a0, double* a1, double& cst, int& mask);

// collision term k of the descriptor: 0 = the coll_* fields, k >= 1 = coll_extra[k - 1]
thip_coll_term collisionTerm(const thip_problem_desc& d, int k);
// the model of collision term `term` (0: the coll_* term, 1 + x: coll_extra[x]),
// with that term's link-pair data (desc.coll_pairs)
std::shared_ptr<CollisionModel> collisionModel(const thip_problem_desc& d, int term, const double* scene);
// CollisionTermInfo::hatch for collision term k: one term object per unit
void addCollisionTerms(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d,
                       const double* scene, int term = 0);
}  // namespace orc
