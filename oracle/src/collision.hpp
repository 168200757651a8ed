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
};

// A contact between a robot link sphere (link_ids[0], active) and a scene
// primitive (link_ids[1], static).
struct Contact
{
  int link = 0, prim = 0, sphere = 0, substate = 0;
  double distance = 0;
  double normal[3];    // from the robot sphere toward the primitive
  double p_robot[3];   // nearest points, world
  double p_prim[3];
  double p_local[3];   // nearest_points_local[0] (robot link frame at the sub-state)
  Iso3 transform;      // robot link pose at the sub-state (discrete) / at the cast's start state (continuous)
  Iso3 cc_transform;   // = transform (discrete) / link pose at the cast's end state (continuous)
  double cc_time = 0;  // interpolation time of the sub-state / of the closest point along the cast
  int cc_type = 0;     // 0 None (single-timestep contactTest), 1 Time0, 2 Time1, 3 Between
};

void spherePrimDistance(const double c[3], double r, const double* prim, double& dist, double n[3],
                        double p_robot[3], double p_prim[3]);
// Swept sphere (center a -> b, radius r: a capsule) vs primitive: the signed
// distance min_t d(a + t (b - a)) and its first minimiser t (see collision.cpp).
void sweptSpherePrimDistance(const double a[3], const double b[3], double r, const double* prim, double& dist,
                             double n[3], double p_robot[3], double p_prim[3], double& t_star);
std::vector<Contact> calcCollisionsSingle(const CollisionModel& cm, const double* q);
std::vector<Contact> calcCollisions(const CollisionModel& cm, const double* q0, const double* q1, bool vars0_fixed,
                                    bool vars1_fixed);
void contactGradient(const CollisionModel& cm, const double* dofvals, const Contact& ct, bool timestep1,
                     double* grad, double& scale);

// collision term k of the descriptor: 0 = the coll_* fields, k >= 1 = coll_extra[k - 1]
thip_coll_term collisionTerm(const thip_problem_desc& d, int k);
std::shared_ptr<CollisionModel> collisionModel(const thip_problem_desc& d, const thip_coll_term& t,
                                               const double* scene);
// CollisionTermInfo::hatch for collision term k: one term object per unit
void addCollisionTerms(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d,
                       const double* scene, int term = 0);
}  // namespace orc
