// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of the LVS-discrete collision term on a primitive scene:
//   DiscreteCollisionEvaluator::CalcCollisions  trajopt/src/collision_terms.cpp:817-898
//   CollisionEvaluator::GetGradient             trajopt/src/collision_terms.cpp:195-242
//   CollisionsToDistanceExpressions             trajopt/src/collision_terms.cpp:341-386
//   CalcDistExpressions{BothFree,..}            trajopt/src/collision_terms.cpp:463-536
//   CollisionCost::convex / value               trajopt/src/collision_terms.cpp:1267-1306
//   removeInvalidContactResults                 trajopt_common/src/collision_utils.cpp:73-114
// Bullet's contactTest is replaced by closed-form sphere-vs-primitive signed
// distance shared with the GPU path ("parity unpinned" against Bullet).
#pragma once
#include <vector>

#include "terms.hpp"

namespace orc
{
void addCollisionTerms(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d,
                       const double* scene);
}
