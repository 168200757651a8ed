#pragma once
#include <vector>

#include "trajopt_ifopt/core/bounds.h"
#include "trajopt_ifopt/core/eigen_types.h"

namespace trajopt_ifopt
{
// |x - lower| below the lower bound, |x - upper| above the upper one, else 0
// (src/utils/ifopt_utils.cpp:122-145)
void calcBoundsViolations(VectorXd& out, const VectorXd& input, const std::vector<Bounds>& bounds);
}  // namespace trajopt_ifopt
