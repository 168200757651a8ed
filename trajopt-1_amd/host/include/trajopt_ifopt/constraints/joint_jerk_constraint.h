#pragma once
#include "trajopt_ifopt/constraints/joint_constraints.h"
