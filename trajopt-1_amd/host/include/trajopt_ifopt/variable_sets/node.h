#pragma once
#include "trajopt_ifopt/variable_sets/nodes_variables.h"
