#pragma once
#include <memory>

#include "trajopt_sqp/qp_problem.h"
#include "trajopt_sqp/types.h"

namespace trajopt_sqp
{
// called after every successful QP step; returning false stops the solve
// (SQPStatus::kStoppedByCallback), include/trajopt_sqp/sqp_callback.h
class SQPCallback
{
public:
  using Ptr = std::shared_ptr<SQPCallback>;
  virtual ~SQPCallback() = default;
  virtual bool execute(const QPProblem& problem, const SQPResults& sqp_results) = 0;
};
}  // namespace trajopt_sqp
