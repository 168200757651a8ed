// ORACLE — test infrastructure only (see sco_expr.hpp header).
#include "collision.hpp"

#include <stdexcept>

namespace orc
{
void addCollisionTerms(TrajProblem&, const std::vector<VarVector>&, const thip_problem_desc&, const double*)
{
  throw std::runtime_error("collision terms: not yet restated in the oracle");
}
}  // namespace orc
