// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// Rounding jitter for the parity gate's oracle-stability proofs
// (tests/parity.py).  The HIP path runs the same algorithm as the oracle with
// a different rounding of every operation: FK in another association order
// (whose rounding the forward-difference CartPose Jacobian amplifies by
// 1/eps = 1e5, to ~1e-11 absolute), ADMM linear algebra in another order (a
// few ulps per KKT solve).  With jitter enabled the oracle re-draws that
// rounding noise: every FD Jacobian entry gets +-jac_abs, every KKT solution
// entry a relative +-kkt_rel, every returned QP solution a relative +-sol_rel
// (the GPU's polished points agree with the oracle's to ~1e-9 relative: the
// delta-regularised polish KKT is ill conditioned), every linearised contact
// expression (collision gradient coefficients and constant: FK and Jacobian
// products in another contraction order) a +-coll_abs, uniform, splitmix64 per
// problem and seed.  Off
// (both 0) unless oracle_set_jitter() was called.
#pragma once
#include <cstdint>

namespace orc
{
struct JitterCfg
{
  double jac_abs = 0;
  double kkt_rel = 0;
  double sol_rel = 0;  // relative jitter of every returned QP solution entry
  double coll_abs = 0;  // absolute jitter of every linearised contact expression's coefficients and constant
  std::uint64_t seed = 0;
};
inline JitterCfg g_jitter;                     // set by oracle_set_jitter before a solve
inline thread_local std::uint64_t t_jitter_state = 0;

inline void jitterSeed(std::uint64_t problem)
{
  t_jitter_state = g_jitter.seed * 0x9E3779B97F4A7C15ULL + problem * 0xBF58476D1CE4E5B9ULL + 1;
}
// uniform in [-1, 1)
inline double jitterU()
{
  std::uint64_t z = (t_jitter_state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return static_cast<double>(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}
}  // namespace orc
