// Host side: per link-pair collision margins and coefficients of a descriptor
// (include/trajopt_hip.h thip_coll_pair; CollisionTermInfo "pairs",
// problem_description.cpp:1686-1719) lowered into the dense table the device
// code reads: entry (s, j) for robot sphere s and
//   j < n_prims:           the pair (link of s, scene primitive j)
//   j = n_prims + s2:      the pair (link of s, link of sphere s2)
// holds (margin, coeff) of that pair -- the term's own dist_pen / coeffs unless
// an entry overrides them (CollisionMarginData / CollisionCoeffData lookups,
// collision_terms.cpp:243-332, 341-386, 1286-1386).  A pair whose coefficient
// is zero to 1e-6 (hasZeroCoeff: almostEqualRelativeAndAbs(coeff, 0),
// trajopt_common/src/collision_types.cpp:47-72) has its contacts dropped by the
// evaluators' filters (collision_terms.cpp:663-670, 846-870, 1078-1100): its
// margin reads -inf, so no distance is below margin + buffer.
#pragma once
#include <cmath>
#include <limits>
#include <string>
#include <vector>

#include "../../include/trajopt_hip.h"

namespace thip
{
// |coeff| at or below this counts as a zero coefficient (tesseract
// almostEqualRelativeAndAbs default max_diff)
constexpr double kZeroCoeff = 1e-6;

inline std::string validate_coll_pairs(const thip_problem_desc& d)
{
  if (d.n_coll_pairs < 0 || d.n_coll_pairs > THIP_MAX_COLL_PAIRS)
    return "collision: n_coll_pairs out of range";
  for (int k = 0; k < d.n_coll_pairs; ++k)
  {
    const thip_coll_pair& e = d.coll_pairs[k];
    const int terms = (d.coll_enabled ? 1 : 0) + d.n_coll_extra;
    if (e.term < 0 || e.term >= terms)
      return "collision: coll_pairs[" + std::to_string(k) + "].term names no collision term";
    if (e.link < 0 || e.link >= d.chain.n_links)
      return "collision: coll_pairs[" + std::to_string(k) + "].link out of range";
    if (e.other >= 0 ? e.other >= d.n_prims : (-1 - e.other) >= d.chain.n_links)
      return "collision: coll_pairs[" + std::to_string(k) + "].other out of range";
    if (!std::isfinite(e.margin) || !std::isfinite(e.coeff))
      return "collision: coll_pairs[" + std::to_string(k) + "] margin / coeff must be finite";
  }
  return "";
}

// The term's table ([n_spheres][n_prims + n_spheres][2]); false (and an empty
// table) when no entry names this term: every pair then takes the term's own
// margin and coefficient and the device reads the scalars.
inline bool coll_pair_table(const thip_problem_desc& d, int term, std::vector<double>& tab)
{
  tab.clear();
  bool any = false;
  for (int k = 0; k < d.n_coll_pairs; ++k)
    any |= d.coll_pairs[k].term == term;
  if (!any)
    return false;
  // term k is the main term only when it is enabled (k == 0 && coll_enabled);
  // the extra terms follow it (term_eval.hip, validate_coll_pairs)
  const bool main_term = d.coll_enabled && term == 0;
  const int extra = term - (d.coll_enabled ? 1 : 0);
  const double m0 = main_term ? d.coll_margin : d.coll_extra[extra].margin;
  const double c0 = main_term ? d.coll_coeff : d.coll_extra[extra].coeff;
  const int ns = d.n_spheres, P = d.n_prims, W = P + ns;
  tab.assign(static_cast<std::size_t>(ns) * W * 2, 0.0);
  for (int s = 0; s < ns; ++s)
    for (int j = 0; j < W; ++j)
    {
      const int la = d.sphere_link[s];
      const bool prim = j < P;
      const int lb = prim ? -1 : d.sphere_link[j - P];
      // a pair set to a zero coefficient is dropped (only set pairs: a zero term
      // coefficient keeps its contacts, CollisionCoeffData::zero_coeff_ holds set pairs)
      double m = m0, cf = c0;
      bool zero = false;
      for (int k = 0; k < d.n_coll_pairs; ++k)  // in order: the last matching entry wins
      {
        const thip_coll_pair& e = d.coll_pairs[k];
        if (e.term != term)
          continue;
        const bool hit = prim ? (e.other == j && e.link == la)
                              : (e.other < 0 && ((e.link == la && -1 - e.other == lb) ||
                                                 (e.link == lb && -1 - e.other == la)));
        if (hit)
        {
          m = e.margin;
          cf = e.coeff;
          zero = std::fabs(e.coeff) <= kZeroCoeff;
        }
      }
      double* out = &tab[(static_cast<std::size_t>(s) * W + j) * 2];
      out[0] = zero ? -std::numeric_limits<double>::infinity() : m;
      out[1] = cf;
    }
  return true;
}
}  // namespace thip
