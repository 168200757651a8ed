// Host side: the self-collision sphere pairs of a descriptor in key order
// (include/trajopt_hip.h self_pair): link pairs as given; inside a pair the
// spheres of link a, then those of link b, in sphere index order -- the
// insertion order of a key's contacts after the sub-state.  The same list the
// oracle's collisionModel builds (oracle/src/collision.cpp).
#pragma once
#include <string>
#include <vector>

#include "../../include/trajopt_hip.h"

namespace thip
{
// sa / sb: the sphere pairs; kp[k] = first pair of key k (n_self_pairs + 1
// entries).  Returns "" or why the descriptor's pairs are refused.
inline std::string self_sphere_pairs(const thip_problem_desc& d, std::vector<int>& sa, std::vector<int>& sb,
                                     std::vector<int>& kp)
{
  sa.clear();
  sb.clear();
  kp.assign(1, 0);
  if (d.n_self_pairs < 0 || d.n_self_pairs > THIP_MAX_SELF_PAIRS)
    return "collision: n_self_pairs out of range";
  for (int k = 0; k < d.n_self_pairs; ++k)
  {
    const int a = d.self_pair[k][0], b = d.self_pair[k][1];
    if (a < 1 || a >= d.chain.n_links || b < 1 || b >= d.chain.n_links || a == b)
      return "collision: bad self-collision link pair " + std::to_string(k);
    for (int i = 0; i < d.n_spheres; ++i)
      if (d.sphere_link[i] == a)
        for (int j = 0; j < d.n_spheres; ++j)
          if (d.sphere_link[j] == b)
          {
            sa.push_back(i);
            sb.push_back(j);
          }
    kp.push_back(static_cast<int>(sa.size()));
  }
  if (static_cast<int>(sa.size()) > THIP_MAX_SELF_SPHERE_PAIRS)
    return "collision: more than THIP_MAX_SELF_SPHERE_PAIRS self-collision sphere pairs";
  return "";
}
}  // namespace thip
