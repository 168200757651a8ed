// ORACLE — test infrastructure only (see sco_expr.hpp header).
#include "collision.hpp"

#include "jitter.hpp"

#include <cmath>
#include <map>
#include <stdexcept>
#include <utility>

namespace orc
{
// ------------------------------------------------------------ signed distance
// Closed-form distance between a robot sphere (center c, radius r) and a scene
// primitive record (16 doubles, include/trajopt_hip.h).  normal points from
// the robot sphere toward the primitive, so d(distance)/d(c) = -normal.
void spherePrimDistance(const double c[3], double r, const double* prim, double& dist, double n[3],
                        double p_robot[3], double p_prim[3])
{
  const int type = static_cast<int>(prim[0]);
  auto sphere_sphere = [&](const double s[3], double rs) {
    double v[3] = { s[0] - c[0], s[1] - c[1], s[2] - c[2] };
    const double L = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (L < 1e-12)
    {
      n[0] = 0;
      n[1] = 0;
      n[2] = 1;
    }
    else
      for (int i = 0; i < 3; ++i)
        n[i] = v[i] / L;
    dist = L - r - rs;
    for (int i = 0; i < 3; ++i)
    {
      p_robot[i] = c[i] + r * n[i];
      p_prim[i] = s[i] - rs * n[i];
    }
  };
  if (type == THIP_PRIM_SPHERE)
  {
    sphere_sphere(prim + 1, prim[4]);
    return;
  }
  if (type == THIP_PRIM_CAPSULE)
  {
    const double* a = prim + 1;
    const double* b = prim + 4;
    const double ab[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] };
    const double den = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
    double t = 0;
    if (den > 1e-24)
      t = ((c[0] - a[0]) * ab[0] + (c[1] - a[1]) * ab[1] + (c[2] - a[2]) * ab[2]) / den;
    t = std::fmin(std::fmax(t, 0.0), 1.0);
    const double s[3] = { a[0] + t * ab[0], a[1] + t * ab[1], a[2] + t * ab[2] };
    sphere_sphere(s, prim[7]);
    return;
  }
  if (type != THIP_PRIM_BOX)
    throw std::runtime_error("unknown scene primitive type");
  const double* ctr = prim + 1;
  const double* R = prim + 4;  // row-major, columns = box axes
  const double* h = prim + 13;
  const double w[3] = { c[0] - ctr[0], c[1] - ctr[1], c[2] - ctr[2] };
  double cl[3];
  for (int i = 0; i < 3; ++i)
    cl[i] = R[0 * 3 + i] * w[0] + R[1 * 3 + i] * w[1] + R[2 * 3 + i] * w[2];
  const bool inside = std::fabs(cl[0]) <= h[0] && std::fabs(cl[1]) <= h[1] && std::fabs(cl[2]) <= h[2];
  double ql[3];
  if (!inside)
  {
    for (int i = 0; i < 3; ++i)
      ql[i] = std::fmin(std::fmax(cl[i], -h[i]), h[i]);
    const double vl[3] = { ql[0] - cl[0], ql[1] - cl[1], ql[2] - cl[2] };
    const double L = std::sqrt(vl[0] * vl[0] + vl[1] * vl[1] + vl[2] * vl[2]);
    for (int i = 0; i < 3; ++i)
      n[i] = (R[i * 3 + 0] * vl[0] + R[i * 3 + 1] * vl[1] + R[i * 3 + 2] * vl[2]) / L;
    dist = L - r;
  }
  else
  {
    int k = 0;
    double depth = h[0] - std::fabs(cl[0]);
    for (int i = 1; i < 3; ++i)
    {
      const double dd = h[i] - std::fabs(cl[i]);
      if (dd < depth)
      {
        depth = dd;
        k = i;
      }
    }
    const double sgn = (cl[k] < 0) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i)
      ql[i] = cl[i];
    ql[k] = sgn * h[k];
    // outward face normal o = sgn R e_k; the normal toward the obstacle is -o
    for (int i = 0; i < 3; ++i)
      n[i] = -sgn * R[i * 3 + k];
    dist = -depth - r;
  }
  for (int i = 0; i < 3; ++i)
  {
    p_prim[i] = ctr[i] + R[i * 3 + 0] * ql[0] + R[i * 3 + 1] * ql[1] + R[i * 3 + 2] * ql[2];
    p_robot[i] = c[i] + r * n[i];
  }
}

// ------------------------------------------------------------ swept sphere
// Bullet's cast (castVsCast on the convex hull of the link shape at the two
// poses) replaced for a sphere: its center moves on the segment a -> b, so
// the swept shape is a capsule.  dist = min over t in [0, 1] of the sphere's
// signed distance at a + t (b - a); t_star is the minimiser chosen by a fixed
// rule (closed form for spheres and capsules; for boxes the smallest value
// among the breakpoints and piecewise stationary points of the box SDF along
// the segment, ties within 1e-14 to the smaller t).  The same rule runs on
// the GPU (collision_device.hpp).
namespace
{
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// Closest points of segments p1 + s d1 and p2 + t d2 (s, t in [0, 1]);
// returns s (Ericson, Real-Time Collision Detection 5.1.9).
double segSegParam(const double p1[3], const double d1[3], const double p2[3], const double d2[3])
{
  const double r[3] = { p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2] };
  const double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  const double eps = 1e-24;
  double s, t;
  if (a <= eps && e <= eps)
    return 0.0;
  if (a <= eps)
    return 0.0;
  const double cc = dot3(d1, r);
  if (e <= eps)
    return std::fmin(std::fmax(-cc / a, 0.0), 1.0);
  const double b = dot3(d1, d2);
  const double denom = a * e - b * b;
  s = (denom > eps) ? std::fmin(std::fmax((b * f - cc * e) / denom, 0.0), 1.0) : 0.0;
  t = (b * s + f) / e;
  if (t < 0.0)
    s = std::fmin(std::fmax(-cc / a, 0.0), 1.0);
  else if (t > 1.0)
    s = std::fmin(std::fmax((b - cc) / a, 0.0), 1.0);
  return s;
}

// Both parameters of the closest points of segments p1 + s d1 and p2 + t d2
// (Ericson 5.1.9, s as segSegParam computes it)
void segSegParams(const double p1[3], const double d1[3], const double p2[3], const double d2[3], double& s, double& t)
{
  const double r[3] = { p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2] };
  const double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  const double eps = 1e-24;
  if (a <= eps && e <= eps)
  {
    s = t = 0.0;
    return;
  }
  if (a <= eps)
  {
    s = 0.0;
    t = std::fmin(std::fmax(f / e, 0.0), 1.0);
    return;
  }
  const double cc = dot3(d1, r);
  if (e <= eps)
  {
    t = 0.0;
    s = std::fmin(std::fmax(-cc / a, 0.0), 1.0);
    return;
  }
  const double b = dot3(d1, d2);
  const double denom = a * e - b * b;
  s = (denom > eps) ? std::fmin(std::fmax((b * f - cc * e) / denom, 0.0), 1.0) : 0.0;
  t = (b * s + f) / e;
  if (t < 0.0)
  {
    t = 0.0;
    s = std::fmin(std::fmax(-cc / a, 0.0), 1.0);
  }
  else if (t > 1.0)
  {
    t = 1.0;
    s = std::fmin(std::fmax((b - cc) / a, 0.0), 1.0);
  }
}
}  // namespace

// Robot sphere a vs robot sphere b (self-collision), both moving: centers
// a0 -> a1 and b0 -> b1 over a cast (a1 = a0, b1 = b0 for one state).  The swept
// shapes are two capsules; their distance is the closest points (sa, sb) of the
// two center segments, each side's own time along its cast (the cast hulls are
// independent, not synchronised).  normal from a toward b.
void selfSphereDistance(const double a0[3], const double a1[3], double ra, const double b0[3], const double b1[3],
                        double rb, bool cast, double& dist, double n[3], double pa[3], double pb[3], double& sa,
                        double& sb)
{
  const double da[3] = { a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2] };
  const double db[3] = { b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2] };
  sa = sb = 0.0;
  if (cast)
    segSegParams(a0, da, b0, db, sa, sb);
  double ca[3], cb[3];
  for (int i = 0; i < 3; ++i)
  {
    ca[i] = a0[i] + sa * da[i];
    cb[i] = b0[i] + sb * db[i];
  }
  const double v[3] = { cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2] };
  const double L = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (L < 1e-12)
  {
    n[0] = 0;
    n[1] = 0;
    n[2] = 1;
  }
  else
    for (int i = 0; i < 3; ++i)
      n[i] = v[i] / L;
  dist = L - ra - rb;
  for (int i = 0; i < 3; ++i)
  {
    pa[i] = ca[i] + ra * n[i];
    pb[i] = cb[i] - rb * n[i];
  }
}

void sweptSpherePrimDistance(const double a[3], const double b[3], double r, const double* prim, double& dist,
                             double n[3], double p_robot[3], double p_prim[3], double& t_star)
{
  const int type = static_cast<int>(prim[0]);
  const double u[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] };
  const double uu = dot3(u, u);
  auto at = [&](double t, double c[3]) {
    for (int i = 0; i < 3; ++i)
      c[i] = a[i] + t * u[i];
  };
  double t = 0.0;
  if (type == THIP_PRIM_SPHERE)
  {
    const double w[3] = { prim[1] - a[0], prim[2] - a[1], prim[3] - a[2] };
    t = (uu > 1e-24) ? std::fmin(std::fmax(dot3(w, u) / uu, 0.0), 1.0) : 0.0;
  }
  else if (type == THIP_PRIM_CAPSULE)
  {
    const double d2[3] = { prim[4] - prim[1], prim[5] - prim[2], prim[6] - prim[3] };
    t = segSegParam(a, u, prim + 1, d2);
  }
  else
  {
    // box: a and u in box coordinates
    const double* ctr = prim + 1;
    const double* R = prim + 4;
    const double* h = prim + 13;
    const double w[3] = { a[0] - ctr[0], a[1] - ctr[1], a[2] - ctr[2] };
    double al[3], ul[3];
    for (int i = 0; i < 3; ++i)
    {
      al[i] = R[0 * 3 + i] * w[0] + R[1 * 3 + i] * w[1] + R[2 * 3 + i] * w[2];
      ul[i] = R[0 * 3 + i] * u[0] + R[1 * 3 + i] * u[1] + R[2 * 3 + i] * u[2];
    }
    // breakpoints where a coordinate crosses a face plane or zero (the kink
    // of |p_i|), sorted
    double bp[11];
    int nb = 0;
    bp[nb++] = 0.0;
    for (int i = 0; i < 3; ++i)
      if (std::fabs(ul[i]) > 1e-300)
        for (int sg = -1; sg <= 1; ++sg)
        {
          const double tb = (sg * h[i] - al[i]) / ul[i];
          if (tb > 0.0 && tb < 1.0)
            bp[nb++] = tb;
        }
    bp[nb++] = 1.0;
    for (int i = 1; i < nb; ++i)  // insertion sort
      for (int j = i; j > 0 && bp[j - 1] > bp[j]; --j)
      {
        const double tmp = bp[j];
        bp[j] = bp[j - 1];
        bp[j - 1] = tmp;
      }
    double cand[48];
    int nc = 0;
    for (int k = 0; k < nb; ++k)
      cand[nc++] = bp[k];
    for (int k = 0; k + 1 < nb; ++k)
    {
      const double t0 = bp[k], t1 = bp[k + 1];
      if (!(t1 > t0))
        continue;
      const double tm = 0.5 * (t0 + t1);
      double sg[3];
      bool out = false;
      for (int i = 0; i < 3; ++i)
      {
        const double pm = al[i] + tm * ul[i];
        sg[i] = (pm < 0) ? -1.0 : 1.0;
        out = out || (std::fabs(pm) > h[i]);
      }
      if (out)
      {
        // outside: minimise sum over the outside axes of (p_i - sg_i h_i)^2
        double num = 0, den = 0;
        for (int i = 0; i < 3; ++i)
        {
          const double pm = al[i] + tm * ul[i];
          if (std::fabs(pm) > h[i])
          {
            num += (al[i] - sg[i] * h[i]) * ul[i];
            den += ul[i] * ul[i];
          }
        }
        if (den > 0)
          cand[nc++] = std::fmin(std::fmax(-num / den, t0), t1);
      }
      else
        // inside: max_i (sg_i p_i - h_i); stationary points where two terms are equal
        for (int i = 0; i < 3; ++i)
          for (int j = i + 1; j < 3; ++j)
          {
            const double den = sg[i] * ul[i] - sg[j] * ul[j];
            if (std::fabs(den) > 1e-300)
            {
              const double tc = (h[i] - h[j] - sg[i] * al[i] + sg[j] * al[j]) / den;
              if (tc > t0 && tc < t1)
                cand[nc++] = tc;
            }
          }
    }
    // the smallest value; among values within 1e-14 of it, the smallest t
    double val[48];
    double best = 0;
    for (int k = 0; k < nc; ++k)
    {
      double c[3], nn[3], pr[3], pp[3];
      at(cand[k], c);
      spherePrimDistance(c, r, prim, val[k], nn, pr, pp);
      best = (k == 0) ? val[k] : std::fmin(best, val[k]);
    }
    double bt = 2.0;
    for (int k = 0; k < nc; ++k)
      if (val[k] <= best + 1e-14 && cand[k] < bt)
        bt = cand[k];
    t = bt;
  }
  double c[3];
  at(t, c);
  spherePrimDistance(c, r, prim, dist, n, p_robot, p_prim);
  t_star = t;
}

namespace
{
// Eigen::VectorXd::LinSpaced(size, low, high)(i) for floating point
// (Eigen 3.4 linspaced_op_impl<Scalar, false>)
double linspaced(int size, double low, double high, int i)
{
  if (size == 1)
    return high;
  const int size1 = size - 1;
  const double step = (high - low) / size1;
  const bool flip = std::fabs(high) < std::fabs(low);
  if (flip)
    return (i == 0) ? low : high - double(size1 - i) * step;
  return (i == size1) ? high : low + double(i) * step;
}

constexpr int kCCNone = 0, kCCTime0 = 1, kCCTime1 = 2, kCCBetween = 3;
}  // namespace

namespace
{
void sphereWorld(const Iso3& T, const double* cl, double* c)
{
  for (int r = 0; r < 3; ++r)
    c[r] = T.R[r * 3 + 0] * cl[0] + T.R[r * 3 + 1] * cl[1] + T.R[r * 3 + 2] * cl[2] + T.t[r];
}

void toLocal(const Iso3& T, const double* p, double* pl)
{
  const double w[3] = { p[0] - T.t[0], p[1] - T.t[1], p[2] - T.t[2] };
  for (int r = 0; r < 3; ++r)
    pl[r] = T.R[0 * 3 + r] * w[0] + T.R[1 * 3 + r] * w[1] + T.R[2 * 3 + r] * w[2];
}

// removeInvalidContactResults (collision_utils.cpp:73-114) at the fixed ends:
// keep a contact when one of its active sides is not at the fixed end
bool keepAtFixedEnds(const Contact& ct, bool vars0_fixed, bool vars1_fixed)
{
  if (!vars0_fixed && !vars1_fixed)
    return true;
  const int ta = ct.cc_type, tb = ct.self() ? ct.cc_type_b : kCCNone;
  if (vars0_fixed && ((ta != kCCNone && ta != kCCTime0) || (tb != kCCNone && tb != kCCTime0)))
    return true;
  if (vars1_fixed && ((ta != kCCNone && ta != kCCTime1) || (tb != kCCNone && tb != kCCTime1)))
    return true;
  return false;
}

// Self contacts of sub-state i (a cast i -> i + 1 when T1 is given) appended to
// their keys' lists.  mode 0: DISCRETE (CCType_None), 1: LVS_DISCRETE (both
// sides at the sub-state's time i dt), 2: LVS_CONTINUOUS (each side its own
// closest-point time, (i + s) dt).
void addSelfContacts(const CollisionModel& cm, const std::vector<Iso3>& T, const std::vector<Iso3>* T1, int i,
                     long last, double dt, int mode, bool vars0_fixed, bool vars1_fixed,
                     std::vector<std::vector<Contact>>& keys)
{
  for (std::size_t j = 0; j < cm.self_a.size(); ++j)
  {
    const int sa = cm.self_a[j], sb = cm.self_b[j];
    const int la = cm.sphere_link[sa], lb = cm.sphere_link[sb];
    // the pair's contact distance (its margin + the buffer); a zero-coefficient
    // pair's contacts are cleared by the filter
    if (cm.hasZeroCoeff(la, lb))
      continue;
    const double margin = cm.marginOf(la, lb), threshold = margin + cm.buffer;
    const Iso3 &Ta = T[static_cast<std::size_t>(la)], &Tb = T[static_cast<std::size_t>(lb)];
    const Iso3& Ta1 = T1 ? (*T1)[static_cast<std::size_t>(la)] : Ta;
    const Iso3& Tb1 = T1 ? (*T1)[static_cast<std::size_t>(lb)] : Tb;
    double a0[3], a1[3], b0[3], b1[3];
    sphereWorld(Ta, cm.sphere_center[sa], a0);
    sphereWorld(Ta1, cm.sphere_center[sa], a1);
    sphereWorld(Tb, cm.sphere_center[sb], b0);
    sphereWorld(Tb1, cm.sphere_center[sb], b1);
    Contact ct;
    double ta = 0, tb = 0;
    selfSphereDistance(a0, a1, cm.sphere_radius[sa], b0, b1, cm.sphere_radius[sb], mode == 2, ct.distance, ct.normal,
                       ct.p_robot, ct.p_prim, ta, tb);
    if (!(ct.distance < threshold))  // contactTest: within the pair's contact distance
      continue;
    ct.link = la;
    ct.sphere = sa;
    ct.prim = -1 - sb;
    ct.link_b = lb;
    ct.sphere_b = sb;
    ct.substate = i;
    ct.transform = Ta;
    ct.cc_transform = Ta1;
    ct.transform_b = Tb;
    ct.cc_transform_b = Tb1;
    toLocal(Ta, ct.p_robot, ct.p_local);
    toLocal(Tb, ct.p_prim, ct.p_local_b);
    if (mode == 0)
    {
      ct.cc_time = ct.cc_time_b = 0;
      ct.cc_type = ct.cc_type_b = kCCNone;
    }
    else if (mode == 1)
    {
      ct.cc_time = ct.cc_time_b = double(i) * dt;
      ct.cc_type = ct.cc_type_b = (i == 0) ? kCCTime0 : ((i == last) ? kCCTime1 : kCCBetween);
    }
    else
    {
      ct.cc_time = (double(i) + ta) * dt;
      ct.cc_time_b = (double(i) + tb) * dt;
      ct.cc_type = (i == 0 && ta == 0.0) ? kCCTime0 : ((i + 1 == last && ta == 1.0) ? kCCTime1 : kCCBetween);
      ct.cc_type_b = (i == 0 && tb == 0.0) ? kCCTime0 : ((i + 1 == last && tb == 1.0) ? kCCTime1 : kCCBetween);
    }
    (void)vars0_fixed;
    (void)vars1_fixed;  // (the evaluator's filter runs after the test: applyContactTest)
    keys[static_cast<std::size_t>(cm.self_key[j])].push_back(ct);
  }
}

// One contactTest call's contacts (the candidates within their pair's contact
// distance, per key in ContactResultMap order), reduced as the request's test
// type returns them (trajopt_hip.h THIP_CONTACT_*: ALL every one, CLOSEST the
// smallest distance per key -- the first on ties --, FIRST the first of the whole
// call), then the evaluator's filter (removeInvalidContactResults,
// collision_utils.cpp:73-114: beyond margin + buffer, at a fixed end) and
// appended to the run's key lists (addInterpolatedCollisionResults,
// collision_terms.cpp:880-897).
void applyContactTest(const CollisionModel& cm, std::map<std::pair<int, int>, std::vector<Contact>>& call_scene,
                      std::vector<std::vector<Contact>>& call_self, bool vars0_fixed, bool vars1_fixed,
                      std::map<std::pair<int, int>, std::vector<Contact>>& results,
                      std::vector<std::vector<Contact>>& self)
{
  auto filter = [&](const Contact& ct) {
    return !(ct.distance > cm.marginOf(ct.link, ct.other()) + cm.buffer) && keepAtFixedEnds(ct, vars0_fixed, vars1_fixed);
  };
  auto closest = [](const std::vector<Contact>& v) {
    std::size_t best = 0;
    for (std::size_t k = 1; k < v.size(); ++k)
      if (v[k].distance < v[best].distance)
        best = k;
    return best;
  };
  if (cm.contact_test == THIP_CONTACT_FIRST)
  {
    const Contact* first = nullptr;
    std::pair<int, int> key;
    int skey = -1;
    for (auto& kv : call_scene)
      if (!kv.second.empty())
      {
        first = &kv.second.front();
        key = kv.first;
        break;
      }
    for (std::size_t k = 0; !first && k < call_self.size(); ++k)
      if (!call_self[k].empty())
      {
        first = &call_self[k].front();
        skey = static_cast<int>(k);
      }
    if (first && filter(*first))
    {
      if (skey < 0)
        results[key].push_back(*first);
      else
        self[static_cast<std::size_t>(skey)].push_back(*first);
    }
    return;
  }
  for (auto& kv : call_scene)
  {
    if (kv.second.empty())
      continue;
    if (cm.contact_test == THIP_CONTACT_CLOSEST)
    {
      const Contact& ct = kv.second[closest(kv.second)];
      if (filter(ct))
        results[kv.first].push_back(ct);
    }
    else
      for (const Contact& ct : kv.second)
        if (filter(ct))
          results[kv.first].push_back(ct);
  }
  for (std::size_t k = 0; k < call_self.size(); ++k)
  {
    if (call_self[k].empty())
      continue;
    if (cm.contact_test == THIP_CONTACT_CLOSEST)
    {
      const Contact& ct = call_self[k][closest(call_self[k])];
      if (filter(ct))
        self[k].push_back(ct);
    }
    else
      for (const Contact& ct : call_self[k])
        if (filter(ct))
          self[k].push_back(ct);
  }
}

// the flattened map: scene keys (link, primitive), then the self keys in order
std::vector<Contact> flatten(std::map<std::pair<int, int>, std::vector<Contact>>& scene,
                             std::vector<std::vector<Contact>>& self)
{
  std::vector<Contact> flat;
  for (auto& kv : scene)
    flat.insert(flat.end(), kv.second.begin(), kv.second.end());
  for (auto& v : self)
    flat.insert(flat.end(), v.begin(), v.end());
  return flat;
}
}  // namespace

// SingleTimestepCollisionEvaluator::CalcCollisions (collision_terms.cpp:653-688):
// FK at one state, contactTest, then the filter drops contacts beyond
// margin + buffer (no cc_type filtering; the results keep CCType_None).
std::vector<Contact> calcCollisionsSingle(const CollisionModel& cm, const double* q)
{
  const thip_chain& ch = *cm.chain;
  std::map<std::pair<int, int>, std::vector<Contact>> results, call;
  std::vector<std::vector<Contact>> self(static_cast<std::size_t>(cm.n_self_keys)), call_self(self.size());
  std::vector<Iso3> T;
  chainFwdKin(ch, q, T);
  for (int s = 0; s < cm.n_spheres; ++s)
  {
    const int link = cm.sphere_link[s];
    const Iso3& Tl = T[static_cast<std::size_t>(link)];
    double c[3];
    sphereWorld(Tl, cm.sphere_center[s], c);
    for (int p = 0; p < cm.n_prims; ++p)
    {
      const int pk = CollisionModel::kScenePair + p;
      if (cm.hasZeroCoeff(link, pk))
        continue;
      const double margin = cm.marginOf(link, pk), threshold = margin + cm.buffer;
      Contact ct;
      spherePrimDistance(c, cm.sphere_radius[s], cm.scene + 16 * p, ct.distance, ct.normal, ct.p_robot, ct.p_prim);
      if (!(ct.distance < threshold))
        continue;
      ct.link = link;
      ct.prim = p;
      ct.sphere = s;
      ct.substate = 0;
      ct.transform = Tl;
      ct.cc_transform = Tl;
      toLocal(Tl, ct.p_robot, ct.p_local);
      ct.cc_time = 0;
      ct.cc_type = 0;  // CCType_None
      call[{ link, p }].push_back(ct);
    }
  }
  addSelfContacts(cm, T, nullptr, 0, 0, 0.0, 0, false, false, call_self);
  applyContactTest(cm, call, call_self, false, false, results, self);
  return flatten(results, self);
}

// DiscreteCollisionEvaluator::CalcCollisions (collision_terms.cpp:817-898) for
// the step pair (q0, q1); results flattened in ContactResultMap order: link
// pair key (robot link, primitive), then the self keys, then insertion
// (sub-state, sphere).
std::vector<Contact> calcCollisions(const CollisionModel& cm, const double* q0, const double* q1, bool vars0_fixed,
                                    bool vars1_fixed)
{
  const thip_chain& ch = *cm.chain;
  const int D = ch.n_dof;
  double dist = 0;
  for (int j = 0; j < D; ++j)
    dist += (q1[j] - q0[j]) * (q1[j] - q0[j]);
  dist = std::sqrt(dist);
  long cnt = 2;
  if (dist > cm.lvs)
    cnt = static_cast<long>(std::ceil(dist / cm.lvs)) + 1;
  const long last = cnt - 1;
  const double dt = 1.0 / double(last);
  // per pair: contact distance margin + buffer (incrementCollisionMargin(buffer));
  // zero-coefficient pairs are cleared by the filter
  std::map<std::pair<int, int>, std::vector<Contact>> results;
  std::vector<std::vector<Contact>> self(static_cast<std::size_t>(cm.n_self_keys));
  std::vector<double> q(static_cast<std::size_t>(D));
  std::vector<Iso3> T;
  if (cm.continuous)
  {
    // CastCollisionEvaluator::CalcCollisions (collision_terms.cpp:1106-1161): one cast per
    // consecutive sub-state pair (a single cast q0 -> q1 when dist <= lvs); the contact's
    // cc_time is the closest point's time along the whole step pair,
    // (i + t) / (cnt - 1) (addInterpolatedCollisionResults, discrete = false)
    std::vector<Iso3> T1;
    std::vector<double> qn(static_cast<std::size_t>(D));
    for (long i = 0; i + 1 < cnt; ++i)
    {
      std::map<std::pair<int, int>, std::vector<Contact>> call;
      std::vector<std::vector<Contact>> call_self(self.size());
      for (int j = 0; j < D; ++j)
      {
        q[static_cast<std::size_t>(j)] = linspaced(static_cast<int>(cnt), q0[j], q1[j], static_cast<int>(i));
        qn[static_cast<std::size_t>(j)] = linspaced(static_cast<int>(cnt), q0[j], q1[j], static_cast<int>(i + 1));
      }
      chainFwdKin(ch, q.data(), T);
      chainFwdKin(ch, qn.data(), T1);
      for (int s = 0; s < cm.n_spheres; ++s)
      {
        const int link = cm.sphere_link[s];
        const Iso3& Ta = T[static_cast<std::size_t>(link)];
        const Iso3& Tb = T1[static_cast<std::size_t>(link)];
        double ca[3], cb[3];
        sphereWorld(Ta, cm.sphere_center[s], ca);
        sphereWorld(Tb, cm.sphere_center[s], cb);
        for (int p = 0; p < cm.n_prims; ++p)
        {
          const int pk = CollisionModel::kScenePair + p;
          if (cm.hasZeroCoeff(link, pk))
            continue;
          const double margin = cm.marginOf(link, pk), threshold = margin + cm.buffer;
          Contact ct;
          double ts = 0;
          sweptSpherePrimDistance(ca, cb, cm.sphere_radius[s], cm.scene + 16 * p, ct.distance, ct.normal, ct.p_robot,
                                  ct.p_prim, ts);
          if (!(ct.distance < threshold))
            continue;
          ct.link = link;
          ct.prim = p;
          ct.sphere = s;
          ct.substate = static_cast<int>(i);
          ct.transform = Ta;
          ct.cc_transform = Tb;
          // nearest_points_local[0] in the link frame at the cast's start state
          toLocal(Ta, ct.p_robot, ct.p_local);
          ct.cc_time = (double(i) + ts) * dt;
          ct.cc_type = (i == 0 && ts == 0.0) ? kCCTime0 : ((i + 1 == last && ts == 1.0) ? kCCTime1 : kCCBetween);
          call[{ link, p }].push_back(ct);
        }
      }
      addSelfContacts(cm, T, &T1, static_cast<int>(i), last, dt, 2, vars0_fixed, vars1_fixed, call_self);
      applyContactTest(cm, call, call_self, vars0_fixed, vars1_fixed, results, self);
    }
    return flatten(results, self);
  }
  for (long i = 0; i < cnt; ++i)
  {
    std::map<std::pair<int, int>, std::vector<Contact>> call;
    std::vector<std::vector<Contact>> call_self(self.size());
    for (int j = 0; j < D; ++j)
      q[static_cast<std::size_t>(j)] = linspaced(static_cast<int>(cnt), q0[j], q1[j], static_cast<int>(i));
    chainFwdKin(ch, q.data(), T);
    for (int s = 0; s < cm.n_spheres; ++s)
    {
      const int link = cm.sphere_link[s];
      const Iso3& Tl = T[static_cast<std::size_t>(link)];
      double c[3];
      sphereWorld(Tl, cm.sphere_center[s], c);
      for (int p = 0; p < cm.n_prims; ++p)
      {
        const int pk = CollisionModel::kScenePair + p;
        if (cm.hasZeroCoeff(link, pk))
          continue;
        const double margin = cm.marginOf(link, pk), threshold = margin + cm.buffer;
        Contact ct;
        spherePrimDistance(c, cm.sphere_radius[s], cm.scene + 16 * p, ct.distance, ct.normal, ct.p_robot,
                           ct.p_prim);
        if (!(ct.distance < threshold))  // contactTest: within the contact distance
          continue;
        ct.link = link;
        ct.prim = p;
        ct.sphere = s;
        ct.substate = static_cast<int>(i);
        ct.transform = Tl;
        ct.cc_transform = Tl;
        // nearest_points_local[0]: the robot point in the link frame
        toLocal(Tl, ct.p_robot, ct.p_local);
        // addInterpolatedCollisionResults(.., discrete = true): active link only
        ct.cc_time = double(i) * dt;
        ct.cc_type = (i == 0) ? kCCTime0 : ((i == last) ? kCCTime1 : kCCBetween);
        // (filter after the test: applyContactTest; the static primitive has CCType_None)
        call[{ link, p }].push_back(ct);
      }
    }
    addSelfContacts(cm, T, nullptr, static_cast<int>(i), last, dt, 1, vars0_fixed, vars1_fixed, call_self);
    applyContactTest(cm, call, call_self, vars0_fixed, vars1_fixed, results, self);
  }
  return flatten(results, self);
}

// CollisionEvaluator::GetGradient (collision_terms.cpp:195-242) for the robot
// link (link_ids[0]): jacobian at the step's own joint values, reference point
// moved to transform.linear() * nearest_points_local (the sub-state pose; for
// discrete-continuous results cc_transform == transform), gradient
// -normal^T J_lin, scale 1 - cc_time (timestep 0) or cc_time (timestep 1).
void contactGradient(const CollisionModel& cm, const double* dofvals, const Contact& ct, bool timestep1,
                     double* grad, double& scale, int side)
{
  const thip_chain& ch = *cm.chain;
  const int D = ch.n_dof;
  double J[6 * THIP_MAX_DOF];
  const bool b = side == 1;
  chainJacobian(ch, dofvals, b ? ct.link_b : ct.link, J);
  // scale 1 and link_transform = transform for CCType_None; otherwise scale
  // (1 - cc_time) / cc_time and link_transform = transform / cc_transform
  // (collision_terms.cpp:214-221)
  const int type = b ? ct.cc_type_b : ct.cc_type;
  const double cc_time = b ? ct.cc_time_b : ct.cc_time;
  const bool none = type == kCCNone;
  const Iso3& lt = (timestep1 && !none) ? (b ? ct.cc_transform_b : ct.cc_transform) : (b ? ct.transform_b : ct.transform);
  const double* pl = b ? ct.p_local_b : ct.p_local;
  double r[3];
  for (int i = 0; i < 3; ++i)
    r[i] = lt.R[i * 3 + 0] * pl[0] + lt.R[i * 3 + 1] * pl[1] + lt.R[i * 3 + 2] * pl[2];
  scale = none ? 1.0 : (timestep1 ? cc_time : (1 - cc_time));
  // gradient = (i == 0 ? -1 : 1) * normal^T J_lin (collision_terms.cpp:232)
  const double sg = b ? 1.0 : -1.0;
  for (int j = 0; j < D; ++j)
  {
    // jacobianChangeRefPoint: J_lin += J_ang x r
    const double wx = J[3 * D + j], wy = J[4 * D + j], wz = J[5 * D + j];
    const double l0 = J[0 * D + j] + (wy * r[2] - wz * r[1]);
    const double l1 = J[1 * D + j] + (wz * r[0] - wx * r[2]);
    const double l2 = J[2 * D + j] + (wx * r[1] - wy * r[0]);
    grad[j] = sg * (ct.normal[0] * l0 + ct.normal[1] * l1 + ct.normal[2] * l2);
  }
}

namespace
{
// parity-gate rounding jitter of a contact expression (jitter.hpp coll_abs)
void jitterContact(int D, double* a0, double* a1, double& cst, int mask)
{
  if (!(g_jitter.coll_abs > 0))
    return;
  for (int j = 0; j < D; ++j)
  {
    if (mask & (1 << j))
      a0[j] += g_jitter.coll_abs * jitterU();
    if (mask & (1 << (D + j)))
      a1[j] += g_jitter.coll_abs * jitterU();
  }
  cst += g_jitter.coll_abs * jitterU();
}
}  // namespace

void contactExpression(const CollisionModel& cm, const Contact& ct, const double* q0, const double* q1, bool use0,
                       bool use1, bool single, double* a0, double* a1, double& cst, int& mask)
{
  const int D = cm.chain->n_dof;
  const int nsides = ct.self() ? 2 : 1;
  mask = 0;
  for (int j = 0; j < D; ++j)
    a0[j] = a1[j] = 0.0;
  // one timestep's part (CollisionsToDistanceExpressions): per side varDot(scale g, vars)
  // and scale * -g.q, the constant summed over the sides from 0
  auto part = [&](const double* q, bool ts1, double* a, int bit0) {
    double c = 0.0;
    for (int side = 0; side < nsides; ++side)
    {
      double g[THIP_MAX_DOF], scale, gd = 0;
      contactGradient(cm, q, ct, ts1, g, scale, side);
      for (int j = 0; j < D; ++j)
      {
        const double av = scale * g[j];
        gd += g[j] * q[j];
        if (std::fabs(av) > 1e-7)  // cleanupAff
        {
          a[j] = (mask & (1 << (bit0 + j))) ? a[j] + av : av;
          mask |= 1 << (bit0 + j);
        }
      }
      c += scale * -gd;
    }
    return c;
  };
  if (single)
  {
    // CalcDistExpressionsSingleTimeStep: 0 + part(x_t), then + d
    cst = 0.0 + part(q0, false, a0, 0);
    cst += ct.distance;
    jitterContact(D, a0, a1, cst, mask);
    return;
  }
  // CalcDistExpressions{BothFree, StartFree, EndFree}: d + part(x_t) + part(x_t+1)
  cst = ct.distance;
  if (use0)
    cst += part(q0, false, a0, 0);
  if (use1)
    cst += part(q1, true, a1, D);
  jitterContact(D, a0, a1, cst, mask);
}

namespace
{
// The distance expressions of one step pair (CollisionEvaluator::CalcDistExpressions,
// LVS_DISCRETE evaluator, collision_terms.cpp:463-536) shared by the cost and
// constraint forms below.
class CollisionPairCalc
{
public:
  CollisionPairCalc(std::shared_ptr<const CollisionModel> cm, VarVector v0, VarVector v1, int type)
    : cm_(std::move(cm)), vars0_(std::move(v0)), vars1_(std::move(v1)), type_(type)
  {
  }

  VarVector vars() const
  {
    VarVector v = vars0_;
    v.insert(v.end(), vars1_.begin(), vars1_.end());
    return v;
  }

  std::vector<Contact> collide(const DblVec& x) const
  {
    const DblVec q0 = getDblVec(x, vars0_), q1 = getDblVec(x, vars1_);
    return calcCollisions(*cm_, q0.data(), q1.data(), type_ == kStartFixedEndFree, type_ == kStartFreeEndFixed);
  }

  // dist = d + sum scale * g (q - q0) over the free ends, cleanupAff'd
  AffExprVector exprs(const DblVec& x, std::vector<Contact>* cts = nullptr) const
  {
    AffExprVector out;
    const auto contacts = collide(x);
    if (cts)
      *cts = contacts;
    const DblVec q0 = getDblVec(x, vars0_), q1 = getDblVec(x, vars1_);
    const int D = cm_->chain->n_dof;
    for (const auto& c : contacts)
    {
      double a0[THIP_MAX_DOF], a1[THIP_MAX_DOF], cst;
      int mask;
      contactExpression(*cm_, c, q0.data(), q1.data(), type_ != kStartFixedEndFree, type_ != kStartFreeEndFixed,
                        false, a0, a1, cst, mask);
      AffExpr e(cst);
      for (int j = 0; j < D; ++j)
        if (mask & (1 << j))
        {
          e.coeffs.push_back(a0[j]);
          e.vars.push_back(vars0_[static_cast<std::size_t>(j)]);
        }
      for (int j = 0; j < D; ++j)
        if (mask & (1 << (D + j)))
        {
          e.coeffs.push_back(a1[j]);
          e.vars.push_back(vars1_[static_cast<std::size_t>(j)]);
        }
      out.push_back(e);
    }
    return out;
  }

  const CollisionModel& model() const { return *cm_; }

  static constexpr int kBothFree = 0, kStartFixedEndFree = 1, kStartFreeEndFixed = 2;

private:
  std::shared_ptr<const CollisionModel> cm_;
  VarVector vars0_, vars1_;
  int type_;
};

// The distance expressions of one waypoint (DISCRETE evaluator,
// CalcDistExpressionsSingleTimeStep, collision_terms.cpp:538-554):
// dist = 0 + g.x - g.q (CollisionsToDistanceExpressions with vars0, scale 1),
// then + d, cleanupAff'd.
class CollisionSingleCalc
{
public:
  CollisionSingleCalc(std::shared_ptr<const CollisionModel> cm, VarVector v0) : cm_(std::move(cm)), vars0_(std::move(v0))
  {
  }

  VarVector vars() const { return vars0_; }

  std::vector<Contact> collide(const DblVec& x) const
  {
    const DblVec q = getDblVec(x, vars0_);
    return calcCollisionsSingle(*cm_, q.data());
  }

  AffExprVector exprs(const DblVec& x, std::vector<Contact>* cts = nullptr) const
  {
    AffExprVector out;
    const auto contacts = collide(x);
    if (cts)
      *cts = contacts;
    const DblVec q = getDblVec(x, vars0_);
    const int D = cm_->chain->n_dof;
    for (const auto& c : contacts)
    {
      double a0[THIP_MAX_DOF], a1[THIP_MAX_DOF], cst;
      int mask;
      contactExpression(*cm_, c, q.data(), q.data(), true, false, true, a0, a1, cst, mask);
      AffExpr e(cst);
      for (int j = 0; j < D; ++j)
        if (mask & (1 << j))
        {
          e.coeffs.push_back(a0[j]);
          e.vars.push_back(vars0_[static_cast<std::size_t>(j)]);
        }
      out.push_back(e);
    }
    return out;
  }

  const CollisionModel& model() const { return *cm_; }

private:
  std::shared_ptr<const CollisionModel> cm_;
  VarVector vars0_;
};

// One CollisionCost term per step pair (CollisionTermInfo::hatch,
// problem_description.cpp:1735-1781) or per free waypoint (DISCRETE, :1782-1796).
template <class Calc>
class CollisionPairCost : public Cost
{
public:
  explicit CollisionPairCost(Calc calc) : calc_(std::move(calc)) {}
  VarVector getVars() override { return calc_.vars(); }

  // CollisionCost::value (collision_terms.cpp:1287-1306): no buffer
  double value(const DblVec& x) override
  {
    const auto contacts = calc_.collide(x);
    const CollisionModel& cm = calc_.model();
    double out = 0;
    for (const auto& c : contacts)
      out += std::fmax(cm.marginOf(c.link, c.other()) - c.distance, 0.0) * cm.coeffOf(c.link, c.other());
    return out;
  }

  // CollisionCost::convex (collision_terms.cpp:1267-1284): hinge(margin - dist) * coeff
  ConvexObjective::Ptr convex(const DblVec& x, Model* model) override
  {
    auto out = std::make_shared<ConvexObjective>(model);
    const CollisionModel& cm = calc_.model();
    std::vector<Contact> cts;
    const AffExprVector ex = calc_.exprs(x, &cts);
    for (std::size_t i = 0; i < ex.size(); ++i)
      out->addHinge(exprSub(AffExpr(cm.marginOf(cts[i].link, cts[i].other())), ex[i]),
                    cm.coeffOf(cts[i].link, cts[i].other()));
    return out;
  }

private:
  Calc calc_;
};

// One CollisionConstraint per step pair (problem_description.cpp:1797-1840,
// prob.addIneqConstraint) or per free waypoint (DISCRETE, :1842-1856).
template <class Calc>
class CollisionPairConstraint : public Constraint
{
public:
  explicit CollisionPairConstraint(Calc calc) : calc_(std::move(calc)) {}
  VarVector getVars() override { return calc_.vars(); }
  ConstraintType type() override { return INEQ; }

  // CollisionConstraint::value (collision_terms.cpp:1366-1386)
  DblVec value(const DblVec& x) override
  {
    const auto contacts = calc_.collide(x);
    const CollisionModel& cm = calc_.model();
    DblVec out;
    for (const auto& c : contacts)
      out.push_back(std::fmax(cm.marginOf(c.link, c.other()) - c.distance, 0.0) * cm.coeffOf(c.link, c.other()));
    return out;
  }

  // CollisionConstraint::convex (collision_terms.cpp:1347-1364): ineq exprMult(margin - dist, coeff)
  ConvexConstraints::Ptr convex(const DblVec& x, Model* model) override
  {
    auto out = std::make_shared<ConvexConstraints>(model);
    const CollisionModel& cm = calc_.model();
    std::vector<Contact> cts;
    const AffExprVector ex = calc_.exprs(x, &cts);
    for (std::size_t i = 0; i < ex.size(); ++i)
      out->addIneqCnt(exprMult(exprSub(AffExpr(cm.marginOf(cts[i].link, cts[i].other())), ex[i]),
                               cm.coeffOf(cts[i].link, cts[i].other())));
    return out;
  }

private:
  Calc calc_;
};
}  // namespace

thip_coll_term collisionTerm(const thip_problem_desc& d, int k)
{
  if (k > 0)
    return d.coll_extra[k - 1];
  thip_coll_term t{};
  t.is_cnt = d.coll_is_cnt;
  t.first_step = d.coll_first_step;
  t.last_step = d.coll_last_step;
  t.n_fixed = d.coll_n_fixed;
  for (int i = 0; i < d.coll_n_fixed && i < THIP_MAX_STEPS; ++i)
    t.fixed_steps[i] = d.coll_fixed_steps[i];
  t.margin = d.coll_margin;
  t.coeff = d.coll_coeff;
  t.buffer = d.coll_buffer;
  t.lvs = d.coll_lvs;
  t.continuous = d.coll_continuous;
  t.contact_test = d.coll_contact_test;
  return t;
}

std::shared_ptr<CollisionModel> collisionModel(const thip_problem_desc& d, int term, const double* scene)
{
  const thip_coll_term t = collisionTerm(d, term);
  auto cm = std::make_shared<CollisionModel>();
  cm->chain = &d.chain;
  cm->n_spheres = d.n_spheres;
  for (int s = 0; s < d.n_spheres; ++s)
  {
    cm->sphere_link[s] = d.sphere_link[s];
    cm->sphere_radius[s] = d.sphere_radius[s];
    for (int i = 0; i < 3; ++i)
      cm->sphere_center[s][i] = d.sphere_center[s][i];
  }
  cm->n_prims = d.n_prims;
  cm->scene_store.assign(scene, scene + 16 * d.n_prims);
  cm->scene = cm->scene_store.data();
  cm->margin = t.margin;
  cm->coeff = t.coeff;
  cm->buffer = t.buffer;
  cm->lvs = t.lvs;
  cm->continuous = t.continuous == 1;
  cm->contact_test = t.contact_test;
  // self pairs in key order: link pairs as given, spheres of a then of b in index order
  for (int k = 0; k < d.n_self_pairs; ++k)
    for (int sa = 0; sa < d.n_spheres; ++sa)
      if (d.sphere_link[sa] == d.self_pair[k][0])
        for (int sb = 0; sb < d.n_spheres; ++sb)
          if (d.sphere_link[sb] == d.self_pair[k][1])
          {
            cm->self_a.push_back(sa);
            cm->self_b.push_back(sb);
            cm->self_key.push_back(k);
          }
  cm->n_self_keys = d.n_self_pairs;
  // "pairs" (problem_description.cpp:1707-1718): setCollisionMargin(link, p, dist_pen)
  // and setCollisionCoeff(link, p, coeffs) per entry, in order (insert_or_assign;
  // a zero coefficient joins zero_coeff_, a nonzero one leaves it)
  for (int k = 0; k < d.n_coll_pairs; ++k)
  {
    const thip_coll_pair& e = d.coll_pairs[k];
    if (e.term != term)
      continue;
    const int b = e.other >= 0 ? CollisionModel::kScenePair + e.other : -1 - e.other;
    const auto key = CollisionModel::key(e.link, b);
    cm->pair_margin[key] = e.margin;
    cm->pair_coeff[key] = e.coeff;
    if (std::fabs(e.coeff - 0.0) <= 1e-6)  // almostEqualRelativeAndAbs(coeff, 0.0)
      cm->zero_coeff.insert(key);
    else
      cm->zero_coeff.erase(key);
  }
  return cm;
}

void addCollisionTerms(TrajProblem& tp, const std::vector<VarVector>& rows, const thip_problem_desc& d,
                       const double* scene, int term)
{
  const thip_coll_term tm = collisionTerm(d, term);
  auto cm = collisionModel(d, term, scene);
  const int first = tm.first_step;
  const int last = (tm.last_step < 0) ? d.n_steps - 1 : tm.last_step;
  auto fixed = [&](int t) {
    for (int k = 0; k < tm.n_fixed; ++k)
      if (tm.fixed_steps[k] == t)
        return true;
    return false;
  };
  if (tm.continuous == 2)
  {
    // DISCRETE: SINGLE_TIME_STEP terms on the free waypoints of [first, last]
    for (int i = first; i <= last; ++i)
    {
      if (fixed(i))
        continue;
      CollisionSingleCalc calc(cm, rows[static_cast<std::size_t>(i)]);
      if (tm.is_cnt)
      {
        auto c = std::make_shared<CollisionPairConstraint<CollisionSingleCalc>>(std::move(calc));
        c->setName("collision_" + std::to_string(i));
        tp.prob->addConstraint(c);
      }
      else
      {
        auto c = std::make_shared<CollisionPairCost<CollisionSingleCalc>>(std::move(calc));
        c->setName("collision_" + std::to_string(i));
        tp.prob->addCost(c);
      }
    }
    return;
  }
  for (int i = first; i < last; ++i)
  {
    const bool cf = fixed(i), nf = fixed(i + 1);
    int type;
    if (!cf && !nf)
      type = CollisionPairCalc::kBothFree;
    else if (cf && nf)
      throw std::runtime_error("Currently two adjacent fixed steps are not supported in collision term.");
    else if (cf)
      type = CollisionPairCalc::kStartFixedEndFree;
    else
      type = CollisionPairCalc::kStartFreeEndFixed;
    CollisionPairCalc calc(cm, rows[static_cast<std::size_t>(i)], rows[static_cast<std::size_t>(i + 1)], type);
    if (tm.is_cnt)
    {
      auto c = std::make_shared<CollisionPairConstraint<CollisionPairCalc>>(std::move(calc));
      c->setName("collision_" + std::to_string(i));
      tp.prob->addConstraint(c);
    }
    else
    {
      auto c = std::make_shared<CollisionPairCost<CollisionPairCalc>>(std::move(calc));
      c->setName("collision_" + std::to_string(i));
      tp.prob->addCost(c);
    }
  }
}

}  // namespace orc
