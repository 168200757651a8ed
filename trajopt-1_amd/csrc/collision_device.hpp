// Device-side collision geometry for the LVS-discrete collision cost
// (config C): closed-form robot-sphere vs scene-primitive signed distance,
// the sub-state interpolation of DiscreteCollisionEvaluator::CalcCollisions
// (trajopt/src/collision_terms.cpp:817-898) and the geometric jacobian used
// by CollisionEvaluator::GetGradient (collision_terms.cpp:195-242).  The
// arithmetic is operation-for-operation that of oracle/src/collision.cpp.
#pragma once
#include "kin_device.hpp"

namespace thip
{
// Primitive record (16 doubles, include/trajopt_hip.h).  normal points from
// the robot sphere toward the primitive; d(dist)/d(center) = -normal.
__device__ inline void sphere_prim_distance(const double c[3], double r, const double* prim, double& dist, double n[3],
                                            double p_robot[3])
{
  const int type = static_cast<int>(prim[0]);
  if (type == THIP_PRIM_SPHERE || type == THIP_PRIM_CAPSULE)
  {
    double s[3], rs;
    if (type == THIP_PRIM_SPHERE)
    {
      s[0] = prim[1];
      s[1] = prim[2];
      s[2] = prim[3];
      rs = prim[4];
    }
    else
    {
      const double* a = prim + 1;
      const double* b = prim + 4;
      const double ab[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] };
      const double den = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
      double t = 0;
      if (den > 1e-24)
        t = ((c[0] - a[0]) * ab[0] + (c[1] - a[1]) * ab[1] + (c[2] - a[2]) * ab[2]) / den;
      t = fmin(fmax(t, 0.0), 1.0);
      s[0] = a[0] + t * ab[0];
      s[1] = a[1] + t * ab[1];
      s[2] = a[2] + t * ab[2];
      rs = prim[7];
    }
    const double v[3] = { s[0] - c[0], s[1] - c[1], s[2] - c[2] };
    const double L = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
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
      p_robot[i] = c[i] + r * n[i];
    return;
  }
  const double* ctr = prim + 1;
  const double* R = prim + 4;
  const double* h = prim + 13;
  const double w[3] = { c[0] - ctr[0], c[1] - ctr[1], c[2] - ctr[2] };
  double cl[3];
  for (int i = 0; i < 3; ++i)
    cl[i] = R[0 * 3 + i] * w[0] + R[1 * 3 + i] * w[1] + R[2 * 3 + i] * w[2];
  const bool inside = fabs(cl[0]) <= h[0] && fabs(cl[1]) <= h[1] && fabs(cl[2]) <= h[2];
  if (!inside)
  {
    double ql[3];
    for (int i = 0; i < 3; ++i)
      ql[i] = fmin(fmax(cl[i], -h[i]), h[i]);
    const double vl[3] = { ql[0] - cl[0], ql[1] - cl[1], ql[2] - cl[2] };
    const double L = sqrt(vl[0] * vl[0] + vl[1] * vl[1] + vl[2] * vl[2]);
    for (int i = 0; i < 3; ++i)
      n[i] = (R[i * 3 + 0] * vl[0] + R[i * 3 + 1] * vl[1] + R[i * 3 + 2] * vl[2]) / L;
    dist = L - r;
  }
  else
  {
    int k = 0;
    double depth = h[0] - fabs(cl[0]);
    for (int i = 1; i < 3; ++i)
    {
      const double dd = h[i] - fabs(cl[i]);
      if (dd < depth)
      {
        depth = dd;
        k = i;
      }
    }
    const double sgn = (cl[k] < 0) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i)
      n[i] = -sgn * R[i * 3 + k];
    dist = -depth - r;
  }
  for (int i = 0; i < 3; ++i)
    p_robot[i] = c[i] + r * n[i];
}

// Swept sphere (center a -> b, radius r: a capsule) vs primitive, the
// restatement of Bullet's cast for a sphere (oracle/src/collision.cpp,
// sweptSpherePrimDistance, the same rule): dist = min over t in [0, 1] of the
// signed distance at a + t (b - a), t_star its minimiser (closed form for
// spheres and capsules; for boxes the smallest value among the breakpoints
// and piecewise stationary points of the box SDF on the segment, ties within
// 1e-14 to the smaller t).
__device__ inline double sseg_param(const double p1[3], const double d1[3], const double p2[3], const double d2[3])
{
  const double r[3] = { p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2] };
  const double a = d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2];
  const double e = d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2];
  const double f = d2[0] * r[0] + d2[1] * r[1] + d2[2] * r[2];
  const double eps = 1e-24;
  if (a <= eps)
    return 0.0;
  const double cc = d1[0] * r[0] + d1[1] * r[1] + d1[2] * r[2];
  if (e <= eps)
    return fmin(fmax(-cc / a, 0.0), 1.0);
  const double b = d1[0] * d2[0] + d1[1] * d2[1] + d1[2] * d2[2];
  const double denom = a * e - b * b;
  double s = (denom > eps) ? fmin(fmax((b * f - cc * e) / denom, 0.0), 1.0) : 0.0;
  const double t = (b * s + f) / e;
  if (t < 0.0)
    s = fmin(fmax(-cc / a, 0.0), 1.0);
  else if (t > 1.0)
    s = fmin(fmax((b - cc) / a, 0.0), 1.0);
  return s;
}

__device__ inline void swept_sphere_prim_distance(const double a[3], const double b[3], double r, const double* prim,
                                                  double& dist, double n[3], double p_robot[3], double& t_star)
{
  const int type = static_cast<int>(prim[0]);
  const double u[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] };
  const double uu = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  double t = 0.0;
  if (type == THIP_PRIM_SPHERE)
  {
    const double w[3] = { prim[1] - a[0], prim[2] - a[1], prim[3] - a[2] };
    t = (uu > 1e-24) ? fmin(fmax((w[0] * u[0] + w[1] * u[1] + w[2] * u[2]) / uu, 0.0), 1.0) : 0.0;
  }
  else if (type == THIP_PRIM_CAPSULE)
  {
    const double d2[3] = { prim[4] - prim[1], prim[5] - prim[2], prim[6] - prim[3] };
    t = sseg_param(a, u, prim + 1, d2);
  }
  else
  {
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
    double bp[11];
    int nb = 0;
    bp[nb++] = 0.0;
    for (int i = 0; i < 3; ++i)
      if (fabs(ul[i]) > 1e-300)
        for (int sg = -1; sg <= 1; ++sg)
        {
          const double tb = (sg * h[i] - al[i]) / ul[i];
          if (tb > 0.0 && tb < 1.0)
            bp[nb++] = tb;
        }
    bp[nb++] = 1.0;
    for (int i = 1; i < nb; ++i)
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
        out = out || (fabs(pm) > h[i]);
      }
      if (out)
      {
        double num = 0, den = 0;
        for (int i = 0; i < 3; ++i)
        {
          const double pm = al[i] + tm * ul[i];
          if (fabs(pm) > h[i])
          {
            num += (al[i] - sg[i] * h[i]) * ul[i];
            den += ul[i] * ul[i];
          }
        }
        if (den > 0)
          cand[nc++] = fmin(fmax(-num / den, t0), t1);
      }
      else
        for (int i = 0; i < 3; ++i)
          for (int j = i + 1; j < 3; ++j)
          {
            const double den = sg[i] * ul[i] - sg[j] * ul[j];
            if (fabs(den) > 1e-300)
            {
              const double tc = (h[i] - h[j] - sg[i] * al[i] + sg[j] * al[j]) / den;
              if (tc > t0 && tc < t1)
                cand[nc++] = tc;
            }
          }
    }
    double val[48];
    double best = 0;
    for (int k = 0; k < nc; ++k)
    {
      const double c[3] = { a[0] + cand[k] * u[0], a[1] + cand[k] * u[1], a[2] + cand[k] * u[2] };
      double nn[3], pr[3];
      sphere_prim_distance(c, r, prim, val[k], nn, pr);
      best = (k == 0) ? val[k] : fmin(best, val[k]);
    }
    double bt = 2.0;
    for (int k = 0; k < nc; ++k)
      if (val[k] <= best + 1e-14 && cand[k] < bt)
        bt = cand[k];
    t = bt;
  }
  const double c[3] = { a[0] + t * u[0], a[1] + t * u[1], a[2] + t * u[2] };
  sphere_prim_distance(c, r, prim, dist, n, p_robot);
  t_star = t;
}

// Both parameters of the closest points of segments p1 + s d1 and p2 + t d2
// (oracle segSegParams; s as sseg_param computes it).
__device__ inline void sseg_params(const double p1[3], const double d1[3], const double p2[3], const double d2[3],
                                   double& s, double& t)
{
  const double r[3] = { p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2] };
  const double a = d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2];
  const double e = d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2];
  const double f = d2[0] * r[0] + d2[1] * r[1] + d2[2] * r[2];
  const double eps = 1e-24;
  if (a <= eps && e <= eps)
  {
    s = t = 0.0;
    return;
  }
  if (a <= eps)
  {
    s = 0.0;
    t = fmin(fmax(f / e, 0.0), 1.0);
    return;
  }
  const double cc = d1[0] * r[0] + d1[1] * r[1] + d1[2] * r[2];
  if (e <= eps)
  {
    t = 0.0;
    s = fmin(fmax(-cc / a, 0.0), 1.0);
    return;
  }
  const double b = d1[0] * d2[0] + d1[1] * d2[1] + d1[2] * d2[2];
  const double denom = a * e - b * b;
  s = (denom > eps) ? fmin(fmax((b * f - cc * e) / denom, 0.0), 1.0) : 0.0;
  t = (b * s + f) / e;
  if (t < 0.0)
  {
    t = 0.0;
    s = fmin(fmax(-cc / a, 0.0), 1.0);
  }
  else if (t > 1.0)
  {
    t = 1.0;
    s = fmin(fmax((b - cc) / a, 0.0), 1.0);
  }
}

// Robot sphere a vs robot sphere b (self-collision), both moving: centers
// a0 -> a1, b0 -> b1 over a cast (a1 = a0, b1 = b0 for one state); the two
// capsules' distance at the closest points (sa, sb) of the center segments,
// each side its own time; normal from a toward b (oracle selfSphereDistance).
__device__ inline void self_sphere_distance(const double a0[3], const double a1[3], double ra, const double b0[3],
                                            const double b1[3], double rb, bool cast, double& dist, double n[3],
                                            double pa[3], double pb[3], double& sa, double& sb)
{
  const double da[3] = { a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2] };
  const double db[3] = { b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2] };
  sa = sb = 0.0;
  if (cast)
    sseg_params(a0, da, b0, db, sa, sb);
  double ca[3], cb[3];
  for (int i = 0; i < 3; ++i)
  {
    ca[i] = a0[i] + sa * da[i];
    cb[i] = b0[i] + sb * db[i];
  }
  const double v[3] = { cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2] };
  const double L = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
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

// A lower bound of the swept distance (segment to the primitive's bounding
// sphere): a candidate whose bound exceeds the contact distance cannot be a
// contact, so the exact cast is skipped.
__device__ inline double swept_lower_bound(const double a[3], const double b[3], double r, const double* prim)
{
  const int type = static_cast<int>(prim[0]);
  double c[3], rad;
  if (type == THIP_PRIM_SPHERE)
  {
    c[0] = prim[1];
    c[1] = prim[2];
    c[2] = prim[3];
    rad = prim[4];
  }
  else if (type == THIP_PRIM_CAPSULE)
  {
    for (int i = 0; i < 3; ++i)
      c[i] = 0.5 * (prim[1 + i] + prim[4 + i]);
    const double hl[3] = { 0.5 * (prim[4] - prim[1]), 0.5 * (prim[5] - prim[2]), 0.5 * (prim[6] - prim[3]) };
    rad = sqrt(hl[0] * hl[0] + hl[1] * hl[1] + hl[2] * hl[2]) + prim[7];
  }
  else
  {
    c[0] = prim[1];
    c[1] = prim[2];
    c[2] = prim[3];
    rad = sqrt(prim[13] * prim[13] + prim[14] * prim[14] + prim[15] * prim[15]);
  }
  const double u[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] };
  const double uu = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  const double w[3] = { c[0] - a[0], c[1] - a[1], c[2] - a[2] };
  const double t = (uu > 1e-24) ? fmin(fmax((w[0] * u[0] + w[1] * u[1] + w[2] * u[2]) / uu, 0.0), 1.0) : 0.0;
  const double v[3] = { w[0] - t * u[0], w[1] - t * u[1], w[2] - t * u[2] };
  // slack for rounding: the bound only filters candidates far from contact
  return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) - rad - r - 1e-9;
}

// Eigen::VectorXd::LinSpaced(size, low, high)(i) (Eigen 3.4 linspaced_op_impl)
__device__ __forceinline__ double linspaced(int size, double low, double high, int i)
{
  if (size == 1)
    return high;
  const int size1 = size - 1;
  const double step = (high - low) / size1;
  const bool flip = fabs(high) < fabs(low);
  if (flip)
    return (i == 0) ? low : high - double(size1 - i) * step;
  return (i == size1) ? high : low + double(i) * step;
}

// Number of LVS sub-states of a step pair (collision_terms.cpp:846-852)
__device__ __forceinline__ int lvs_count(const double* q0, const double* q1, int D, double lvs)
{
  double dist = 0;
  for (int j = 0; j < D; ++j)
    dist += (q1[j] - q0[j]) * (q1[j] - q0[j]);
  dist = sqrt(dist);
  long cnt = 2;
  if (dist > lvs)
    cnt = static_cast<long>(ceil(dist / lvs)) + 1;
  return static_cast<int>(cnt);
}

// Geometric jacobian of link `link` at q (world frame, reference point =
// link origin): J[6][D] row-major (linear rows 0-2, angular 3-5); columns of
// joints off the link's path from the root are zero.
__device__ inline void chain_jacobian(const thip_chain& ch, const double* q, int link, double* J)
{
  const int D = ch.n_dof;
  const unsigned path = chain_path(ch, link);
  Pose T[THIP_MAX_LINKS];
  pose_load(T[0], ch.base_pose);
  int prev = 0;  // the path's previous link
  for (int k = 1; k <= link; ++k)
  {
    if (!((path >> k) & 1u))
      continue;
    Pose O, Tn;
    pose_load(O, ch.joint_origin[k]);
    pose_mul(T[prev], O, Tn);
    prev = k;
    const int type = ch.joint_type[k];
    if (type == THIP_JOINT_REVOLUTE || type == THIP_JOINT_CONTINUOUS)
    {
      Pose M;
      rot_axis_angle(ch.joint_axis[k], q[ch.joint_dof[k]], M.r);
      M.t[0] = M.t[1] = M.t[2] = 0;
      pose_mul(Tn, M, T[k]);
    }
    else if (type == THIP_JOINT_PRISMATIC)
    {
      Pose M;
      const double v = q[ch.joint_dof[k]];
      M.r[0] = M.r[4] = M.r[8] = 1;
      M.r[1] = M.r[2] = M.r[3] = M.r[5] = M.r[6] = M.r[7] = 0;
      M.t[0] = ch.joint_axis[k][0] * v;
      M.t[1] = ch.joint_axis[k][1] * v;
      M.t[2] = ch.joint_axis[k][2] * v;
      pose_mul(Tn, M, T[k]);
    }
    else
      T[k] = Tn;
  }
  for (int e = 0; e < 6 * D; ++e)
    J[e] = 0.0;
  const double* p = T[link].t;
  for (int k = 1; k <= link; ++k)
  {
    const int type = ch.joint_type[k];
    if (type == THIP_JOINT_FIXED || !((path >> k) & 1u))
      continue;
    const double* ax = ch.joint_axis[k];
    double a[3];
    for (int r = 0; r < 3; ++r)
      a[r] = T[k].r[r * 3 + 0] * ax[0] + T[k].r[r * 3 + 1] * ax[1] + T[k].r[r * 3 + 2] * ax[2];
    const int j = ch.joint_dof[k];
    if (type == THIP_JOINT_PRISMATIC)
    {
      for (int r = 0; r < 3; ++r)
        J[r * D + j] = a[r];
      continue;
    }
    const double d[3] = { p[0] - T[k].t[0], p[1] - T[k].t[1], p[2] - T[k].t[2] };
    J[0 * D + j] = a[1] * d[2] - a[2] * d[1];
    J[1 * D + j] = a[2] * d[0] - a[0] * d[2];
    J[2 * D + j] = a[0] * d[1] - a[1] * d[0];
    for (int r = 0; r < 3; ++r)
      J[(3 + r) * D + j] = a[r];
  }
}

}  // namespace thip
