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

// Geometric jacobian of chain link `link` at q (world frame, reference point =
// link origin): J[6][D] row-major (linear rows 0-2, angular 3-5).
__device__ inline void chain_jacobian(const thip_chain& ch, const double* q, int link, double* J)
{
  const int D = ch.n_dof;
  Pose T[THIP_MAX_LINKS];
  pose_load(T[0], ch.base_pose);
  for (int k = 1; k <= link; ++k)
  {
    Pose O, Tn;
    pose_load(O, ch.joint_origin[k]);
    pose_mul(T[k - 1], O, Tn);
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
    if (type == THIP_JOINT_FIXED)
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
