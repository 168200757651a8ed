// Device kinematics and pose-error arithmetic (fp64, one thread per pose).
//
// GPU side of the tesseract arithmetic the reference calls
// (trajopt/src/kinematic_terms.cpp:189-370): kinematic-tree FK, the
// transform error target^-1 * source with the rotation-vector conventions of
// tesseract's calcRotationalError / calcRotationalError2, and the
// forward-difference error delta used by CartPoseJacCalculator.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/trajopt_hip.h"

namespace thip
{
struct Pose
{
  double r[9];
  double t[3];
};

__device__ __forceinline__ void pose_load(Pose& p, const double* s)
{
#pragma unroll
  for (int i = 0; i < 3; ++i)
  {
    p.r[3 * i + 0] = s[4 * i + 0];
    p.r[3 * i + 1] = s[4 * i + 1];
    p.r[3 * i + 2] = s[4 * i + 2];
    p.t[i] = s[4 * i + 3];
  }
}

__device__ __forceinline__ void pose_mul(const Pose& a, const Pose& b, Pose& c)
{
#pragma unroll
  for (int i = 0; i < 3; ++i)
  {
#pragma unroll
    for (int k = 0; k < 3; ++k)
      c.r[3 * i + k] = a.r[3 * i + 0] * b.r[0 + k] + a.r[3 * i + 1] * b.r[3 + k] + a.r[3 * i + 2] * b.r[6 + k];
    c.t[i] = a.r[3 * i + 0] * b.t[0] + a.r[3 * i + 1] * b.t[1] + a.r[3 * i + 2] * b.t[2] + a.t[i];
  }
}

__device__ __forceinline__ void pose_inv(const Pose& a, Pose& c)
{
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      c.r[3 * i + k] = a.r[3 * k + i];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    c.t[i] = -(c.r[3 * i + 0] * a.t[0] + c.r[3 * i + 1] * a.t[1] + c.r[3 * i + 2] * a.t[2]);
}

// Eigen AngleAxis::toRotationMatrix
__device__ __forceinline__ void rot_axis_angle(const double* ax, double ang, double* R)
{
  double s, c;
  sincos(ang, &s, &c);
  const double sa0 = s * ax[0], sa1 = s * ax[1], sa2 = s * ax[2];
  const double ca0 = (1 - c) * ax[0], ca1 = (1 - c) * ax[1], ca2 = (1 - c) * ax[2];
  double tmp = ca0 * ax[1];
  R[1] = tmp - sa2;
  R[3] = tmp + sa2;
  tmp = ca0 * ax[2];
  R[2] = tmp + sa1;
  R[6] = tmp - sa1;
  tmp = ca1 * ax[2];
  R[5] = tmp - sa0;
  R[7] = tmp + sa0;
  R[0] = ca0 * ax[0] + c;
  R[4] = ca1 * ax[1] + c;
  R[8] = ca2 * ax[2] + c;
}

// Links on the path root -> `link` (bit k set for link k >= 1): the joints
// whose motion moves the link.  A serial chain has every link below `link`.
__device__ __forceinline__ unsigned chain_path(const thip_chain& ch, int link)
{
  unsigned path = 0;
  for (int k = link; k > 0; k = ch.parent[k])
    path |= 1u << k;
  return path;
}

// World pose of link `upto` at joint values q: the joints of its path from
// the root, in order (parent[k] < k).
__device__ inline void chain_fk(const thip_chain& ch, const double* q, int upto, Pose& out)
{
  static_assert(THIP_MAX_LINKS <= 32, "path mask");
  const unsigned path = chain_path(ch, upto);
  Pose T;
  pose_load(T, ch.base_pose);
  for (int k = 1; k <= upto; ++k)
  {
    if (!((path >> k) & 1u))
      continue;
    Pose O, Tn;
    pose_load(O, ch.joint_origin[k]);
    pose_mul(T, O, Tn);
    const int type = ch.joint_type[k];
    if (type == THIP_JOINT_REVOLUTE || type == THIP_JOINT_CONTINUOUS)
    {
      Pose M;
      rot_axis_angle(ch.joint_axis[k], q[ch.joint_dof[k]], M.r);
      M.t[0] = M.t[1] = M.t[2] = 0;
      pose_mul(Tn, M, T);
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
      pose_mul(Tn, M, T);
    }
    else
      T = Tn;
  }
  out = T;
}

// rotation vector of R: quaternion (Shoemake branches as Eigen), AngleAxis
// conversion, tesseract sign fix and wrap into [-pi, pi] (two_pi = false) or
// [0, 2pi] (two_pi = true)
__device__ inline void rot_error(const double* R, double* out, bool two_pi)
{
  double w, v[3];
  double t = R[0] + R[4] + R[8];
  if (t > 0)
  {
    t = sqrt(t + 1.0);
    w = 0.5 * t;
    t = 0.5 / t;
    v[0] = (R[7] - R[5]) * t;
    v[1] = (R[2] - R[6]) * t;
    v[2] = (R[3] - R[1]) * t;
  }
  else
  {
    int i = 0;
    if (R[4] > R[0])
      i = 1;
    if (R[8] > R[4 * i])
      i = 2;
    const int j = (i + 1) % 3;
    const int k = (j + 1) % 3;
    t = sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
    v[i] = 0.5 * t;
    t = 0.5 / t;
    w = (R[3 * k + j] - R[3 * j + k]) * t;
    v[j] = (R[3 * j + i] + R[3 * i + j]) * t;
    v[k] = (R[3 * k + i] + R[3 * i + k]) * t;
  }
  double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < 2.220446049250313e-16)
  {
    const double sc = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
    if (sc > 0)
    {
      const double a = v[0] / sc, b = v[1] / sc, c = v[2] / sc;
      n = sc * sqrt(a * a + b * b + c * c);
    }
    else
      n = 0;
  }
  double ang, ax0, ax1, ax2;
  if (n != 0)
  {
    ang = 2 * atan2(n, fabs(w));
    const double sg = (w < 0) ? -1.0 : 1.0;
    ax0 = sg * v[0] / n;
    ax1 = sg * v[1] / n;
    ax2 = sg * v[2] / n;
  }
  else
  {
    ang = 0;
    ax0 = 1;
    ax1 = ax2 = 0;
  }
  const double dot = v[0] * ax0 + v[1] * ax1 + v[2] * ax2;
  const double s = (dot < 0) ? -1.0 : 1.0;
  ang = s * ang;
  ax0 = s * ax0;
  ax1 = s * ax1;
  ax2 = s * ax2;
  const double tp = 2.0 * M_PI;
  ang = copysign(fmod(fabs(ang), tp), ang);
  if (two_pi)
  {
    if (ang < 0)
      ang += tp;
    else if (ang > tp)
      ang -= tp;
  }
  else
  {
    if (ang < -M_PI)
      ang += tp;
    else if (ang > M_PI)
      ang -= tp;
  }
  out[0] = ax0 * ang;
  out[1] = ax1 * ang;
  out[2] = ax2 * ang;
}

// err = [ (T1^-1 T2).t ; rotvec((T1^-1 T2).R) ]  (calcTransformError); T1inv given
__device__ inline void transform_error(const Pose& T1inv, const Pose& T2, double* err)
{
  Pose E;
  pose_mul(T1inv, T2, E);
  err[0] = E.t[0];
  err[1] = E.t[1];
  err[2] = E.t[2];
  rot_error(E.r, err + 3, false);
}

// tesseract applyTolerances: 0 inside [lower, upper], else the excess past the band
__device__ inline void apply_tolerances(double* err, const double* lower, const double* upper)
{
  for (int i = 0; i < 6; ++i)
    err[i] = (err[i] < lower[i]) ? err[i] - lower[i] : ((err[i] > upper[i]) ? err[i] - upper[i] : 0.0);
}

// Tolerance-aware calcJacobianTransformErrorDiff(target, source, source_perturbed,
// lower, upper) given pe = target^-1 source, ppe = target^-1 source_perturbed: both
// errors with the [-pi, pi] rotation vector, or the continuous [0, 2 pi) one for
// both when a component jumps by more than pi, banded, then differenced (the same
// restatement as oracle/src/kin.cpp calcJacobianTransformErrorDiffTol).
__device__ inline void transform_error_diff_tol(const Pose& pe, const Pose& ppe, const double* lower,
                                                const double* upper, double* diff)
{
  double e0[6], e1[6];
  for (int i = 0; i < 3; ++i)
  {
    e0[i] = pe.t[i];
    e1[i] = ppe.t[i];
  }
  rot_error(pe.r, e0 + 3, false);
  rot_error(ppe.r, e1 + 3, false);
  bool wrap = false;
  for (int i = 3; i < 6; ++i)
    wrap = wrap || fabs(e1[i] - e0[i]) > M_PI;
  if (wrap)
  {
    rot_error(pe.r, e0 + 3, true);
    rot_error(ppe.r, e1 + 3, true);
  }
  apply_tolerances(e0, lower, upper);
  apply_tolerances(e1, lower, upper);
  for (int i = 0; i < 6; ++i)
    diff[i] = e1[i] - e0[i];
}

}  // namespace thip
