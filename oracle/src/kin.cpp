// ORACLE — test infrastructure only (see sco_expr.hpp header).
#include "kin.hpp"

#include <cmath>

namespace orc
{
Iso3 mul(const Iso3& a, const Iso3& b)
{
  Iso3 c{};
  for (int r = 0; r < 3; ++r)
  {
    for (int k = 0; k < 3; ++k)
      c.R[r * 3 + k] = a.R[r * 3 + 0] * b.R[0 * 3 + k] + a.R[r * 3 + 1] * b.R[1 * 3 + k] + a.R[r * 3 + 2] * b.R[2 * 3 + k];
    c.t[r] = a.R[r * 3 + 0] * b.t[0] + a.R[r * 3 + 1] * b.t[1] + a.R[r * 3 + 2] * b.t[2] + a.t[r];
  }
  return c;
}

Iso3 inverse(const Iso3& a)
{
  Iso3 c{};
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k)
      c.R[r * 3 + k] = a.R[k * 3 + r];
  for (int r = 0; r < 3; ++r)
    c.t[r] = -(c.R[r * 3 + 0] * a.t[0] + c.R[r * 3 + 1] * a.t[1] + c.R[r * 3 + 2] * a.t[2]);
  return c;
}

Iso3 axisAngle(const double axis[3], double angle)
{
  Iso3 m = Iso3::identity();
  const double s = std::sin(angle), c = std::cos(angle);
  const double sa[3] = { s * axis[0], s * axis[1], s * axis[2] };
  const double ca[3] = { (1 - c) * axis[0], (1 - c) * axis[1], (1 - c) * axis[2] };
  double tmp = ca[0] * axis[1];
  m.R[0 * 3 + 1] = tmp - sa[2];
  m.R[1 * 3 + 0] = tmp + sa[2];
  tmp = ca[0] * axis[2];
  m.R[0 * 3 + 2] = tmp + sa[1];
  m.R[2 * 3 + 0] = tmp - sa[1];
  tmp = ca[1] * axis[2];
  m.R[1 * 3 + 2] = tmp - sa[0];
  m.R[2 * 3 + 1] = tmp + sa[0];
  m.R[0] = ca[0] * axis[0] + c;
  m.R[4] = ca[1] * axis[1] + c;
  m.R[8] = ca[2] * axis[2] + c;
  return m;
}

void quatFromMatrix(const double R[9], double q[4])
{
  // q = (w, x, y, z); coefficient index i of (x, y, z) -> q[1 + i]
  auto M = [&](int r, int c) { return R[r * 3 + c]; };
  double t = M(0, 0) + M(1, 1) + M(2, 2);
  if (t > 0)
  {
    t = std::sqrt(t + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[1] = (M(2, 1) - M(1, 2)) * t;
    q[2] = (M(0, 2) - M(2, 0)) * t;
    q[3] = (M(1, 0) - M(0, 1)) * t;
  }
  else
  {
    int i = 0;
    if (M(1, 1) > M(0, 0))
      i = 1;
    if (M(2, 2) > M(i, i))
      i = 2;
    const int j = (i + 1) % 3;
    const int k = (j + 1) % 3;
    t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
    q[1 + i] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (M(k, j) - M(j, k)) * t;
    q[1 + j] = (M(j, i) + M(i, j)) * t;
    q[1 + k] = (M(k, i) + M(i, k)) * t;
  }
}

// Eigen AngleAxis(quaternion) + tesseract sign/wrap handling
static void rotErr(const double R[9], double out[3], bool zero_to_two_pi)
{
  double q[4];
  quatFromMatrix(R, q);
  double n = std::sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 2.220446049250313e-16)
  {
    const double sc = std::fmax(std::fabs(q[1]), std::fmax(std::fabs(q[2]), std::fabs(q[3])));
    if (sc > 0)
    {
      const double a = q[1] / sc, b = q[2] / sc, c = q[3] / sc;
      n = sc * std::sqrt(a * a + b * b + c * c);
    }
    else
      n = 0;
  }
  double angle, axis[3];
  if (n != 0)
  {
    angle = 2 * std::atan2(n, std::fabs(q[0]));
    const double sgn = (q[0] < 0) ? -1.0 : 1.0;
    for (int i = 0; i < 3; ++i)
      axis[i] = sgn * q[1 + i] / n;
  }
  else
  {
    angle = 0;
    axis[0] = 1;
    axis[1] = axis[2] = 0;
  }
  const double dot = q[1] * axis[0] + q[2] * axis[1] + q[3] * axis[2];
  const double s = (dot < 0) ? -1.0 : 1.0;
  angle = s * angle;
  for (double& a : axis)
    a = s * a;
  const double two_pi = 2.0 * M_PI;
  angle = std::copysign(std::fmod(std::fabs(angle), two_pi), angle);
  if (zero_to_two_pi)
  {
    if (angle < 0)
      angle += two_pi;
    else if (angle > two_pi)
      angle -= two_pi;
  }
  else
  {
    if (angle < -M_PI)
      angle += two_pi;
    else if (angle > M_PI)
      angle -= two_pi;
  }
  for (int i = 0; i < 3; ++i)
    out[i] = axis[i] * angle;
}

void calcRotationalError(const double R[9], double out[3]) { rotErr(R, out, false); }
void calcRotationalError2(const double R[9], double out[3]) { rotErr(R, out, true); }

void calcTransformError(const Iso3& t1, const Iso3& t2, double err[6])
{
  const Iso3 e = mul(inverse(t1), t2);
  err[0] = e.t[0];
  err[1] = e.t[1];
  err[2] = e.t[2];
  calcRotationalError(e.R, err + 3);
}

void calcJacobianTransformErrorDiff(const Iso3& target, const Iso3& source, const Iso3& source_pert, double err[6])
{
  calcJacobianTransformErrorDiff(target, target, source, source_pert, err);
}

// the 4-pose form [ext] used by DynamicCartPoseJacCalculator (kinematic_terms.cpp:170-177):
// both frames perturbed, err2(target_pert^-1 source_pert) - err2(target^-1 source)
void calcJacobianTransformErrorDiff(const Iso3& target, const Iso3& target_pert, const Iso3& source,
                                    const Iso3& source_pert, double err[6])
{
  const Iso3 pe = mul(inverse(target), source);
  const Iso3 ppe = mul(inverse(target_pert), source_pert);
  for (int i = 0; i < 3; ++i)
    err[i] = ppe.t[i] - pe.t[i];
  double r0[3], r1[3];
  calcRotationalError2(pe.R, r0);
  calcRotationalError2(ppe.R, r1);
  for (int i = 0; i < 3; ++i)
    err[3 + i] = r1[i] - r0[i];
}

// The tolerance-aware error difference of tesseract's 5-argument
// calcJacobianTransformErrorDiff [ext, unpinned; called at kinematic_terms.cpp:319-339]:
// both errors [t; rotvec] with the rotation vector in [-pi, pi] (calcTransformError),
// switched to the continuous [0, 2 pi) form (calcRotationalError2) for both when the
// perturbation crosses the wrap (a component jumps by more than pi), then
// applyTolerances on both; returns perturbed - unperturbed.  Pinned by
// kinematic_costs_unit.cpp:79-254 (zero rows inside the band, FD consistency).
void calcJacobianTransformErrorDiffTol(const Iso3& target, const Iso3& source, const Iso3& source_pert,
                                       const double* lower, const double* upper, double err[6])
{
  calcJacobianTransformErrorDiffTol(target, target, source, source_pert, lower, upper, err);
}

void calcJacobianTransformErrorDiffTol(const Iso3& target, const Iso3& target_pert, const Iso3& source,
                                       const Iso3& source_pert, const double* lower, const double* upper,
                                       double err[6])
{
  const Iso3 pe = mul(inverse(target), source);
  const Iso3 ppe = mul(inverse(target_pert), source_pert);
  double e0[6], e1[6];
  for (int i = 0; i < 3; ++i)
  {
    e0[i] = pe.t[i];
    e1[i] = ppe.t[i];
  }
  calcRotationalError(pe.R, e0 + 3);
  calcRotationalError(ppe.R, e1 + 3);
  bool wrap = false;
  for (int i = 3; i < 6; ++i)
    wrap = wrap || std::fabs(e1[i] - e0[i]) > M_PI;
  if (wrap)
  {
    calcRotationalError2(pe.R, e0 + 3);
    calcRotationalError2(ppe.R, e1 + 3);
  }
  applyTolerances(e0, lower, upper, 6);
  applyTolerances(e1, lower, upper, 6);
  for (int i = 0; i < 6; ++i)
    err[i] = e1[i] - e0[i];
}

void applyTolerances(double err[6], const double* lower, const double* upper, int n)
{
  for (int i = 0; i < n; ++i)
  {
    if (err[i] < lower[i])
      err[i] = err[i] - lower[i];
    else if (err[i] > upper[i])
      err[i] = err[i] - upper[i];
    else
      err[i] = 0;
  }
}

void chainFwdKin(const thip_chain& chain, const double* q, std::vector<Iso3>& out)
{
  out.resize(static_cast<std::size_t>(chain.n_links));
  out[0] = Iso3::from12(chain.base_pose);
  for (int k = 1; k < chain.n_links; ++k)
  {
    Iso3 t = mul(out[static_cast<std::size_t>(parentOf(chain, k))], Iso3::from12(chain.joint_origin[k]));
    const int type = chain.joint_type[k];
    if (type == THIP_JOINT_REVOLUTE || type == THIP_JOINT_CONTINUOUS)
      t = mul(t, axisAngle(chain.joint_axis[k], q[chain.joint_dof[k]]));
    else if (type == THIP_JOINT_PRISMATIC)
    {
      Iso3 m = Iso3::identity();
      for (int i = 0; i < 3; ++i)
        m.t[i] = chain.joint_axis[k][i] * q[chain.joint_dof[k]];
      t = mul(t, m);
    }
    out[static_cast<std::size_t>(k)] = t;
  }
}

void chainJacobian(const thip_chain& chain, const double* q, int link, double* J)
{
  std::vector<Iso3> T;
  chainFwdKin(chain, q, T);
  const int D = chain.n_dof;
  for (int e = 0; e < 6 * D; ++e)
    J[e] = 0.0;
  const double* p = T[static_cast<std::size_t>(link)].t;
  // the joints on the link's path from the root (a tree: other branches do
  // not move it)
  std::vector<char> on_path(static_cast<std::size_t>(chain.n_links), 0);
  for (int k = link; k > 0; k = parentOf(chain, k))
    on_path[static_cast<std::size_t>(k)] = 1;
  for (int k = 1; k <= link; ++k)
  {
    const int type = chain.joint_type[k];
    if (type == THIP_JOINT_FIXED || !on_path[static_cast<std::size_t>(k)])
      continue;
    const Iso3& Tk = T[static_cast<std::size_t>(k)];
    const double* ax = chain.joint_axis[k];
    double a[3];
    for (int r = 0; r < 3; ++r)
      a[r] = Tk.R[r * 3 + 0] * ax[0] + Tk.R[r * 3 + 1] * ax[1] + Tk.R[r * 3 + 2] * ax[2];
    const int j = chain.joint_dof[k];
    if (type == THIP_JOINT_PRISMATIC)
    {
      for (int r = 0; r < 3; ++r)
        J[r * D + j] = a[r];
      continue;
    }
    const double d[3] = { p[0] - Tk.t[0], p[1] - Tk.t[1], p[2] - Tk.t[2] };
    J[0 * D + j] = a[1] * d[2] - a[2] * d[1];
    J[1 * D + j] = a[2] * d[0] - a[0] * d[2];
    J[2 * D + j] = a[0] * d[1] - a[1] * d[0];
    for (int r = 0; r < 3; ++r)
      J[(3 + r) * D + j] = a[r];
  }
}

}  // namespace orc
