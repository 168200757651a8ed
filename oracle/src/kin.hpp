// ORACLE — test infrastructure only (see sco_expr.hpp header).
//
// CPU restatement of the kinematics / pose-error arithmetic the reference
// delegates to tesseract [ext, not under /root/reference]:
//   JointGroup::calcFwdKin (kinematic tree, URDF joint semantics)
//     call sites trajopt/src/kinematic_terms.cpp:255,355; collision_terms.cpp:882
//   tesseract::common::calcTransformError, calcRotationalError(2),
//   calcJacobianTransformErrorDiff, applyTolerances
//     call sites trajopt/src/kinematic_terms.cpp:84-92,175,218-245,321,339
// The Eigen primitives they rest on (Quaternion-from-matrix, AngleAxis from
// quaternion / to rotation matrix, Isometry inverse) are restated with Eigen's
// published formulas. Pinned by the reference's kinematic_costs_unit semantics
// (FD consistency, AngleAxis(-0.1, x) -> err[3] = -0.1); exact values vs
// tesseract are "parity unpinned".
#pragma once
#include <array>
#include <vector>

#include "../../include/trajopt_hip.h"

namespace orc
{
// parent link of k >= 1: thip_chain.parent when the chain is a tree, else k - 1
// (a zero-initialised chain is serial, include/trajopt_hip.h)
inline int parentOf(const thip_chain& c, int k) { return c.is_tree ? c.parent[k] : k - 1; }

struct Iso3
{
  // row-major R (3x3) and t
  double R[9];
  double t[3];
  static Iso3 identity()
  {
    Iso3 a{};
    a.R[0] = a.R[4] = a.R[8] = 1;
    return a;
  }
  static Iso3 from12(const double* p)  // [R | t] row-major 3x4
  {
    Iso3 a{};
    for (int r = 0; r < 3; ++r)
    {
      for (int c = 0; c < 3; ++c)
        a.R[r * 3 + c] = p[r * 4 + c];
      a.t[r] = p[r * 4 + 3];
    }
    return a;
  }
  void to12(double* p) const
  {
    for (int r = 0; r < 3; ++r)
    {
      for (int c = 0; c < 3; ++c)
        p[r * 4 + c] = R[r * 3 + c];
      p[r * 4 + 3] = t[r];
    }
  }
};

Iso3 mul(const Iso3& a, const Iso3& b);
Iso3 inverse(const Iso3& a);
Iso3 axisAngle(const double axis[3], double angle);  // Eigen AngleAxis::toRotationMatrix
// Quaternion (w, x, y, z) from a rotation matrix (Eigen quaternionbase_assign_impl<.,3,3>)
void quatFromMatrix(const double R[9], double q[4]);
void calcRotationalError(const double R[9], double out[3]);   // angle in [-pi, pi]
void calcRotationalError2(const double R[9], double out[3]);  // angle in [0, 2pi]
void calcTransformError(const Iso3& t1, const Iso3& t2, double err[6]);
void calcJacobianTransformErrorDiff(const Iso3& target, const Iso3& source, const Iso3& source_pert, double err[6]);
void applyTolerances(double err[6], const double* lower, const double* upper, int n);
void calcJacobianTransformErrorDiffTol(const Iso3& target, const Iso3& source, const Iso3& source_pert,
                                       const double* lower, const double* upper, double err[6]);
void calcJacobianTransformErrorDiff(const Iso3& target, const Iso3& target_pert, const Iso3& source,
                                    const Iso3& source_pert, double err[6]);
void calcJacobianTransformErrorDiffTol(const Iso3& target, const Iso3& target_pert, const Iso3& source,
                                       const Iso3& source_pert, const double* lower, const double* upper,
                                       double err[6]);

// link poses of the chain at q: out[n_links]
void chainFwdKin(const thip_chain& chain, const double* q, std::vector<Iso3>& out);

// Geometric jacobian (world frame, reference point = origin of `link`) at q:
// J[6][n_dof] row-major, rows 0-2 linear, 3-5 angular; revolute column
// [a x (p - o); a], prismatic [a; 0] (tesseract JointGroup::calcJacobian [ext])
void chainJacobian(const thip_chain& chain, const double* q, int link, double* J);

}  // namespace orc
