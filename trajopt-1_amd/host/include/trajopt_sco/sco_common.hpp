// trajopt_sco/include/trajopt_sco/sco_common.hpp (vector helpers and aliases)
// restated without Eigen for the MI355X build's host library.
#pragma once
#include <cmath>
#include <cstddef>
#include <string>
#include <vector>

namespace sco
{
using DblVec = std::vector<double>;
using IntVec = std::vector<int>;
using SizeTVec = std::vector<std::size_t>;
using StrVec = std::vector<std::string>;

inline double vecSum(const DblVec& v)
{
  double out = 0;
  for (double x : v)
    out += x;
  return out;
}
inline double vecAbsSum(const DblVec& v)
{
  double out = 0;
  for (double x : v)
    out += std::fabs(x);
  return out;
}
inline double pospart(double x) { return (x > 0) ? x : 0; }
inline double sq(double x) { return x * x; }
inline double vecHingeSum(const DblVec& v)
{
  double out = 0;
  for (double x : v)
    out += pospart(x);
  return out;
}
inline double vecMax(const DblVec& v)
{
  double out = -HUGE_VAL;
  for (double x : v)
    out = (x > out) ? x : out;
  return out;
}
inline double vecDot(const DblVec& a, const DblVec& b)
{
  double out = 0;
  for (std::size_t i = 0; i < a.size() && i < b.size(); ++i)
    out += a[i] * b[i];
  return out;
}
}  // namespace sco
