// trajopt_ifopt::Bounds (trajopt_ifopt/src/core/bounds.cpp:24-84): the type of a
// row's bounds (equality when |upper - lower| < 1e-8, values beyond +-1e20 are
// infinite) decides how trajopt_sqp lowers it (slack variables per row).
#pragma once
#include <cmath>

namespace trajopt_ifopt
{
enum class BoundsType
{
  kEquality,
  kRangeBound,
  kLowerBound,
  kUpperBound,
  kUnbounded
};

bool isFinite(double value);

class Bounds
{
public:
  Bounds(double lower = 0.0, double upper = 0.0);
  void set(double lower, double upper);
  void setLower(double lower);
  void setUpper(double upper);
  double getLower() const { return lower_; }
  double getUpper() const { return upper_; }
  BoundsType getType() const { return type_; }
  void operator+=(double scalar);
  void operator-=(double scalar);

private:
  double lower_, upper_;
  BoundsType type_{ BoundsType::kEquality };
  void updateType();
};

extern const Bounds NoBound;
extern const Bounds BoundZero;
extern const Bounds BoundGreaterZero;
extern const Bounds BoundSmallerZero;
}  // namespace trajopt_ifopt
