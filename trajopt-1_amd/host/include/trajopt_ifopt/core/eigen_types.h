// trajopt_ifopt's matrix types (trajopt_ifopt/include/trajopt_ifopt/core/eigen_types.h)
// without Eigen: VectorXd is a std::vector<double>, Jacobian a row-major sparse
// matrix filled the way the reference's constraint sets fill Eigen's
// (startVec(row) / insertBack(row, col) = value / finalize, columns ascending
// inside a row), so a user ConstraintSet's getJacobian() reads the same.
#pragma once
#include <cstddef>
#include <stdexcept>
#include <vector>

namespace trajopt_ifopt
{
using VectorXd = std::vector<double>;
using Index = long;

class Jacobian
{
public:
  Jacobian() = default;
  Jacobian(Index rows, Index cols) : rows_(rows), cols_(cols), outer_(static_cast<std::size_t>(rows) + 1, 0) {}
  Index rows() const { return rows_; }
  Index cols() const { return cols_; }
  Index outerSize() const { return rows_; }
  Index nonZeros() const { return static_cast<Index>(inner_.size()); }
  void reserve(Index nnz)
  {
    inner_.reserve(static_cast<std::size_t>(nnz));
    values_.reserve(static_cast<std::size_t>(nnz));
  }
  // Eigen's low-level filling API: rows in order, columns ascending inside a row
  void startVec(Index row)
  {
    if (row < cur_ || row >= rows_)
      throw std::runtime_error("Jacobian::startVec: rows must be started in order");
    for (Index r = cur_ + 1; r <= row; ++r)
      outer_[static_cast<std::size_t>(r)] = static_cast<long>(inner_.size());
    cur_ = row;
    row_start_ = static_cast<Index>(inner_.size());
  }
  double& insertBack(Index row, Index col)
  {
    if (row != cur_ || col < 0 || col >= cols_ || (static_cast<Index>(inner_.size()) > row_start_ && inner_.back() >= col))
      throw std::runtime_error("Jacobian::insertBack: entries of the started row in ascending column order");
    inner_.push_back(col);
    values_.push_back(0.0);
    return values_.back();
  }
  void finalize()
  {
    for (Index r = cur_ + 1; r <= rows_; ++r)
      outer_[static_cast<std::size_t>(r)] = static_cast<long>(inner_.size());
    cur_ = rows_;
  }
  // row r spans [rowBegin(r), rowEnd(r)) of col() / value()
  Index rowBegin(Index r) const { return outer_[static_cast<std::size_t>(r)]; }
  Index rowEnd(Index r) const { return outer_[static_cast<std::size_t>(r) + 1]; }
  Index col(Index e) const { return inner_[static_cast<std::size_t>(e)]; }
  double value(Index e) const { return values_[static_cast<std::size_t>(e)]; }
  double& valueRef(Index e) { return values_[static_cast<std::size_t>(e)]; }

private:
  Index rows_ = 0, cols_ = 0, cur_ = -1, row_start_ = 0;
  std::vector<long> outer_{ 0 };
  std::vector<Index> inner_;
  std::vector<double> values_;
};
}  // namespace trajopt_ifopt
