// Row-major dense matrix (reference: qmf/Matrix.h:27-88) and the symmetric solve used as
// the host fallback for rows whose system is not positive definite (Matrix.cpp:81-96).
#pragma once

#include <vector>

#include <qmf/Types.h>
#include <qmf/Vector.h>

namespace qmf {

class Matrix {
 public:
  using value_type = Double;

  Matrix(const size_t nrows, const size_t ncols);
  Matrix(const Matrix&) = default;
  Matrix& operator=(const Matrix&) = default;
  Matrix(Matrix&&) = default;
  Matrix& operator=(Matrix&&) = default;

  Double operator()(const size_t r, const size_t c) const { return data_[r * ncols_ + c]; }
  Double& operator()(const size_t r, const size_t c) { return data_[r * ncols_ + c]; }

  size_t nrows() const { return nrows_; }
  size_t ncols() const { return ncols_; }

  void clear() { std::fill(data_.begin(), data_.end(), Double()); }

  Matrix transpose() const;
  Matrix operator+(const Matrix& X) const;

  Double* data() { return data_.data(); }
  const Double* data() const { return data_.data(); }
  Double* data(const size_t r) { return &data_[r * ncols_]; }
  const Double* data(const size_t r) const { return &data_[r * ncols_]; }

 private:
  size_t nrows_;
  size_t ncols_;
  std::vector<Double> data_;
};

// Solves A x = b for a symmetric (possibly indefinite) A.  Aborts if A is singular, as the
// reference's CHECK on dsysv's info does.
Vector linearSymmetricSolve(Matrix A, Vector b);

}  // namespace qmf
