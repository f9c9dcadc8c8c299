#include <qmf/Matrix.h>

#include <algorithm>
#include <cmath>

#include <qmf/utils/Log.h>

namespace qmf {

Matrix::Matrix(const size_t nrows, const size_t ncols)
    : nrows_(nrows), ncols_(ncols), data_(nrows * ncols, 0.0) {
  CHECK_GT(nrows * ncols, 0) << "matrix's dimensions should be positive";
}

Matrix Matrix::transpose() const {
  Matrix T(ncols_, nrows_);
  for (size_t i = 0; i < nrows_; ++i)
    for (size_t j = 0; j < ncols_; ++j) T(j, i) = (*this)(i, j);
  return T;
}

Matrix Matrix::operator+(const Matrix& X) const {
  CHECK_EQ(nrows_, X.nrows());
  CHECK_EQ(ncols_, X.ncols());
  Matrix S(nrows_, ncols_);
  for (size_t i = 0; i < data_.size(); ++i) S.data_[i] = data_[i] + X.data_[i];
  return S;
}

// Gaussian elimination with partial pivoting in fp64.  Only reached for the rare rows the
// device flags as not positive definite, so a simple O(n³) host solve is enough.
Vector linearSymmetricSolve(Matrix A, Vector b) {
  CHECK_EQ(A.nrows(), A.ncols()) << "A should be squared";
  CHECK_EQ(A.nrows(), b.size()) << "b should have the same number of rows as A";
  const size_t n = A.nrows();
  for (size_t c = 0; c < n; ++c) {
    size_t piv = c;
    for (size_t r = c + 1; r < n; ++r)
      if (std::fabs(A(r, c)) > std::fabs(A(piv, c))) piv = r;
    CHECK(A(piv, c) != 0.0) << "linear solve failed: singular matrix";
    if (piv != c) {
      for (size_t j = 0; j < n; ++j) std::swap(A(c, j), A(piv, j));
      std::swap(b(c), b(piv));
    }
    const Double inv = 1.0 / A(c, c);
    for (size_t r = c + 1; r < n; ++r) {
      const Double f = A(r, c) * inv;
      if (f == 0.0) continue;
      for (size_t j = c; j < n; ++j) A(r, j) -= f * A(c, j);
      b(r) -= f * b(c);
    }
  }
  Vector x(n);
  for (size_t i = n; i-- > 0;) {
    Double s = b(i);
    for (size_t j = i + 1; j < n; ++j) s -= A(i, j) * x(j);
    x(i) = s / A(i, i);
  }
  return x;
}

}  // namespace qmf
