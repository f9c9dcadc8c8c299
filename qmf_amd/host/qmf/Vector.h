// Dense vector (reference: qmf/Vector.h:25-47).
#pragma once

#include <vector>

#include <qmf/Types.h>

namespace qmf {

class Vector {
 public:
  explicit Vector(const size_t n) : data_(n, 0.0) {}

  Double operator()(const size_t i) const { return data_[i]; }
  Double& operator()(const size_t i) { return data_[i]; }
  size_t size() const { return data_.size(); }
  Double* data() { return data_.data(); }
  const Double* data() const { return data_.data(); }

 private:
  std::vector<Double> data_;
};

}  // namespace qmf
