// Host-side factor matrix + optional biases (reference: qmf/FactorData.h:28-142).  The
// engines keep the authoritative copy on the device and refresh this mirror on demand.
#pragma once

#include <cstdio>
#include <fstream>
#include <string>

#include <qmf/Matrix.h>
#include <qmf/Vector.h>
#include <qmf/utils/Log.h>

namespace qmf {

class FactorData {
 public:
  FactorData(const size_t nelems, const size_t nfactors, const bool withBiases = false)
      : withBiases_(withBiases), factors_(nelems, nfactors), biases_(withBiases ? nelems : 0) {}

  Double at(const size_t idx, const size_t fidx) const { return factors_(idx, fidx); }
  Double& at(const size_t idx, const size_t fidx) { return factors_(idx, fidx); }

  Double biasAt(const size_t idx) const { return withBiases_ ? biases_(idx) : 0.0; }
  Double& biasAt(const size_t idx) {
    CHECK(withBiases_) << "can't access bias when withBiases = false";
    return biases_(idx);
  }

  template <typename FuncT>
  void setFactors(FuncT func) {
    for (size_t idx = 0; idx < nelems(); ++idx)
      for (size_t fidx = 0; fidx < nfactors(); ++fidx) factors_(idx, fidx) = func(idx, fidx);
  }

  // zero fill
  void setFactors() { factors_.clear(); }

  // One "%lf" per line, row-major in idx order (FactorData.h:74-100).  A short file logs
  // an error and leaves the remaining factors unchanged; a malformed line aborts.
  void setFactors(const std::string& fileName) {
    std::ifstream fin(fileName);
    std::string line;
    size_t count = 0;
    for (size_t idx = 0; idx < nelems(); ++idx) {
      for (size_t fidx = 0; fidx < nfactors(); ++fidx) {
        if (!std::getline(fin, line)) {
          LOG(ERROR) << "read uniform data from " << fileName << " failed.";
          return;
        }
        double value = 0.0;
        const int result = sscanf(line.c_str(), "%lf", &value);
        CHECK_EQ(result, 1) << "the file format is incorrect: " << line;
        factors_(idx, fidx) = value;
        ++count;
      }
    }
    LOG(INFO) << "initialized factor from file size: " << count;
  }

  template <typename FuncT>
  void setBiases(FuncT func) {
    for (size_t idx = 0; idx < biases_.size(); ++idx) biases_(idx) = func(idx);
  }

  size_t nelems() const { return factors_.nrows(); }
  size_t nfactors() const { return factors_.ncols(); }
  bool withBiases() const { return withBiases_; }

  const Matrix& getFactors() const { return factors_; }
  Matrix& getFactors() { return factors_; }
  const Vector& getBiases() const { return biases_; }
  Vector& getBiases() { return biases_; }

 private:
  const bool withBiases_;
  Matrix factors_;
  Vector biases_;
};

}  // namespace qmf
