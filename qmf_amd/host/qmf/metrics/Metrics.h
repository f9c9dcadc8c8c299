// Per-user ranking/regression metrics (reference: qmf/metrics/Metrics.h:27-88,
// Metrics.cpp:27-164).  Labels > 0 are positives.  Host-side: evaluated on eval epochs only.
#pragma once

#include <vector>

#include <qmf/Types.h>
#include <qmf/utils/ParallelExecutor.h>

namespace qmf {

class Metric {
 public:
  virtual ~Metric() = default;
  virtual Double compute(const std::vector<Double>& labels,
                         const std::vector<Double>& scores) const = 0;
  // mean over users
  virtual Double compute(const std::vector<std::vector<Double>>& labels,
                         const std::vector<std::vector<Double>>& scores) const;
  virtual Double compute(const std::vector<std::vector<Double>>& labels,
                         const std::vector<std::vector<Double>>& scores,
                         ParallelExecutor& parallel) const;
};

class MeanSquaredError : public Metric {
 public:
  using Metric::compute;
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
};

class AUC : public Metric {
 public:
  using Metric::compute;
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
};

class Precision : public Metric {
 public:
  using Metric::compute;
  explicit Precision(const size_t k) : k_(k) {}
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;

 private:
  const size_t k_;
};

class Recall : public Metric {
 public:
  using Metric::compute;
  explicit Recall(const size_t k) : k_(k) {}
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;

 private:
  const size_t k_;
};

class AveragePrecision : public Metric {
 public:
  using Metric::compute;
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
};

}  // namespace qmf
