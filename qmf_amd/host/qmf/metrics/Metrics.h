// Per-user ranking/regression metrics (reference: qmf/metrics/Metrics.h:27-88,
// Metrics.cpp:27-164).  Labels > 0 are positives.  Host-side: evaluated on eval epochs only.
#pragma once

#include <vector>

#include <qmf/Types.h>
#include <qmf/utils/ParallelExecutor.h>

namespace qmf {

// One test user's ranking over all nitems items, as reduced on the device
// (qmfx_eval_ranks, csrc/eval.hip) instead of a dense score vector.  Every metric is a
// function of these: the reference sorts (score, label > 0) pairs descending, so the
// positives' places in that order are fixed by how many items score strictly higher.
struct RankedUser {
  size_t nitems = 0;
  Double sse = 0.0;                 // Σ_i (label_i − score_i)² over all items
  std::vector<int64_t> positions;   // 0-based places of the positives, ascending

  // positives (label > 0) with their scores and the count of items scored strictly higher
  void setPositives(const std::vector<Double>& scores, const std::vector<int64_t>& above);
};

class Metric {
 public:
  virtual ~Metric() = default;
  virtual Double compute(const std::vector<Double>& labels,
                         const std::vector<Double>& scores) const = 0;
  // the same value from the device-reduced ranking (addition to the reference API)
  virtual Double compute(const RankedUser& user) const = 0;
  virtual Double compute(const std::vector<RankedUser>& users, ParallelExecutor& parallel) const;
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
  Double compute(const RankedUser& user) const override;
};

class AUC : public Metric {
 public:
  using Metric::compute;
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
  Double compute(const RankedUser& user) const override;
};

class Precision : public Metric {
 public:
  using Metric::compute;
  explicit Precision(const size_t k) : k_(k) {}
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
  Double compute(const RankedUser& user) const override;

 private:
  const size_t k_;
};

class Recall : public Metric {
 public:
  using Metric::compute;
  explicit Recall(const size_t k) : k_(k) {}
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
  Double compute(const RankedUser& user) const override;

 private:
  const size_t k_;
};

class AveragePrecision : public Metric {
 public:
  using Metric::compute;
  Double compute(const std::vector<Double>& labels,
                 const std::vector<Double>& scores) const override;
  Double compute(const RankedUser& user) const override;
};

}  // namespace qmf
