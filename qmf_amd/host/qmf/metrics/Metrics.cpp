#include <qmf/metrics/Metrics.h>

#include <algorithm>
#include <functional>
#include <utility>

#include <qmf/utils/Log.h>

namespace qmf {

namespace {

using Scored = std::vector<std::pair<Double, bool>>;

// (score, is_positive) pairs and the positive count
Scored scorePairs(const std::vector<Double>& labels, const std::vector<Double>& scores,
                  int32_t* npos) {
  CHECK_EQ(labels.size(), scores.size());
  Scored s;
  s.reserve(labels.size());
  int32_t pos = 0;
  for (size_t i = 0; i < labels.size(); ++i) {
    const bool p = labels[i] > 0.0;
    pos += p;
    s.emplace_back(scores[i], p);
  }
  if (npos) *npos = pos;
  return s;
}

// positives among the k best-scored (ties broken by the pair order, as the reference)
int64_t positivesInTopK(Scored& s, size_t k) {
  std::nth_element(s.begin(), s.begin() + k, s.end(), std::greater<std::pair<Double, bool>>());
  return std::count_if(s.begin(), s.begin() + k, [](const auto& p) { return p.second; });
}

}  // namespace

Double Metric::compute(const std::vector<std::vector<Double>>& labels,
                       const std::vector<std::vector<Double>>& scores) const {
  CHECK_EQ(labels.size(), scores.size());
  CHECK_GT(labels.size(), 0);
  Double sum = 0.0;
  for (size_t u = 0; u < labels.size(); ++u) sum += compute(labels[u], scores[u]);
  return sum / labels.size();
}

Double Metric::compute(const std::vector<std::vector<Double>>& labels,
                       const std::vector<std::vector<Double>>& scores,
                       ParallelExecutor& parallel) const {
  CHECK_EQ(labels.size(), scores.size());
  CHECK_GT(labels.size(), 0);
  const Double total = parallel.mapReduce(
    labels.size(), [&](const size_t u) { return compute(labels[u], scores[u]); },
    std::plus<Double>(), 0.0);
  return total / labels.size();
}

Double MeanSquaredError::compute(const std::vector<Double>& labels,
                                 const std::vector<Double>& scores) const {
  CHECK_EQ(labels.size(), scores.size());
  CHECK_GT(labels.size(), 0);
  Double sum = 0.0;
  for (size_t i = 0; i < labels.size(); ++i) {
    const Double d = labels[i] - scores[i];
    sum += d * d;
  }
  return sum / labels.size();
}

Double AUC::compute(const std::vector<Double>& labels, const std::vector<Double>& scores) const {
  int32_t pos = 0;
  Scored s = scorePairs(labels, scores, &pos);
  const int32_t neg = static_cast<int32_t>(labels.size()) - pos;
  if (pos == 0 || neg == 0) {
    LOG(ERROR) << "AUC needs at least 1 example in each class";
    return 1.0;
  }
  std::sort(s.begin(), s.end(), std::greater<std::pair<Double, bool>>());
  // each negative adds the true-positive rate reached before it, times 1/neg
  int32_t tp = 0;
  Double auc = 0.0;
  for (const auto& p : s) {
    if (p.second)
      ++tp;
    else
      auc += static_cast<Double>(tp) / pos / neg;
  }
  return auc;
}

Double Precision::compute(const std::vector<Double>& labels,
                          const std::vector<Double>& scores) const {
  CHECK_EQ(labels.size(), scores.size());
  CHECK_GE(labels.size(), k_) << "P@k needs at least k ranked elements";
  Scored s = scorePairs(labels, scores, nullptr);
  return static_cast<Double>(positivesInTopK(s, k_)) / k_;
}

Double Recall::compute(const std::vector<Double>& labels, const std::vector<Double>& scores) const {
  CHECK_EQ(labels.size(), scores.size());
  CHECK_GE(labels.size(), k_) << "R@k needs at least k ranked elements";
  int32_t pos = 0;
  Scored s = scorePairs(labels, scores, &pos);
  CHECK_GT(pos, 0) << "R@k needs at least 1 positive";
  return static_cast<Double>(positivesInTopK(s, k_)) / pos;
}

Double AveragePrecision::compute(const std::vector<Double>& labels,
                                 const std::vector<Double>& scores) const {
  int32_t pos = 0;
  Scored s = scorePairs(labels, scores, &pos);
  CHECK_GT(pos, 0) << "AP needs at least 1 positive";
  std::sort(s.begin(), s.end(), std::greater<std::pair<Double, bool>>());
  Double ap = 0.0;
  int32_t seen = 0;
  for (size_t r = 0; r < s.size(); ++r)
    if (s[r].second) ap += static_cast<Double>(++seen) / (r + 1);
  return ap / pos;
}

}  // namespace qmf
