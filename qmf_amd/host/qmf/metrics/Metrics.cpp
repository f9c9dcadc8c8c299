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

int64_t positivesBefore(const RankedUser& u, size_t k) {
  return std::lower_bound(u.positions.begin(), u.positions.end(), static_cast<int64_t>(k)) -
         u.positions.begin();
}

}  // namespace

void RankedUser::setPositives(const std::vector<Double>& scores,
                              const std::vector<int64_t>& above) {
  CHECK_EQ(scores.size(), above.size());
  std::vector<size_t> ord(scores.size());
  for (size_t p = 0; p < ord.size(); ++p) ord[p] = p;
  std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return scores[a] > scores[b]; });
  // equal-scored positives are equal (score, true) pairs: they fill the places
  // above, above + 1, ... in any order
  positions.resize(ord.size());
  for (size_t r = 0; r < ord.size(); ++r) {
    const bool tie = r > 0 && scores[ord[r]] == scores[ord[r - 1]];
    positions[r] = tie ? positions[r - 1] + 1 : above[ord[r]];
  }
}

Double Metric::compute(const std::vector<RankedUser>& users, ParallelExecutor& parallel) const {
  CHECK_GT(users.size(), 0);
  const Double total = parallel.mapReduce(
    users.size(), [&](const size_t u) { return compute(users[u]); }, std::plus<Double>(), 0.0);
  return total / users.size();
}

Double MeanSquaredError::compute(const RankedUser& u) const {
  CHECK_GT(u.nitems, 0);
  return u.sse / u.nitems;
}

Double AUC::compute(const RankedUser& u) const {
  const int64_t pos = static_cast<int64_t>(u.positions.size());
  const int64_t neg = static_cast<int64_t>(u.nitems) - pos;
  if (pos == 0 || neg == 0) {
    LOG(ERROR) << "AUC needs at least 1 example in each class";
    return 1.0;
  }
  // the negatives between the m-th and (m+1)-th positive each add m/pos/neg
  Double auc = 0.0;
  for (int64_t m = 1; m <= pos; ++m) {
    const int64_t next = m < pos ? u.positions[m] : static_cast<int64_t>(u.nitems);
    const int64_t negs = next - u.positions[m - 1] - 1;
    auc += static_cast<Double>(negs) * (static_cast<Double>(m) / pos / neg);
  }
  return auc;
}

Double Precision::compute(const RankedUser& u) const {
  CHECK_GE(u.nitems, k_) << "P@k needs at least k ranked elements";
  return static_cast<Double>(positivesBefore(u, k_)) / k_;
}

Double Recall::compute(const RankedUser& u) const {
  CHECK_GE(u.nitems, k_) << "R@k needs at least k ranked elements";
  CHECK_GT(u.positions.size(), 0) << "R@k needs at least 1 positive";
  return static_cast<Double>(positivesBefore(u, k_)) / u.positions.size();
}

Double AveragePrecision::compute(const RankedUser& u) const {
  CHECK_GT(u.positions.size(), 0) << "AP needs at least 1 positive";
  Double ap = 0.0;
  for (size_t m = 0; m < u.positions.size(); ++m)
    ap += static_cast<Double>(m + 1) / (u.positions[m] + 1);
  return ap / u.positions.size();
}

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
