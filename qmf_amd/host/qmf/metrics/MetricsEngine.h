// Metric bookkeeping for the engines (reference: qmf/metrics/MetricsEngine.h:30-137,
// MetricsEngine.cpp:21-47).  Records (epoch, value) per "<prefix><metric>" key and logs
// "epoch E: recorded metric KEY = V".
#pragma once

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include <qmf/Types.h>
#include <qmf/metrics/MetricsManager.h>
#include <qmf/utils/Log.h>

namespace qmf {

struct MetricsConfig {
  size_t numTestUsers;
  bool alwaysCompute;
  int32_t seed;
};

class MetricsEngine {
 public:
  // keeps a copy of `config` (the reference keeps a reference, which dangles for the
  // defaulted argument)
  MetricsEngine(const MetricsConfig& config = {}, const bool log = true);

  const MetricsConfig& config() const { return config_; }

  bool addTrainMetric(const std::string& m) { return addMetric(trainMetrics_, m); }
  bool addTestMetric(const std::string& m) { return addMetric(testMetrics_, m); }
  bool addTrainAvgMetric(const std::string& m) { return addMetric(trainAvgMetrics_, m); }
  bool addTestAvgMetric(const std::string& m) { return addMetric(testAvgMetrics_, m); }

  void computeAndRecordTrainMetrics(const size_t epoch, const std::vector<Double>& labels,
                                    const std::vector<Double>& scores) {
    computeAndRecord(trainMetrics_, "train_", epoch, labels, scores);
  }
  void computeAndRecordTestMetrics(const size_t epoch, const std::vector<Double>& labels,
                                   const std::vector<Double>& scores) {
    computeAndRecord(testMetrics_, "test_", epoch, labels, scores);
  }
  template <typename... Args>
  void computeAndRecordTrainAvgMetrics(const size_t epoch, Args&... args) {
    computeAndRecord(trainAvgMetrics_, "train_avg_", epoch, args...);
  }
  template <typename... Args>
  void computeAndRecordTestAvgMetrics(const size_t epoch, Args&... args) {
    computeAndRecord(testAvgMetrics_, "test_avg_", epoch, args...);
  }

  const std::vector<std::string>& trainMetrics() const { return trainMetrics_; }
  const std::vector<std::string>& testMetrics() const { return testMetrics_; }
  const std::vector<std::string>& trainAvgMetrics() const { return trainAvgMetrics_; }
  const std::vector<std::string>& testAvgMetrics() const { return testAvgMetrics_; }

  using MetricVector = std::vector<std::pair<size_t, Double>>;
  // recorded values per key (e.g. "test_avg_auc")
  const std::unordered_map<std::string, MetricVector>& recorded() const { return metricsMap_; }

 private:
  bool addMetric(std::vector<std::string>& metrics, const std::string& metric);

  template <typename... Args>
  void computeAndRecord(const std::vector<std::string>& metrics, const std::string& prefix,
                        const size_t epoch, Args&... args) {
    for (const auto& name : metrics) {
      const auto& m = MetricsManager::get().getMetric(name);
      CHECK(m) << "missing metric " << prefix + name;
      recordMetric(prefix + name, epoch, m->compute(args...));
    }
  }

  void recordMetric(const std::string& key, const size_t epoch, const Double val);

  const MetricsConfig config_;
  const bool log_;
  std::vector<std::string> trainMetrics_;
  std::vector<std::string> trainAvgMetrics_;
  std::vector<std::string> testMetrics_;
  std::vector<std::string> testAvgMetrics_;
  std::unordered_map<std::string, MetricVector> metricsMap_;
};

}  // namespace qmf
