// Registry of metric objects by name (reference: qmf/metrics/MetricsManager.h:28-68,
// MetricsManager.cpp:27-95): "mse", "auc", "ap" built in; "p@k" / "r@k" created on demand.
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

#include <qmf/metrics/Metrics.h>

namespace qmf {

namespace detail {
// "<name>@<k>" -> (name, k); false when there is no '@' after a non-empty name or k is
// not a number
bool parseAtKMetric(const std::string& name, std::string& metricName, size_t& k);
}  // namespace detail

class MetricsManager {
 public:
  MetricsManager();
  MetricsManager(const MetricsManager&) = delete;
  MetricsManager(MetricsManager&&) = delete;
  MetricsManager& operator=(const MetricsManager&) = delete;
  MetricsManager& operator=(MetricsManager&&) = delete;

  void init();
  bool initFromName(const std::string& name) const;

  template <typename MetricT, typename... Args>
  void registerMetric(const std::string& name, Args&&... args) const {
    std::lock_guard<std::mutex> g(mu_);
    metrics_.emplace(name, std::make_unique<MetricT>(std::forward<Args>(args)...));
  }

  // nullptr-holding reference when the metric does not exist
  const std::unique_ptr<Metric>& getMetric(const std::string& name) const;
  bool exists(const std::string& name) const;

  static const MetricsManager& get();

 private:
  mutable std::mutex mu_;
  mutable std::unordered_map<std::string, std::unique_ptr<Metric>> metrics_;
};

}  // namespace qmf
