#include <qmf/metrics/MetricsEngine.h>

namespace qmf {

MetricsEngine::MetricsEngine(const MetricsConfig& config, const bool log)
    : config_(config), log_(log) {}

bool MetricsEngine::addMetric(std::vector<std::string>& metrics, const std::string& metric) {
  if (!MetricsManager::get().exists(metric)) return false;
  metrics.push_back(metric);
  return true;
}

void MetricsEngine::recordMetric(const std::string& key, const size_t epoch, const Double val) {
  metricsMap_[key].emplace_back(epoch, val);
  if (log_) LOG(INFO) << "epoch " << epoch << ": recorded metric " << key << " = " << val;
}

}  // namespace qmf
