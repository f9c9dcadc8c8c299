#include <qmf/metrics/MetricsManager.h>

#include <exception>

namespace qmf {

namespace {
const std::unique_ptr<Metric> kNoMetric;
}

MetricsManager::MetricsManager() { init(); }

void MetricsManager::init() {
  registerMetric<MeanSquaredError>("mse");
  registerMetric<AUC>("auc");
  registerMetric<AveragePrecision>("ap");
}

namespace detail {
bool parseAtKMetric(const std::string& name, std::string& metricName, size_t& k) {
  const auto at = name.find('@');
  if (at == 0 || at == std::string::npos) return false;
  metricName = name.substr(0, at);
  try {
    k = std::stoul(name.substr(at + 1));
  } catch (const std::exception&) {
    return false;
  }
  return true;
}
}  // namespace detail

bool MetricsManager::initFromName(const std::string& name) const {
  std::string base;
  size_t k = 0;
  if (!detail::parseAtKMetric(name, base, k)) return false;
  if (base == "p")
    registerMetric<Precision>(name, k);
  else if (base == "r")
    registerMetric<Recall>(name, k);
  else
    return false;
  return true;
}

const std::unique_ptr<Metric>& MetricsManager::getMetric(const std::string& name) const {
  if (!exists(name)) return kNoMetric;
  std::lock_guard<std::mutex> g(mu_);
  return metrics_.find(name)->second;
}

bool MetricsManager::exists(const std::string& name) const {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (metrics_.count(name)) return true;
  }
  return initFromName(name);
}

const MetricsManager& MetricsManager::get() {
  static MetricsManager instance;
  return instance;
}

}  // namespace qmf
