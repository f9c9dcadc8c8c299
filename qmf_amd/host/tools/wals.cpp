// `wals` command line, drop-in for the reference's qmf/wals.cpp:26-107: same flags, same
// log lines and output files.  Additions: --device, --precision (32 | 64), --ngpus.
#include <chrono>
#include <cstdlib>
#include <fstream>
#include <memory>

#include <qmf/DatasetReader.h>
#include <qmf/metrics/MetricsEngine.h>
#include <qmf/utils/Flags.h>
#include <qmf/utils/Log.h>
#include <qmf/utils/Util.h>
#include <qmf/wals/WALSEngine.h>

// model arguments
DEFINE_uint64(nepochs, 10, "number of epochs for ALS");
DEFINE_uint64(nfactors, 30, "dimension of learned factors");
DEFINE_double(regularization_lambda, 0.05, "regularization param");
DEFINE_double(confidence_weight, 40, "confidence weight");
DEFINE_double(init_distribution_bound, 0.01, "init distirbution bound");
DEFINE_string(distribution_file, "", "uniform distribution file, for repeatable result");
// settings
DEFINE_int32(nthreads, 16, "number of host threads (ingest, evaluation, output)");
DEFINE_int32(device, qmf::DeviceOptions::envInt("QMF_DEVICE", 0), "GPU ordinal");
DEFINE_int32(precision, qmf::DeviceOptions::envInt("QMF_PRECISION", 64),
             "device arithmetic: 64 (fp64, the reference's Double; default) or 32 (fp32)");
DEFINE_int32(ngpus, qmf::DeviceOptions::envInt("QMF_NGPUS", 1),
             "GPUs to split the rows over (devices --device .. --device+ngpus-1, RCCL "
             "all-gather per half-epoch)");
// datasets
DEFINE_string(train_dataset, "", "filename of training dataset");
DEFINE_string(test_dataset, "", "filename of test dataset");
// metrics
DEFINE_string(test_avg_metrics, "", "comma-separated list of test metrics (averaged per-user)");
DEFINE_int32(eval_seed, 42, "random seed for picking test users");
DEFINE_uint64(num_test_users, 0, "# users to use for computing test avg metrics (0 = all users)");
DEFINE_bool(test_always, false,
            "whether to compute test avg metrics after each epoch (if false, only computes at "
            "the end)");
// model output
DEFINE_string(user_factors, "", "filename of user factors");
DEFINE_string(item_factors, "", "filename of item factors");

namespace {
// QMF_TIMINGS=1 (an addition; unset, the output is the reference's): one "timing:" log line per
// phase with its wall time, read by tools/bench_cli.py
bool timings() {
  static const bool on = std::getenv("QMF_TIMINGS") && std::atoi(std::getenv("QMF_TIMINGS")) > 0;
  return on;
}
double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
long long fileBytes(const std::string& f) {
  std::ifstream s(f, std::ios::binary | std::ios::ate);
  return s ? static_cast<long long>(s.tellg()) : 0;
}
}  // namespace

int main(int argc, char** argv) {
  if (!qmf::flags::parse(&argc, &argv, "wals")) return 1;
  if (FLAGS_user_factors.empty() || FLAGS_item_factors.empty()) {
    LOG(WARNING) << "warning: missing model output filenames! (use options --{user,item}_factors)";
  }
  qmf::WALSConfig config{FLAGS_nepochs,
                         FLAGS_nfactors,
                         FLAGS_regularization_lambda,
                         FLAGS_confidence_weight,
                         FLAGS_init_distribution_bound,
                         FLAGS_distribution_file};
  qmf::MetricsConfig metricsConfig{FLAGS_num_test_users, FLAGS_test_always, FLAGS_eval_seed};
  const auto metricsEngine = std::make_unique<qmf::MetricsEngine>(metricsConfig);
  for (const auto& metric : qmf::split(FLAGS_test_avg_metrics, ',')) {
    CHECK(metricsEngine->addTestAvgMetric(metric)) << "metric " << metric << " is not available";
  }
  qmf::DeviceOptions device;
  device.device = FLAGS_device;
  device.precision = FLAGS_precision;
  device.ngpus = FLAGS_ngpus;
  qmf::WALSEngine engine(config, metricsEngine, static_cast<size_t>(FLAGS_nthreads), device);

  LOG(INFO) << "loading training data";
  double t0 = now();
  qmf::DatasetReader trainReader(FLAGS_train_dataset);
  {
    const auto data = trainReader.readAll();
    const double t1 = now();
    if (timings())
      LOG(INFO) << "timing: parse " << t1 - t0 << " s, " << fileBytes(FLAGS_train_dataset)
                << " bytes, " << data.size() << " lines";
    engine.init(data);
    if (timings()) LOG(INFO) << "timing: init " << now() - t1 << " s";
  }
  if (!FLAGS_test_dataset.empty()) {
    LOG(INFO) << "loading test data";
    qmf::DatasetReader testReader(FLAGS_test_dataset);
    engine.initTest(testReader.readAll());
  }
  LOG(INFO) << "training";
  t0 = now();
  engine.optimize();
  if (timings()) LOG(INFO) << "timing: optimize " << now() - t0 << " s, " << FLAGS_nepochs << " epochs";
  if (!FLAGS_user_factors.empty() && !FLAGS_item_factors.empty()) {
    LOG(INFO) << "saving model output";
    t0 = now();
    engine.saveUserFactors(FLAGS_user_factors);
    engine.saveItemFactors(FLAGS_item_factors);
    if (timings())
      LOG(INFO) << "timing: save " << now() - t0 << " s, "
                << fileBytes(FLAGS_user_factors) + fileBytes(FLAGS_item_factors) << " bytes";
  }
  return 0;
}
