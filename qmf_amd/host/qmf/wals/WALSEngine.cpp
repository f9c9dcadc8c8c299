#include <qmf/wals/WALSEngine.h>

#include <limits>
#include <random>

#include <qmf/Matrix.h>
#include <qmf/utils/Log.h>

namespace qmf {

WALSEngine::WALSEngine(const WALSConfig& config,
                       const std::unique_ptr<MetricsEngine>& metricsEngine,
                       const size_t nthreads,
                       const DeviceOptions& device)
    : config_(config), metricsEngine_(metricsEngine), deviceOptions_(device),
      parallel_(nthreads) {
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty() &&
      metricsEngine_->config().numTestUsers == 0) {
    LOG(WARNING) << "computing average test metrics on all users can be slow! "
                    "Set numTestUsers > 0 to sample some of them";
  }
}

WALSEngine::~WALSEngine() = default;

void WALSEngine::init(const std::vector<DatasetElem>& dataset) {
  CHECK(!userFactors_ && !itemFactors_) << "engine was already initialized with train data";
  CHECK_GT(config_.nfactors, 0);
  CHECK(!dataset.empty()) << "empty train dataset";
  CHECK_GE(deviceOptions_.ngpus, 1) << "--ngpus must be at least 1";
  if (deviceOptions_.ngpus > 1) {
    int visible = 0;
    QMFX_CHECK(qmfx_device_count(&visible));
    CHECK_LE(deviceOptions_.device + deviceOptions_.ngpus, visible)
        << "--ngpus " << deviceOptions_.ngpus << " from --device " << deviceOptions_.device
        << " needs " << deviceOptions_.device + deviceOptions_.ngpus << " GPUs; " << visible
        << " visible";
  }
  dev_ = std::make_unique<DeviceContext>(deviceOptions_, config_.nfactors);
  ranks_.assign(1, dev_->get());
  for (int r = 1; r < deviceOptions_.ngpus; ++r) {
    peers_.push_back(std::make_unique<DeviceContext>(deviceOptions_, config_.nfactors, r));
    ranks_.push_back(peers_.back()->get());
  }
  qmfx_ctx* c = dev_->get();
  if (dataset.size() < static_cast<size_t>(std::numeric_limits<int32_t>::max())) {
    // ids, idx and both CSR orientations built on the device (qmfx_group_signals)
    int64_t nu = 0, ni = 0;
    QMFX_CHECK(qmfx_group_signals(c, dataset.data(), static_cast<int64_t>(dataset.size()), &nu,
                                  &ni));
    std::vector<int64_t> uids(static_cast<size_t>(nu)), iids(static_cast<size_t>(ni));
    QMFX_CHECK(qmfx_get_ids(c, QMFX_USERS, uids.data()));
    QMFX_CHECK(qmfx_get_ids(c, QMFX_ITEMS, iids.data()));
    userIndex_.assignSorted(std::move(uids));
    itemIndex_.assignSorted(std::move(iids));
    // the other ranks copy rank 0's CSR device to device over xGMI (one sort, no further
    // host→device uploads); qmfx_dist_init_all then keeps each rank's shard
    for (size_t r = 1; r < ranks_.size(); ++r) QMFX_CHECK(qmfx_import_signals(ranks_[r], c));
  } else {
    // beyond the device sort's 32-bit item count: the same grouping on the host
    SignalCsr byUser, byItem;
    groupSignals(dataset, userIndex_, itemIndex_, byUser, byItem, parallel_.nthreads());
    for (qmfx_ctx* rc : ranks_) {
      QMFX_CHECK(qmfx_set_shape(rc, static_cast<int64_t>(nusers()),
                                static_cast<int64_t>(nitems())));
      QMFX_CHECK(qmfx_upload_csr(rc, QMFX_USERS, byUser.rowptr.data(), byUser.col.data(),
                                 byUser.val.data(), static_cast<int64_t>(byUser.nnz())));
      QMFX_CHECK(qmfx_upload_csr(rc, QMFX_ITEMS, byItem.rowptr.data(), byItem.col.data(),
                                 byItem.val.data(), static_cast<int64_t>(byItem.nnz())));
    }
  }

  userFactors_ = std::make_unique<FactorData>(nusers(), config_.nfactors);
  itemFactors_ = std::make_unique<FactorData>(nitems(), config_.nfactors);
  if (config_.DistributionFile.empty()) {
    // not reproducible by design (random_device), as in the reference (WALSEngine.cpp:56-63)
    std::random_device rd;
    std::mt19937 gen(rd());
    std::uniform_real_distribution<Double> distr(-config_.initDistributionBound,
                                                 config_.initDistributionBound);
    itemFactors_->setFactors([&](auto...) { return distr(gen); });
  } else {
    itemFactors_->setFactors(config_.DistributionFile);
  }

  for (qmfx_ctx* rc : ranks_) {
    QMFX_CHECK(qmfx_set_factors(rc, QMFX_USERS, userFactors_->getFactors().data()));
    QMFX_CHECK(qmfx_set_factors(rc, QMFX_ITEMS, itemFactors_->getFactors().data()));
  }
  if (ranks_.size() > 1) {
    QMFX_CHECK(qmfx_dist_init_all(ranks_.data(), static_cast<int>(ranks_.size())));
    LOG(INFO) << "rows partitioned over " << ranks_.size() << " GPUs (devices "
              << deviceOptions_.device << ".." << deviceOptions_.device + ranks_.size() - 1
              << "), RCCL all-gather per half-epoch";
  }
  hostStale_ = false;
}

void WALSEngine::initTest(const std::vector<DatasetElem>& testDataset) {
  CHECK(testUsers_.empty()) << "engine was already initialized with test data";
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty()) {
    initAvgTestData(testUsers_, testLabels_, testScores_, testDataset, userIndex_, itemIndex_,
                    metricsEngine_->config().numTestUsers, metricsEngine_->config().seed);
  }
}

void WALSEngine::reportFailedRows(const int side) {
  int64_t count = 0;
  for (qmfx_ctx* rc : ranks_) {  // each rank flags the rows it solved
    int64_t n = 0;
    QMFX_CHECK(qmfx_wals_failed_rows(rc, nullptr, 0, &n));
    count += n;
  }
  if (count == 0) return;
  // the device re-solved them in fp64 with a pivoted factorization (dsysv_'s role,
  // Matrix.cpp:81-96) inside the half; a singular one fails qmfx_wals_half itself
  LOG(WARNING) << count << (side == QMFX_USERS ? " user" : " item")
               << " systems are not positive definite; re-solved with pivoting on the device";
  pivotedRows_ += static_cast<size_t>(count);
}

Double WALSEngine::iterate(const int side) {
  Double sum = 0.0;
  if (ranks_.size() > 1)
    QMFX_CHECK(qmfx_wals_half_multi(ranks_.data(), static_cast<int>(ranks_.size()), side,
                                    config_.confidenceWeight, config_.regularizationLambda, &sum));
  else
    QMFX_CHECK(qmfx_wals_half(dev_->get(), side, config_.confidenceWeight,
                              config_.regularizationLambda, &sum));
  reportFailedRows(side);
  hostStale_ = true;
  lastLoss_ = sum / (static_cast<Double>(nusers()) * static_cast<Double>(nitems()));
  return lastLoss_;
}

void WALSEngine::optimize() {
  CHECK(userFactors_ && itemFactors_) << "no factor data, have you initialized the engine?";
  for (size_t epoch = 1; epoch <= config_.nepochs; ++epoch) {
    iterate(QMFX_USERS);                    // item factors fixed
    const Double loss = iterate(QMFX_ITEMS);  // user factors fixed
    LOG(INFO) << "epoch " << epoch << ": train loss = " << loss;
    evaluate(epoch);
  }
  for (qmfx_ctx* rc : ranks_) QMFX_CHECK(qmfx_sync(rc));
}

void WALSEngine::syncHost() const {
  if (!hostStale_ || !dev_) return;
  QMFX_CHECK(qmfx_get_factors(dev_->get(), QMFX_USERS, userFactors_->getFactors().data()));
  QMFX_CHECK(qmfx_get_factors(dev_->get(), QMFX_ITEMS, itemFactors_->getFactors().data()));
  hostStale_ = false;
}

void WALSEngine::evaluate(const size_t epoch) {
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty() && !testUsers_.empty() &&
      (metricsEngine_->config().alwaysCompute || epoch == config_.nepochs)) {
    LOG(INFO) << "do compute evaluate ...";
    computeTestRanks(dev_->get(), false, testUsers_, testLabels_, testRanks_);
    metricsEngine_->computeAndRecordTestAvgMetrics(epoch, testRanks_, parallel_);
  }
}

const FactorData& WALSEngine::userFactors() const {
  CHECK(userFactors_) << "user factors wasn't initialized";
  syncHost();
  return *userFactors_;
}

const FactorData& WALSEngine::itemFactors() const {
  CHECK(itemFactors_) << "item factors wasn't initialized";
  syncHost();
  return *itemFactors_;
}

void WALSEngine::saveUserFactors(const std::string& fileName) const {
  saveFactors(userFactors(), userIndex_, fileName);
}

void WALSEngine::saveItemFactors(const std::string& fileName) const {
  saveFactors(itemFactors(), itemIndex_, fileName);
}

size_t WALSEngine::nusers() const { return userIndex_.size(); }
size_t WALSEngine::nitems() const { return itemIndex_.size(); }

}  // namespace qmf
