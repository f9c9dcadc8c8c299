#include <qmf/bpr/BPREngine.h>

#include <algorithm>

#include <qmf/utils/Log.h>

namespace qmf {

BPREngine::BPREngine(const BPRConfig& config,
                     const std::unique_ptr<MetricsEngine>& metricsEngine,
                     const size_t evalNumNeg,
                     const int32_t evalSeed,
                     const size_t nthreads,
                     const DeviceOptions& device)
    : config_(config), metricsEngine_(metricsEngine), evalNumNeg_(evalNumNeg),
      evalSeed_(evalSeed), deviceOptions_(device), parallel_(nthreads),
      gen_(std::random_device()()) {
  if (config_.numHogwildThreads > nthreads) {
    LOG(WARNING) << "number of hogwild threads should be smaller than number of "
                    "threads in the threadpool";
  }
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty() &&
      metricsEngine_->config().numTestUsers == 0) {
    LOG(WARNING) << "computing average test metrics on all users can be slow! "
                    "Set numTestUsers > 0 to sample some of them";
  }
}

BPREngine::~BPREngine() = default;

size_t BPREngine::nusers() const { return userIndex_.size(); }
size_t BPREngine::nitems() const { return itemIndex_.size(); }

BPREngine::PositiveSets BPREngine::buildSets(const std::vector<std::pair<size_t, size_t>>& pairs,
                                             const size_t nusers) {
  PositiveSets s;
  s.rowptr.assign(nusers + 1, 0);
  for (const auto& p : pairs) ++s.rowptr[p.first + 1];
  for (size_t u = 0; u < nusers; ++u) s.rowptr[u + 1] += s.rowptr[u];
  std::vector<int64_t> fill(s.rowptr.begin(), s.rowptr.end() - 1);
  s.items.resize(pairs.size());
  for (const auto& p : pairs) s.items[fill[p.first]++] = p.second;
  // sort + dedupe each row, then compact
  int64_t w = 0;
  for (size_t u = 0; u < nusers; ++u) {
    const int64_t b = s.rowptr[u], e = s.rowptr[u + 1];
    std::sort(s.items.begin() + b, s.items.begin() + e);
    const int64_t n = std::unique(s.items.begin() + b, s.items.begin() + e) - (s.items.begin() + b);
    std::move(s.items.begin() + b, s.items.begin() + b + n, s.items.begin() + w);
    s.rowptr[u] = w;
    w += n;
  }
  s.rowptr[nusers] = w;
  s.items.resize(static_cast<size_t>(w));
  return s;
}

bool BPREngine::PositiveSets::contains(const size_t u, const size_t i) const {
  return std::binary_search(items.begin() + rowptr[u], items.begin() + rowptr[u + 1], i);
}

size_t BPREngine::sampleRandomNegative(const size_t userIdx, std::mt19937& gen,
                                       const PositiveSets& sets) const {
  // the reference would spin forever here; abort instead
  CHECK_LT(sets.count(userIdx), nitems()) << "user idx " << userIdx
                                          << " has every item as a positive";
  std::uniform_int_distribution<> dis(0, static_cast<int>(nitems()) - 1);
  size_t neg;
  do {
    neg = dis(gen);
  } while (sets.contains(userIdx, neg));
  return neg;
}

void BPREngine::init(const std::vector<DatasetElem>& dataset) {
  initHost(dataset);
  initDevice();
}

void BPREngine::initHost(const std::vector<DatasetElem>& dataset) {
  CHECK(!userFactors_ && !itemFactors_) << "engine was already initialized with train data";
  for (const auto& e : dataset) {
    if (e.value < 1.0) continue;
    const size_t u = userIndex_.getOrSetIdx(e.userId);
    const size_t i = itemIndex_.getOrSetIdx(e.itemId);
    data_.emplace_back(u, i);
  }
  itemMap_ = buildSets(data_, nusers());

  // evaluation set: every positive × evalNumNeg negatives, mt19937(evalSeed)
  {
    std::mt19937 gen(evalSeed_);
    evalSet_.reserve(data_.size() * evalNumNeg_);
    for (const auto& p : data_)
      for (size_t j = 0; j < evalNumNeg_; ++j)
        evalSet_.push_back(PosNegTriplet{p.first, p.second,
                                         sampleRandomNegative(p.first, gen, itemMap_)});
  }

  learningRate_ = config_.initLearningRate;
  userFactors_ = std::make_unique<FactorData>(nusers(), config_.nfactors);
  itemFactors_ = std::make_unique<FactorData>(nitems(), config_.nfactors, config_.useBiases);
  std::uniform_real_distribution<Double> distr(-config_.initDistributionBound,
                                               config_.initDistributionBound);
  auto unif = [&](auto...) { return distr(gen_); };
  userFactors_->setFactors(unif);
  itemFactors_->setFactors(unif);
  if (config_.useBiases) itemFactors_->setBiases(unif);
}

void BPREngine::initDevice() {
  // Hogwild across GPUs would need cross-device atomics: BPR runs on one GPU (replicas only)
  CHECK_EQ(deviceOptions_.ngpus, 1) << "BPR runs on one GPU (QMF_NGPUS / --ngpus is WALS only)";
  dev_ = std::make_unique<DeviceContext>(deviceOptions_, config_.nfactors);
  qmfx_ctx* c = dev_->get();
  QMFX_CHECK(qmfx_set_shape(c, static_cast<int64_t>(nusers()), static_cast<int64_t>(nitems())));
  std::vector<int64_t> pu(data_.size()), pi(data_.size());
  for (size_t e = 0; e < data_.size(); ++e) {
    pu[e] = static_cast<int64_t>(data_[e].first);
    pi[e] = static_cast<int64_t>(data_[e].second);
  }
  QMFX_CHECK(qmfx_bpr_set_positives(c, pu.data(), pi.data(), static_cast<int64_t>(pu.size())));
  QMFX_CHECK(qmfx_set_factors(c, QMFX_USERS, userFactors_->getFactors().data()));
  QMFX_CHECK(qmfx_set_factors(c, QMFX_ITEMS, itemFactors_->getFactors().data()));
  std::vector<Double> zeros;
  const Double* bias = itemFactors_->getBiases().data();
  if (!config_.useBiases) {
    zeros.assign(nitems(), 0.0);
    bias = zeros.data();
  }
  QMFX_CHECK(qmfx_bpr_set_biases(c, bias));
  hostStale_ = false;
}

void BPREngine::initTest(const std::vector<DatasetElem>& testDataset) {
  CHECK(testEvalSet_.empty()) << "engine was already initialzied with test data";
  std::vector<std::pair<size_t, size_t>> valid;
  valid.reserve(testDataset.size());
  for (const auto& e : testDataset) {
    if (e.value < 1.0) continue;
    const size_t u = userIndex_.idx(e.userId);
    const size_t i = itemIndex_.idx(e.itemId);
    if (u == IdIndex::missingIdx || i == IdIndex::missingIdx) continue;
    valid.emplace_back(u, i);
  }
  testItemMap_ = buildSets(valid, nusers());
  std::mt19937 gen(evalSeed_);
  testEvalSet_.reserve(evalNumNeg_ * valid.size());
  for (const auto& p : valid)
    for (size_t j = 0; j < evalNumNeg_; ++j)
      testEvalSet_.push_back(PosNegTriplet{p.first, p.second,
                                           sampleRandomNegative(p.first, gen, testItemMap_)});
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty()) {
    initAvgTestData(testUsers_, testLabels_, testScores_, testDataset, userIndex_, itemIndex_,
                    metricsEngine_->config().numTestUsers, metricsEngine_->config().seed);
  }
}

void BPREngine::optimize() {
  CHECK(userFactors_ && itemFactors_) << "no factor data, have you initialized the engine?";
  for (size_t epoch = 1; epoch <= config_.nepochs; ++epoch) {
    // the reference visits positives in file order in epoch 1 and shuffles after each
    // epoch; the device kernel visits them in a seeded permutation from epoch 2 on
    const uint64_t seed = (static_cast<uint64_t>(gen_()) << 32) | gen_();
    const int shuffle = config_.shuffleTrainingSet && epoch > 1 ? 1 : 0;
    QMFX_CHECK(qmfx_bpr_epoch(dev_->get(), seed, static_cast<int>(config_.numNegativeSamples),
                              learningRate_, config_.biasLambda, config_.userLambda,
                              config_.itemLambda, config_.useBiases ? 1 : 0, shuffle));
    hostStale_ = true;
    evaluate(epoch);
    if (config_.decayRate < 1.0) learningRate_ *= config_.decayRate;
  }
  QMFX_CHECK(qmfx_sync(dev_->get()));
}

Double BPREngine::evalLoss(const int slot, const std::vector<PosNegTriplet>& set) const {
  if (set.empty()) return -1.0;
  Double sum = 0.0;
  QMFX_CHECK(qmfx_bpr_eval(dev_->get(), slot, reinterpret_cast<const int64_t*>(set.data()),
                           static_cast<int64_t>(set.size()), config_.useBiases ? 1 : 0, &sum));
  return sum / set.size();
}

void BPREngine::evaluate(const size_t epoch) {
  // mean log(1 + exp(−x̂)) over the fixed evaluation triplets (BPREngine.cpp:246-264)
  lastTrainLoss_ = evalLoss(0, evalSet_);
  lastTestLoss_ = evalLoss(1, testEvalSet_);
  LOG(INFO) << "epoch " << epoch << ": train loss = " << lastTrainLoss_
            << ", test loss = " << lastTestLoss_;
  if (metricsEngine_ && !metricsEngine_->testAvgMetrics().empty() && !testUsers_.empty() &&
      (metricsEngine_->config().alwaysCompute || epoch == config_.nepochs)) {
    computeTestRanks(dev_->get(), itemFactors_->withBiases(), testUsers_, testLabels_, testRanks_);
    metricsEngine_->computeAndRecordTestAvgMetrics(epoch, testRanks_, parallel_);
  }
}

void BPREngine::syncHost() const {
  if (!hostStale_ || !dev_) return;
  QMFX_CHECK(qmfx_get_factors(dev_->get(), QMFX_USERS, userFactors_->getFactors().data()));
  QMFX_CHECK(qmfx_get_factors(dev_->get(), QMFX_ITEMS, itemFactors_->getFactors().data()));
  if (config_.useBiases)
    QMFX_CHECK(qmfx_bpr_get_biases(dev_->get(), itemFactors_->getBiases().data()));
  hostStale_ = false;
}

const FactorData& BPREngine::userFactors() const {
  CHECK(userFactors_) << "user factors wasn't initialized";
  syncHost();
  return *userFactors_;
}

const FactorData& BPREngine::itemFactors() const {
  CHECK(itemFactors_) << "item factors wasn't initialized";
  syncHost();
  return *itemFactors_;
}

void BPREngine::saveUserFactors(const std::string& fileName) const {
  saveFactors(userFactors(), userIndex_, fileName);
}

void BPREngine::saveItemFactors(const std::string& fileName) const {
  saveFactors(itemFactors(), itemIndex_, fileName);
}

}  // namespace qmf
