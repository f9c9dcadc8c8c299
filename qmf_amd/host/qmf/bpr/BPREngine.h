// Bayesian Personalised Ranking engine, drop-in for the reference's qmf::BPREngine
// (qmf/bpr/BPREngine.h:38-162, BPREngine.cpp:24-278, BPREngine-inl.h:23-60).
//
// Host side (bit-identical to the reference): positives (value ≥ 1) in file order with
// first-appearance idx, the evaluation triplets drawn with mt19937(evalSeed) and
// uniform_int_distribution<int>(0, nitems−1) with rejection against the user's positives,
// factor init from a random_device-seeded mt19937 in the reference's order, lr decay.
// Device side: each epoch is one Hogwild kernel over all positives × numNegativeSamples
// (qmfx_bpr_epoch), the per-epoch evaluation losses are a device reduction (qmfx_bpr_eval).
#pragma once

#include <memory>
#include <random>
#include <string>
#include <vector>

#include <qmf/Device.h>
#include <qmf/Engine.h>
#include <qmf/FactorData.h>
#include <qmf/Types.h>
#include <qmf/metrics/MetricsEngine.h>
#include <qmf/utils/IdIndex.h>
#include <qmf/utils/ParallelExecutor.h>

namespace qmf {

struct BPRConfig {
  size_t nepochs;
  size_t nfactors;
  Double initLearningRate;
  Double biasLambda;
  Double userLambda;
  Double itemLambda;
  Double decayRate;
  bool useBiases;
  Double initDistributionBound;
  size_t numNegativeSamples;
  size_t numHogwildThreads;  // accepted for compatibility; the device runs every positive in parallel
  bool shuffleTrainingSet;
};

class BPREngine : public Engine {
 public:
  explicit BPREngine(const BPRConfig& config,
                     const std::unique_ptr<MetricsEngine>& metricsEngine,
                     const size_t evalNumNeg = 3,
                     const int32_t evalSeed = 42,
                     const size_t nthreads = 16,
                     const DeviceOptions& device = DeviceOptions());
  ~BPREngine() override;

  void init(const std::vector<DatasetElem>& dataset) override;
  void initTest(const std::vector<DatasetElem>& testDataset) override;
  void optimize() override;
  void evaluate(const size_t epoch) override;

  size_t nusers() const;
  size_t nitems() const;

  void saveUserFactors(const std::string& fileName) const override;
  void saveItemFactors(const std::string& fileName) const override;

  // --- additions (not in the reference API) ---
  struct PosNegTriplet {
    size_t userIdx;
    size_t posItemIdx;
    size_t negItemIdx;
  };
  const std::vector<PosNegTriplet>& evalSet() const { return evalSet_; }
  const std::vector<PosNegTriplet>& testEvalSet() const { return testEvalSet_; }
  const FactorData& userFactors() const;
  const FactorData& itemFactors() const;
  const IdIndex& userIndex() const { return userIndex_; }
  const IdIndex& itemIndex() const { return itemIndex_; }
  // mean eval losses of the last evaluate() (−1 when the set is empty)
  Double lastTrainLoss() const { return lastTrainLoss_; }
  Double lastTestLoss() const { return lastTestLoss_; }
  Double learningRate() const { return learningRate_; }
  // Overrides the seed of the factor initialisation and of the per-epoch device sampling
  // (the reference seeds it from std::random_device).  Call before init().
  void seed(uint32_t s) { gen_.seed(s); }

 private:
  // per-user sorted distinct positive items: membership test for negative sampling
  struct PositiveSets {
    std::vector<int64_t> rowptr;
    std::vector<size_t> items;
    bool contains(size_t u, size_t i) const;
    size_t count(size_t u) const { return static_cast<size_t>(rowptr[u + 1] - rowptr[u]); }
  };
  // host bookkeeping of init() (indexes, positives, evaluation set, factor init), then the
  // device upload
  void initHost(const std::vector<DatasetElem>& dataset);
  void initDevice();
  static PositiveSets buildSets(const std::vector<std::pair<size_t, size_t>>& pairs,
                                size_t nusers);
  // BPREngine-inl.h:48-60 (same distribution object and call sequence)
  size_t sampleRandomNegative(size_t userIdx, std::mt19937& gen, const PositiveSets& sets) const;
  void syncHost() const;
  Double evalLoss(int slot, const std::vector<PosNegTriplet>& set) const;

  const BPRConfig& config_;
  const std::unique_ptr<MetricsEngine>& metricsEngine_;
  const size_t evalNumNeg_;
  const int32_t evalSeed_;
  DeviceOptions deviceOptions_;
  mutable ParallelExecutor parallel_;
  std::mt19937 gen_;
  Double learningRate_ = 0.0;
  std::unique_ptr<DeviceContext> dev_;

  std::vector<std::pair<size_t, size_t>> data_;  // (userIdx, posItemIdx) in file order
  std::vector<PosNegTriplet> evalSet_;
  std::vector<PosNegTriplet> testEvalSet_;
  PositiveSets itemMap_;
  PositiveSets testItemMap_;

  IdIndex userIndex_;
  IdIndex itemIndex_;
  mutable std::unique_ptr<FactorData> userFactors_;
  mutable std::unique_ptr<FactorData> itemFactors_;
  mutable bool hostStale_ = false;

  std::vector<size_t> testUsers_;
  std::vector<std::vector<Double>> testLabels_;
  std::vector<std::vector<Double>> testScores_;
  std::vector<RankedUser> testRanks_;

  Double lastTrainLoss_ = -1.0;
  Double lastTestLoss_ = -1.0;

  friend class BPREngineTestPeer;
};

static_assert(sizeof(BPREngine::PosNegTriplet) == 3 * sizeof(int64_t),
              "triplets cross the C ABI as int64[3]");

}  // namespace qmf
