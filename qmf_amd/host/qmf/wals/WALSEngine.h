// Implicit-feedback ALS engine, drop-in for the reference's qmf::WALSEngine
// (qmf/wals/WALSEngine.h:35-143, WALSEngine.cpp:24-355).  Same constructor, methods,
// logging and output files; the epoch loop runs on an MI355X through the qmfx C ABI
// (include/qmfx.h): both CSR orientations and both factor matrices stay resident in HBM,
// one qmfx_wals_half call per half-epoch.  The host keeps the id indexes and a mirror of
// the factors that is refreshed when something reads it (evaluation, saving).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include <qmf/Device.h>
#include <qmf/Engine.h>
#include <qmf/FactorData.h>
#include <qmf/Types.h>
#include <qmf/metrics/MetricsEngine.h>
#include <qmf/utils/IdIndex.h>
#include <qmf/utils/ParallelExecutor.h>
#include <qmf/wals/Signals.h>

namespace qmf {

struct WALSConfig {
  size_t nepochs;
  size_t nfactors;
  Double regularizationLambda;
  Double confidenceWeight;
  Double initDistributionBound;
  std::string DistributionFile;
};

class WALSEngine : public Engine {
 public:
  // `config` and `metricsEngine` are kept by reference (caller-owned), as in the reference.
  // `nthreads` sizes the host-side work (ingest, evaluation, output formatting).
  explicit WALSEngine(const WALSConfig& config,
                      const std::unique_ptr<MetricsEngine>& metricsEngine,
                      const size_t nthreads = 16,
                      const DeviceOptions& device = DeviceOptions());
  ~WALSEngine() override;

  void init(const std::vector<DatasetElem>& dataset) override;
  void initTest(const std::vector<DatasetElem>& testDataset) override;
  void optimize() override;
  void evaluate(const size_t epoch) override;

  size_t nusers() const;
  size_t nitems() const;

  void saveUserFactors(const std::string& fileName) const override;
  void saveItemFactors(const std::string& fileName) const override;

  // --- additions (not in the reference API) ---
  // host copies of the current factors (synchronised from the device on access)
  const FactorData& userFactors() const;
  const FactorData& itemFactors() const;
  const IdIndex& userIndex() const { return userIndex_; }
  const IdIndex& itemIndex() const { return itemIndex_; }
  // the loss the last half-epoch returned (Σ row losses / (nusers · nitems))
  Double lastLoss() const { return lastLoss_; }
  // rows re-solved with pivoting (on the device) because their system was not positive
  // definite
  size_t pivotedRows() const { return pivotedRows_; }
  qmfx_ctx* deviceContext() const { return dev_ ? dev_->get() : nullptr; }

 private:
  // one half-epoch: solve every row of `side` with the other side fixed; returns the
  // loss normalised as WALSEngine::iterate does (WALSEngine.cpp:215)
  Double iterate(int side);
  // logs the rows of the last half whose system was not positive definite (the device
  // re-solved them with pivoting inside the half)
  void reportFailedRows(int side);
  void syncHost() const;

  const WALSConfig& config_;
  const std::unique_ptr<MetricsEngine>& metricsEngine_;
  DeviceOptions deviceOptions_;
  mutable ParallelExecutor parallel_;
  std::unique_ptr<DeviceContext> dev_;
  // --ngpus > 1: the other ranks' contexts (dev_ is rank 0); all are passed to
  // qmfx_wals_half_multi in rank order
  std::vector<std::unique_ptr<DeviceContext>> peers_;
  std::vector<qmfx_ctx*> ranks_;

  IdIndex userIndex_;
  IdIndex itemIndex_;
  mutable std::unique_ptr<FactorData> userFactors_;
  mutable std::unique_ptr<FactorData> itemFactors_;
  mutable bool hostStale_ = false;

  std::vector<size_t> testUsers_;
  std::vector<std::vector<Double>> testLabels_;
  std::vector<std::vector<Double>> testScores_;
  std::vector<RankedUser> testRanks_;

  Double lastLoss_ = 0.0;
  size_t pivotedRows_ = 0;
};

}  // namespace qmf
