// Base class of the drop-in engines (reference: qmf/Engine.h:32-96, Engine.cpp:27-122).
// Non-copyable, non-movable; errors abort through CHECK as in the reference.
#pragma once

#include <ostream>
#include <string>
#include <vector>

#include <qmf/DatasetReader.h>
#include <qmf/FactorData.h>
#include <qmf/metrics/Metrics.h>
#include <qmf/Types.h>
#include <qmf/utils/IdIndex.h>
#include <qmf/utils/ParallelExecutor.h>
#include <qmfx.h>

namespace qmf {

class Engine {
 public:
  Engine() = default;
  virtual ~Engine() = default;
  Engine(const Engine&) = delete;
  Engine(Engine&&) = delete;
  Engine& operator=(const Engine&) = delete;
  Engine& operator=(Engine&&) = delete;

  virtual void init(const std::vector<DatasetElem>& dataset) {}
  virtual void initTest(const std::vector<DatasetElem>& testDataset) {}
  virtual void optimize() {}
  virtual void evaluate(const size_t epoch) {}
  virtual void saveUserFactors(const std::string& fileName) const {}
  virtual void saveItemFactors(const std::string& fileName) const {}

 protected:
  // test users (those with at least one known (user, item) test pair), optionally a
  // sample of numTestUsers of them shuffled with mt19937(seed), and their dense label rows
  static void initAvgTestData(std::vector<size_t>& testUsers,
                              std::vector<std::vector<Double>>& testLabels,
                              std::vector<std::vector<Double>>& testScores,
                              const std::vector<DatasetElem>& testDataset,
                              const IdIndex& userIndex,
                              const IdIndex& itemIndex,
                              const size_t numTestUsers = 0,
                              const int32_t seed = 0);

  // scores[u][i] = bias_i + <user_u, item_i> for every test user and item
  static void computeTestScores(std::vector<std::vector<Double>>& testScores,
                                const std::vector<size_t>& testUsers,
                                const FactorData& userFactors,
                                const FactorData& itemFactors,
                                ParallelExecutor& parallel);

  // Device evaluation (addition to the reference API): the same per-user metrics without the
  // dense score matrix.  The non-zero test labels go to the device once (as a CSR over the
  // test users); each call scores the context's current factors there and returns one
  // RankedUser per test user (include/qmfx.h qmfx_eval_ranks).
  void computeTestRanks(qmfx_ctx* ctx, bool useBiases, const std::vector<size_t>& testUsers,
                        const std::vector<std::vector<Double>>& testLabels,
                        std::vector<RankedUser>& ranks);

  // "<id>[ <bias>] <f0> ... <fk-1>\n" per idx, std::fixed with 9 decimals
  static void saveFactors(const FactorData& factorData, const IdIndex& index,
                          const std::string& fileName);
  static void saveFactors(const FactorData& factorData, const IdIndex& index, std::ostream& out);

  friend class EngineTestPeer;

 private:
  struct TestLabelCsr {
    std::vector<int64_t> rowptr, items;
    std::vector<Double> values;
    size_t npos = 0;
    bool uploaded = false;
  } testCsr_;
};

}  // namespace qmf
