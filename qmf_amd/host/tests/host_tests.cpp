// CPU tests of the drop-in host library: the reference's own unit tests re-expressed
// (qmf/test/*.cpp, cited per case) plus equivalence checks for the parallel paths.
// No GPU is touched: engines are exercised through their host-side bookkeeping only.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <random>
#include <sstream>

#include <qmf/DatasetReader.h>
#include <qmf/Engine.h>
#include <qmf/FactorData.h>
#include <qmf/Matrix.h>
#include <qmf/bpr/BPREngine.h>
#include <qmf/metrics/Metrics.h>
#include <qmf/metrics/MetricsEngine.h>
#include <qmf/metrics/MetricsManager.h>
#include <qmf/utils/Flags.h>
#include <qmf/utils/IdIndex.h>
#include <qmf/utils/ParallelExecutor.h>
#include <qmf/utils/Util.h>
#include <qmf/wals/Signals.h>

#include "testing.h"

namespace qmf {

class EngineTestPeer : public Engine {
 public:
  using Engine::computeTestScores;
  using Engine::initAvgTestData;
  using Engine::saveFactors;
};

class BPREngineTestPeer {
 public:
  static void initHost(BPREngine& e, const std::vector<DatasetElem>& d) { e.initHost(d); }
  static const BPREngine::PositiveSets& itemMap(const BPREngine& e) { return e.itemMap_; }
  static const BPREngine::PositiveSets& testItemMap(const BPREngine& e) { return e.testItemMap_; }
  static const FactorData& U(const BPREngine& e) { return *e.userFactors_; }
  static const FactorData& I(const BPREngine& e) { return *e.itemFactors_; }
  static size_t ndata(const BPREngine& e) { return e.data_.size(); }
};

}  // namespace qmf

using namespace qmf;

static std::string tmpPath(const char* tag) {
  return std::string("/tmp/qmf_host_test_") + std::to_string(getpid()) + "_" + tag;
}

// ---- utils (UtilTest.cpp:23-32, ParallelExecutorTest.cpp) ---------------------------------
TEST(Util, split) {
  using vec = std::vector<std::string>;
  EXPECT_TRUE(split("", ',') == vec({}));
  EXPECT_TRUE(split("hello", ',') == vec({"hello"}));
  EXPECT_TRUE(split("hello,world", ',') == vec({"hello", "world"}));
  EXPECT_TRUE(split("hello,world,!", ',') == vec({"hello", "world", "!"}));
  EXPECT_TRUE(split("hello world !", ' ') == vec({"hello", "world", "!"}));
  EXPECT_TRUE(split("a,", ',') == vec({"a", ""}));
}

TEST(ParallelExecutor, executeAndMapReduce) {
  for (size_t nt : {1, 2, 3, 8, 17}) {
    ParallelExecutor px(nt);
    std::vector<int> hit(1000, 0);
    px.execute(hit.size(), [&](size_t t) { hit[t] += 1; });
    bool all = true;
    for (int h : hit) all = all && h == 1;
    EXPECT_TRUE(all);
    const long s = px.mapReduce(1001, [](size_t t) { return (long)t; }, std::plus<long>(), 0L);
    EXPECT_EQ(s, 1000L * 1001 / 2);
    std::vector<long> v(37);
    for (size_t i = 0; i < v.size(); ++i) v[i] = (long)i;
    // unlike the reference's block split, no tail element is dropped
    EXPECT_EQ(px.mapReduce(v, [](long x) { return x; }, std::plus<long>(), 0L), 36L * 37 / 2);
  }
}

TEST(IdIndex, basics) {
  IdIndex ix;
  EXPECT_EQ(ix.getOrSetIdx(7), 0u);
  EXPECT_EQ(ix.getOrSetIdx(-3), 1u);
  EXPECT_EQ(ix.getOrSetIdx(7), 0u);
  EXPECT_EQ(ix.size(), 2u);
  EXPECT_EQ(ix.id(1), -3);
  EXPECT_EQ(ix.idx(99), IdIndex::missingIdx);
  ix.assignSorted({-5, 2, 9});
  EXPECT_EQ(ix.idx(9), 2u);
  EXPECT_EQ(ix.idx(7), IdIndex::missingIdx);
}

TEST(Flags, gflagsSyntax) {
  EXPECT_EQ(flags::set("no_such_flag", "1").empty(), false);
}

// ---- FactorData (FactorDataTest.cpp:23-62) -------------------------------------------------
TEST(FactorData, withBiases) {
  FactorData fd(3, 2, true);
  EXPECT_EQ(fd.nelems(), 3u);
  EXPECT_EQ(fd.nfactors(), 2u);
  fd.at(0, 0) = 1.5;
  fd.at(2, 1) = 3.0;
  fd.biasAt(2) = -0.5;
  EXPECT_DOUBLE_EQ(fd.at(0, 0), 1.5);
  EXPECT_DOUBLE_EQ(fd.at(2, 1), 3.0);
  EXPECT_DOUBLE_EQ(fd.biasAt(2), -0.5);
  fd.setFactors([](size_t i, size_t f) { return 2.0 * i + f; });
  fd.setBiases([](size_t i) { return 42.0 + i; });
  for (size_t i = 0; i < 3; ++i) {
    EXPECT_DOUBLE_EQ(fd.biasAt(i), 42.0 + i);
    for (size_t f = 0; f < 2; ++f) EXPECT_DOUBLE_EQ(fd.at(i, f), 2.0 * i + f);
  }
}

TEST(FactorData, noBiases) {
  FactorData fd(3, 2, false);
  EXPECT_FALSE(fd.withBiases());
  const FactorData& cfd = fd;
  EXPECT_DOUBLE_EQ(cfd.biasAt(1), 0.0);
  EXPECT_DEATH(fd.biasAt(0) = 1.0);
}

TEST(FactorData, distributionFile) {
  // FactorData.h:74-100: row-major "%lf" lines; a short file leaves the rest untouched
  const std::string p = tmpPath("dist");
  {
    std::ofstream f(p);
    for (int i = 0; i < 5; ++i) f << (0.001 * (i + 1)) << "\n";
  }
  FactorData fd(3, 2);
  fd.setFactors([](size_t, size_t) { return 7.0; });
  fd.setFactors(p);
  EXPECT_DOUBLE_EQ(fd.at(0, 0), 0.001);
  EXPECT_DOUBLE_EQ(fd.at(0, 1), 0.002);
  EXPECT_DOUBLE_EQ(fd.at(2, 0), 0.005);
  EXPECT_DOUBLE_EQ(fd.at(2, 1), 7.0);
  {
    std::ofstream f(p);
    f << "0.5\nabc\n";
  }
  EXPECT_DEATH(fd.setFactors(p));
  std::remove(p.c_str());
}

// ---- Matrix (MatrixTest.cpp:23-116) ---------------------------------------------------------
TEST(Matrix, transposeAndAdd) {
  Matrix X(3, 2);
  for (size_t i = 0; i < 3; ++i)
    for (size_t j = 0; j < 2; ++j) X(i, j) = 10.0 * i + j;
  const Matrix T = X.transpose();
  EXPECT_EQ(T.nrows(), 2u);
  EXPECT_DOUBLE_EQ(T(1, 2), 21.0);
  const Matrix S = X + X;
  EXPECT_DOUBLE_EQ(S(2, 1), 42.0);
  EXPECT_DEATH(Matrix(0, 3));
}

TEST(Matrix, linearSolve) {
  // symmetric indefinite A with entries U(−1, 1): residual within 1e-8 (MatrixTest.cpp:92-116)
  const size_t n = 50;
  std::mt19937 gen(123);
  std::uniform_real_distribution<Double> distr(-1.0, 1.0);
  Matrix A(n, n);
  Vector b(n);
  for (size_t i = 0; i < n; ++i) {
    b(i) = distr(gen);
    for (size_t j = i; j < n; ++j) A(i, j) = A(j, i) = distr(gen);
  }
  const Vector x = linearSymmetricSolve(A, b);
  EXPECT_EQ(x.size(), n);
  for (size_t i = 0; i < n; ++i) {
    Double prod = 0.0;
    for (size_t j = 0; j < n; ++j) prod += A(i, j) * x(j);
    EXPECT_NEAR(b(i), prod, 1e-8);
  }
  Matrix Z(2, 2);
  EXPECT_DEATH(linearSymmetricSolve(Z, Vector(2)));
}

// ---- DatasetReader (DatasetReaderTest.cpp:23-58) -------------------------------------------
TEST(DatasetReader, readOne) {
  DatasetReader r(std::make_unique<std::istringstream>("1 2 3"));
  DatasetElem e;
  EXPECT_TRUE(r.readOne(e));
  EXPECT_EQ(e.userId, 1);
  EXPECT_EQ(e.itemId, 2);
  EXPECT_DOUBLE_EQ(e.value, 3.0);
  EXPECT_FALSE(r.readOne(e));
}

TEST(DatasetReader, readOneBadFormat) {
  DatasetReader r(std::make_unique<std::istringstream>("1 3"));
  DatasetElem e;
  EXPECT_DEATH(r.readOne(e));
}

TEST(DatasetReader, readAll) {
  std::string s;
  for (int i = 0; i < 5; ++i) s += "1 2 3\n";
  DatasetReader r(std::make_unique<std::istringstream>(s));
  const auto d = r.readAll();
  EXPECT_EQ(d.size(), 5u);
  for (const auto& e : d) EXPECT_TRUE(e.userId == 1 && e.itemId == 2 && e.value == 3.0);
}

TEST(DatasetReader, parallelFileParseEqualsSequential) {
  // > 1 MiB so several threads parse; odd whitespace, signs, exponents, CRLF, no final '\n'
  std::mt19937_64 g(5);
  std::string text;
  const char* sep[] = {" ", "\t", "  ", " \t "};
  while (text.size() < (5u << 20)) {
    const long long u = (long long)(g() % 2000000) - 1000000;
    const long long i = (long long)(g() >> 1);
    char vb[64];
    // (kinds 4-9: the forms the in-place parser hands to the strtod path — hex, inf / nan,
    // out of range, subnormal, trailing garbage — and a fraction strtoll stops at)
    const int kind = (int)(g() % 10);
    if (kind == 0) std::snprintf(vb, sizeof vb, "%d", (int)(g() % 6));
    if (kind == 1) std::snprintf(vb, sizeof vb, "%.17g", (double)(g() % 100000) / 7.0);
    if (kind == 2) std::snprintf(vb, sizeof vb, "%.3e", -(double)(g() % 1000));
    if (kind == 3) std::snprintf(vb, sizeof vb, "+%u.5", (unsigned)(g() % 9));
    if (kind == 4) std::snprintf(vb, sizeof vb, "0x1.8p%d", (int)(g() % 8));
    if (kind == 5) std::snprintf(vb, sizeof vb, "%s", (g() & 1) ? "inf" : "-nan");
    if (kind == 6) std::snprintf(vb, sizeof vb, "1e%d", 300 + (int)(g() % 20));
    if (kind == 7) std::snprintf(vb, sizeof vb, "%.3e", 1e-300 * (double)(g() % 1000) * 1e-10);
    if (kind == 8) std::snprintf(vb, sizeof vb, "%u.25abc,x", (unsigned)(g() % 9));
    if (kind == 9) std::snprintf(vb, sizeof vb, ".%u", (unsigned)(g() % 100));
    // (the item field occasionally carries a fraction: "%lld" stops at the '.', and "%lf"
    // then reads the fraction as the value — the value field is dropped by the scan)
    const bool frac = g() % 16 == 0;
    text += (g() % 3 == 0 ? " " : "") + std::to_string(u) + sep[g() % 4] + std::to_string(i) +
            (frac ? std::string(".75") : std::string("")) + sep[g() % 4] + vb +
            (g() % 5 == 0 ? "\r\n" : "\n");
  }
  text += "42 43 44";  // last line without newline
  const std::string p = tmpPath("ds");
  {
    std::ofstream f(p, std::ios::binary);
    f << text;
  }
  std::vector<DatasetElem> seq;
  {
    DatasetReader r(std::make_unique<std::istringstream>(text));
    DatasetElem e;
    while (r.readOne(e)) seq.push_back(e);
  }
  const auto par = DatasetReader(p).readAll();
  EXPECT_EQ(par.size(), seq.size());
  bool same = par.size() == seq.size();
  for (size_t k = 0; same && k < seq.size(); ++k)
    same = par[k].userId == seq[k].userId && par[k].itemId == seq[k].itemId &&
           std::memcmp(&par[k].value, &seq[k].value, 8) == 0;
  EXPECT_TRUE(same);
  // an empty line in the middle aborts, like sscanf's result != 3
  {
    std::ofstream f(p, std::ios::binary);
    f << "1 2 3\n\n4 5 6\n";
  }
  EXPECT_DEATH(DatasetReader(p).readAll());
  std::remove(p.c_str());
  // a missing file reads as empty (the reference's ifstream just fails)
  EXPECT_EQ(DatasetReader(tmpPath("missing")).readAll().size(), 0u);
}

// ---- metrics (MetricsTest.cpp:23-87, MetricsManagerTest.cpp:23-44) -----------------------
// The statistics qmfx_eval_ranks reduces on the device, formed here by brute force
static RankedUser rankedOf(const std::vector<Double>& l, const std::vector<Double>& s) {
  RankedUser r;
  r.nitems = l.size();
  std::vector<Double> ps;
  std::vector<int64_t> ab;
  for (size_t i = 0; i < l.size(); ++i) {
    r.sse += (l[i] - s[i]) * (l[i] - s[i]);
    if (l[i] > 0.0) {
      ps.push_back(s[i]);
      ab.push_back(std::count_if(s.begin(), s.end(), [&](Double x) { return x > s[i]; }));
    }
  }
  r.setPositives(ps, ab);
  return r;
}

// dense (reference) value; the ranked path must agree
static Double one(const Metric& m, std::vector<Double> l, std::vector<Double> s) {
  const Double dense = m.compute(l, s);
  EXPECT_NEAR(m.compute(rankedOf(l, s)), dense, 1e-12 * std::fabs(dense) + 1e-15);
  return dense;
}

TEST(Metrics, knownAnswers) {
  MeanSquaredError mse;
  EXPECT_DOUBLE_EQ(one(mse, {1.0, 0.0}, {0.5, 0.5}), 0.25);
  EXPECT_DOUBLE_EQ(one(mse, {1.0, 0.0, 1.0}, {0.0, 1.0, 2.0}), 1.0);
  std::vector<std::vector<Double>> L = {{1.0, 0.0}, {1.0, 0.0, 1.0}};
  std::vector<std::vector<Double>> S = {{0.5, 0.5}, {0.0, 1.0, 2.0}};
  EXPECT_DOUBLE_EQ(mse.compute(L, S), 0.5 * (0.25 + 1.0));
  ParallelExecutor px(3);
  EXPECT_DOUBLE_EQ(mse.compute(L, S, px), 0.5 * (0.25 + 1.0));
  AUC auc;
  EXPECT_DOUBLE_EQ(one(auc, {1.0, 0.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(auc, {0.0, 1.0}, {3.0, 2.0}), 0.0);
  EXPECT_DOUBLE_EQ(one(auc, {1.0, 1.0, 0.0}, {3.0, 2.0, 0.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(auc, {1.0, 0.0, 1.0}, {3.0, 2.0, 0.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(auc, {0.0, 1.0, 1.0}, {3.0, 2.0, 0.0}), 0.0);
  Precision p1(1), p2(2);
  EXPECT_DOUBLE_EQ(one(p1, {1.0, 0.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(p1, {1.0, 1.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(p1, {0.0, 1.0}, {3.0, 2.0}), 0.0);
  EXPECT_DOUBLE_EQ(one(p2, {1.0, 0.0}, {3.0, 2.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(p2, {1.0, 1.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(p2, {0.0, 1.0}, {3.0, 2.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(p2, {0.0, 1.0, 0.0}, {3.0, 2.0, 1.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(p2, {0.0, 1.0, 0.0}, {3.0, 1.0, 2.0}), 0.0);
  Recall r1(1), r2(2);
  EXPECT_DOUBLE_EQ(one(r1, {1.0, 0.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(r1, {1.0, 1.0}, {3.0, 2.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(r1, {0.0, 1.0}, {3.0, 2.0}), 0.0);
  EXPECT_DOUBLE_EQ(one(r2, {1.0, 0.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(r2, {1.0, 1.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(r2, {0.0, 1.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(r2, {0.0, 1.0, 0.0}, {3.0, 2.0, 1.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(r2, {0.0, 1.0, 0.0}, {3.0, 1.0, 2.0}), 0.0);
  AveragePrecision ap;
  EXPECT_DOUBLE_EQ(one(ap, {1.0, 0.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(ap, {1.0, 1.0}, {3.0, 2.0}), 1.0);
  EXPECT_DOUBLE_EQ(one(ap, {0.0, 1.0}, {3.0, 2.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(ap, {0.0, 1.0, 0.0}, {3.0, 2.0, 1.0}), 0.5);
  EXPECT_DOUBLE_EQ(one(ap, {0.0, 1.0, 0.0}, {3.0, 1.0, 2.0}), 1.0 / 3);
  EXPECT_DEATH(one(ap, {0.0, 0.0}, {1.0, 2.0}));
  EXPECT_DEATH(one(p2, {1.0}, {1.0}));
}

// Ranked (device-statistics) metrics equal the dense ones, ties and negative labels included
TEST(Metrics, rankedEqualsDense) {
  std::mt19937 gen(7);
  MeanSquaredError mse;
  AUC auc;
  AveragePrecision ap;
  const Double labelSet[] = {-1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 2.0};
  for (int trial = 0; trial < 400; ++trial) {
    const size_t n = 1 + gen() % 60;
    std::vector<Double> l(n), s(n);
    for (size_t i = 0; i < n; ++i) {
      l[i] = labelSet[gen() % 7];
      s[i] = trial % 2 ? static_cast<Double>(gen() % 5) : std::ldexp(gen() % 100000, -7);
    }
    const bool anyPos = std::any_of(l.begin(), l.end(), [](Double x) { return x > 0.0; });
    one(mse, l, s);
    if (anyPos && std::any_of(l.begin(), l.end(), [](Double x) { return x <= 0.0; }))
      one(auc, l, s);
    if (anyPos) one(ap, l, s);
    for (size_t k : {1, 2, 5, 10}) {
      if (n < k) continue;
      one(Precision(k), l, s);
      if (anyPos) one(Recall(k), l, s);
    }
  }
  // mean over users through the executor
  std::vector<RankedUser> users = {rankedOf({1.0, 0.0}, {0.5, 0.5}),
                                   rankedOf({1.0, 0.0, 1.0}, {0.0, 1.0, 2.0})};
  ParallelExecutor px(2);
  EXPECT_DOUBLE_EQ(mse.compute(users, px), 0.5 * (0.25 + 1.0));
  EXPECT_DEATH(ap.compute(rankedOf({0.0, 0.0}, {1.0, 2.0})));
  EXPECT_DEATH(Precision(2).compute(rankedOf({1.0}, {1.0})));
}

TEST(MetricsManager, parseAndExists) {
  std::string name;
  size_t k = 0;
  EXPECT_TRUE(detail::parseAtKMetric("p@5", name, k));
  EXPECT_TRUE(name == "p" && k == 5);
  EXPECT_FALSE(detail::parseAtKMetric("p5", name, k));
  EXPECT_FALSE(detail::parseAtKMetric("@5", name, k));
  EXPECT_FALSE(detail::parseAtKMetric("p@", name, k));
  const auto& m = MetricsManager::get();
  for (const char* n : {"mse", "auc", "ap", "p@5", "p@10", "r@5", "r@10"}) EXPECT_TRUE(m.exists(n));
  EXPECT_FALSE(m.exists("q@5"));
  EXPECT_FALSE(m.exists("ndcg"));
  EXPECT_TRUE(m.getMetric("nope") == nullptr);
  MetricsConfig mc{0, false, 42};
  MetricsEngine me(mc, false);
  EXPECT_TRUE(me.addTestAvgMetric("auc"));
  EXPECT_FALSE(me.addTestAvgMetric("bogus"));
  std::vector<std::vector<Double>> L = {{1.0, 0.0}}, S = {{3.0, 2.0}};
  ParallelExecutor px(2);
  me.computeAndRecordTestAvgMetrics(3, L, S, px);
  EXPECT_DOUBLE_EQ(me.recorded().at("test_avg_auc").at(0).second, 1.0);
}

// ---- Engine (EngineTest.cpp:27-139) ---------------------------------------------------------
TEST(Engine, initAvgTestData) {
  IdIndex ui, ii;
  for (int64_t id : {1, 2, 3}) ui.getOrSetIdx(id);
  for (int64_t id : {1, 2, 4, 3}) ii.getOrSetIdx(id);
  std::vector<DatasetElem> test = {{1, 4}, {2, 1}, {4, 2}, {1, 5}};
  std::vector<size_t> users;
  std::vector<std::vector<Double>> labels, scores;
  EngineTestPeer::initAvgTestData(users, labels, scores, test, ui, ii);
  EXPECT_EQ(users.size(), 2u);
  EXPECT_EQ(labels.size(), 2u);
  EXPECT_EQ(scores.size(), 2u);
  for (size_t t = 0; t < users.size(); ++t) {
    EXPECT_EQ(labels[t].size(), ii.size());
    const int64_t want = ui.id(users[t]) == 1 ? 4 : 1;  // user 1 -> item 4, user 2 -> item 1
    for (size_t i = 0; i < ii.size(); ++i)
      EXPECT_DOUBLE_EQ(labels[t][i], i == ii.idx(want) ? 1.0 : 0.0);
  }
  // sampling keeps numTestUsers of them
  std::vector<size_t> u2;
  std::vector<std::vector<Double>> l2, s2;
  EngineTestPeer::initAvgTestData(u2, l2, s2, test, ui, ii, 1, 7);
  EXPECT_EQ(u2.size(), 1u);
}

TEST(Engine, computeTestScores) {
  const size_t k = 3, nu = 4, ni = 5;
  const std::vector<size_t> users = {2, 0};
  FactorData U(nu, k), I(ni, k, true);
  int val = 0;
  auto setter = [&val](auto...) { return (Double)++val; };
  U.setFactors(setter);
  I.setFactors(setter);
  I.setBiases(setter);
  std::vector<std::vector<Double>> scores(users.size(), std::vector<Double>(ni));
  for (size_t nt : {1, 2, 4}) {
    ParallelExecutor px(nt);
    EngineTestPeer::computeTestScores(scores, users, U, I, px);
    for (size_t t = 0; t < users.size(); ++t)
      for (size_t i = 0; i < ni; ++i) {
        Double r = I.biasAt(i);
        for (size_t f = 0; f < k; ++f) r += U.at(users[t], f) * I.at(i, f);
        EXPECT_DOUBLE_EQ(scores[t][i], r);
      }
  }
}

TEST(Engine, saveFactors) {
  IdIndex ix;
  ix.getOrSetIdx(3);
  ix.getOrSetIdx(5);
  {
    FactorData fd(2, 3);
    fd.setFactors([](size_t i, size_t j) { return (Double)(i * 3 + j); });
    std::ostringstream out;
    EngineTestPeer::saveFactors(fd, ix, out);
    EXPECT_EQ(out.str(), std::string("3 0.000000000 1.000000000 2.000000000\n5 "
                                     "3.000000000 4.000000000 5.000000000\n"));
  }
  {
    FactorData fd(2, 3, true);
    fd.setFactors([](size_t i, size_t j) { return (Double)(i * 3 + j); });
    fd.setBiases([](size_t i) { return 5.0 + i; });
    std::ostringstream out;
    EngineTestPeer::saveFactors(fd, ix, out);
    EXPECT_EQ(out.str(), std::string("3 5.000000000 0.000000000 1.000000000 2.000000000\n5 "
                                     "6.000000000 3.000000000 4.000000000 5.000000000\n"));
  }
  // the parallel writer equals the reference's ostream << fixed << setprecision(9)
  const size_t n = 40000;
  IdIndex big;
  std::mt19937_64 g(3);
  for (size_t i = 0; i < n; ++i) big.getOrSetIdx((int64_t)(g() >> 2) - (int64_t)(i % 3) * (1LL << 60));
  FactorData fd(n, 3, true);
  std::normal_distribution<Double> nd(0.0, 1.0);
  // (the writer formats with std::to_chars: every magnitude from 1e-14 to 1e22, values on a
  // %.9f rounding boundary, ±0, ±inf, NaN and 1e300 — printf's own path — must match)
  const Double special[] = {-0.0, 0.0, 0.0000000005, -0.0000000015, 2.5e-10, 0.1234567895,
                            1e15 + 0.5, 1e22, -1e300, INFINITY, -INFINITY, NAN, 4.9e-324};
  fd.setFactors([&](size_t i, size_t j) {
    if (i % 977 == 0) return -0.0;
    if (i % 101 == 0) return special[(i / 101 + j) % (sizeof(special) / sizeof(special[0]))];
    return nd(g) * std::pow(10.0, (double)(i % 37) - 14);
  });
  fd.setBiases([&](size_t) { return nd(g); });
  std::ostringstream fast, ref;
  EngineTestPeer::saveFactors(fd, big, fast);
  ref << std::fixed << std::setprecision(9);
  for (size_t i = 0; i < n; ++i) {
    ref << big.id(i) << ' ' << fd.biasAt(i);
    for (size_t f = 0; f < 3; ++f) ref << ' ' << fd.at(i, f);
    ref << '\n';
  }
  EXPECT_TRUE(fast.str() == ref.str());
  FactorData wrong(3, 3);
  std::ostringstream sink;
  EXPECT_DEATH(EngineTestPeer::saveFactors(wrong, ix, sink));
}

// ---- WALS grouping (WALSEngineTest.cpp:29-84) -----------------------------------------------
TEST(WALS, groupSignalsLayout) {
  std::vector<DatasetElem> d = {{1, 1}, {1, 2}, {1, 3}, {2, 1}, {2, 3}, {3, 4}};
  IdIndex ui, ii;
  SignalCsr bu, bi;
  groupSignals(d, ui, ii, bu, bi, 4);
  EXPECT_EQ(ui.size(), 3u);
  EXPECT_EQ(ii.size(), 4u);
  EXPECT_TRUE(bu.rowptr == std::vector<int64_t>({0, 3, 5, 6}));
  EXPECT_TRUE(bu.col == std::vector<int32_t>({0, 1, 2, 0, 2, 3}));
  EXPECT_TRUE(bi.rowptr == std::vector<int64_t>({0, 2, 3, 5, 6}));
  EXPECT_TRUE(bi.col == std::vector<int32_t>({0, 1, 0, 0, 1, 2}));
  for (size_t i = 0; i < 3; ++i) EXPECT_EQ(ui.id(i), (int64_t)i + 1);
  for (size_t i = 0; i < 4; ++i) EXPECT_EQ(ii.id(i), (int64_t)i + 1);
}

TEST(WALS, groupSignalsSignedIdsAndDuplicates) {
  // ids sort as signed int64; duplicates stay, in input order
  std::vector<DatasetElem> d = {{5, -2, 1.0}, {-9, 7, 2.0}, {5, -2, 3.0},
                                {INT64_MAX, INT64_MIN, 4.0}, {5, 7, 5.0}};
  IdIndex ui, ii;
  SignalCsr bu, bi;
  groupSignals(d, ui, ii, bu, bi, 3);
  EXPECT_TRUE(ui.ids() == std::vector<int64_t>({-9, 5, INT64_MAX}));
  EXPECT_TRUE(ii.ids() == std::vector<int64_t>({INT64_MIN, -2, 7}));
  EXPECT_TRUE(bu.rowptr == std::vector<int64_t>({0, 1, 4, 5}));
  EXPECT_TRUE(bu.col == std::vector<int32_t>({2, 1, 1, 2, 0}));
  EXPECT_TRUE(bu.val == std::vector<Double>({2.0, 1.0, 3.0, 5.0, 4.0}));
  EXPECT_TRUE(bi.rowptr == std::vector<int64_t>({0, 1, 3, 5}));
  EXPECT_TRUE(bi.col == std::vector<int32_t>({2, 1, 1, 0, 1}));
  EXPECT_TRUE(bi.val == std::vector<Double>({4.0, 1.0, 3.0, 2.0, 5.0}));
}

TEST(WALS, sortedUniqueMatchesStd) {
  std::mt19937_64 g(9);
  std::vector<int64_t> v(300000);
  for (auto& x : v) x = (int64_t)(g() % 50000) - 25000;
  auto ref = v;
  std::sort(ref.begin(), ref.end());
  ref.erase(std::unique(ref.begin(), ref.end()), ref.end());
  for (size_t nt : {1, 2, 5, 8}) EXPECT_TRUE(sortedUnique(v, nt) == ref);
}

// ---- BPR host bookkeeping (BPREngineTest.cpp:27-78) -----------------------------------------
TEST(BPR, initHost) {
  BPRConfig config{};
  config.nfactors = 30;
  config.initDistributionBound = 0.1;
  const std::unique_ptr<MetricsEngine> none;
  BPREngine e(config, none, /*evalNumNeg=*/2);
  std::vector<DatasetElem> d = {{3, 2}, {5, 2}, {3, 4}, {6, 2}, {7, 10}, {8, 10, 0.5}};
  BPREngineTestPeer::initHost(e, d);
  EXPECT_EQ(e.nusers(), 4u);  // value < 1 dropped
  EXPECT_EQ(e.nitems(), 3u);
  EXPECT_EQ(BPREngineTestPeer::ndata(e), 5u);
  EXPECT_EQ(BPREngineTestPeer::U(e).nelems(), 4u);
  EXPECT_EQ(BPREngineTestPeer::I(e).nfactors(), 30u);
  EXPECT_EQ(e.userIndex().idx(3), 0u);  // first-appearance order
  EXPECT_EQ(e.itemIndex().idx(10), 2u);
  const auto& im = BPREngineTestPeer::itemMap(e);
  const size_t u3 = e.userIndex().idx(3);
  EXPECT_EQ(im.count(u3), 2u);
  EXPECT_TRUE(im.contains(u3, e.itemIndex().idx(2)) && im.contains(u3, e.itemIndex().idx(4)));
  EXPECT_EQ(e.evalSet().size(), 2u * 5);
  for (const auto& t : e.evalSet()) {
    EXPECT_TRUE(im.contains(t.userIdx, t.posItemIdx));
    EXPECT_FALSE(im.contains(t.userIdx, t.negItemIdx));
  }
  for (size_t i = 0; i < 4; ++i)
    for (size_t f = 0; f < 30; ++f) EXPECT_TRUE(std::fabs(BPREngineTestPeer::U(e).at(i, f)) <= 0.1);
  std::vector<DatasetElem> td = {{5, 4}, {3, 10}, {6, 12}, {8, 13}};
  // initTest needs only host state: the metrics engine is absent
  e.initTest(td);
  const auto& tm = BPREngineTestPeer::testItemMap(e);
  EXPECT_EQ(tm.count(u3), 1u);
  EXPECT_TRUE(tm.contains(u3, e.itemIndex().idx(10)));
  EXPECT_EQ(e.testEvalSet().size(), 2u * 2);
  for (const auto& t : e.testEvalSet()) {
    EXPECT_TRUE(tm.contains(t.userIdx, t.posItemIdx));
    EXPECT_FALSE(tm.contains(t.userIdx, t.negItemIdx));
  }
  // the evaluation set depends only on evalSeed (mt19937), never on the factor seed
  BPREngine e2(config, none, 2);
  e2.seed(12345);
  BPREngineTestPeer::initHost(e2, d);
  bool same = e2.evalSet().size() == e.evalSet().size();
  for (size_t t = 0; same && t < e.evalSet().size(); ++t)
    same = e2.evalSet()[t].negItemIdx == e.evalSet()[t].negItemIdx;
  EXPECT_TRUE(same);
}

TEST(BPR, userWithEveryItemAborts) {
  BPRConfig config{};
  config.nfactors = 4;
  const std::unique_ptr<MetricsEngine> none;
  BPREngine e(config, none, 1);
  std::vector<DatasetElem> d = {{1, 1}, {1, 2}};
  EXPECT_DEATH(BPREngineTestPeer::initHost(e, d));
}

int main(int argc, char** argv) { return testing::runAll(argc, argv); }
