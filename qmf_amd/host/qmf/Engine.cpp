#include <qmf/Engine.h>

#include <charconv>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <random>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include <qmf/Device.h>
#include <qmf/utils/Log.h>

namespace qmf {

void Engine::initAvgTestData(std::vector<size_t>& testUsers,
                             std::vector<std::vector<Double>>& testLabels,
                             std::vector<std::vector<Double>>& testScores,
                             const std::vector<DatasetElem>& testDataset,
                             const IdIndex& userIndex,
                             const IdIndex& itemIndex,
                             const size_t numTestUsers,
                             const int32_t seed) {
  // The user order is the iteration order of an unordered_set filled in dataset order,
  // then (optionally) a mt19937(seed) shuffle: the same containers and calls as the
  // reference (Engine.cpp:35-52) so the sampled users coincide.
  std::unordered_set<size_t> seen;
  for (const auto& e : testDataset) {
    const size_t u = userIndex.idx(e.userId);
    const size_t i = itemIndex.idx(e.itemId);
    if (u != IdIndex::missingIdx && i != IdIndex::missingIdx) seen.insert(u);
  }
  testUsers.assign(seen.begin(), seen.end());
  if (numTestUsers > 0 && numTestUsers < testUsers.size()) {
    std::shuffle(testUsers.begin(), testUsers.end(), std::mt19937(seed));
    testUsers.resize(numTestUsers);
    testUsers.shrink_to_fit();
  }
  std::unordered_map<size_t, size_t> slot;
  testLabels.reserve(testUsers.size());
  testScores.reserve(testUsers.size());
  for (size_t t = 0; t < testUsers.size(); ++t) {
    slot[testUsers[t]] = t;
    testLabels.emplace_back(itemIndex.size());
    testScores.emplace_back(itemIndex.size());
  }
  for (const auto& e : testDataset) {
    const size_t u = userIndex.idx(e.userId);
    const size_t i = itemIndex.idx(e.itemId);
    if (u == IdIndex::missingIdx || i == IdIndex::missingIdx) continue;
    const auto it = slot.find(u);
    if (it != slot.end()) testLabels[it->second][i] = e.value;
  }
}

void Engine::computeTestScores(std::vector<std::vector<Double>>& testScores,
                               const std::vector<size_t>& testUsers,
                               const FactorData& userFactors,
                               const FactorData& itemFactors,
                               ParallelExecutor& parallel) {
  const size_t k = userFactors.nfactors();
  const size_t ni = itemFactors.nelems();
  parallel.execute(testUsers.size(), [&](const size_t t) {
    const Double* u = userFactors.getFactors().data(testUsers[t]);
    auto& scores = testScores[t];
    for (size_t i = 0; i < ni; ++i) {
      const Double* q = itemFactors.getFactors().data(i);
      Double s = itemFactors.withBiases() ? itemFactors.biasAt(i) : 0.0;
      for (size_t f = 0; f < k; ++f) s += u[f] * q[f];
      scores[i] = s;
    }
  });
}

void Engine::computeTestRanks(qmfx_ctx* ctx, bool useBiases,
                              const std::vector<size_t>& testUsers,
                              const std::vector<std::vector<Double>>& testLabels,
                              std::vector<RankedUser>& ranks) {
  CHECK_EQ(testUsers.size(), testLabels.size());
  const size_t nt = testUsers.size();
  auto& L = testCsr_;
  if (!L.uploaded) {
    L.rowptr.assign(1, 0);
    for (const auto& row : testLabels) {
      for (size_t i = 0; i < row.size(); ++i)
        if (row[i] != 0.0) {
          L.items.push_back(static_cast<int64_t>(i));
          L.values.push_back(row[i]);
          L.npos += row[i] > 0.0;
        }
      L.rowptr.push_back(static_cast<int64_t>(L.items.size()));
    }
    const std::vector<int64_t> users(testUsers.begin(), testUsers.end());
    QMFX_CHECK(qmfx_eval_set_labels(ctx, static_cast<int64_t>(nt), users.data(),
                                    L.rowptr.data(), L.items.data(), L.values.data()));
    L.uploaded = true;
  }
  std::vector<double> lscore(L.items.size()), sq(nt);
  std::vector<int64_t> above(L.npos);
  QMFX_CHECK(qmfx_eval_ranks(ctx, useBiases ? 1 : 0, lscore.data(), above.data(), sq.data()));
  ranks.assign(nt, RankedUser());
  size_t p = 0;
  for (size_t t = 0; t < nt; ++t) {
    RankedUser& r = ranks[t];
    r.nitems = testLabels[t].size();
    // Σ score² over all items, with the labelled items' terms swapped for (label − score)²
    Double sse = sq[t];
    std::vector<Double> ps;
    std::vector<int64_t> ab;
    for (int64_t e = L.rowptr[t]; e < L.rowptr[t + 1]; ++e) {
      const Double l = L.values[e], s = lscore[e];
      sse += (l - s) * (l - s) - s * s;
      if (l > 0.0) {
        ps.push_back(s);
        ab.push_back(above[p++]);
      }
    }
    r.sse = sse;
    r.setPositives(ps, ab);
  }
}

namespace {

// " %.9f" of x appended to s.  std::to_chars with a precision renders the exact decimal value
// of x correctly rounded, as glibc's printf does, so the text is the same byte for byte (the
// host tests compare them over random and edge values); a value that does not fit the buffer
// (|x| ≥ 1e290) takes printf itself.
inline void appendFixed9(std::string& s, Double x) {
  char buf[320];
  buf[0] = ' ';
  const auto r = std::to_chars(buf + 1, buf + sizeof(buf), x, std::chars_format::fixed, 9);
  if (r.ec == std::errc()) {
    s.append(buf, r.ptr);
    return;
  }
  std::string big(static_cast<size_t>(std::snprintf(nullptr, 0, " %.9f", x)) + 1, '\0');
  std::snprintf(&big[0], big.size(), " %.9f", x);
  big.pop_back();
  s += big;
}

// Formats rows [b, e) exactly as `out << std::fixed << std::setprecision(9)` would:
// libstdc++ renders fixed doubles through printf("%.*f").
void formatRows(const FactorData& fd, const IdIndex& index, size_t b, size_t e, std::string& s) {
  char buf[32];
  const size_t k = fd.nfactors();
  s.reserve(s.size() + (e - b) * (k * 13 + 24));
  for (size_t idx = b; idx < e; ++idx) {
    s.append(buf, std::to_chars(buf, buf + sizeof(buf), static_cast<long long>(index.id(idx))).ptr);
    if (fd.withBiases()) appendFixed9(s, fd.biasAt(idx));
    const Double* row = fd.getFactors().data(idx);
    for (size_t f = 0; f < k; ++f) appendFixed9(s, row[f]);
    s.push_back('\n');
  }
}

}  // namespace

void Engine::saveFactors(const FactorData& factorData, const IdIndex& index,
                         const std::string& fileName) {
  std::ofstream fout(fileName);
  saveFactors(factorData, index, fout);
}

void Engine::saveFactors(const FactorData& factorData, const IdIndex& index, std::ostream& out) {
  CHECK_EQ(factorData.nelems(), index.size());
  const size_t n = factorData.nelems();
  // format blocks of rows in parallel, write them in order
  const size_t block = 1 << 14;
  const size_t nblocks = (n + block - 1) / block;
  const unsigned hc = std::thread::hardware_concurrency();
  const size_t nt = std::max<size_t>(1, std::min<size_t>(hc ? hc : 1, 32));
  for (size_t b0 = 0; b0 < nblocks; b0 += nt) {
    const size_t nb = std::min(nt, nblocks - b0);
    std::vector<std::string> parts(nb);
    ParallelExecutor::run(nb, [&](const size_t t) {
      const size_t b = (b0 + t) * block;
      formatRows(factorData, index, b, std::min(n, b + block), parts[t]);
    });
    for (const auto& p : parts) out.write(p.data(), static_cast<std::streamsize>(p.size()));
  }
}

}  // namespace qmf
