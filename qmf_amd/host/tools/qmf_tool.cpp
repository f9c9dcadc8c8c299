// Host-side inspection tool used by the parity tests: dumps the drop-in library's
// bookkeeping (no GPU involved) so it can be compared with the oracle's restatement of
// the reference.  Output: one line per array, "<name> <n> v0 v1 ...".
//   qmf_tool wals-csr <dataset>                           ids + both CSR orientations
//   qmf_tool bpr-sets <train> <test|-> <evalNumNeg> <seed>  BPR indexes + evaluation sets
//   qmf_tool gen-dataset <nusers> <nitems> <nnz> <seed> <out>  a synthetic `u i w` text file
//     (nnz distinct pairs in a seeded pseudo-random order, w in 1..5; tools/bench_cli.py)
//   qmf_tool read-seq <file>   the reference's reader loop (getline + sscanf per line,
//     qmf/DatasetReader.cpp:29-59) on one thread: prints "<lines> <seconds>"
#include <charconv>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <thread>
#include <string>
#include <vector>

#include <qmf/DatasetReader.h>
#include <qmf/bpr/BPREngine.h>
#include <qmf/wals/Signals.h>

namespace qmf {
class BPREngineTestPeer {
 public:
  static void initHost(BPREngine& e, const std::vector<DatasetElem>& d) { e.initHost(d); }
};
}  // namespace qmf

template <typename T>
static void dump(const char* name, const std::vector<T>& v) {
  std::printf("%s %zu", name, v.size());
  for (const T& x : v) {
    if (std::is_floating_point<T>::value)
      std::printf(" %.17g", (double)x);
    else
      std::printf(" %lld", (long long)x);
  }
  std::printf("\n");
}

static uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// Line j holds the pair key (a·j + b) mod (nusers·nitems) with a coprime to the key space, so
// the nnz pairs are distinct; written by several threads, each formatting its own chunk.
static int genDataset(long long nu, long long ni, long long nnz, unsigned long long seed,
                      const char* out) {
  const unsigned long long space = (unsigned long long)nu * (unsigned long long)ni;
  if (nu <= 0 || ni <= 0 || nnz <= 0 || (unsigned long long)nnz > space) return 2;
  unsigned long long a = (mix64(seed) % space) | 1;
  while (std::gcd(a, space) != 1) a += 2;
  const unsigned long long b = mix64(seed + 1) % space;
  const int nt = 16;
  std::vector<std::string> parts(nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      const long long j0 = nnz * t / nt, j1 = nnz * (t + 1) / nt;
      std::string& o = parts[t];
      o.reserve((size_t)(j1 - j0) * 18);
      char buf[64];
      for (long long j = j0; j < j1; ++j) {
        const unsigned long long key =
            (unsigned long long)(((unsigned __int128)a * (unsigned long long)j + b) % space);
        char* p = buf;
        p = std::to_chars(p, buf + 24, (long long)(key / ni)).ptr;  // ≤ 20 digits each
        *p++ = ' ';
        p = std::to_chars(p, p + 24, (long long)(key % ni)).ptr;
        *p++ = ' ';
        *p++ = (char)('1' + mix64(seed ^ (unsigned long long)j) % 5);
        *p++ = '\n';
        o.append(buf, p);
      }
    });
  for (auto& x : th) x.join();
  FILE* f = std::fopen(out, "wb");
  if (!f) return 1;
  for (const auto& o : parts) std::fwrite(o.data(), 1, o.size(), f);
  return std::fclose(f) == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !std::strcmp(argv[1], "read-seq")) {
    const auto t0 = std::chrono::steady_clock::now();
    qmf::DatasetReader r(argv[2]);
    qmf::DatasetElem e;
    long long n = 0;
    while (r.readOne(e)) ++n;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%lld %.3f\n", n, s);
    return 0;
  }
  if (argc >= 7 && !std::strcmp(argv[1], "gen-dataset"))
    return genDataset(std::atoll(argv[2]), std::atoll(argv[3]), std::atoll(argv[4]),
                      std::strtoull(argv[5], nullptr, 10), argv[6]);
  if (argc >= 3 && !std::strcmp(argv[1], "wals-csr")) {
    const auto ds = qmf::DatasetReader(argv[2]).readAll();
    qmf::IdIndex ui, ii;
    qmf::SignalCsr bu, bi;
    qmf::groupSignals(ds, ui, ii, bu, bi, 8);
    dump("uids", ui.ids());
    dump("iids", ii.ids());
    dump("urowptr", bu.rowptr);
    dump("ucol", bu.col);
    dump("uval", bu.val);
    dump("irowptr", bi.rowptr);
    dump("icol", bi.col);
    dump("ival", bi.val);
    return 0;
  }
  if (argc >= 6 && !std::strcmp(argv[1], "bpr-sets")) {
    const auto ds = qmf::DatasetReader(argv[2]).readAll();
    qmf::BPRConfig config{};
    config.nfactors = 1;
    config.initDistributionBound = 0.01;
    const std::unique_ptr<qmf::MetricsEngine> none;
    qmf::BPREngine e(config, none, std::stoul(argv[4]), std::stoi(argv[5]), 1);
    qmf::BPREngineTestPeer::initHost(e, ds);
    if (std::strcmp(argv[3], "-")) e.initTest(qmf::DatasetReader(argv[3]).readAll());
    dump("uids", e.userIndex().ids());
    dump("iids", e.itemIndex().ids());
    std::vector<int64_t> t;
    for (const auto& x : e.evalSet()) t.insert(t.end(), {(int64_t)x.userIdx, (int64_t)x.posItemIdx, (int64_t)x.negItemIdx});
    dump("eval", t);
    t.clear();
    for (const auto& x : e.testEvalSet()) t.insert(t.end(), {(int64_t)x.userIdx, (int64_t)x.posItemIdx, (int64_t)x.negItemIdx});
    dump("testeval", t);
    return 0;
  }
  std::fprintf(stderr, "usage: qmf_tool wals-csr <dataset> | bpr-sets <train> <test|-> <evalNumNeg> <seed>\n");
  return 2;
}
