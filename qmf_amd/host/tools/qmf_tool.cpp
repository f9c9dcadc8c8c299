// Host-side inspection tool used by the parity tests: dumps the drop-in library's
// bookkeeping (no GPU involved) so it can be compared with the oracle's restatement of
// the reference.  Output: one line per array, "<name> <n> v0 v1 ...".
//   qmf_tool wals-csr <dataset>                           ids + both CSR orientations
//   qmf_tool bpr-sets <train> <test|-> <evalNumNeg> <seed>  BPR indexes + evaluation sets
#include <cstdio>
#include <cstring>
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

int main(int argc, char** argv) {
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
