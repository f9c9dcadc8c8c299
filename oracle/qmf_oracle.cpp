// =====================================================================================
//  qmf oracle — TEST INFRASTRUCTURE ONLY.
//
//  A CPU restatement of the reference (taozhijiang/qmf) algorithm for the WALS / BPR hot
//  path.  It is the checker for parity tests (tests/), for __graft_entry__.smoke() and the
//  `cpu_baseline` leg of bench.py.  Nothing in the product path (qmf_amd/, include/, the
//  wals/bpr CLIs) links, loads or calls this file.
//
//  Every function names the reference file:line it restates (paths relative to the
//  reference root).  Arithmetic is fp64 (qmf/Types.h:24) with the reference's loop orders,
//  so that results match the reference CPU/LAPACK path to rounding.
//
//  Parity pins (see tests/test_oracle.py and DESIGN.md §Oracle):
//    * reference unit-test known answers: WALSEngineTest.cpp:29-84 (CSR layout),
//      :112-143 (XtX), :145-205 (x = 0.4/1.12), MatrixTest.cpp:92-116 (dsysv residual),
//      EngineTest.cpp:113-139 (output text, checked on the product writer);
//    * reference outputs measured by the survey (epoch-1 loss
//      1.81858, epoch-10 loss 0.574536 on the seeded ML-100K-shaped synthetic).
//  The reference itself is not buildable in this image (it needs glog, gflags and a
//  system LAPACK, none of which is installed) — see DESIGN.md.
//
//  LAPACK dsysv_ (third-party, not vendored; README.md:25 names liblapack-dev) is
//  restated as netlib's unblocked Bunch-Kaufman dsytf2 + dsytrs for uplo='U', which is
//  what dsysv_ runs when lwork = n is below the blocked-path workspace (Matrix.cpp:81-96).
// =====================================================================================
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <random>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <dlfcn.h>

namespace orc {

// ---- IdIndex (qmf/utils/IdIndex.h:27-62, IdIndex.cpp:21-31) ------------------------
struct IdIndex {
  std::vector<int64_t> ids;
  std::unordered_map<int64_t, size_t> map;
  static constexpr size_t missing = std::numeric_limits<size_t>::max();
  size_t getOrSetIdx(int64_t id) {
    auto it = map.find(id);
    if (it != map.end()) return it->second;
    size_t idx = ids.size();
    ids.push_back(id);
    map.emplace(id, idx);
    return idx;
  }
  size_t idx(int64_t id) const {
    auto it = map.find(id);
    return it == map.end() ? missing : it->second;
  }
};

struct Elem {  // DatasetElem (qmf/DatasetReader.h:29-33)
  int64_t userId;
  int64_t itemId;
  double value;
};

struct Signal {  // WALSEngine.h:67-70
  int64_t id;
  double value;
};
struct SignalGroup {  // WALSEngine.h:72-75
  int64_t sourceId;
  std::vector<Signal> group;
};

// ---- groupSignals / sortDataset (WALSEngine.cpp:130-163) ----------------------------
static void groupSignals(std::vector<SignalGroup>& signals, IdIndex& index,
                         std::vector<Elem>& dataset) {
  std::sort(dataset.begin(), dataset.end(), [](const Elem& x, const Elem& y) {
    if (x.userId != y.userId) return x.userId < y.userId;
    return x.itemId < y.itemId;
  });
  const int64_t invalid = std::numeric_limits<int64_t>::min();
  int64_t prev = invalid;
  std::vector<Signal> group;
  for (const auto& e : dataset) {
    if (e.userId != prev) {
      if (prev != invalid) signals.push_back(SignalGroup{prev, group});
      prev = e.userId;
      group.clear();
    }
    group.push_back(Signal{e.itemId, e.value});
  }
  if (prev != invalid) signals.push_back(SignalGroup{prev, group});
  for (size_t i = 0; i < signals.size(); ++i) index.getOrSetIdx(signals[i].sourceId);
}

// ---- LAPACK dsysv_ restatement (netlib dsytf2 + dsytrs, uplo = 'U') ------------------
// a: column-major n×n, only the upper triangle is read/written. 1-based formulas.
static int dsytf2_upper(int n, double* a, int* ipiv) {
#define A_(i, j) a[((j)-1) * (size_t)n + ((i)-1)]
  const double alpha = (1.0 + std::sqrt(17.0)) / 8.0;
  int info = 0;
  int k = n;
  while (k >= 1) {
    int kstep = 1;
    double absakk = std::fabs(A_(k, k));
    int imax = 0;
    double colmax = 0.0;
    if (k > 1) {
      imax = 1;
      double m = std::fabs(A_(1, k));
      for (int i = 2; i <= k - 1; ++i) {
        if (std::fabs(A_(i, k)) > m) { m = std::fabs(A_(i, k)); imax = i; }
      }
      colmax = m;
    }
    int kp;
    if (std::max(absakk, colmax) == 0.0 || std::isnan(absakk)) {
      if (info == 0) info = k;
      kp = k;
    } else {
      if (absakk >= alpha * colmax) {
        kp = k;
      } else {
        // rowmax = largest off-diagonal in row imax
        double rowmax = 0.0;
        int jmax = imax + 1;
        {
          double m = -1.0;
          for (int j = imax + 1; j <= k; ++j) {
            if (std::fabs(A_(imax, j)) > m) { m = std::fabs(A_(imax, j)); jmax = j; }
          }
          rowmax = m;
        }
        if (imax > 1) {
          int jm = 1;
          double m = std::fabs(A_(1, imax));
          for (int j = 2; j <= imax - 1; ++j) {
            if (std::fabs(A_(j, imax)) > m) { m = std::fabs(A_(j, imax)); jm = j; }
          }
          rowmax = std::max(rowmax, m);
        }
        (void)jmax;
        if (absakk >= alpha * colmax * (colmax / rowmax)) {
          kp = k;
        } else if (std::fabs(A_(imax, imax)) >= alpha * rowmax) {
          kp = imax;
        } else {
          kp = imax;
          kstep = 2;
        }
      }
      const int kk = k - kstep + 1;
      if (kp != kk) {
        for (int i = 1; i <= kp - 1; ++i) std::swap(A_(i, kk), A_(i, kp));
        for (int j = kp + 1; j <= kk - 1; ++j) std::swap(A_(j, kk), A_(kp, j));
        std::swap(A_(kk, kk), A_(kp, kp));
        if (kstep == 2) std::swap(A_(k - 1, k), A_(kp, k));
      }
      if (kstep == 1) {
        // dsyr: A := A - (1/D(k)) W(k) W(k)^T ; then scale column k
        const double r1 = 1.0 / A_(k, k);
        for (int j = 1; j <= k - 1; ++j) {
          if (A_(j, k) != 0.0) {
            const double temp = -r1 * A_(j, k);
            for (int i = 1; i <= j; ++i) A_(i, j) += A_(i, k) * temp;
          }
        }
        for (int i = 1; i <= k - 1; ++i) A_(i, k) *= r1;
      } else if (k > 2) {
        double d12 = A_(k - 1, k);
        const double d22 = A_(k - 1, k - 1) / d12;
        const double d11 = A_(k, k) / d12;
        const double t = 1.0 / (d11 * d22 - 1.0);
        d12 = t / d12;
        for (int j = k - 2; j >= 1; --j) {
          const double wkm1 = d12 * (d11 * A_(j, k - 1) - A_(j, k));
          const double wk = d12 * (d22 * A_(j, k) - A_(j, k - 1));
          for (int i = j; i >= 1; --i) A_(i, j) = A_(i, j) - A_(i, k) * wk - A_(i, k - 1) * wkm1;
          A_(j, k) = wk;
          A_(j, k - 1) = wkm1;
        }
      }
    }
    if (kstep == 1) {
      ipiv[k - 1] = kp;
    } else {
      ipiv[k - 1] = -kp;
      ipiv[k - 2] = -kp;
    }
    k -= kstep;
  }
  return info;
}

static void dsytrs_upper(int n, const double* a, const int* ipiv, double* b) {
  int k = n;
  while (k >= 1) {
    if (ipiv[k - 1] > 0) {
      const int kp = ipiv[k - 1];
      if (kp != k) std::swap(b[k - 1], b[kp - 1]);
      for (int i = 1; i <= k - 1; ++i) b[i - 1] -= A_(i, k) * b[k - 1];
      b[k - 1] /= A_(k, k);
      k -= 1;
    } else {
      const int kp = -ipiv[k - 1];
      if (kp != k - 1) std::swap(b[k - 2], b[kp - 1]);
      for (int i = 1; i <= k - 2; ++i) b[i - 1] -= A_(i, k) * b[k - 1];
      for (int i = 1; i <= k - 2; ++i) b[i - 1] -= A_(i, k - 1) * b[k - 2];
      const double akm1k = A_(k - 1, k);
      const double akm1 = A_(k - 1, k - 1) / akm1k;
      const double ak = A_(k, k) / akm1k;
      const double denom = akm1 * ak - 1.0;
      const double bkm1 = b[k - 2] / akm1k;
      const double bk = b[k - 1] / akm1k;
      b[k - 2] = (ak * bkm1 - bk) / denom;
      b[k - 1] = (akm1 * bk - bkm1) / denom;
      k -= 2;
    }
  }
  k = 1;
  while (k <= n) {
    if (ipiv[k - 1] > 0) {
      double s = 0.0;
      for (int i = 1; i <= k - 1; ++i) s += A_(i, k) * b[i - 1];
      b[k - 1] -= s;
      const int kp = ipiv[k - 1];
      if (kp != k) std::swap(b[k - 1], b[kp - 1]);
      k += 1;
    } else {
      double s = 0.0;
      for (int i = 1; i <= k - 1; ++i) s += A_(i, k) * b[i - 1];
      b[k - 1] -= s;
      s = 0.0;
      for (int i = 1; i <= k - 1; ++i) s += A_(i, k + 1) * b[i - 1];
      b[k] -= s;
      const int kp = -ipiv[k - 1];
      if (kp != k) std::swap(b[k - 1], b[kp - 1]);
      k += 2;
    }
  }
#undef A_
}

// linearSymmetricSolve (Matrix.cpp:81-96): A row-major n×n, b length n; returns info.
// Optional cross-check: when ORC_LAPACK names a LAPACK shared library (e.g. MKL's
// libmkl_rt), its dsysv_ is called with the reference's exact arguments instead of the
// restatement below.  Used only by tests to pin the restatement; never by default.
typedef void (*dsysv_fn)(char*, int*, int*, double*, int*, int*, double*, int*, double*, int*,
                         int*);
static dsysv_fn external_dsysv() {
  static dsysv_fn fn = []() -> dsysv_fn {
    const char* path = std::getenv("ORC_LAPACK");
    if (!path || !*path) return nullptr;
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return nullptr;
    return (dsysv_fn)dlsym(h, "dsysv_");
  }();
  return fn;
}

static int linearSymmetricSolve(const std::vector<double>& A, std::vector<double>& b, int n) {
  // A = A.transpose(); the column-major view of the transposed row-major copy is A itself.
  std::vector<double> At(A.size());
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) At[(size_t)j * n + i] = A[(size_t)i * n + j];
  // column-major element (i,j) at At[j*n+i]... At row-major (r,c) holds A(c,r); read as
  // column-major M(i,j) = data[j*n + i] = At(j,i) = A(i,j).
  std::vector<int> ipiv(n);
  if (dsysv_fn f = external_dsysv()) {  // Matrix.cpp:92-93 argument list
    int nn = n, nrhs = 1, info = 0;
    std::vector<double> work(n);
    char uplo[] = "Upper";
    f(uplo, &nn, &nrhs, At.data(), &nn, ipiv.data(), b.data(), &nn, work.data(), &nn, &info);
    return info;
  }
  int info = dsytf2_upper(n, At.data(), ipiv.data());
  if (info != 0) return info;
  dsytrs_upper(n, At.data(), ipiv.data(), b.data());
  return 0;
}

// ---- WALS engine restatement ----------------------------------------------------------
struct Wals {
  int k;
  double lambda, alpha;
  IdIndex userIndex, itemIndex;
  std::vector<SignalGroup> userSignals, itemSignals;
  std::vector<double> U, I;  // row-major n×k (FactorData, FactorData.h:28-36)
};

// WALSEngine::computeXtX(const Matrix&, Matrix*) with OMP_NUM_THREADS=1 (WALSEngine.cpp:246-264)
static void computeXtX(const std::vector<double>& X, size_t nrows, int k, std::vector<double>& out) {
  out.assign((size_t)k * k, 0.0);
  for (size_t r = 0; r < nrows; ++r) {
    const double* x = &X[r * k];
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < k; ++j) out[(size_t)i * k + j] += x[i] * x[j];
  }
}

// Index whose ids are the idx themselves (synthetic CSRs, where id = row/column index):
// the same lookups as IdIndex without building a hash over 10^7 ids for a row-sample check.
struct IdentityIndex {
  size_t idx(int64_t id) const { return (size_t)id; }
};

// WALSEngine::updateFactorsForOne (Matrix& overload, WALSEngine.cpp:266-310)
template <class LIndex, class RIndex>
static double updateFactorsForOne(std::vector<double>& X, const LIndex& leftIndex,
                                  const std::vector<double>& Y, const RIndex& rightIndex,
                                  const SignalGroup& sg, std::vector<double> A /*YtY by value*/,
                                  double alpha, double lambda, int n, int* info_out) {
  double loss = 0.0;
  std::vector<double> b(n, 0.0);
  for (const auto& s : sg.group) {
    const size_t r = rightIndex.idx(s.id);
    const double* y = &Y[r * n];
    for (int i = 0; i < n; ++i) {
      b[i] += y[i] * (1.0 + alpha * s.value);
      for (int j = 0; j < n; ++j) A[(size_t)i * n + j] += y[i] * alpha * s.value * y[j];
    }
    loss += 1.0 + alpha * s.value;
  }
  std::vector<double> B = A;
  for (int i = 0; i < n; ++i) A[(size_t)i * n + i] += lambda;
  std::vector<double> x = b;
  const int info = linearSymmetricSolve(A, x, n);
  if (info_out) *info_out = info;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) loss += B[(size_t)i * n + j] * x[i] * x[j];
  for (int i = 0; i < n; ++i) loss -= 2 * x[i] * b[i];
  const size_t leftIdx = leftIndex.idx(sg.sourceId);
  for (int i = 0; i < n; ++i) X[leftIdx * n + i] = x[i];
  return loss;
}

// WALSEngine::iterate (WALSEngine.cpp:165-218) with ParallelExecutor::mapReduce's strided
// task split and reduction order (ParallelExecutor-inl.h:37-58).
static double iterate(Wals& w, int side, int nthreads, int* bad_info) {
  std::vector<double>& X = side == 0 ? w.U : w.I;
  const std::vector<double>& Y = side == 0 ? w.I : w.U;
  const IdIndex& leftIndex = side == 0 ? w.userIndex : w.itemIndex;
  const IdIndex& rightIndex = side == 0 ? w.itemIndex : w.userIndex;
  const std::vector<SignalGroup>& sig = side == 0 ? w.userSignals : w.itemSignals;
  const int k = w.k;
  std::fill(X.begin(), X.end(), 0.0);
  std::vector<double> YtY;
  computeXtX(Y, rightIndex.ids.size(), k, YtY);
  if (nthreads < 1) nthreads = 1;
  const size_t ntasks = sig.size();
  std::vector<double> partial(nthreads, 0.0);
  std::vector<int> infos(nthreads, 0);
  auto worker = [&](int t) {
    double res = 0.0;
    for (size_t task = t; task < ntasks; task += nthreads) {
      int info = 0;
      res = res + updateFactorsForOne(X, leftIndex, Y, rightIndex, sig[task], YtY, w.alpha,
                                      w.lambda, k, &info);
      if (info != 0) infos[t] = info;
    }
    partial[t] = res;
  };
  if (nthreads == 1) {
    worker(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
  }
  double loss = 0.0;
  for (int t = 0; t < nthreads; ++t) loss = loss + partial[t];
  if (bad_info) {
    *bad_info = 0;
    for (int t = 0; t < nthreads; ++t)
      if (infos[t]) *bad_info = infos[t];
  }
  return loss / (double)w.userIndex.ids.size() / (double)w.itemIndex.ids.size();
}

// ---- BPR update rule (BPREngine.cpp:178-244) ----------------------------------------
static double predictDifference(const double* U, const double* I, const double* bias, int k,
                                size_t u, size_t p, size_t n, bool useBiases) {
  double pred = 0.0;
  if (useBiases) pred += bias[p] - bias[n];
  for (int i = 0; i < k; ++i) pred += U[u * k + i] * (I[p * k + i] - I[n * k + i]);
  return pred;
}

}  // namespace orc

using namespace orc;

extern "C" {

// ---- WALS handle ---------------------------------------------------------------------
// WALSEngine::init (WALSEngine.cpp:37-69): copy dataset, group by user, swap ids, group by
// item, allocate factors (zeros).  Item-factor init is done by the caller (set/load).
void* orc_wals_create(const int64_t* uid, const int64_t* iid, const double* val, int64_t n,
                      int k, double lambda, double alpha) {
  auto* w = new Wals();
  w->k = k;
  w->lambda = lambda;
  w->alpha = alpha;
  std::vector<Elem> ds((size_t)n);
  for (int64_t e = 0; e < n; ++e) ds[e] = Elem{uid[e], iid[e], val[e]};
  groupSignals(w->userSignals, w->userIndex, ds);
  for (auto& e : ds) std::swap(e.userId, e.itemId);
  groupSignals(w->itemSignals, w->itemIndex, ds);
  w->U.assign(w->userIndex.ids.size() * (size_t)k, 0.0);
  w->I.assign(w->itemIndex.ids.size() * (size_t)k, 0.0);
  return w;
}

// Build directly from a CSR whose ids are the row / column indices (used for the CPU
// baseline on device-generated synthetic data).  Signals keep the CSR order, which is
// ascending column index = ascending id, exactly as groupSignals would produce.
void* orc_wals_create_csr(int64_t nusers, int64_t nitems, const int64_t* urowptr,
                          const int32_t* ucol, const double* uval, const int64_t* irowptr,
                          const int32_t* icol, const double* ival, int k, double lambda,
                          double alpha) {
  auto* w = new Wals();
  w->k = k;
  w->lambda = lambda;
  w->alpha = alpha;
  for (int64_t u = 0; u < nusers; ++u) w->userIndex.getOrSetIdx(u);
  for (int64_t i = 0; i < nitems; ++i) w->itemIndex.getOrSetIdx(i);
  w->userSignals.resize(nusers);
  for (int64_t u = 0; u < nusers; ++u) {
    w->userSignals[u].sourceId = u;
    for (int64_t e = urowptr[u]; e < urowptr[u + 1]; ++e)
      w->userSignals[u].group.push_back(Signal{ucol[e], uval[e]});
  }
  w->itemSignals.resize(nitems);
  for (int64_t i = 0; i < nitems; ++i) {
    w->itemSignals[i].sourceId = i;
    for (int64_t e = irowptr[i]; e < irowptr[i + 1]; ++e)
      w->itemSignals[i].group.push_back(Signal{icol[e], ival[e]});
  }
  w->U.assign((size_t)nusers * k, 0.0);
  w->I.assign((size_t)nitems * k, 0.0);
  return w;
}

void orc_wals_destroy(void* h) { delete static_cast<Wals*>(h); }
int64_t orc_wals_nusers(void* h) { return (int64_t) static_cast<Wals*>(h)->userIndex.ids.size(); }
int64_t orc_wals_nitems(void* h) { return (int64_t) static_cast<Wals*>(h)->itemIndex.ids.size(); }
int64_t orc_wals_nnz(void* h) {
  int64_t s = 0;
  for (auto& g : static_cast<Wals*>(h)->userSignals) s += (int64_t)g.group.size();
  return s;
}

void orc_wals_ids(void* h, int side, int64_t* out) {
  auto* w = static_cast<Wals*>(h);
  const auto& ids = side == 0 ? w->userIndex.ids : w->itemIndex.ids;
  std::copy(ids.begin(), ids.end(), out);
}

// CSR of the signal groups in reference order; colidx = idx of the other side.
void orc_wals_csr(void* h, int side, int64_t* rowptr, int64_t* colidx, double* vals) {
  auto* w = static_cast<Wals*>(h);
  const auto& sig = side == 0 ? w->userSignals : w->itemSignals;
  const IdIndex& other = side == 0 ? w->itemIndex : w->userIndex;
  int64_t e = 0;
  rowptr[0] = 0;
  for (size_t r = 0; r < sig.size(); ++r) {
    for (const auto& s : sig[r].group) {
      colidx[e] = (int64_t)other.idx(s.id);
      vals[e] = s.value;
      ++e;
    }
    rowptr[r + 1] = e;
  }
}

void orc_wals_set_factors(void* h, int side, const double* f) {
  auto* w = static_cast<Wals*>(h);
  auto& X = side == 0 ? w->U : w->I;
  std::copy(f, f + X.size(), X.begin());
}

void orc_wals_get_factors(void* h, int side, double* out) {
  auto* w = static_cast<Wals*>(h);
  auto& X = side == 0 ? w->U : w->I;
  std::copy(X.begin(), X.end(), out);
}

// FactorData::setFactors(const std::string&) (FactorData.h:74-100): one %lf per line,
// row-major in idx order; a short file stops early leaving the rest untouched.
// Returns the number of values read, or -1 on a malformed line (reference: CHECK abort).
int64_t orc_wals_load_distribution_file(void* h, int side, const char* path) {
  auto* w = static_cast<Wals*>(h);
  auto& X = side == 0 ? w->U : w->I;
  std::ifstream fin(path);
  std::string line;
  int64_t count = 0;
  for (size_t e = 0; e < X.size(); ++e) {
    if (!std::getline(fin, line)) return count;
    double v = 0.0;
    if (sscanf(line.c_str(), "%lf", &v) != 1) return -1;
    X[e] = v;
    ++count;
  }
  return count;
}

// One half-epoch.  side 0 = solve users (items fixed), 1 = solve items.
double orc_wals_iterate(void* h, int side, int nthreads, int* bad_info) {
  return iterate(*static_cast<Wals*>(h), side, nthreads, bad_info);
}

// WALSEngine::optimize (WALSEngine.cpp:82-96): per epoch user half then item half; the
// logged loss is the item-half's.  losses[e] receives epoch e+1's item-half loss.
void orc_wals_optimize(void* h, int nepochs, int nthreads, double* losses) {
  auto* w = static_cast<Wals*>(h);
  for (int e = 0; e < nepochs; ++e) {
    iterate(*w, 0, nthreads, nullptr);
    losses[e] = iterate(*w, 1, nthreads, nullptr);
  }
}

// CPU baseline on a bounded sample: time YtY of the fixed side and the solve of every
// `stride`-th row of side `side` (reference per-row work: hash lookups, k×k copies, Gram,
// dsysv).  Rows are run by `nthreads` threads with the reference's strided split.
void orc_wals_time_sample(void* h, int side, int nthreads, int64_t stride, double* t_yty,
                          double* t_rows, int64_t* rows_done) {
  auto* w = static_cast<Wals*>(h);
  std::vector<double>& X = side == 0 ? w->U : w->I;
  const std::vector<double>& Y = side == 0 ? w->I : w->U;
  const IdIndex& leftIndex = side == 0 ? w->userIndex : w->itemIndex;
  const IdIndex& rightIndex = side == 0 ? w->itemIndex : w->userIndex;
  const auto& sig = side == 0 ? w->userSignals : w->itemSignals;
  const int k = w->k;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<double> YtY;
  computeXtX(Y, rightIndex.ids.size(), k, YtY);
  auto t1 = std::chrono::steady_clock::now();
  std::vector<size_t> rows;
  for (size_t r = 0; r < sig.size(); r += (size_t)stride) rows.push_back(r);
  auto worker = [&](int t) {
    double res = 0.0;
    for (size_t task = t; task < rows.size(); task += nthreads)
      res = res + updateFactorsForOne(X, leftIndex, Y, rightIndex, sig[rows[task]], YtY,
                                      w->alpha, w->lambda, k, nullptr);
    (void)res;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
  for (auto& x : th) x.join();
  auto t2 = std::chrono::steady_clock::now();
  *t_yty = std::chrono::duration<double>(t1 - t0).count();
  *t_rows = std::chrono::duration<double>(t2 - t1).count();
  *rows_done = (int64_t)rows.size();
}

// ---- building blocks exposed for known-answer tests -----------------------------------
void orc_xtx(const double* X, int64_t n, int k, double* out) {
  std::vector<double> x(X, X + n * k), o;
  computeXtX(x, (size_t)n, k, o);
  std::copy(o.begin(), o.end(), out);
}

// linearSymmetricSolve on a row-major matrix; b is overwritten with x. Returns info.
int orc_linear_symmetric_solve(const double* A, double* b, int n) {
  std::vector<double> a(A, A + (size_t)n * n), x(b, b + n);
  int info = linearSymmetricSolve(a, x, n);
  std::copy(x.begin(), x.end(), b);
  return info;
}

// updateFactorsForOne on explicit inputs: Y (nY×k), the row's signals as (Y row index,
// value) pairs, YtY (k×k).  Writes x (k) and returns the row loss.
double orc_update_one(const double* Y, int64_t nY, int k, const int64_t* cols,
                      const double* vals, int64_t nnz, const double* YtY, double alpha,
                      double lambda, double* x_out) {
  IdIndex left, right;
  left.getOrSetIdx(0);
  for (int64_t i = 0; i < nY; ++i) right.getOrSetIdx(i);
  SignalGroup sg{0, {}};
  for (int64_t e = 0; e < nnz; ++e) sg.group.push_back(Signal{cols[e], vals[e]});
  std::vector<double> X((size_t)k, 0.0), y(Y, Y + nY * k), g(YtY, YtY + (size_t)k * k);
  double loss = updateFactorsForOne(X, left, y, right, sg, g, alpha, lambda, k, nullptr);
  std::copy(X.begin(), X.end(), x_out);
  return loss;
}

// Parity checker at full size: re-solves `nrows` rows of a CSR (ids = indices) with
// updateFactorsForOne against the given fixed side Y (nY×k, the device's own values), with
// YtY = computeXtX(Y) summed over `nthreads` row blocks (fixed order; the serial sum differs
// only by rounding).  Writes x (nrows×k) and the row losses.  Returns the first nonzero
// dsysv info, or 0.
int orc_solve_rows(const double* Y, int64_t nY, int k, const int64_t* rowptr,
                   const int32_t* col, const double* val, const int64_t* rows, int64_t nrows,
                   double alpha, double lambda, int nthreads, double* x_out, double* loss_out) {
  if (nthreads < 1) nthreads = 1;
  std::vector<double> y(Y, Y + (size_t)nY * k);
  std::vector<std::vector<double>> part((size_t)nthreads);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t]() {
        const int64_t b = nY * t / nthreads, e = nY * (t + 1) / nthreads;
        std::vector<double> sub(y.begin() + b * k, y.begin() + e * k);
        computeXtX(sub, (size_t)(e - b), k, part[(size_t)t]);
      });
    for (auto& x : th) x.join();
  }
  std::vector<double> YtY((size_t)k * k, 0.0);
  for (int t = 0; t < nthreads; ++t)
    for (size_t i = 0; i < YtY.size(); ++i) YtY[i] += part[(size_t)t][i];
  const IdentityIndex ident;
  std::vector<int> infos((size_t)nthreads, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t]() {
      std::vector<double> X((size_t)k, 0.0);
      struct One {
        size_t idx(int64_t) const { return 0; }
      } one;
      for (int64_t q = t; q < nrows; q += nthreads) {
        const int64_t r = rows[q];
        SignalGroup sg{r, {}};
        for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e)
          sg.group.push_back(Signal{col[e], val[e]});
        int info = 0;
        loss_out[q] = updateFactorsForOne(X, one, y, ident, sg, YtY, alpha, lambda, k, &info);
        if (info) infos[(size_t)t] = info;
        std::copy(X.begin(), X.end(), x_out + q * k);
      }
    });
  for (auto& x : th) x.join();
  for (int v : infos)
    if (v) return v;
  return 0;
}

// ---- BPR -------------------------------------------------------------------------------
double orc_bpr_predict_difference(const double* U, const double* I, const double* bias, int k,
                                  int64_t u, int64_t p, int64_t n, int useBiases) {
  return predictDifference(U, I, bias, k, u, p, n, useBiases != 0);
}

// BPREngine::update (BPREngine.cpp:178-220), applied to triplets in order.
// Returns 0, or 1 if a derivative was not finite (reference CHECK abort).
int orc_bpr_update_seq(double* U, double* I, double* bias, int k, const int64_t* trip,
                       int64_t ntrip, double lr, double biasLambda, double userLambda,
                       double itemLambda, int useBiases) {
  for (int64_t t = 0; t < ntrip; ++t) {
    const size_t u = trip[3 * t], p = trip[3 * t + 1], n = trip[3 * t + 2];
    const double x = predictDifference(U, I, bias, k, u, p, n, useBiases != 0);
    const double e = 1.0 / (1.0 + std::exp(x));  // lossDerivative (:237-244)
    if (!std::isfinite(e)) return 1;
    if (useBiases) {
      double step = lr * (e - biasLambda * bias[p]);
      bias[p] += step;
      step = lr * (-e - biasLambda * bias[n]);
      bias[n] += step;
    }
    for (int i = 0; i < k; ++i) {
      const double step = lr * (e * (I[p * k + i] - I[n * k + i]) - userLambda * U[u * k + i]);
      U[u * k + i] += step;
    }
    for (int i = 0; i < k; ++i) {
      const double step = lr * (e * U[u * k + i] - itemLambda * I[p * k + i]);
      I[p * k + i] += step;
    }
    for (int i = 0; i < k; ++i) {
      const double step = lr * (-e * U[u * k + i] - itemLambda * I[n * k + i]);
      I[n * k + i] += step;
    }
  }
  return 0;
}

// Sum of log(1 + exp(-x̂)) over triplets (BPREngine::loss / evaluate, :237-274), serial.
double orc_bpr_loss_sum(const double* U, const double* I, const double* bias, int k,
                        const int64_t* trip, int64_t ntrip, int useBiases) {
  double s = 0.0;
  for (int64_t t = 0; t < ntrip; ++t) {
    const double x = predictDifference(U, I, bias, k, trip[3 * t], trip[3 * t + 1],
                                       trip[3 * t + 2], useBiases != 0);
    s += std::log(1.0 + std::exp(-x));
  }
  return s;
}

// BPREngine::init (BPREngine.cpp:63-90) and initTest (:92-131) bookkeeping with
// sampleRandomNegative (BPREngine-inl.h:48-60): first-appearance indexes, value < 1
// dropped, per-user unordered_set of positives, the evaluation triplets from
// mt19937(evalSeed) + uniform_int_distribution<int>(0, nitems − 1) with rejection.
// Outputs: index sizes and ids, eval / test-eval triplets (u, p, n).  Returns 1 (instead
// of spinning forever like the reference) when some user has every item as a positive.
// One BPR epoch as BPREngine::optimize runs it with numHogwildThreads = T > 1
// (BPREngine.cpp:146-176): T contiguous blocks of floor(N/T) positives (the tail is dropped,
// as in the reference), each block on its own thread (iterateBlock, BPREngine-inl.h:31-46),
// numNeg negatives per positive rejection-sampled against the user's unordered_set
// (sampleRandomNegative, -inl.h:48-60), update() on shared rows without locks, then the
// eval-set loss (evaluate, :246-274) by a T-way mapReduce.  The reference shares one
// mt19937 across threads (a data race); here each thread seeds its own (seed + block), which
// can only make this baseline faster.  CPU BASELINE ONLY: the factor races make the result
// nondeterministic, like the reference's.  Returns the elapsed seconds of the update part
// in *t_update and of the evaluation in *t_eval; the eval loss sum in *eval_loss.
int orc_bpr_hogwild_epoch(double* U, double* I, double* bias, int k, const int64_t* pos_user,
                          const int64_t* pos_item, int64_t npos, int64_t nusers, int64_t nitems,
                          int numNeg, int nthreads, uint64_t seed, double lr, double biasLambda,
                          double userLambda, double itemLambda, int useBiases,
                          const int64_t* evalSet, int64_t nEval, double* t_update,
                          double* t_eval, double* eval_loss) {
  if (nthreads < 1) nthreads = 1;
  // itemMap_ (BPREngine.cpp:79-82): per-user unordered_set of positive items
  std::vector<std::unordered_set<size_t>> itemMap((size_t)nusers);
  for (int64_t e = 0; e < npos; ++e) itemMap[(size_t)pos_user[e]].insert((size_t)pos_item[e]);
  std::atomic<int> bad{0};
  auto t0 = std::chrono::steady_clock::now();
  const int64_t block = npos / nthreads;
  auto worker = [&](int t) {
    std::mt19937 gen((uint32_t)(seed + (uint64_t)t));
    std::uniform_int_distribution<> dis(0, (int)nitems - 1);
    for (int64_t i = t * block; i < (t + 1) * block; ++i) {
      const size_t u = (size_t)pos_user[i], p = (size_t)pos_item[i];
      const auto& set = itemMap[u];
      for (int j = 0; j < numNeg; ++j) {
        size_t n;
        do {
          n = (size_t)dis(gen);
        } while (set.count(n) > 0);
        const int64_t trip[3] = {(int64_t)u, (int64_t)p, (int64_t)n};
        if (orc_bpr_update_seq(U, I, bias, k, trip, 1, lr, biasLambda, userLambda, itemLambda,
                               useBiases))
          bad = 1;
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
  }
  auto t1 = std::chrono::steady_clock::now();
  std::vector<double> part((size_t)nthreads, 0.0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t]() {
        double s = 0.0;
        for (int64_t q = t; q < nEval; q += nthreads) {
          const double x = predictDifference(U, I, bias, k, (size_t)evalSet[3 * q],
                                             (size_t)evalSet[3 * q + 1], (size_t)evalSet[3 * q + 2],
                                             useBiases != 0);
          s += std::log(1.0 + std::exp(-x));
        }
        part[(size_t)t] = s;
      });
    for (auto& x : th) x.join();
  }
  double loss = 0.0;
  for (double v : part) loss += v;
  auto t2 = std::chrono::steady_clock::now();
  *t_update = std::chrono::duration<double>(t1 - t0).count();
  *t_eval = std::chrono::duration<double>(t2 - t1).count();
  *eval_loss = loss;
  return bad.load();
}

int orc_bpr_sets(const int64_t* users, const int64_t* items, const double* vals, int64_t n,
                 const int64_t* tusers, const int64_t* titems, const double* tvals, int64_t tn,
                 int64_t evalNumNeg, int32_t evalSeed, int64_t* nusers, int64_t* nitems,
                 int64_t* uids, int64_t* iids, int64_t* evalSet, int64_t* nEval,
                 int64_t* testEvalSet, int64_t* nTestEval) {
  IdIndex ui, ii;
  std::vector<std::pair<size_t, size_t>> data;
  for (int64_t e = 0; e < n; ++e) {
    if (vals[e] < 1.0) continue;
    const size_t u = ui.getOrSetIdx(users[e]);
    const size_t p = ii.getOrSetIdx(items[e]);
    data.emplace_back(u, p);
  }
  std::vector<std::unordered_set<size_t>> itemMap(ui.ids.size());
  for (const auto& d : data) itemMap[d.first].insert(d.second);
  const size_t ni = ii.ids.size();
  auto sample = [ni](const std::unordered_set<size_t>& pos, std::mt19937& gen,
                     size_t* out) -> bool {
    if (pos.size() >= ni) return false;
    std::uniform_int_distribution<> dis(0, static_cast<int>(ni) - 1);
    size_t neg;
    do {
      neg = dis(gen);
    } while (pos.count(neg) > 0);
    *out = neg;
    return true;
  };
  {
    std::mt19937 gen(evalSeed);
    int64_t w = 0;
    for (const auto& d : data)
      for (int64_t j = 0; j < evalNumNeg; ++j) {
        size_t neg;
        if (!sample(itemMap[d.first], gen, &neg)) return 1;
        evalSet[3 * w] = (int64_t)d.first;
        evalSet[3 * w + 1] = (int64_t)d.second;
        evalSet[3 * w + 2] = (int64_t)neg;
        ++w;
      }
    *nEval = w;
  }
  {
    std::vector<std::unordered_set<size_t>> testMap(ui.ids.size());
    std::vector<std::pair<size_t, size_t>> valid;
    for (int64_t e = 0; e < tn; ++e) {
      if (tvals[e] < 1.0) continue;
      const size_t u = ui.idx(tusers[e]);
      const size_t p = ii.idx(titems[e]);
      if (u == IdIndex::missing || p == IdIndex::missing) continue;
      testMap[u].insert(p);
      valid.emplace_back(u, p);
    }
    std::mt19937 gen(evalSeed);
    int64_t w = 0;
    for (const auto& d : valid)
      for (int64_t j = 0; j < evalNumNeg; ++j) {
        size_t neg;
        if (!sample(testMap[d.first], gen, &neg)) return 1;
        testEvalSet[3 * w] = (int64_t)d.first;
        testEvalSet[3 * w + 1] = (int64_t)d.second;
        testEvalSet[3 * w + 2] = (int64_t)neg;
        ++w;
      }
    *nTestEval = w;
  }
  *nusers = (int64_t)ui.ids.size();
  *nitems = (int64_t)ni;
  std::copy(ui.ids.begin(), ui.ids.end(), uids);
  std::copy(ii.ids.begin(), ii.ids.end(), iids);
  return 0;
}

}  // extern "C"
