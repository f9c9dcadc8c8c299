#include <qmf/wals/Signals.h>

#include <algorithm>
#include <limits>

#include <qmf/utils/Log.h>
#include <qmf/utils/ParallelExecutor.h>

namespace qmf {

std::vector<int64_t> sortedUnique(std::vector<int64_t> ids, size_t nthreads) {
  const size_t n = ids.size();
  const size_t nt = std::max<size_t>(1, std::min(nthreads, n / 65536 + 1));
  // sort + dedupe chunks in parallel; the distinct ids are usually far fewer than nnz
  std::vector<std::vector<int64_t>> parts(nt);
  ParallelExecutor::run(nt, [&](const size_t t) {
    auto& p = parts[t];
    p.assign(ids.begin() + n * t / nt, ids.begin() + n * (t + 1) / nt);
    std::sort(p.begin(), p.end());
    p.erase(std::unique(p.begin(), p.end()), p.end());
  });
  std::vector<int64_t>().swap(ids);
  // pairwise merges
  while (parts.size() > 1) {
    const size_t half = parts.size() / 2;
    std::vector<std::vector<int64_t>> next(parts.size() - half);
    ParallelExecutor::run(half, [&](const size_t t) {
      auto& a = parts[2 * t];
      auto& b = parts[2 * t + 1];
      auto& m = next[t];
      m.resize(a.size() + b.size());
      m.erase(std::set_union(a.begin(), a.end(), b.begin(), b.end(), m.begin()), m.end());
      std::vector<int64_t>().swap(a);
      std::vector<int64_t>().swap(b);
    });
    if (parts.size() % 2) next.back() = std::move(parts.back());
    parts.swap(next);
  }
  return parts.empty() ? std::vector<int64_t>() : std::move(parts[0]);
}

namespace {

// CSR of (row[e], col[e], val[e]) with rows in idx order and, inside each row, entries by
// ascending col, equal cols in input order (stable)
void buildCsr(const std::vector<int32_t>& row, const std::vector<int32_t>& col,
              const std::vector<DatasetElem>& ds, size_t nrows, SignalCsr& out,
              size_t nthreads) {
  const size_t nnz = row.size();
  out.rowptr.assign(nrows + 1, 0);
  for (size_t e = 0; e < nnz; ++e) ++out.rowptr[static_cast<size_t>(row[e]) + 1];
  for (size_t r = 0; r < nrows; ++r) out.rowptr[r + 1] += out.rowptr[r];
  std::vector<int64_t> fill(out.rowptr.begin(), out.rowptr.end() - 1);
  std::vector<int64_t> src(nnz);  // input position per CSR slot (stable scatter)
  for (size_t e = 0; e < nnz; ++e) src[fill[row[e]]++] = static_cast<int64_t>(e);
  std::vector<int64_t>().swap(fill);
  out.col.resize(nnz);
  out.val.resize(nnz);
  ParallelExecutor px(nthreads);
  const size_t chunk = 4096;
  px.execute((nrows + chunk - 1) / chunk, [&](const size_t task) {
    std::vector<std::pair<int32_t, int64_t>> buf;
    const size_t rb = task * chunk, re = std::min(nrows, rb + chunk);
    for (size_t r = rb; r < re; ++r) {
      const int64_t b = out.rowptr[r], e = out.rowptr[r + 1];
      buf.clear();
      for (int64_t p = b; p < e; ++p) buf.emplace_back(col[src[p]], src[p]);
      // (col, input position) order = ascending id with duplicates in input order
      std::sort(buf.begin(), buf.end());
      for (int64_t p = b; p < e; ++p) {
        out.col[p] = buf[p - b].first;
        out.val[p] = ds[buf[p - b].second].value;
      }
    }
  });
}

}  // namespace

void groupSignals(const std::vector<DatasetElem>& dataset, IdIndex& userIndex,
                  IdIndex& itemIndex, SignalCsr& byUser, SignalCsr& byItem, size_t nthreads) {
  const size_t nnz = dataset.size();
  std::vector<int64_t> uids(nnz), iids(nnz);
  ParallelExecutor px(nthreads);
  px.execute(nthreads, [&](const size_t t) {
    for (size_t e = nnz * t / nthreads; e < nnz * (t + 1) / nthreads; ++e) {
      uids[e] = dataset[e].userId;
      iids[e] = dataset[e].itemId;
    }
  });
  uids = sortedUnique(std::move(uids), nthreads);
  iids = sortedUnique(std::move(iids), nthreads);
  CHECK_LT(uids.size(), static_cast<size_t>(std::numeric_limits<int32_t>::max()));
  CHECK_LT(iids.size(), static_cast<size_t>(std::numeric_limits<int32_t>::max()));
  std::vector<int32_t> uidx(nnz), iidx(nnz);
  px.execute(nthreads, [&](const size_t t) {
    for (size_t e = nnz * t / nthreads; e < nnz * (t + 1) / nthreads; ++e) {
      uidx[e] = static_cast<int32_t>(
        std::lower_bound(uids.begin(), uids.end(), dataset[e].userId) - uids.begin());
      iidx[e] = static_cast<int32_t>(
        std::lower_bound(iids.begin(), iids.end(), dataset[e].itemId) - iids.begin());
    }
  });
  buildCsr(uidx, iidx, dataset, uids.size(), byUser, nthreads);
  buildCsr(iidx, uidx, dataset, iids.size(), byItem, nthreads);
  userIndex.assignSorted(std::move(uids));
  itemIndex.assignSorted(std::move(iids));
}

}  // namespace qmf
