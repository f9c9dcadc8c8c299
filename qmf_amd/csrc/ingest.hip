// Device ingest: raw (user id, item id, value) records → the two CSR orientations and the
// ascending id tables, on the GPU.
//
// Reference (taozhijiang/qmf):
//   WALSEngine::init             qmf/wals/WALSEngine.cpp:37-69   (index build + grouping)
//   WALSEngine::groupSignals     qmf/wals/WALSEngine.cpp:130-150 (std::sort by (id, id), group)
//   WALSEngine::sortDataset      qmf/wals/WALSEngine.cpp:152-163
//   IdIndex (idx = rank of the id among the distinct ids)  qmf/utils/IdIndex.cpp:21-31
//
// Same result as the host restatement (host/qmf/wals/Signals.cpp): rows in ascending-id
// order, each row's entries by ascending column id, duplicates of a (u, i) pair kept in
// input order.  Here that is
//   1. distinct ids per side: radix sort of the signed 64-bit ids + unique;
//   2. idx of every record on both sides: a lower bound in the id table;
//   3. per orientation, a STABLE radix sort of the 64-bit keys (row idx << 32 | col idx)
//      carrying the record position, so equal keys (duplicates) keep input order;
//   4. rowptr by a lower bound per row, col = low word of the key, val = value[position].
// Records cross the ABI in the reference's packed 24-byte DatasetElem layout
// (qmf/DatasetReader.h:29-33: int64 userId, int64 itemId, double value).
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "kernels.h"

namespace qmfx {

namespace {

inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// packed 24-byte records → user ids, item ids (and the value, in the context precision)
template <typename T>
__global__ void unpack_records_kernel(const uint64_t* rec, int64_t n, int64_t* uid,
                                      int64_t* iid, T* val) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint64_t* r = rec + 3 * e;
  uid[e] = (int64_t)r[0];
  iid[e] = (int64_t)r[1];
  val[e] = (T)__longlong_as_double((long long)r[2]);
}

// idx[e] = rank of id[e] in the ascending table (the id is present)
__global__ void rank_ids_kernel(const int64_t* id, int64_t n, const int64_t* table,
                                int64_t m, int32_t* idx) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t x = id[e];
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (table[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  idx[e] = (int32_t)lo;
}

__global__ void make_keys_kernel(const int32_t* row, const int32_t* col, int64_t n,
                                 uint64_t* key, int32_t* pos) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  key[e] = ((uint64_t)(uint32_t)row[e] << 32) | (uint32_t)col[e];
  pos[e] = (int32_t)e;
}

// rowptr[r] = first position whose key's row ≥ r (r = 0..nrows)
__global__ void rowptr_kernel(const uint64_t* key, int64_t n, int64_t nrows, int64_t* rowptr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  const uint64_t target = (uint64_t)r << 32;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = lo;
}

template <typename T>
__global__ void gather_entries_kernel(const uint64_t* key, const int32_t* pos, const T* val,
                                      int64_t n, int32_t* col, T* out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  col[p] = (int32_t)(uint32_t)key[p];
  out[p] = val[pos[p]];
}

int bits_for(int64_t n) {  // bits needed for the values 0..n-1
  int b = 1;
  while (b < 62 && ((int64_t)1 << b) < n) ++b;
  return b;
}

struct DevTmp {  // hipcub temporary storage, grown on demand
  void* p = nullptr;
  size_t cap = 0;
  hipError_t need(size_t b) {
    if (b <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, b);
    if (e == hipSuccess) cap = b;
    return e;
  }
  ~DevTmp() {
    if (p) (void)hipFree(p);
  }
};

#define IGCHK(x)                     \
  do {                               \
    hipError_t e_ = (x);             \
    if (e_ != hipSuccess) return e_; \
  } while (0)

// distinct ids of `id` (ascending, signed order) → *table (allocated here, ≥ *m entries)
hipError_t distinct_ids(const int64_t* id, int64_t n, int64_t** table, int64_t* m, DevTmp& tmp,
                        hipStream_t s) {
  int64_t *sorted = nullptr, *uniq = nullptr;
  IGCHK(hipMalloc(&sorted, (size_t)n * 8));
  IGCHK(hipMalloc(&uniq, (size_t)n * 8 + 16));
  *table = uniq;  // owned by the caller from here on
  int64_t* d_num = uniq + n;
  size_t t1 = 0, t2 = 0;
  IGCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, id, sorted, (int)n, 0, 64, s));
  IGCHK(hipcub::DeviceSelect::Unique(nullptr, t2, sorted, uniq, d_num, (int)n, s));
  IGCHK(tmp.need(t1 > t2 ? t1 : t2));
  t1 = t2 = tmp.cap;
  IGCHK(hipcub::DeviceRadixSort::SortKeys(tmp.p, t1, id, sorted, (int)n, 0, 64, s));
  IGCHK(hipcub::DeviceSelect::Unique(tmp.p, t2, sorted, uniq, d_num, (int)n, s));
  IGCHK(hipMemcpyAsync(m, d_num, 8, hipMemcpyDeviceToHost, s));
  IGCHK(hipStreamSynchronize(s));
  (void)hipFree(sorted);
  return hipSuccess;
}

// one orientation: rows by `row` idx (nrows of them), entries by `col` idx
template <typename T>
hipError_t orient(const int32_t* row, const int32_t* col, const T* val, int64_t n,
                  int64_t nrows, int64_t* rowptr, int32_t* out_col, T* out_val, DevTmp& tmp,
                  hipStream_t s) {
  uint64_t *k0 = nullptr, *k1 = nullptr;
  int32_t *p0 = nullptr, *p1 = nullptr;
  IGCHK(hipMalloc(&k0, (size_t)n * 8));
  IGCHK(hipMalloc(&k1, (size_t)n * 8));
  IGCHK(hipMalloc(&p0, (size_t)n * 4));
  IGCHK(hipMalloc(&p1, (size_t)n * 4));
  hipLaunchKernelGGL(make_keys_kernel, dim3(nblk(n)), dim3(256), 0, s, row, col, n, k0, p0);
  IGCHK(hipGetLastError());
  // the sort covers the column word and the row's bits; LSD radix sort is stable
  const int end_bit = 32 + bits_for(nrows);
  size_t t = 0;
  IGCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t, k0, k1, p0, p1, (int)n, 0, end_bit, s));
  IGCHK(tmp.need(t));
  t = tmp.cap;
  IGCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, t, k0, k1, p0, p1, (int)n, 0, end_bit, s));
  hipLaunchKernelGGL(rowptr_kernel, dim3(nblk(nrows + 1)), dim3(256), 0, s, k1, n, nrows, rowptr);
  IGCHK(hipGetLastError());
  hipLaunchKernelGGL((gather_entries_kernel<T>), dim3(nblk(n)), dim3(256), 0, s, k1, p1, val, n,
                     out_col, out_val);
  IGCHK(hipGetLastError());
  IGCHK(hipStreamSynchronize(s));
  (void)hipFree(k0);
  (void)hipFree(k1);
  (void)hipFree(p0);
  (void)hipFree(p1);
  return hipSuccess;
}

template <typename T>
hipError_t group_records_t(const void* d_records, int64_t n, IngestOut& o, hipStream_t s) {
  DevTmp tmp;
  int64_t *uid = nullptr, *iid = nullptr;
  T* val = nullptr;
  IGCHK(hipMalloc(&uid, (size_t)n * 8));
  IGCHK(hipMalloc(&iid, (size_t)n * 8));
  IGCHK(hipMalloc(&val, (size_t)n * sizeof(T)));
  hipLaunchKernelGGL((unpack_records_kernel<T>), dim3(nblk(n)), dim3(256), 0, s,
                     (const uint64_t*)d_records, n, uid, iid, val);
  IGCHK(hipGetLastError());
  IGCHK(distinct_ids(uid, n, &o.ids[0], &o.n[0], tmp, s));
  IGCHK(distinct_ids(iid, n, &o.ids[1], &o.n[1], tmp, s));
  if (o.n[0] > 0x7fffffffll || o.n[1] > 0x7fffffffll) return hipErrorInvalidValue;
  int32_t *uidx = nullptr, *iidx = nullptr;
  IGCHK(hipMalloc(&uidx, (size_t)n * 4));
  IGCHK(hipMalloc(&iidx, (size_t)n * 4));
  hipLaunchKernelGGL(rank_ids_kernel, dim3(nblk(n)), dim3(256), 0, s, uid, n, o.ids[0], o.n[0], uidx);
  hipLaunchKernelGGL(rank_ids_kernel, dim3(nblk(n)), dim3(256), 0, s, iid, n, o.ids[1], o.n[1], iidx);
  IGCHK(hipGetLastError());
  IGCHK(hipStreamSynchronize(s));
  (void)hipFree(uid);
  (void)hipFree(iid);
  for (int side = 0; side < 2; ++side) {
    IGCHK(hipMalloc(&o.rowptr[side], (size_t)(o.n[side] + 1) * 8));
    IGCHK(hipMalloc(&o.col[side], (size_t)n * 4));
    IGCHK(hipMalloc(&o.val[side], (size_t)n * sizeof(T)));
  }
  IGCHK(orient<T>(uidx, iidx, val, n, o.n[0], o.rowptr[0], o.col[0], (T*)o.val[0], tmp, s));
  IGCHK(orient<T>(iidx, uidx, val, n, o.n[1], o.rowptr[1], o.col[1], (T*)o.val[1], tmp, s));
  (void)hipFree(uidx);
  (void)hipFree(iidx);
  (void)hipFree(val);
  return hipSuccess;
}

}  // namespace

hipError_t group_records(const void* d_records, int64_t n, int prec, IngestOut& out,
                         hipStream_t s) {
  if (n <= 0 || n > 0x7fffffffll) return hipErrorInvalidValue;  // hipcub: int item counts
  return prec == 32 ? group_records_t<float>(d_records, n, out, s)
                    : group_records_t<double>(d_records, n, out, s);
}

}  // namespace qmfx
