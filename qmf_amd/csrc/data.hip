// Device-side data preparation: synthetic interaction matrices (SURVEY.md §8(d) recipe:
// uniform (u, i) pairs without replacement, w ∈ 1..5), CSR construction from sorted
// 64-bit (row, col) keys in both orientations, and uniform factor initialisation.
//
// The reference builds its per-user / per-item signal groups by std::sort of the dataset
// (WALSEngine.cpp:130-163); here, for data generated on the device, the same "sort by
// (row id, col id), group by row" is a radix sort of 64-bit keys followed by a
// lower-bound per row.  Row and column indices are the ids, so id ordering is preserved.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "kernels.h"

namespace qmfx {

__global__ void synth_keys_kernel(uint64_t* keys, int64_t n, uint64_t space, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = mix64(seed ^ mix64((uint64_t)i));
  keys[i] = (uint64_t)(((unsigned __int128)h * space) >> 64);
}

// Skewed variant (SURVEY.md §8(d) "Zipf(s) item popularity"): the user is uniform, the item
// rank r follows the continuous Zipf(s) inverse CDF on [1, nitems + 1) (s = 1:
// P(r) = ln((r+2)/(r+1)) / ln(nitems+1)), and ranks are scattered over item ids by the
// bijection item = (pa·r + pb) mod nitems (gcd(pa, nitems) = 1), so popular items are not
// all at the low ids.
__global__ void synth_keys_zipf_kernel(uint64_t* keys, int64_t n, uint64_t nusers,
                                       uint64_t nitems, double s, uint64_t pa, uint64_t pb,
                                       uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h1 = mix64(seed ^ mix64((uint64_t)i));
  const uint64_t h2 = mix64(h1 ^ 0x2545f4914f6cdd1dull);
  const uint64_t u = (uint64_t)(((unsigned __int128)h1 * nusers) >> 64);
  const double u01 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
  const double top = (double)nitems + 1.0;
  double x;
  if (fabs(s - 1.0) < 1e-12) {
    x = exp(u01 * log(top));
  } else {
    const double e = 1.0 - s;
    x = pow((pow(top, e) - 1.0) * u01 + 1.0, 1.0 / e);
  }
  uint64_t r = x >= 1.0 ? (uint64_t)x - 1 : 0;
  if (r >= nitems) r = nitems - 1;
  const uint64_t it = (uint64_t)(((unsigned __int128)pa * r + pb) % nitems);
  keys[i] = u * nitems + it;
}

__global__ void rowptr_from_keys_kernel(const uint64_t* keys, int64_t nnz, int64_t nrows,
                                        uint64_t ncols, int64_t* rowptr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  const uint64_t target = (uint64_t)r * ncols;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = lo;
}

__global__ void col_from_keys_kernel(const uint64_t* keys, int64_t nnz, uint64_t ncols,
                                     int32_t* col) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nnz) col[i] = (int32_t)(keys[i] % ncols);
}

// key = row·ncols + col  →  transposed key = col·nrows + row
__global__ void transpose_keys_kernel(const uint64_t* keys, int64_t nnz, uint64_t ncols,
                                      uint64_t nrows, uint64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nnz) out[i] = (keys[i] % ncols) * nrows + keys[i] / ncols;
}

// value of pair (u, i) = 1 + hash(u·nitems + i) mod 5, identical in both orientations.
template <typename T>
__global__ void synth_values_kernel(const uint64_t* keys, int64_t n, uint64_t div,
                                    uint64_t nitems, int user_major, uint64_t seed, T* val) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint64_t a = keys[e] / div, b = keys[e] % div;
  const uint64_t u = user_major ? a : b, it = user_major ? b : a;
  val[e] = (T)(1 + mix64(seed ^ (u * nitems + it)) % 5);
}

template <typename T>
__global__ void fill_uniform_kernel(T* X, int64_t n, int kp, int k, double bound, uint64_t seed) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * kp) return;
  const int64_t r = idx / kp;
  const int c = (int)(idx % kp);
  if (c >= k) {
    X[idx] = T(0);
    return;
  }
  const uint64_t h = mix64(seed ^ mix64((uint64_t)(r * k + c)));
  const double u01 = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  X[idx] = (T)((2.0 * u01 - 1.0) * bound);
}

static inline unsigned nb(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_synth_keys(uint64_t* keys, int64_t n, uint64_t space, uint64_t seed,
                             hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(synth_keys_kernel, dim3(nb(n)), dim3(256), 0, s, keys, n, space, seed);
  return hipGetLastError();
}

hipError_t launch_synth_keys_zipf(uint64_t* keys, int64_t n, uint64_t nusers, uint64_t nitems,
                                  double zipf_s, uint64_t seed, hipStream_t s) {
  // a multiplier coprime to nitems near nitems·(golden ratio − 1)
  uint64_t pa = (uint64_t)((double)nitems * 0.6180339887498949) | 1ull;
  auto gcd = [](uint64_t a, uint64_t b) {
    while (b) {
      const uint64_t t = a % b;
      a = b;
      b = t;
    }
    return a;
  };
  if (nitems <= 1) pa = 1;
  while (nitems > 1 && gcd(pa, nitems) != 1) pa += 2;
  const uint64_t pb = mix64(seed ^ 0x7a1full) % (nitems ? nitems : 1);
  if (n > 0)
    hipLaunchKernelGGL(synth_keys_zipf_kernel, dim3(nb(n)), dim3(256), 0, s, keys, n, nusers,
                       nitems, zipf_s, pa % (nitems ? nitems : 1), pb, seed);
  return hipGetLastError();
}

hipError_t build_csr_from_sorted_keys(const uint64_t* keys, int64_t nnz, int64_t nrows,
                                      uint64_t ncols, int64_t* rowptr, int32_t* col,
                                      hipStream_t s) {
  hipLaunchKernelGGL(rowptr_from_keys_kernel, dim3(nb(nrows + 1)), dim3(256), 0, s, keys, nnz,
                     nrows, ncols, rowptr);
  if (nnz > 0)
    hipLaunchKernelGGL(col_from_keys_kernel, dim3(nb(nnz)), dim3(256), 0, s, keys, nnz, ncols, col);
  return hipGetLastError();
}

hipError_t launch_transpose_keys(const uint64_t* keys, int64_t nnz, uint64_t ncols,
                                 uint64_t nrows, uint64_t* out, hipStream_t s) {
  if (nnz > 0)
    hipLaunchKernelGGL(transpose_keys_kernel, dim3(nb(nnz)), dim3(256), 0, s, keys, nnz, ncols,
                       nrows, out);
  return hipGetLastError();
}

template <typename T>
static hipError_t synth_values(const uint64_t* keys, int64_t n, uint64_t div, uint64_t nitems,
                               int user_major, uint64_t seed, T* val, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL((synth_values_kernel<T>), dim3(nb(n)), dim3(256), 0, s, keys, n, div,
                       nitems, user_major, seed, val);
  return hipGetLastError();
}
hipError_t launch_synth_values_any(const uint64_t* keys, int64_t n, uint64_t div,
                                   uint64_t nitems, int user_major, uint64_t seed, void* val,
                                   int prec, hipStream_t s) {
  return prec == 32 ? synth_values<float>(keys, n, div, nitems, user_major, seed, (float*)val, s)
                    : synth_values<double>(keys, n, div, nitems, user_major, seed, (double*)val, s);
}

hipError_t launch_fill_uniform_f32(float* X, int64_t n, int kp, int k, double bound,
                                   uint64_t seed, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(fill_uniform_kernel<float>, dim3(nb(n * kp)), dim3(256), 0, s, X, n, kp, k,
                       bound, seed);
  return hipGetLastError();
}
hipError_t launch_fill_uniform_f64(double* X, int64_t n, int kp, int k, double bound,
                                   uint64_t seed, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(fill_uniform_kernel<double>, dim3(nb(n * kp)), dim3(256), 0, s, X, n, kp,
                       k, bound, seed);
  return hipGetLastError();
}

// Radix sort of 64-bit keys (in place via a scratch buffer of equal size) and in-place
// unique; *n_out receives the unique count.  `scratch` must hold n keys.
hipError_t sort_unique_keys(uint64_t* keys, uint64_t* scratch, int64_t n, int64_t* n_out,
                            int end_bit, hipStream_t s) {
  size_t tmp_sort = 0, tmp_uniq = 0;
  // hipcub takes int item counts; sort in one call when n fits, else fail loudly.
  if (n > 0x7fffffffll) return hipErrorInvalidValue;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_sort, keys, scratch, (int)n, 0, end_bit, s);
  if (e != hipSuccess) return e;
  int64_t* d_num = nullptr;
  e = hipcub::DeviceSelect::Unique(nullptr, tmp_uniq, scratch, keys, d_num, (int)n, s);
  if (e != hipSuccess) return e;
  const size_t tmp = tmp_sort > tmp_uniq ? tmp_sort : tmp_uniq;
  void* d_tmp = nullptr;
  const size_t num_off = (tmp + 15) & ~(size_t)15;
  if ((e = hipMallocAsync(&d_tmp, num_off + 64, s)) != hipSuccess) return e;
  d_num = (int64_t*)((char*)d_tmp + num_off);
  e = hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp_sort, keys, scratch, (int)n, 0, end_bit, s);
  if (e == hipSuccess) e = hipcub::DeviceSelect::Unique(d_tmp, tmp_uniq, scratch, keys, d_num, (int)n, s);
  if (e == hipSuccess) e = hipMemcpyAsync(n_out, d_num, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFreeAsync(d_tmp, s);
  return e;
}

// Stable sort of keys only (for the transposed orientation; keys are unique already).
hipError_t sort_keys(uint64_t* keys, uint64_t* scratch, int64_t n, int end_bit, hipStream_t s) {
  if (n > 0x7fffffffll) return hipErrorInvalidValue;
  size_t tmp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, keys, scratch, (int)n, 0, end_bit, s);
  if (e != hipSuccess) return e;
  void* d_tmp = nullptr;
  if ((e = hipMallocAsync(&d_tmp, tmp + 16, s)) != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp, keys, scratch, (int)n, 0, end_bit, s);
  if (e == hipSuccess) e = hipMemcpyAsync(keys, scratch, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s);
  (void)hipFreeAsync(d_tmp, s);
  return e;
}

}  // namespace qmfx
