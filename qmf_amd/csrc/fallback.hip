// Rows whose system the Cholesky kernels cannot factor (a non-positive pivot: some
// 1 + αv < 0, λ ≤ 0, or fp32 rounding on a nearly singular system) are re-solved here, on
// the device, in fp64 with a pivoted factorization — what the reference's dsysv_ does for
// every row (Bunch-Kaufman LDLᵀ, Matrix.cpp:81-96; here Gaussian elimination with partial
// pivoting: the same solution to rounding, and the same failure on an exactly singular
// system, which the reference turns into CHECK(info == 0) and the ABI into an error).
//
// Reference: updateFactorsForOne, qmf/wals/WALSEngine.cpp:266-310
//   A = YᵀY + Σ α v y yᵀ + λI,  b = Σ (1 + α v) y,  x = A⁻¹b,
//   loss = Σ(1 + αv) + xᵀ(A − λI)x − 2xᵀb = Σ(1 + αv) − xᵀb − λ‖x‖²   (A x = b).
//
// Runs per solve piece, after the row kernels and before the piece's all-gather, so a
// re-solved row is broadcast like every other row.  Cost when no row failed: one pass over
// the piece's status words.  One 256-thread workgroup per failed row, the system in a
// per-workgroup fp64 scratch ((KP + 3)·KP doubles, L2-resident); signals are staged 16 at a
// time through LDS.
#include "common.h"
#include "kernels.h"

namespace qmfx {

namespace {

constexpr int FB_THREADS = 256;
constexpr int FB_CHUNK = 16;

__device__ double block_argmax_abs(const double* A, int KP, int j, int tid, double* red_v,
                                   int* red_i, int& piv) {
  double best = -1.0;
  int bi = j;
  for (int i = j + tid; i < KP; i += FB_THREADS) {
    const double v = fabs(A[(size_t)i * KP + j]);
    if (v > best) {
      best = v;
      bi = i;
    }
  }
  red_v[tid] = best;
  red_i[tid] = bi;
  __syncthreads();
  for (int s = FB_THREADS / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const double o = red_v[tid + s];
      const int oi = red_i[tid + s];
      // ties: the smallest row index (LAPACK's idamax convention)
      if (o > red_v[tid] || (o == red_v[tid] && oi < red_i[tid])) {
        red_v[tid] = o;
        red_i[tid] = oi;
      }
    }
    __syncthreads();
  }
  piv = red_i[0];
  const double r = red_v[0];
  __syncthreads();
  return r;
}

// Builds A (KP×KP, row-major; padding diagonal 1), b and Σc of `row` into scratch.
template <typename T>
__device__ void build_system(const FallbackArgs<T>& a, int64_t beg, int64_t end, double* A,
                             double* b, double& csum, double (*ys)[256], double* ws,
                             double* cs, int tid) {
  const int KP = a.kp, k = a.k;
  for (int idx = tid; idx < KP * KP; idx += FB_THREADS) {
    const int i = idx / KP, j = idx % KP;
    double v = (i < k && j < k) ? (double)a.G[idx] : 0.0;
    if (i == j) v += i < k ? (double)a.lambda : 1.0;
    A[idx] = v;
  }
  for (int i = tid; i < KP; i += FB_THREADS) b[i] = 0.0;
  double cacc = 0.0;
  __syncthreads();
  for (int64_t base = beg; base < end; base += FB_CHUNK) {
    const int m = (int)(end - base < FB_CHUNK ? end - base : FB_CHUNK);
    for (int idx = tid; idx < FB_CHUNK * KP; idx += FB_THREADS) {
      const int e = idx / KP, j = idx % KP;
      ys[e][j] = (e < m && j < k) ? (double)a.Y[(size_t)(uint32_t)a.col[base + e] * KP + j] : 0.0;
    }
    if (tid < FB_CHUNK) {
      const double v = tid < m ? (double)a.val[base + tid] : 0.0;
      ws[tid] = tid < m ? (double)a.alpha * v : 0.0;
      cs[tid] = tid < m ? 1.0 + (double)a.alpha * v : 0.0;
    }
    __syncthreads();
    for (int idx = tid; idx < KP * KP; idx += FB_THREADS) {
      const int i = idx / KP, j = idx % KP;
      double s = 0.0;
#pragma unroll
      for (int e = 0; e < FB_CHUNK; ++e) s += ws[e] * ys[e][i] * ys[e][j];
      A[idx] += s;
    }
    for (int i = tid; i < KP; i += FB_THREADS) {
      double s = 0.0;
#pragma unroll
      for (int e = 0; e < FB_CHUNK; ++e) s += cs[e] * ys[e][i];
      b[i] += s;
    }
    if (tid == 0)
      for (int e = 0; e < m; ++e) cacc += cs[e];
    __syncthreads();
  }
  csum = cacc;  // valid on thread 0
}

}  // namespace

// Scans slots [slot_begin, slot_begin + nslots) of the order list; each workgroup takes a
// contiguous share and solves its flagged rows one after another.
template <typename T>
__global__ __launch_bounds__(FB_THREADS) void wals_fallback_kernel(FallbackArgs<T> a) {
  __shared__ double ys[FB_CHUNK][256];
  __shared__ double ws[FB_CHUNK], cs[FB_CHUNK];
  __shared__ double red_v[FB_THREADS];
  __shared__ int red_i[FB_THREADS];
  __shared__ int list[FB_THREADS];
  __shared__ int nlist;
  __shared__ int sing;
  const int tid = threadIdx.x;
  const int KP = a.kp;
  double* A = a.scratch + (size_t)blockIdx.x * (size_t)(KP + 3) * KP;
  double* b = A + (size_t)KP * KP;
  double* b0 = b + KP;
  double* x = b0 + KP;
  const int64_t share = (a.nslots + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = a.slot_begin + share * blockIdx.x;
  const int64_t s1 = min(a.slot_begin + a.nslots, s0 + share);
  for (int64_t base = s0; base < s1; base += FB_THREADS) {
    if (tid == 0) nlist = 0;
    __syncthreads();
    const int64_t slot = base + tid;
    if (slot < s1 && a.status[a.desc[slot].row] != 0) list[atomicAdd(&nlist, 1)] = (int)(slot - base);
    __syncthreads();
    const int cnt = nlist;
    for (int li = 0; li < cnt; ++li) {
      const RowDesc d = a.desc[base + list[li]];
      double csum = 0.0;
      build_system<T>(a, d.beg, d.beg + d.n, A, b, csum, ys, ws, cs, tid);
      for (int i = tid; i < KP; i += FB_THREADS) b0[i] = b[i];
      if (tid == 0) sing = 0;
      __syncthreads();
      // Gaussian elimination with partial pivoting, rows swapped in place
      for (int j = 0; j < KP; ++j) {
        int p = j;
        const double pv = block_argmax_abs(A, KP, j, tid, red_v, red_i, p);
        if (pv == 0.0) {
          if (tid == 0) sing = 1;
          break;
        }
        if (p != j) {
          for (int m = j + tid; m < KP; m += FB_THREADS) {
            const double t = A[(size_t)j * KP + m];
            A[(size_t)j * KP + m] = A[(size_t)p * KP + m];
            A[(size_t)p * KP + m] = t;
          }
          if (tid == 0) {
            const double t = b[j];
            b[j] = b[p];
            b[p] = t;
          }
        }
        __syncthreads();
        const double inv = 1.0 / A[(size_t)j * KP + j];
        for (int i = j + 1 + tid; i < KP; i += FB_THREADS) A[(size_t)i * KP + j] *= inv;
        __syncthreads();
        const int m = KP - j - 1;
        for (int idx = tid; idx < m * m; idx += FB_THREADS) {
          const int i = j + 1 + idx / m, c = j + 1 + idx % m;
          A[(size_t)i * KP + c] -= A[(size_t)i * KP + j] * A[(size_t)j * KP + c];
        }
        for (int i = j + 1 + tid; i < KP; i += FB_THREADS) b[i] -= A[(size_t)i * KP + j] * b[j];
        __syncthreads();
      }
      __syncthreads();
      const bool singular = sing != 0;
      // back substitution, column-oriented
      if (!singular) {
        for (int i = KP - 1; i >= 0; --i) {
          if (tid == 0) x[i] = b[i] / A[(size_t)i * KP + i];
          __syncthreads();
          const double xi = x[i];
          for (int r = tid; r < i; r += FB_THREADS) b[r] -= A[(size_t)r * KP + i] * xi;
          __syncthreads();
        }
      }
      double xb = 0.0, xx = 0.0;
      for (int i = tid; i < KP; i += FB_THREADS) {
        const double xi = singular ? 0.0 : x[i];
        a.X[(size_t)d.row * KP + i] = (T)xi;
        xb += xi * b0[i];
        xx += xi * xi;
      }
      red_v[tid] = xb;
      __syncthreads();
      for (int s = FB_THREADS / 2; s > 0; s >>= 1) {
        if (tid < s) red_v[tid] += red_v[tid + s];
        __syncthreads();
      }
      xb = red_v[0];
      __syncthreads();
      red_v[tid] = xx;
      __syncthreads();
      for (int s = FB_THREADS / 2; s > 0; s >>= 1) {
        if (tid < s) red_v[tid] += red_v[tid + s];
        __syncthreads();
      }
      xx = red_v[0];
      if (tid == 0) {
        a.rowloss[d.row] = singular ? 0.0 : csum - xb - (double)a.lambda * xx;
        a.status[d.row] = singular ? 2 : 1;
        atomicAdd((unsigned long long*)&a.counters[0], 1ull);
        if (singular) atomicAdd((unsigned long long*)&a.counters[1], 1ull);
      }
      __syncthreads();
    }
  }
}

// A (k×k row-major, λ included), b and Σc of one row, for qmfx_wals_row_system.
template <typename T>
__global__ __launch_bounds__(FB_THREADS) void wals_system_kernel(FallbackArgs<T> a, int64_t beg,
                                                                 int64_t end, double* out) {
  __shared__ double ys[FB_CHUNK][256];
  __shared__ double ws[FB_CHUNK], cs[FB_CHUNK];
  const int tid = threadIdx.x;
  const int KP = a.kp, k = a.k;
  double* A = a.scratch;
  double* b = A + (size_t)KP * KP;
  double csum = 0.0;
  build_system<T>(a, beg, end, A, b, csum, ys, ws, cs, tid);
  __syncthreads();
  for (int idx = tid; idx < k * k; idx += FB_THREADS)
    out[idx] = A[(size_t)(idx / k) * KP + idx % k];
  for (int i = tid; i < k; i += FB_THREADS) out[(size_t)k * k + i] = b[i];
  if (tid == 0) out[(size_t)k * k + k] = csum;
}

// End-of-half status in one block for one async copy to pinned host memory: the loss sum,
// the re-solved and singular row counts, and the YᵀY + λI factorization flag.
__global__ void half_status_kernel(const double* loss, const unsigned long long* fb,
                                   const int32_t* chol, double* out) {
  if (threadIdx.x == 0) {
    out[0] = loss[0];
    out[1] = (double)fb[0];
    out[2] = (double)fb[1];
    out[3] = chol ? (double)chol[0] : 0.0;
  }
}

hipError_t launch_half_status(const double* loss, const unsigned long long* fb,
                              const int32_t* chol, double* out, hipStream_t s) {
  hipLaunchKernelGGL(half_status_kernel, dim3(1), dim3(64), 0, s, loss, fb, chol, out);
  return hipGetLastError();
}

int fallback_grid(int64_t nslots) {
  const int64_t g = (nslots + 4095) / 4096;
  return (int)(g < 1 ? 1 : (g > FB_MAX_GRID ? FB_MAX_GRID : g));
}

template <typename T>
static hipError_t fallback(const FallbackArgs<T>& a, hipStream_t s) {
  if (a.nslots <= 0) return hipSuccess;
  if (a.kp > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wals_fallback_kernel<T>, dim3(fallback_grid(a.nslots)), dim3(FB_THREADS), 0,
                     s, a);
  return hipGetLastError();
}
template <typename T>
static hipError_t system(const FallbackArgs<T>& a, int64_t beg, int64_t end, double* out,
                         hipStream_t s) {
  if (a.kp > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wals_system_kernel<T>, dim3(1), dim3(FB_THREADS), 0, s, a, beg, end, out);
  return hipGetLastError();
}

hipError_t launch_wals_fallback(const FallbackArgs<float>& a, hipStream_t s) { return fallback(a, s); }
hipError_t launch_wals_fallback(const FallbackArgs<double>& a, hipStream_t s) { return fallback(a, s); }
hipError_t launch_wals_system(const FallbackArgs<float>& a, int64_t beg, int64_t end, double* out,
                              hipStream_t s) {
  return system(a, beg, end, out, s);
}
hipError_t launch_wals_system(const FallbackArgs<double>& a, int64_t beg, int64_t end,
                              double* out, hipStream_t s) {
  return system(a, beg, end, out, s);
}

}  // namespace qmfx
