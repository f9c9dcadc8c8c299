// Test-set ranking statistics on the device: the reference's evaluation step
// (Engine::computeTestScores, Engine.cpp:73-96, followed by the per-user metrics of
// Metrics.cpp:27-164) without the dense n_test × n_items score matrix.
//
// Every metric the reference offers (mse, auc, ap, p@k, r@k) is a function of, per test
// user: Σ_i (label_i − score_i)², the scores of the positives (label > 0), and for each
// positive the number of items scored strictly higher.  (Ties: the reference sorts
// (score, is_positive) pairs descending, so an equal-scored negative ranks below a positive
// and equal-scored positives are interchangeable.)  The device computes exactly those:
//
//   eval_label_kernel  one thread per labelled (user, item): its score;
//   eval_rank_kernel   a tile of item rows staged through LDS, 16 test users per workgroup;
//                      each lane scores one item for 4 users, accumulates Σ score², and
//                      counts, per positive of those users, the items scored above it
//                      (wave ballot + popcount into LDS counters, flushed once per chunk).
//
// Scores are formed as the reference does — bias (or 0), then one rounded multiply and one
// rounded add per factor in factor order, no fused multiply-add — so they equal the host's
// double scores bit for bit (the factors are the same values in fp32 or fp64 storage), and
// the rank counts are exact.  Bound: fp64 VALU (2 instructions per multiply-add).
#include "common.h"
#include "kernels.h"

namespace qmfx {
namespace {

constexpr int EV_TI = 64;               // items per tile (one per lane)
constexpr int EV_UW = 4;                // test users per wave
constexpr int EV_W = 4;                 // waves per workgroup
constexpr int EV_UG = EV_UW * EV_W;     // test users per workgroup
constexpr int EV_KC = 64;               // factor columns per LDS stage
constexpr int EV_CAP = 2048;            // positives of a workgroup counted in LDS
constexpr int EV_KMAX = 256;

#pragma clang fp contract(off)
__device__ __forceinline__ double mul_add_rn(double s, double a, double b) {
  const double p = a * b;
  return s + p;
}
#pragma clang fp contract(on)

template <typename T>
__global__ __launch_bounds__(256) void eval_label_kernel(EvalArgs<T> a) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= a.nlab) return;
  const int64_t i = a.lab_item[e];
  const T* u = a.U + a.users[a.lab_slot[e]] * (int64_t)a.kp;
  const T* q = a.I + i * (int64_t)a.kp;
  double s = a.bias ? (double)a.bias[i] : 0.0;
  for (int f = 0; f < a.k; ++f) s = mul_add_rn(s, (double)u[f], (double)q[f]);
  a.lab_score[e] = s;
  const int64_t p = a.lab_pidx[e];
  if (p >= 0) a.pscore[p] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void eval_rank_kernel(EvalArgs<T> a) {
  __shared__ T tile[EV_TI][EV_KC + 1];
  __shared__ double us[EV_UG][EV_KMAX];
  __shared__ uint32_t cnt[EV_CAP];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.y * EV_UG;
  const int64_t i0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t i1 = i0 + a.chunk < a.nitems ? i0 + a.chunk : a.nitems;
  const int64_t tl = t0 + EV_UG < a.ntest ? t0 + EV_UG : a.ntest;
  const int64_t pb = a.pptr[t0], pe = a.pptr[tl];

  for (int x = threadIdx.x; x < EV_CAP; x += 256) cnt[x] = 0;
  for (int x = threadIdx.x; x < EV_UG * a.k; x += 256) {
    const int g = x / a.k, f = x - g * a.k;
    us[g][f] = t0 + g < a.ntest ? (double)a.U[a.users[t0 + g] * (int64_t)a.kp + f] : 0.0;
  }

  double sq[EV_UW];
#pragma unroll
  for (int g = 0; g < EV_UW; ++g) sq[g] = 0.0;

  for (int64_t ib = i0; ib < i1; ib += EV_TI) {
    const int64_t item = ib + lane;
    const bool valid = item < i1;
    double acc[EV_UW];
    const double b0 = (a.bias && valid) ? (double)a.bias[item] : 0.0;
#pragma unroll
    for (int g = 0; g < EV_UW; ++g) acc[g] = b0;
    for (int f0 = 0; f0 < a.k; f0 += EV_KC) {
      const int kc = a.k - f0 < EV_KC ? a.k - f0 : EV_KC;
      __syncthreads();
      for (int x = threadIdx.x; x < EV_TI * EV_KC; x += 256) {
        const int r = x / EV_KC, cc = x - r * EV_KC;
        tile[r][cc] = (ib + r < i1 && cc < kc) ? a.I[(ib + r) * a.kp + f0 + cc] : (T)0;
      }
      __syncthreads();
      const double* u0 = &us[w * EV_UW][f0];
#pragma unroll 4
      for (int f = 0; f < kc; ++f) {
        const double q = (double)tile[lane][f];
#pragma unroll
        for (int g = 0; g < EV_UW; ++g) acc[g] = mul_add_rn(acc[g], u0[g * EV_KMAX + f], q);
      }
    }
#pragma unroll
    for (int g = 0; g < EV_UW; ++g) {
      const int64_t t = t0 + w * EV_UW + g;
      if (t >= a.ntest) break;  // uniform over the wave
      const double s = acc[g];
      if (valid) sq[g] += s * s;
      const int64_t qb = a.pptr[t], qe = a.pptr[t + 1];
      for (int64_t p = qb; p < qe; ++p) {
        const uint64_t m = __ballot(valid && s > a.pscore[p]);
        if (lane == 0 && m) {
          const uint32_t c = (uint32_t)__popcll(m);
          if (p - pb < EV_CAP)
            atomicAdd(&cnt[p - pb], c);
          else
            atomicAdd((unsigned long long*)&a.above[p], (unsigned long long)c);
        }
      }
    }
  }

  // Σ score² of each user over this chunk: fixed-order wave sum, one slot per (chunk, user)
#pragma unroll
  for (int g = 0; g < EV_UW; ++g) {
    const int64_t t = t0 + w * EV_UW + g;
    const double v = wave_sum(sq[g]);
    if (lane == 0 && t < a.ntest) a.sq_part[(int64_t)blockIdx.x * a.ntest + t] = v;
  }
  __syncthreads();
  const int64_t np = pe - pb < EV_CAP ? pe - pb : EV_CAP;
  for (int64_t x = threadIdx.x; x < np; x += 256)
    if (cnt[x]) atomicAdd((unsigned long long*)&a.above[pb + x], (unsigned long long)cnt[x]);
}

template <typename T>
hipError_t eval_ranks(const EvalArgs<T>& a0, hipStream_t s) {
  if (a0.k > EV_KMAX) return hipErrorInvalidValue;
  EvalArgs<T> a = a0;
  if (a.nlab > 0)
    hipLaunchKernelGGL(eval_label_kernel<T>, dim3((unsigned)((a.nlab + 255) / 256)), dim3(256),
                       0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || a.ntest == 0 || a.nitems == 0) return e;
  const int64_t groups = (a.ntest + EV_UG - 1) / EV_UG;
  const int64_t nchunk = eval_chunks(a.ntest, a.nitems);
  a.chunk = ((a.nitems + nchunk - 1) / nchunk + EV_TI - 1) / EV_TI * EV_TI;
  if (groups > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(eval_rank_kernel<T>, dim3((unsigned)nchunk, (unsigned)groups), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

}  // namespace

// Item chunks per user group: about 4096 workgroups over the grid, ≥ one tile per chunk.
// The host sizes the Σ score² partial buffer [chunks][ntest] with the same function.
int64_t eval_chunks(int64_t ntest, int64_t nitems) {
  const int64_t groups = (ntest + EV_UG - 1) / EV_UG;
  const int64_t tiles = (nitems + EV_TI - 1) / EV_TI;
  int64_t n = 4096 / (groups > 0 ? groups : 1);
  if (n < 1) n = 1;
  if (n > tiles) n = tiles;
  if (n < 1) n = 1;
  // the chunk is rounded up to whole tiles: drop chunks that would start past the end
  const int64_t chunk = ((nitems + n - 1) / n + EV_TI - 1) / EV_TI * EV_TI;
  return chunk > 0 ? (nitems + chunk - 1) / chunk : 1;
}

hipError_t launch_eval_ranks(const EvalArgs<float>& a, hipStream_t s) { return eval_ranks(a, s); }
hipError_t launch_eval_ranks(const EvalArgs<double>& a, hipStream_t s) { return eval_ranks(a, s); }

}  // namespace qmfx
