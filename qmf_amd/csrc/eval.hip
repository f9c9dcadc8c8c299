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
//   eval_users_kernel  the test users' factor rows as doubles, [groups·32][k] (zero padded);
//   eval_rank_kernel   a tile of item rows staged through LDS, 32 test users per workgroup;
//                      each lane scores one item for the 8 users of its wave — their factor
//                      values are wave-uniform, read through the scalar cache straight into
//                      SGPR operands, so LDS only carries the item tile — accumulates Σ
//                      score², and counts, per positive of those users, the items scored
//                      above it (wave ballot + popcount into LDS counters, flushed once per
//                      chunk).
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
constexpr int EV_UW = 8;                // test users per wave
constexpr int EV_W = 4;                 // waves per workgroup
constexpr int EV_UG = EV_UW * EV_W;     // test users per workgroup
constexpr int EV_KC = 64;               // factor columns per LDS stage
constexpr int EV_CAP = 2048;            // positives of a workgroup counted in LDS
constexpr int EV_KMAX = 256;
constexpr int EV_TS = EV_KC + 2;        // tile row stride (even: 8-byte aligned pairs)

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
__global__ __launch_bounds__(256) void eval_users_kernel(EvalArgs<T> a) {
  // layout [t / 8][f][t % 8] (t relative to the batch's first user): one wave's 8 users at
  // factor f are 64 contiguous bytes
  const int64_t tr = blockIdx.x;
  const int64_t t = a.t_base + tr;
  const T* u = a.U + (t < a.ntest ? a.users[t] * (int64_t)a.kp : 0);
  double* o = a.udbl + (tr / EV_UW) * a.k * EV_UW + (tr % EV_UW);
  for (int f = threadIdx.x; f < a.k; f += blockDim.x)
    o[f * EV_UW] = t < a.ntest ? (double)u[f] : 0.0;
}

template <typename T>
__global__ __launch_bounds__(256) void eval_rank_kernel(EvalArgs<T> a) {
  __shared__ T tile[EV_TI * EV_TS];
  __shared__ uint32_t cnt[EV_CAP];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t0 = a.t_base + (int64_t)blockIdx.y * EV_UG;
  const int64_t tw = t0 + w * EV_UW;  // first user of this wave
  const int64_t i0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t i1 = i0 + a.chunk < a.nitems ? i0 + a.chunk : a.nitems;
  const int64_t tl = t0 + EV_UG < a.ntest ? t0 + EV_UG : a.ntest;
  const int64_t pb = a.pptr[t0], pe = a.pptr[tl];  // (scalar: kernel arguments only)
  // wave-uniform rows, read through the constant address space so they become scalar loads
  // (the kernel's own global stores would otherwise keep them on the vector path)
  typedef const __attribute__((address_space(4))) double* cdptr;
  const cdptr ud = (cdptr)(a.udbl + (tw - a.t_base) * a.k);  // [f][8] for this wave's users
  const cdptr ps = (cdptr)a.pscore;  // written by eval_label_kernel (an earlier launch)
  typedef const __attribute__((address_space(4))) int64_t* ciptr;
  const ciptr pp = (ciptr)a.pptr;

  for (int x = threadIdx.x; x < EV_CAP; x += 256) cnt[x] = 0;

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
        tile[r * EV_TS + cc] = (ib + r < i1 && cc < kc) ? a.I[(ib + r) * a.kp + f0 + cc] : (T)0;
      }
      __syncthreads();
      const T* q = &tile[lane * EV_TS];
      const cdptr u0 = ud + f0 * EV_UW;
      if (kc == EV_KC) {
        // full stage, fully unrolled: every user value is an s_load at an immediate offset
#pragma unroll
        for (int f = 0; f < EV_KC; ++f) {
          const double qf = (double)q[f];
#pragma unroll
          for (int g = 0; g < EV_UW; ++g) acc[g] = mul_add_rn(acc[g], u0[f * EV_UW + g], qf);
        }
      } else {
        for (int f = 0; f < kc; ++f) {
          const double qf = (double)q[f];
#pragma unroll
          for (int g = 0; g < EV_UW; ++g) acc[g] = mul_add_rn(acc[g], u0[f * EV_UW + g], qf);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < EV_UW; ++g) {
      const int64_t t = tw + g;
      if (t >= a.ntest) break;  // uniform over the wave
      const double s = acc[g];
      if (valid) sq[g] += s * s;
      const int64_t qb = pp[t], qe = pp[t + 1];
      // positives' scores through the scalar cache, four at a time
      for (int64_t p0 = qb; p0 < qe; p0 += 4) {
        double sp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) sp[j] = p0 + j < qe ? ps[p0 + j] : 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t p = p0 + j;
          if (p >= qe) break;
          const uint64_t m = __ballot(valid && s > sp[j]);
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
  }

  // Σ score² of each user over this chunk: fixed-order wave sum, one slot per (chunk, user)
#pragma unroll
  for (int g = 0; g < EV_UW; ++g) {
    const int64_t t = tw + g;
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
  // test users in batches of eval_batch_groups() groups (grid.y ≤ 65535; the users' fp64
  // rows in udbl are staged per batch)
  const int64_t bg = eval_batch_groups();
  for (int64_t g0 = 0; g0 < groups; g0 += bg) {
    const int64_t ng = groups - g0 < bg ? groups - g0 : bg;
    a.t_base = g0 * EV_UG;
    hipLaunchKernelGGL(eval_users_kernel<T>, dim3((unsigned)(ng * EV_UG)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(eval_rank_kernel<T>, dim3((unsigned)nchunk, (unsigned)ng), dim3(256), 0,
                       s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

// User groups (of EV_UG test users) per rank-kernel launch: the grid's y limit
// (QMFX_EVAL_BATCH_GROUPS lowers it for the tests).
int64_t eval_batch_groups() {
  int64_t g = 65535;
  if (const char* e = std::getenv("QMFX_EVAL_BATCH_GROUPS"))
    if (std::atoll(e) > 0 && std::atoll(e) < g) g = std::atoll(e);
  return g;
}

// rows of the per-batch fp64 user scratch (udbl)
int64_t eval_user_rows(int64_t ntest) {
  const int64_t rows = (ntest + EV_UG - 1) / EV_UG * EV_UG;
  const int64_t cap = eval_batch_groups() * EV_UG;
  return rows < cap ? rows : cap;
}

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
