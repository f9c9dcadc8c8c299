// BPR hot path on MI355X: Hogwild! SGD over (user, positive, negative) triplets.
//
// Reference (taozhijiang/qmf):
//   BPREngine::update             qmf/bpr/BPREngine.cpp:178-220
//   predictDifference/loss/deriv  qmf/bpr/BPREngine.cpp:222-244
//   optimize / iterateBlock       qmf/bpr/BPREngine.cpp:146-176, BPREngine-inl.h:31-46
//   sampleRandomNegative          qmf/bpr/BPREngine-inl.h:48-60
//
// One wave64 owns one positive at a time; lanes hold factor elements (KP ≤ 64·E).  The
// user's positive item set is staged in registers (64 per pass) so the rejection test of a
// sampled negative is one compare + ballot instead of a hash probe.  Waves update factor
// rows without locks (Hogwild, as the reference's threads do); within a wave the update
// order matches BPREngine::update exactly (p_u from the old q, q_i / q_n from the new p_u).
#include "common.h"
#include "kernels.h"

namespace qmfx {

template <typename T, int E>
struct Row {
  T v[E];
};

// Factor rows and biases are shared by all waves of the epoch (Hogwild).  The per-CU vector
// L1 is not coherent across CUs: a plain load can return a row another CU updated long
// ago, and writing it back would erase that update.  Relaxed agent-scope atomics go to the
// coherent L2 (no ordering is implied, exactly Hogwild's contract).
template <typename T>
__device__ __forceinline__ T ld_shared(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_shared(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int E>
__device__ __forceinline__ void load_row(Row<T, E>& r, const T* base, int lane, int kp) {
#pragma unroll
  for (int e = 0; e < E; ++e)
    r.v[e] = (lane + 64 * e < kp) ? ld_shared(base + lane + 64 * e) : T(0);
}
template <typename T, int E>
__device__ __forceinline__ void store_row(const Row<T, E>& r, T* base, int lane, int kp) {
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (lane + 64 * e < kp) st_shared(base + lane + 64 * e, r.v[e]);
}

// One SGD step on (u, p, n).  Returns false if the derivative was not finite.
template <typename T, int E>
__device__ __forceinline__ bool bpr_step(const BprArgs<T>& a, int64_t u, int64_t p, int64_t n,
                                         int lane) {
  const int kp = a.kp;
  Row<T, E> pu, qp, qn;
  load_row(pu, a.U + u * kp, lane, kp);
  load_row(qp, a.I + p * kp, lane, kp);
  load_row(qn, a.I + n * kp, lane, kp);
  T part = T(0);
#pragma unroll
  for (int e = 0; e < E; ++e) part += pu.v[e] * (qp.v[e] - qn.v[e]);
  T x = wave_sum(part);
  T bp = T(0), bn = T(0);
  if (a.use_biases) {
    bp = ld_shared(a.bias + p);
    bn = ld_shared(a.bias + n);
    x += bp - bn;
  }
  const T ex = exp(x);
  const T eg = T(1) / (T(1) + ex);
  if (!isfinite(eg)) return false;
  const T lr = a.lr;
  if (a.use_biases && lane == 0) {
    st_shared(a.bias + p, bp + lr * (eg - a.bias_lambda * bp));
    st_shared(a.bias + n, bn + lr * (-eg - a.bias_lambda * bn));
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const T pu_new = pu.v[e] + lr * (eg * (qp.v[e] - qn.v[e]) - a.user_lambda * pu.v[e]);
    const T qp_new = qp.v[e] + lr * (eg * pu_new - a.item_lambda * qp.v[e]);
    const T qn_new = qn.v[e] + lr * (-eg * pu_new - a.item_lambda * qn.v[e]);
    pu.v[e] = pu_new;
    qp.v[e] = qp_new;
    qn.v[e] = qn_new;
  }
  store_row(pu, a.U + u * kp, lane, kp);
  store_row(qp, a.I + p * kp, lane, kp);
  store_row(qn, a.I + n * kp, lane, kp);
  return true;
}

// Rejection-samples a negative for user u: uniform in [0, nitems) and not in the user's
// positive set (sorted list urowptr/uitems).  Counter-based, so every (positive, j) draw is
// reproducible for a given seed.
__device__ __forceinline__ int64_t sample_negative(const int32_t* items, int64_t cnt,
                                                   int64_t nitems, uint64_t key, int lane) {
  for (uint32_t attempt = 0;; ++attempt) {
    const uint64_t h = mix64(key ^ ((uint64_t)attempt << 48) ^ 0x5bd1e995ull);
    const int64_t cand = (int64_t)(((unsigned __int128)h * (uint64_t)nitems) >> 64);
    bool hit = false;
    for (int64_t base = 0; base < cnt; base += 64) {
      const int64_t j = base + lane;
      const bool m = j < cnt && items[j] == cand;
      if (__any(m)) {
        hit = true;
        break;
      }
    }
    if (!hit || attempt >= 4096) return cand;
  }
}

template <typename T, int E>
__global__ __launch_bounds__(64) void bpr_epoch_kernel(BprArgs<T> a) {
  const int lane = threadIdx.x;
  const int64_t nwaves = (int64_t)gridDim.x;
  bool ok = true;
  for (int64_t i = blockIdx.x; i < a.npos; i += nwaves) {
    const int64_t slot = (int64_t)(((unsigned __int128)a.perm_a * (uint64_t)i + a.perm_b) %
                                   (uint64_t)a.npos);
    const int64_t u = a.pos_user[slot];
    const int64_t p = a.pos_item[slot];
    const int64_t rb = a.urowptr[u];
    const int64_t cnt = a.urowptr[u + 1] - rb;
    for (int j = 0; j < a.num_neg; ++j) {
      const uint64_t key = mix64(a.seed ^ mix64((uint64_t)slot * 64ull + (uint64_t)j));
      const int64_t n = sample_negative(a.uitems + rb, cnt, a.nitems, key, lane);
      ok &= bpr_step<T, E>(a, u, p, n, lane);
    }
  }
  if (!ok && lane == 0) *a.bad = 1;
}

// Applies a given triplet sequence in order with a single wave (exact reference order).
template <typename T, int E>
__global__ __launch_bounds__(64) void bpr_apply_kernel(BprArgs<T> a, const int64_t* trip,
                                                       int64_t n) {
  const int lane = threadIdx.x;
  bool ok = true;
  for (int64_t t = 0; t < n; ++t) ok &= bpr_step<T, E>(a, trip[3 * t], trip[3 * t + 1],
                                                       trip[3 * t + 2], lane);
  if (!ok && lane == 0) *a.bad = 1;
}

// Σ log(1 + exp(−x̂)) over eval triplets (BPREngine::evaluate :246-274): one wave per
// triplet, per-block partials, then a fixed-order sum.
template <typename T, int E>
__global__ __launch_bounds__(256) void bpr_eval_kernel(const T* U, const T* I, const T* bias,
                                                       const int64_t* trip, int64_t n, int kp,
                                                       int use_biases, double* partial) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  double s = 0.0;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < n; t += nw) {
    const int64_t u = trip[3 * t], p = trip[3 * t + 1], q = trip[3 * t + 2];
    T part = T(0);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int f = lane + 64 * e;
      if (f < kp) part += U[u * kp + f] * (I[p * kp + f] - I[q * kp + f]);
    }
    T x = wave_sum(part);
    if (use_biases) x += bias[p] - bias[q];
    s += log(1.0 + exp(-(double)x));
  }
  if (lane == 0) red[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void sum_partials_kernel(const double* partial, int n, double* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += partial[i];
    *out = s;
  }
}


#define QMFX_E_SWITCH(KP, CALL)          \
  switch ((KP + 63) / 64) {              \
    case 1: return CALL(1);              \
    case 2: return CALL(2);              \
    case 3: return CALL(3);              \
    case 4: return CALL(4);              \
    default: return hipErrorInvalidValue; \
  }

template <typename T, int E>
static hipError_t bpr_epoch(const BprArgs<T>& a, hipStream_t s) {
  hipLaunchKernelGGL((bpr_epoch_kernel<T, E>), dim3(a.waves), dim3(64), 0, s, a);
  return hipGetLastError();
}
template <typename T, int E>
static hipError_t bpr_apply(const BprArgs<T>& a, const int64_t* trip, int64_t n,
                            hipStream_t s) {
  hipLaunchKernelGGL((bpr_apply_kernel<T, E>), dim3(1), dim3(64), 0, s, a, trip, n);
  return hipGetLastError();
}
template <typename T, int E>
static hipError_t bpr_eval(const T* U, const T* I, const T* bias, const int64_t* trip,
                           int64_t n, int kp, int use_biases, double* partial, double* out,
                           hipStream_t s) {
  const int grid = 1024;
  hipLaunchKernelGGL((bpr_eval_kernel<T, E>), dim3(grid), dim3(256), 0, s, U, I, bias, trip, n,
                     kp, use_biases, partial);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, s, partial, grid, out);
  return hipGetLastError();
}

hipError_t launch_bpr_epoch_f32(const BprArgs<float>& a, int kp, hipStream_t s) {
#define CALL(E) bpr_epoch<float, E>(a, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_epoch_f64(const BprArgs<double>& a, int kp, hipStream_t s) {
#define CALL(E) bpr_epoch<double, E>(a, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_apply_f32(const BprArgs<float>& a, const int64_t* trip, int64_t n, int kp,
                                hipStream_t s) {
#define CALL(E) bpr_apply<float, E>(a, trip, n, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_apply_f64(const BprArgs<double>& a, const int64_t* trip, int64_t n,
                                int kp, hipStream_t s) {
#define CALL(E) bpr_apply<double, E>(a, trip, n, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_eval_f32(const float* U, const float* I, const float* bias,
                               const int64_t* trip, int64_t n, int kp, int use_biases,
                               double* partial, double* out, hipStream_t s) {
#define CALL(E) bpr_eval<float, E>(U, I, bias, trip, n, kp, use_biases, partial, out, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_eval_f64(const double* U, const double* I, const double* bias,
                               const int64_t* trip, int64_t n, int kp, int use_biases,
                               double* partial, double* out, hipStream_t s) {
#define CALL(E) bpr_eval<double, E>(U, I, bias, trip, n, kp, use_biases, partial, out, s)
  QMFX_E_SWITCH(kp, CALL)
#undef CALL
}

}  // namespace qmfx
