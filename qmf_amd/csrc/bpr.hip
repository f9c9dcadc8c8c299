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
#include "rowsolve.h"

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
// Adds (r − r0) to the shared row with L2 atomics: a concurrent wave's update of the same row
// is kept instead of being overwritten (the C4 "wavefront-atomic" SGD).  Used for the item
// rows, and for the user row when some user is heavy (BprArgs::atomic_user); otherwise the
// user row is stored plainly and a rare concurrent update of one user is overwritten, as with
// the reference's unsynchronised threads.  Only the read that formed the gradient can be
// stale, as in the reference's threads.
template <typename T, int E>
__device__ __forceinline__ void add_row(const Row<T, E>& r, const Row<T, E>& r0, T* base,
                                        int lane, int kp) {
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (lane + 64 * e < kp) unsafeAtomicAdd(base + lane + 64 * e, r.v[e] - r0.v[e]);
}

// x̂ of one (u, p, n) step summed over the wave: 16-lane DPP row sums, then the four rows'
// sums in a fixed order (no LDS round trips; the value is wave-uniform)
template <typename T>
__device__ __forceinline__ T wave_total(T v) {
  v = row16_sum(v);
  return (readlane(v, 0) + readlane(v, 16)) + (readlane(v, 32) + readlane(v, 48));
}
// lossDerivative (BPREngine.cpp:240-244): 1 / (1 + e^x̂).  fp32: the hardware exp2 and
// reciprocal (≤ 1 ulp each); fp64: exact library calls
__device__ __forceinline__ float neg_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(x));
}
__device__ __forceinline__ double neg_sigmoid(double x) { return 1.0 / (1.0 + exp(x)); }

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
  T x = wave_total(part);
  T bp = T(0), bn = T(0);
  if (a.use_biases) {
    bp = ld_shared(a.bias + p);
    bn = ld_shared(a.bias + n);
    x += bp - bn;
  }
  const T eg = neg_sigmoid(x);
  if (!isfinite(eg)) return false;
  const T lr = a.lr;
  // p == n (possible only in a caller-given sequence: sampled negatives are never positives):
  // the reference updates q_n in place after q_p, so q_n's step starts from the new q_p
  const bool same = p == n;
  if (a.use_biases && lane == 0) {
    const T bp_new = bp + lr * (eg - a.bias_lambda * bp);
    const T bn_old = same ? bp_new : bn;
    st_shared(a.bias + p, bp_new);
    st_shared(a.bias + n, bn_old + lr * (-eg - a.bias_lambda * bn_old));
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const T pu_new = pu.v[e] + lr * (eg * (qp.v[e] - qn.v[e]) - a.user_lambda * pu.v[e]);
    const T qp_new = qp.v[e] + lr * (eg * pu_new - a.item_lambda * qp.v[e]);
    const T qn_old = same ? qp_new : qn.v[e];
    const T qn_new = qn_old + lr * (-eg * pu_new - a.item_lambda * qn_old);
    pu.v[e] = pu_new;
    qp.v[e] = qp_new;
    qn.v[e] = qn_new;
  }
  store_row(pu, a.U + u * kp, lane, kp);
  if (!same) store_row(qp, a.I + p * kp, lane, kp);
  store_row(qn, a.I + n * kp, lane, kp);
  return true;
}

// murmur3 32-bit finaliser (a bijection of uint32)
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  return x ^ (x >> 16);
}

// Negative sampling (sampleRandomNegative, BPREngine-inl.h:48-60, which draws from
// mt19937): counter-based instead, so every draw is reproducible for a given seed.  Positive
// slot s has the 64-bit key mix64(seed_key ^ s) (one splitmix64 per positive); draw j,
// attempt t of it is fmix32(fold(key) + (4099·j + t)·φ) scaled to [0, nitems) — a bijection
// of the counter, all in 32-bit scalar arithmetic.
__device__ __forceinline__ uint32_t draw_hash(uint32_t fk, uint32_t ctr) {
  return fmix32(fk + ctr * 0x9e3779b9u);
}
__device__ __forceinline__ int64_t draw_candidate(uint32_t fk, uint32_t ctr, uint32_t nitems) {
  return (int64_t)(((uint64_t)draw_hash(fk, ctr) * nitems) >> 32);
}

// Rejection-samples a negative for user u: uniform in [0, nitems) and not in the user's
// positive set (sorted list urowptr/uitems).  fk = the positive's folded key, ctr0 = 4099·j.
__device__ __forceinline__ int64_t sample_negative(const int32_t* items, int64_t cnt,
                                                   uint32_t nitems, uint32_t fk, uint32_t ctr0,
                                                   int lane) {
  for (uint32_t attempt = 0;; ++attempt) {
    const int64_t cand = draw_candidate(fk, ctr0 + attempt, nitems);
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

// Draws the negative for (slot, j) against the user's positives: the first 64 are staged in
// `mine` (one per lane); longer lists are scanned from memory.
template <typename A>
__device__ __forceinline__ int64_t draw_negative_t(const A& a, const int32_t* items, int64_t cnt,
                                                   int32_t mine, uint32_t fk, uint32_t ctr0,
                                                   int lane) {
  const uint32_t ni = (uint32_t)a.nitems;
  if (cnt > 64) return sample_negative(items, cnt, ni, fk, ctr0, lane);
  for (uint32_t attempt = 0;; ++attempt) {
    const int64_t cand = draw_candidate(fk, ctr0 + attempt, ni);
    if (!__any(mine == (int32_t)cand) || attempt >= 4096) return cand;
  }
}

// One positive's SGD steps (u, p, n_j), j = 0..num_neg-1, with the rows in registers: p_u
// and q_p are loaded once and carried through the steps, as one thread of the reference
// sees its own writes (BPREngine::update :178-220 per step); the negatives are drawn first
// and their rows loaded together (a repeated negative takes the updated row of its earlier
// draw).  Each item row's net change is added to memory after its last update (add_row);
// the user row is stored (or added, for heavy users) at the end.
template <typename T, int E>
__device__ __forceinline__ bool bpr_positive(const BprArgs<T>& a, int64_t u, int64_t p,
                                             const int64_t (&n)[4], int nn, int lane) {
  const int kp = a.kp;
  Row<T, E> pu, qp, qn[4], pu0, qp0, qn0[4];
  load_row(pu0, a.U + u * kp, lane, kp);
  load_row(qp0, a.I + p * kp, lane, kp);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < nn) load_row(qn0[j], a.I + n[j] * kp, lane, kp);
  pu = pu0;
  qp = qp0;
#pragma unroll
  for (int j = 0; j < 4; ++j) qn[j] = qn0[j];
  T bp0 = T(0), bn0[4] = {T(0), T(0), T(0), T(0)};
  if (a.use_biases) {
    bp0 = ld_shared(a.bias + p);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < nn) bn0[j] = ld_shared(a.bias + n[j]);
  }
  T bp = bp0, bn[4] = {bn0[0], bn0[1], bn0[2], bn0[3]};
  bool ok = true;
  const T lr = a.lr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nn) break;
    // a negative drawn twice continues from its updated row
#pragma unroll
    for (int i = 0; i < j; ++i)
      if (n[i] == n[j]) {
        qn[j] = qn[i];
        qn0[j] = qn0[i];
        bn[j] = bn[i];
        bn0[j] = bn0[i];
      }
    T part = T(0);
#pragma unroll
    for (int e = 0; e < E; ++e) part += pu.v[e] * (qp.v[e] - qn[j].v[e]);
    T x = wave_total(part);
    if (a.use_biases) x += bp - bn[j];
    const T eg = neg_sigmoid(x);
    if (!isfinite(eg)) {
      ok = false;
      continue;  // the reference aborts (CHECK); the row is left as it was
    }
    if (a.use_biases) {
      bp = bp + lr * (eg - a.bias_lambda * bp);
      bn[j] = bn[j] + lr * (-eg - a.bias_lambda * bn[j]);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const T pu_new = pu.v[e] + lr * (eg * (qp.v[e] - qn[j].v[e]) - a.user_lambda * pu.v[e]);
      const T qp_new = qp.v[e] + lr * (eg * pu_new - a.item_lambda * qp.v[e]);
      const T qn_new = qn[j].v[e] + lr * (-eg * pu_new - a.item_lambda * qn[j].v[e]);
      pu.v[e] = pu_new;
      qp.v[e] = qp_new;
      qn[j].v[e] = qn_new;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nn) break;
    bool last = true;
#pragma unroll
    for (int i = j + 1; i < 4; ++i)
      if (i < nn && n[i] == n[j]) last = false;
    if (last) {
      add_row(qn[j], qn0[j], a.I + n[j] * kp, lane, kp);
      if (a.use_biases && lane == 0) unsafeAtomicAdd(a.bias + n[j], bn[j] - bn0[j]);
    }
  }
  // the user row with a plain (relaxed, L2-coherent) store while two waves rarely hold the
  // same user: the host sets atomic_user when the heaviest user's share of the positives
  // times the concurrent waves exceeds 1% (C4's uniform users: ≈0.4%), and an overwrite is
  // then exactly the reference's Hogwild store; the item rows keep the atomic adds (100K
  // items under 4096 waves collide often).  One of five atomic rows per positive fewer: the
  // epoch is bound by the ≈1.3 TB/s chip-wide float-atomic rate.
  if (a.atomic_user)
    add_row(pu, pu0, a.U + u * kp, lane, kp);
  else
    store_row(pu, a.U + u * kp, lane, kp);
  add_row(qp, qp0, a.I + p * kp, lane, kp);
  if (a.use_biases && lane == 0) unsafeAtomicAdd(a.bias + p, bp - bp0);
  return ok;
}

// Hogwild epoch: each wave walks positives i = wave, wave + nwaves, ... in the epoch's
// permuted order.  Positive i's data arrives through a 3-stage prefetch, one stage per
// iteration: (user, item) three positives ahead, the user's CSR range two ahead, its staged
// positive list one ahead.  They are issued before the current positive's row loads, so
// each iteration waits for about one memory latency instead of a chain of dependent loads.
template <typename T, int E>
__global__ __launch_bounds__(64) void bpr_epoch_kernel(BprArgs<T> a) {
  const int lane = threadIdx.x;
  const int64_t nw = (int64_t)gridDim.x;
  // slot of positive i = (perm_a·i + perm_b) mod npos: one 128-bit reduction per wave, then
  // a running sum (step = perm_a·nw mod npos; positives past the end get valid, unused slots)
  const uint64_t np = (uint64_t)a.npos;
  const uint64_t step = (uint64_t)(((unsigned __int128)a.perm_a * (uint64_t)gridDim.x) % np);
  auto advance = [&](uint64_t sl) {
    sl += step;
    return sl >= np ? sl - np : sl;
  };
  int64_t i = blockIdx.x;
  if (i >= a.npos) return;
  bool ok = true;
  const uint64_t seed_key = mix64(a.seed ^ 0xb5ad4eceda1ce2a9ull);
  // stage 0 (current): everything; stage 1: + CSR range; stage 2: (user, item)
  uint64_t s0 = (uint64_t)(((unsigned __int128)a.perm_a * (uint64_t)i + a.perm_b) % np);
  uint64_t s1 = advance(s0), s2 = advance(s1), s3 = s2;
  int64_t slot0 = (int64_t)s0, u0 = a.pos_user[slot0], p0 = a.pos_item[slot0];
  int64_t rb0 = a.urowptr[u0], cnt0 = a.urowptr[u0 + 1] - rb0;
  // (every lane loads: an unconditional load keeps the wait counts exact)
  int32_t mine0 = a.uitems[rb0 + (lane < cnt0 ? lane : 0)];
  mine0 = lane < cnt0 ? mine0 : -1;
  int64_t slot1 = (int64_t)s1, u1 = a.pos_user[slot1], p1 = a.pos_item[slot1];
  int64_t rb1 = a.urowptr[u1], cnt1 = a.urowptr[u1 + 1] - rb1;
  int64_t slot2 = (int64_t)s2, u2 = a.pos_user[slot2], p2 = a.pos_item[slot2];
  for (; i < a.npos; i += nw) {
    s3 = advance(s3);
    const int64_t slot3 = (int64_t)s3;
    const int64_t u3 = a.pos_user[slot3], p3 = a.pos_item[slot3];
    const int64_t rb2 = a.urowptr[u2], cnt2 = a.urowptr[u2 + 1] - rb2;
    int32_t mine1 = a.uitems[rb1 + (lane < cnt1 ? lane : 0)];
    const uint64_t pkey = mix64(seed_key ^ (uint64_t)slot0);
    const uint32_t fk = (uint32_t)pkey ^ (uint32_t)(pkey >> 32);
    for (int j0 = 0; j0 < a.num_neg; j0 += 4) {
      const int nn = a.num_neg - j0 < 4 ? a.num_neg - j0 : 4;
      int64_t n[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < nn)
          n[j] = draw_negative_t(a, a.uitems + rb0, cnt0, mine0, fk, 4099u * (uint32_t)(j0 + j), lane);
      ok &= bpr_positive<T, E>(a, u0, p0, n, nn, lane);
    }
    mine1 = lane < cnt1 ? mine1 : -1;
    slot0 = slot1, u0 = u1, p0 = p1, rb0 = rb1, cnt0 = cnt1, mine0 = mine1;
    slot1 = slot2, u1 = u2, p1 = p2, rb1 = rb2, cnt1 = cnt2;
    slot2 = slot3, u2 = u3, p2 = p3;
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

// Σ log(1 + exp(−x̂)) over eval triplets (BPREngine::evaluate :246-274).  Each wave scores
// four triplets at a time, 16 lanes per triplet and NT = KP/16 contiguous factors per lane
// (one 16-B load per row and lane at k = 64), so 4× as many rows are in flight as with a
// wave per triplet; per-block partials, then a fixed-order sum.
template <typename T, int NT>
__global__ __launch_bounds__(256) void bpr_eval_kernel(const T* U, const T* I, const T* bias,
                                                       const int64_t* trip, int64_t n, int kp,
                                                       int use_biases, double* partial) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int64_t stride = (int64_t)gridDim.x * 16;
  double s = 0.0;
  for (int64_t t = ((int64_t)blockIdx.x * 4 + w) * 4 + g; t < n; t += stride) {
    const int64_t u = trip[3 * t], p = trip[3 * t + 1], q = trip[3 * t + 2];
    const T* pu = U + u * kp + c * NT;
    const T* qp = I + p * kp + c * NT;
    const T* qn = I + q * kp + c * NT;
    T part = T(0);
#pragma unroll
    for (int e = 0; e < NT; ++e) part += pu[e] * (qp[e] - qn[e]);
    T x = row16_sum(part);
    if (use_biases) x += bias[p] - bias[q];
    if (c == 0) s += log(1.0 + exp(-(double)x));
  }
  s = wave_sum(s);
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

#define QMFX_NT_SWITCH(KP, CALL)                                            \
  switch ((KP) / 16) {                                                      \
    case 1: return CALL(1);   case 2: return CALL(2);   case 3: return CALL(3);   \
    case 4: return CALL(4);   case 5: return CALL(5);   case 6: return CALL(6);   \
    case 7: return CALL(7);   case 8: return CALL(8);   case 9: return CALL(9);   \
    case 10: return CALL(10); case 11: return CALL(11); case 12: return CALL(12); \
    case 13: return CALL(13); case 14: return CALL(14); case 15: return CALL(15); \
    case 16: return CALL(16);                                               \
    default: return hipErrorInvalidValue;                                   \
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
template <typename T, int NT>
static hipError_t bpr_eval(const T* U, const T* I, const T* bias, const int64_t* trip,
                           int64_t n, int kp, int use_biases, double* partial, double* out,
                           hipStream_t s) {
  const int grid = 1024;  // = the context's partial buffer
  hipLaunchKernelGGL((bpr_eval_kernel<T, NT>), dim3(grid), dim3(256), 0, s, U, I, bias, trip, n,
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
#define CALL(NT) bpr_eval<float, NT>(U, I, bias, trip, n, kp, use_biases, partial, out, s)
  QMFX_NT_SWITCH(kp, CALL)
#undef CALL
}
hipError_t launch_bpr_eval_f64(const double* U, const double* I, const double* bias,
                               const int64_t* trip, int64_t n, int kp, int use_biases,
                               double* partial, double* out, hipStream_t s) {
#define CALL(NT) bpr_eval<double, NT>(U, I, bias, trip, n, kp, use_biases, partial, out, s)
  QMFX_NT_SWITCH(kp, CALL)
#undef CALL
}

}  // namespace qmfx
