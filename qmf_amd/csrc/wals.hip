// WALS hot path on MI355X (gfx950).
//
// Reference path (taozhijiang/qmf):
//   WALSEngine::iterate             qmf/wals/WALSEngine.cpp:165-218
//   WALSEngine::computeXtX          qmf/wals/WALSEngine.cpp:246-264
//   WALSEngine::updateFactorsForOne qmf/wals/WALSEngine.cpp:266-310
//   linearSymmetricSolve → dsysv_   qmf/Matrix.cpp:81-96
//
// Per solved row r with signals e (fixed-side rows y_e, weights w_e = αv_e, c_e = 1 + αv_e):
//   A = M + Σ_e w_e y_e y_eᵀ,  M = YᵀY + λI,  b = Σ_e c_e y_e,  x = A⁻¹ b,
//   loss_r = Σc + xᵀ(A − λI)x − 2xᵀb = Σc − xᵀb − λ‖x‖²      (since Ax = b).
// Two mathematically identical ways to get x, chosen per row by its signal count n:
//   * direct (n large):  the k×k Gram of the row, then a register-tile Cholesky;
//   * whitened (n ≤ k/2, n ≤ 64): with M = L Lᵀ and Z = Y L⁻ᵀ (one GEMM per half),
//       A = L (I + Zₛᵀ W Zₛ) Lᵀ and, by the push-through identity,
//       x = L⁻ᵀ Zₛᵀ u  with  (W_P⁻¹ + K_PP) u_P = W_P⁻¹ c_P − K_PQ 1_Q,  u_Q = 1,
//     where K = Zₛ Zₛᵀ (n×n), P = signals with w > 0, Q = signals with w = 0 (c = 1).
//     The n×n system replaces the k×k one; x' = Zₛᵀu is mapped back by x = L⁻ᵀ x'
//     (a GEMM over those rows).  xᵀb = x'ᵀ(Zₛᵀc).
//
// Data layout in HBM: factors row-major [n][KP], KP = 16·NT ≥ k, zero padding columns;
// interactions CSR (int64 rowptr, int32 column, value v).  The padded part of every system
// is the identity, so padded solution entries are exactly zero.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "rowsolve.h"

namespace qmfx {



// (split3 / mma_split6: the fp32-accurate split-bf16 products, rowsolve.h)

// ---------------------------------------------------------------------------------------
// Register-tile Cholesky + solve, shared by both row kernels (one wave64 per system).
//   In:  acc = lower 16×16 tiles of an SPD matrix of size 16·NT (diagonal tiles full);
//        S.bw = right-hand side (written and synchronised by the caller).
//   Out: S.xs = solution; S.bw = L⁻¹ b.  `bad` set on a non-positive pivot.
// Right-looking over 16-column panels.  A panel is factored with its rows spread over the
// lanes: per column one broadcast (readlane) of the diagonal block's column, issued
// before the pivot is known, and unconditional FMAs (rows above the pivot only touch
// their dead upper part); the forward solve rides along as one more register per row.
// The trailing update A(I,J) −= L(I,p)L(J,p)ᵀ is 4 MFMAs per tile with operands staged
// through LDS; off-diagonal L tiles return to the registers.  The diagonal L blocks go to
// LDS transposed and column-scaled, Lt[q][c] = L[c][q]/L[q][q] (q < c, 0 elsewhere), so
// the backward substitution is one readlane + one FMA per column.
// ---------------------------------------------------------------------------------------
#ifndef QMFX_CHOL_PK
#define QMFX_CHOL_PK 1
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T>
struct CholLd {
  // padded LDS row of a panel: fp32 rows are 16-B aligned and conflict-free for the
  // b128 row accesses and the MFMA-layout tile accesses used here
  static constexpr int PLD = sizeof(T) == 4 ? 20 : 17;
};

template <typename T, int NT>
struct CholShared {
  static constexpr int PLD = CholLd<T>::PLD;
  T panel[16 * NT * PLD];
  T Lt[NT * 16 * PLD];
  T bw[16 * NT];
  T xs[16 * NT];
  T invd[16 * NT];
};

// 16 consecutive values of an LDS row (b128 accesses for fp32)
template <typename T>
__device__ __forceinline__ void lds_row_load(const T* src, T (&v)[16]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 x = reinterpret_cast<const f32x4*>(src)[j];
      v[4 * j] = x[0], v[4 * j + 1] = x[1], v[4 * j + 2] = x[2], v[4 * j + 3] = x[3];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = src[j];
  }
}
template <typename T>
__device__ __forceinline__ void lds_row_store(T* dst, const T (&v)[16]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      reinterpret_cast<f32x4*>(dst)[j] = f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) dst[j] = v[j];
  }
}

// LDS ordering inside chol_solve: the whole workgroup when it is one wave (WS = false), or
// only the calling wave (WS = true: one wave of a multi-wave workgroup runs the solve; LDS
// accesses of one wave execute in order, so draining them and pinning the compiler's order
// is enough).
template <bool WS>
__device__ __forceinline__ void csync() {
  if constexpr (WS) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

template <typename T, int NT, bool WS = false>
__device__ __forceinline__ void chol_solve(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                           CholShared<T, NT>& S, int lane, int& bad) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr int SLOTS = (KP + 63) / 64;
  constexpr int PLD = CholShared<T, NT>::PLD;
  const int cl = lane & 15;
  const int kk = lane >> 4;
#pragma unroll
  for (int p = 0; p < NT; ++p) {
    const int R = KP - 16 * p;
#pragma unroll
    for (int I = p; I < NT; ++I) {
      const int t = tile_index(I, p);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        S.panel[(16 * (I - p) + M::crow(lane, r)) * PLD + cl] = acc[t][r];
    }
    csync<WS>();
    T pa[SLOTS][16];
    T pb[SLOTS];
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int q = lane + 64 * s;
      const int qq = q < R ? q : 0;
      lds_row_load(&S.panel[qq * PLD], pa[s]);
      pb[s] = S.bw[16 * p + qq];
    }
    // lanes 0..15 collect the panel's 1/L[c][c] and y_c (lane c), stored once per panel
    T invv = T(0), yv = T(0);
    {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        // A[m][c] of the diagonal block's rows, broadcast before the pivot is known: the
        // update uses L[q][c]·L[m][c] = (A[q][c]/d)·A[m][c]
        // (constant trip counts with a predicate: the loops must unroll fully before c is
        // known, or the compiler falls back to indexed register access)
        T am[16];
#pragma unroll
        for (int m = 1; m < 16; ++m)
          if (m > c) am[m] = readlane(pa[0][c], m);
        const T d = readlane(pa[0][c], c);
        const T bc = readlane(pb[0], c);
        T ljj, inv;
        pivot_sqrt(d, ljj, inv);
        (void)ljj;
        const bool me = lane == c;
        invv = me ? inv : invv;
        yv = me ? bc * inv : yv;
        // every row takes lq = A[q][c]/L[c][c]: below the pivot that is L[q][c], at the
        // pivot √d; rows above only change their dead upper part (and their pb, which is
        // no longer read: y comes from yv)
#pragma unroll
        for (int s = 0; s < SLOTS; ++s) {
          if (64 * s < R) {
            const T lq = pa[s][c] * inv;
            const T lqs = lq * inv;
            pa[s][c] = lq;
            pb[s] -= lqs * bc;
#if QMFX_CHOL_PK
            if constexpr (sizeof(T) == 4) {
              // packed pairs: one v_pk_fma_f32 per two columns (same rounding as two FMAs)
#pragma unroll
              for (int m = 0; m < 16; m += 2) {
                if (m > c) {
                  f32x2 v = {pa[s][m], pa[s][m + 1]};
                  const f32x2 a2 = {am[m], am[m + 1]};
                  v = __builtin_elementwise_fma(f32x2{-lqs, -lqs}, a2, v);
                  pa[s][m] = v[0];
                  pa[s][m + 1] = v[1];
                } else if (m + 1 > c) {
                  pa[s][m + 1] -= lqs * am[m + 1];
                }
              }
            } else
#endif
            {
#pragma unroll
              for (int m = 1; m < 16; ++m)
                if (m > c) pa[s][m] -= lqs * am[m];
            }
          }
        }
        // one column per scheduling window: readlanes hoisted across columns exhaust the
        // SGPRs.  The fence pins every slot's updates inside the window; without it the
        // compiler defers the slots past the diagonal block (rows ≥ 64) to the end of the
        // panel and spills all 15·16 broadcasts (SGPR spill + readlane + s_nop per FMA).
#pragma unroll
        for (int s = 1; s < SLOTS; ++s) {
          if (64 * s < R) {
#pragma unroll
            for (int m = 0; m < 16; ++m)
              if (m >= c) asm volatile("" : "+v"(pa[s][m]));
            asm volatile("" : "+v"(pb[s]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // a pivot that is not positive (or not finite) leaves 1/√d outside (0, ∞)
    bad |= __any(lane < 16 && !(invv > T(0) && invv < __builtin_huge_val())) ? 1 : 0;
    if (lane < 16) {
      S.invd[16 * p + lane] = invv;
      S.bw[16 * p + lane] = yv;
    }
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int q = lane + 64 * s;
      if (q < R) lds_row_store(&S.panel[q * PLD], pa[s]);
      if (q >= 16 && q < R) S.bw[16 * p + q] = pb[s];
    }
    csync<WS>();
    // diagonal block → Lt (transposed, scaled by the column's 1/L[q][q], zero on and above
    // the diagonal)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = lane + 64 * it;
      const int r = idx >> 4, c = idx & 15;
      S.Lt[(p * 16 + c) * PLD + r] = c < r ? S.panel[r * PLD + c] * S.invd[16 * p + c] : T(0);
    }
    T fr[NT][4];
#pragma unroll
    for (int I = p + 1; I < NT; ++I) {
#pragma unroll
      for (int s = 0; s < 4; ++s) fr[I][s] = S.panel[(16 * (I - p) + cl) * PLD + 4 * s + kk];
    }
#pragma unroll
    for (int I = p + 1; I < NT; ++I) {
      const int t = tile_index(I, p);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[t][r] = S.panel[(16 * (I - p) + M::crow(lane, r)) * PLD + cl];
#pragma unroll
      for (int J = p + 1; J <= I; ++J) {
        const int tj = tile_index(I, J);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[tj] = M::mma(-fr[I][s], fr[J][s], acc[tj]);
      }
    }
    csync<WS>();
  }
  // backward solve Lᵀ x = y by 16-blocks from the bottom: lane cl carries row cl of the
  // block scaled by its own 1/L[cl][cl]; column c then finishes x_c (readlane) and
  // removes it from the rows above with the scaled Lt (one FMA)
#pragma unroll
  for (int I = NT - 1; I >= 0; --I) {
    T part = T(0);
#pragma unroll
    for (int J = I + 1; J < NT; ++J) {
      const int t = tile_index(J, I);
#pragma unroll
      for (int r = 0; r < 4; ++r) part += acc[t][r] * S.xs[16 * J + M::crow(lane, r)];
    }
    part += shfl_xor(part, 16);
    part += shfl_xor(part, 32);
    T vm = (S.bw[16 * I + cl] - part) * S.invd[16 * I + cl];
    T lt[16];
    lds_row_load(&S.Lt[(16 * I + cl) * PLD], lt);
#pragma unroll
    for (int c = 15; c >= 0; --c) vm -= lt[c] * readlane(vm, c);
    if (lane < 16) S.xs[16 * I + lane] = vm;
    csync<WS>();
  }
}

// Factor-index permutation of the fp32 direct path.  Lane column c of "virtual" block B
// holds physical factor π(16B + c) = 16·W·(B / W) + W·c + (B mod W), so that one lane's
// W consecutive physical factors (one 16·W-byte load) feed W different MFMA blocks.  The
// Gram, the Cholesky and the right-hand side all live in the virtual order; the base
// YᵀY + λI is read through π and x is scattered back through π.
template <int NT>
struct Perm {
  static constexpr int W = (NT % 4 == 0) ? 4 : (NT % 2 == 0 ? 2 : 1);
  // the split-bf16 Gram pays from NT = 6 up; at k ≤ 64 the f32 loop keeps 3 waves/SIMD
  template <typename T>
  static constexpr bool split = sizeof(T) == 4 && NT >= 6;
  __device__ static __forceinline__ int phys(int v) {
    const int B = v >> 4, c = v & 15;
    return 16 * W * (B / W) + W * c + (B % W);
  }
};

// Direct-row Gram, fp32 on the bf16 matrix cores: 32 signals per step, lane (c, g) owns
// signals 8g..8g+7 of the step and virtual column c of every block.  Operands are √w·y
// (w = αv ≥ 0), so A and B are the same split values: A += Σ w y yᵀ; b = Σ c y from the
// raw rows.  The row's (column, value) pairs are staged through LDS 64 at a time (one
// coalesced load per lane, a chunk ahead), and each lane reads its 8 as two b128 pairs.
// Signals past the row's end point at the fixed side's all-zero row a.zrow with v = 0,
// so they add exactly nothing and need no masking.  Σc is summed at staging.  Pipeline:
// the rows of step s+1 are in flight while step s's MFMAs run.  A negative weight (1 + αv
// may still be > 0) sets `negw`; the caller flags the row for the host solve.
#ifndef QMFX_GRAM_HEAD
#define QMFX_GRAM_HEAD 100
#endif
#ifndef QMFX_GRAM_VALU
#define QMFX_GRAM_VALU 2
#endif
template <int NT>
__device__ __forceinline__ void gram_split_bf16(const SolveArgs<float>& a, int64_t beg,
                                                int64_t end, f32x4 (&acc)[NT * (NT + 1) / 2],
                                                float (&bpart)[NT], double& csum, int& negw,
                                                int lane, int (&mcol)[2][64],
                                                float (&mval)[2][64]) {
  constexpr int KP = 16 * NT;
  constexpr int W = Perm<NT>::W;
  constexpr int NG = NT / W;
  using vecW = float __attribute__((ext_vector_type(W)));
  const int c = lane & 15;
  const int g = lane >> 4;
  const int n = (int)(end - beg);
  const int nsteps = (n + 31) >> 5;
  const int nchunks = (n + 63) >> 6;
  float cs = 0.f;
  int pc = a.zrow;
  float pv = 0.f;
  auto fetch = [&](int ch) {  // this lane's signal of chunk ch → (pc, pv)
    const int e = 64 * ch + lane;
    const bool ok = e < n;
    pc = ok ? a.col[beg + e] : a.zrow;
    pv = ok ? a.val[beg + e] : 0.f;
  };
  auto stage = [&](int ch) {  // (pc, pv) of chunk ch → LDS
    const bool ok = 64 * ch + lane < n;
    cs += ok ? 1.f + a.alpha * pv : 0.f;
    mcol[ch & 1][lane] = pc;
    mval[ch & 1][lane] = pv;
  };
  auto read_meta = [&](int st, int (&col)[8], float (&val)[8]) {
    const int o = 32 * (st & 1) + 8 * g;
    const int4 c0 = *reinterpret_cast<const int4*>(&mcol[(st >> 1) & 1][o]);
    const int4 c1 = *reinterpret_cast<const int4*>(&mcol[(st >> 1) & 1][o + 4]);
    const float4 v0 = *reinterpret_cast<const float4*>(&mval[(st >> 1) & 1][o]);
    const float4 v1 = *reinterpret_cast<const float4*>(&mval[(st >> 1) & 1][o + 4]);
    col[0] = c0.x, col[1] = c0.y, col[2] = c0.z, col[3] = c0.w;
    col[4] = c1.x, col[5] = c1.y, col[6] = c1.z, col[7] = c1.w;
    val[0] = v0.x, val[1] = v0.y, val[2] = v0.z, val[3] = v0.w;
    val[4] = v1.x, val[5] = v1.y, val[6] = v1.z, val[7] = v1.w;
  };
  auto load_rows = [&](const int (&col)[8], vecW (&y)[8][NG]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#ifdef QMFX_EXP_LOCAL_GATHER  // timing experiment: every gather hits a few cached rows
      const vecW* yr =
          reinterpret_cast<const vecW*>(a.Y + (uint64_t)(uint32_t)(col[j] & 63) * KP) + c;
#else
      const vecW* yr =
          reinterpret_cast<const vecW*>(a.Y + (uint64_t)(uint32_t)col[j] * KP) + c;
#endif
#pragma unroll
      for (int G = 0; G < NG; ++G) y[j][G] = yr[16 * G];
    }
  };
  if (nsteps == 0) return;
  // prologue: chunks 0 (and 1) staged, chunk 2 in flight, step 0's rows in flight
  fetch(0);
  stage(0);
  if (nchunks > 1) {
    fetch(1);
    stage(1);
  }
  if (nchunks > 2) fetch(2);
  // One step: the next step's rows go out first (into the other buffer, whose rows were
  // consumed one step ago), then each block is split right before the tiles of its block
  // row, so the split VALU of block I+1 issues in the free cycles of row I's MFMAs.  The
  // two buffers swap roles by a 2× unroll (no register copies).
  auto step = [&](int st, vecW (&yc)[8][NG], float (&vc)[8], vecW (&yn)[8][NG],
                  float (&vn)[8]) {
    if (st + 1 < nsteps) {
      if (((st + 1) & 1) == 0) {
        // step st+1 opens chunk k = (st+1)/2: stage chunk k+1, fetch chunk k+2
        const int k = (st + 1) >> 1;
        if (k + 1 < nchunks) stage(k + 1);
        if (k + 2 < nchunks) fetch(k + 2);
      }
      int cn[8];
      read_meta(st + 1, cn, vn);
      load_rows(cn, yn);
    }
    float sw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float w = a.alpha * vc[j];
      const float cw = 1.f + w;
      negw |= w < 0.f;
      sw[j] = fast_sqrt(fabsf(w));
#pragma unroll
      for (int G = 0; G < NG; ++G)
#pragma unroll
        for (int m = 0; m < W; ++m) bpart[W * G + m] += cw * yc[j][G][m];
    }
    Split3 sp[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = sw[j] * yc[j][I / W][I % W];
      split3(x, sp[I]);
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        acc[t] = mma_split6(sp[I], sp[J], acc[t]);
      }
    }
    // issue order: the sqrt/rhs VALU and block 0's split up front, then one MFMA and two
    // VALU at a time (an MFMA holds the vector issue for 8 of its 16 cycles)
    __builtin_amdgcn_sched_group_barrier(0x2, QMFX_GRAM_HEAD, 0);
#pragma unroll
    for (int i = 0; i < 6 * NT * (NT + 1) / 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x2, QMFX_GRAM_VALU, 0);
    }
  };
  int col0[8];
  float val0[8], val1[8];
  vecW y0[8][NG], y1[8][NG];
  read_meta(0, col0, val0);
  load_rows(col0, y0);
  for (int st = 0; st < nsteps; st += 2) {
    step(st, y0, val0, y1, val1);
    if (st + 1 < nsteps) step(st + 1, y1, val1, y0, val0);
  }
  const double tot = wave_sum((double)cs);
  csum += lane == 0 ? tot : 0.0;  // the caller sums the cl == 0 lanes
}

// ---------------------------------------------------------------------------------------
// Direct row kernel: one wave64 per row (slot order heaviest-first).  Gram
// A = G + λI + Σ w y yᵀ accumulated into the lower tiles held in registers, starting from
// the tile image of G + λI (gimg_kernel: one coalesced 16-B load per tile and lane);
// b = Σ c y and Σc on the side.  (A persistent variant that prefetched the next row's
// descriptor measured slower: the trace showed the gathers' latency is a small part of a
// row, and a fixed grid loses the dispatcher's balancing.)
// ---------------------------------------------------------------------------------------
#ifndef QMFX_WAVES_NT8
#define QMFX_WAVES_NT8 1
#endif
// waves per SIMD the direct kernel is compiled for: fp32 split-Gram and fp64 k > 64 tilings
// keep their accumulators in the whole (VGPR + AGPR) register file of one wave
template <typename T, int NT>
constexpr int direct_waves() {
  return Perm<NT>::template split<T> ? QMFX_WAVES_NT8 : (sizeof(T) == 8 && NT > 4 ? 1 : 2);
}

template <typename T, int NT, bool TRACE>
__global__ __launch_bounds__(64, (direct_waves<T, NT>()))
void wals_direct_kernel(SolveArgs<T> a) {
  // fp32 at NT = 8: the split-bf16 Gram keeps 144 accumulator + 96 operand + 128 row
  // registers live: one wave per SIMD with the whole register file (QMFX_WAVES_NT8 = 1)
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  __shared__ __attribute__((aligned(16))) CholShared<T, NT> S;
  __shared__ __attribute__((aligned(16))) T borig[KP];
  __shared__ __attribute__((aligned(16))) int mcol[2][64];
  __shared__ __attribute__((aligned(16))) float mval[2][64];

  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  {
    const RowDesc d = a.desc[a.row_begin + blockIdx.x];
    const int64_t row = d.row;
    const int64_t beg = d.beg;
    const int64_t end = beg + d.n;
    uint64_t tr[5] = {0, 0, 0, 0, 0};
    if (TRACE) tr[0] = __builtin_amdgcn_s_memtime();

    acc_t acc[NTT];
    {
      // buffer loads: the tile offset rides in the scalar offset, so no per-tile address
      // registers are kept
      constexpr int AB = (int)sizeof(acc_t);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.Gimg, (short)0, NTT * 64 * AB, 0x00020000);
#pragma unroll
      for (int t = 0; t < NTT; ++t) {
#pragma unroll
        for (int h = 0; h < AB / 16; ++h) {
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * AB + 16 * h,
                                                                t * 64 * AB, 0);
          if constexpr (sizeof(T) == 4) {
            acc[t] = __builtin_bit_cast(acc_t, v);
          } else {
            const double lo = __builtin_bit_cast(double, (unsigned long long)v[0] |
                                                             ((unsigned long long)v[1] << 32));
            const double hi = __builtin_bit_cast(double, (unsigned long long)v[2] |
                                                             ((unsigned long long)v[3] << 32));
            acc[t][2 * h] = lo;
            acc[t][2 * h + 1] = hi;
          }
        }
      }
    }
    if (TRACE) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tr[1] = __builtin_amdgcn_s_memtime();
    }
    T bpart[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) bpart[c] = T(0);
    double csum = 0.0;
    int negw = 0;
    if constexpr (Perm<NT>::template split<T>) {
      gram_split_bf16<NT>(a, beg, end, acc, bpart, csum, negw, lane, mcol, mval);
    } else
    for (int64_t base = beg; base < end; base += 64) {
      const int nst = (int)(end - base < 64 ? end - base : 64);
      const int cr = lane < nst ? a.col[base + lane] : 0;
      const T vr = lane < nst ? a.val[base + lane] : T(0);
      bool valid = kk < nst;
      T v = __shfl(vr, kk, 64);
      T yn[NT];
      {
        const T* yrow = a.Y + (uint64_t)(uint32_t)__shfl(cr, kk, 64) * KP + cl;
#pragma unroll
        for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
      }
      for (int s = 0; 4 * s < nst; ++s) {
        T yv[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) yv[q] = valid ? yn[q] : T(0);
        const T w = valid ? a.alpha * v : T(0);
        const T cw = valid ? T(1) + a.alpha * v : T(0);
        const int jn = 4 * (s + 1) + kk;
        const bool vn = jn < nst;
        if (4 * (s + 1) < nst) {
          const int cn = __shfl(cr, jn < 64 ? jn : 0, 64);
          v = __shfl(vr, jn < 64 ? jn : 0, 64);
          const T* yrow = a.Y + (uint64_t)(uint32_t)(vn ? cn : cr) * KP + cl;
#pragma unroll
          for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
        }
        valid = vn;
#pragma unroll
        for (int q = 0; q < NT; ++q) bpart[q] += cw * yv[q];
        csum += (double)cw;
#pragma unroll
        for (int I = 0; I < NT; ++I) {
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const int t = tile_index(I, J);
            acc[t] = M::mma(yv[I], w * yv[J], acc[t]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      bpart[q] += shfl_xor(bpart[q], 16);
      bpart[q] += shfl_xor(bpart[q], 32);
      if (kk == 0) {
        borig[16 * q + cl] = bpart[q];
        S.bw[16 * q + cl] = bpart[q];
      }
    }
    csum = wave_sum(cl == 0 ? csum : 0.0);  // each k-slot row counted once
    int bad = __any(negw) ? 1 : 0;  // split Gram with a negative weight: solved on the host
    __syncthreads();
    if (TRACE) tr[2] = __builtin_amdgcn_s_memtime();
    chol_solve<T, NT>(acc, S, lane, bad);
    if (TRACE) tr[3] = __builtin_amdgcn_s_memtime();

    double xb = 0.0, xx = 0.0;
    for (int j = lane; j < KP; j += 64) {
      const T xj = S.xs[j];
      // a failed row stores x = 0 (loss term 0), like the whitened kernel; the caller
      // re-solves it
      a.X[row * KP + (Perm<NT>::template split<T> ? Perm<NT>::phys(j) : j)] = bad ? T(0) : xj;
      xb += (double)xj * (double)borig[j];
      xx += (double)xj * (double)xj;
    }
    xb = wave_sum(xb);
    xx = wave_sum(xx);
    if (lane == 0) {
      a.rowloss[row] = bad ? 0.0 : csum - xb - (double)a.lambda * xx;
      if (bad && a.status) a.status[row] = 1;
    }
    if (TRACE && lane == 0) {
      tr[4] = __builtin_amdgcn_s_memtime();
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* o = a.trace + 8 * (a.row_begin + blockIdx.x);
#pragma unroll
      for (int j = 0; j < 5; ++j) o[j] = tr[j];
      o[5] = hw | ((uint64_t)xcc << 32);
      o[6] = (uint64_t)d.n;
      o[7] = (uint64_t)row;
    }
  }
}

// G + λI (padding diagonal: 1) in the direct kernel's accumulator-tile order:
// img[(t·64 + lane)·4 + r] = acc[t][r] of `lane`, in the kernel's virtual index space.
template <typename T, int NT>
__global__ void gimg_kernel(const T* G, int k, double lambda, T* img) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NTT * 256) return;
  const int r = idx & 3, lane = (idx >> 2) & 63, t = idx >> 8;
  int I = 0;
  while (tile_index(I + 1, 0) <= t) ++I;
  const int J = t - tile_index(I, 0);
  const int i = M::crow(lane, r), cl = lane & 15;
  const int pi = Perm<NT>::template split<T> ? Perm<NT>::phys(16 * I + i) : 16 * I + i;
  const int pj = Perm<NT>::template split<T> ? Perm<NT>::phys(16 * J + cl) : 16 * J + cl;
  double g = (double)G[(int64_t)pi * KP + pj];
  if (I == J && i == cl) g += (pi < k) ? lambda : 1.0;
  img[idx] = (T)g;
}

// ---------------------------------------------------------------------------------------
// Whitened row kernel (n ≤ 16·NTN signals, n ≤ KP/2).  One wave64 per row.  The row's
// whitened fixed-side rows z_e (KP values each) are loaded ONCE into registers in MFMA
// operand order (lane (i, g) holds z_{16I+i}[16q + 4g .. +3] for every I, q), so that
//   K = Zₛ Zₛᵀ         — NTN(NTN+1)/2 tiles × KP/4 steps of 16x16x4 MFMA from registers,
//   x' = Zₛᵀu, Zₛᵀc   — per-lane FMAs + 16-lane DPP row sums,
// and the HBM traffic per signal is one gathered row, as in the direct kernel.
// Writes x' (whitened); whiten_kernel<UNWHITEN> maps it to x = L⁻ᵀ x' and adds −λ‖x‖².
// ---------------------------------------------------------------------------------------
// minimum waves per SIMD of the NTN = 4 tiling (timing experiments: 1 lifts the 256-VGPR cap)
#ifndef QMFX_WB4_MIN_WAVES
#define QMFX_WB4_MIN_WAVES 2
#endif
template <typename T, int NTK, int NTN, bool TRACE>
__global__ __launch_bounds__(64, NTK > 8 ? 1 : (NTN == 4 ? QMFX_WB4_MIN_WAVES : 2))
void wals_woodbury_kernel(SolveArgs<T> a) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  using v4 = typename M::acc_t;  // 4-wide vector of T
  constexpr int KP = 16 * NTK;
  constexpr int NTT = NTN * (NTN + 1) / 2;
  __shared__ __attribute__((aligned(16))) CholShared<T, NTN> S;
  __shared__ __attribute__((aligned(16))) T gq[16 * NTN];

  // one row per wave: the slot's descriptor, then its signals (lane = signal)
  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t i = blockIdx.x;
  const RowDesc dn = a.desc[a.row_begin + i];
  const int64_t row = dn.row;
  const int n = dn.n;  // ≤ 16·NTN by bucketing
  uint64_t tr[5] = {0, 0, 0, 0, 0};
  if (TRACE) tr[0] = __builtin_amdgcn_s_memtime();

  // signal e = lane: column, weight, confidence
  const bool mine = lane < n;
  const int cr = mine ? a.col[dn.beg + lane] : a.zrow;
  const T vr = mine ? a.val[dn.beg + lane] : T(0);
  const T wl = mine ? a.alpha * vr : T(0);
  const T cwl = mine ? T(1) + a.alpha * vr : T(0);
  const bool isP = mine && wl > T(0);
  const bool isQ = mine && wl == T(0);
  int bad = __any(mine && wl < T(0)) ? 1 : 0;  // negative confidence: not SPD in this form
  const uint64_t mQ = __ballot(isQ);
  const bool hasQ = mQ != 0;

  // gather Zₛ into registers: zr[I][q] = z_{16I+cl}[16q + 4kk .. +3].  Padding signals
  // (e ≥ n) load the all-zero row a.zrow, so their K rows and columns are exactly 0.
  v4 zr[NTN][NTK];
#pragma unroll
  for (int I = 0; I < NTN; ++I) {
    const int ce = __shfl(cr, 16 * I + cl, 64);
    const v4* zrow = reinterpret_cast<const v4*>(a.Y + (uint64_t)(uint32_t)ce * KP) + kk;
#pragma unroll
    for (int q = 0; q < NTK; ++q) zr[I][q] = zrow[4 * q];
  }
  if (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[1] = __builtin_amdgcn_s_memtime();
  }
  // K = Zₛ Zₛᵀ (lower tiles); the summation index j = 16q + 4kk + comp is the same for the
  // A and B operands, so its order within a step does not matter
  acc_t acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0, 0, 0, 0};
  if constexpr (sizeof(T) == 4) {
    // fp32: 32-deep chunks on the bf16 matrix cores, exact 3-way split (see split3):
    // chunk s takes the lane's columns q = 2s, 2s+1 (8 values) as its k-slice
    constexpr int NS = (NTK + 1) / 2;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      Split3 sp[NTN];
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        float x[8];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          x[c4] = zr[I][2 * s][c4];
          x[4 + c4] = (2 * s + 1 < NTK) ? zr[I][(2 * s + 1) % NTK][c4] : 0.f;
        }
        split3(x, sp[I]);
      }
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          const int t = tile_index(I, J);
          acc[t] = mma_split6(sp[I], sp[J], acc[t]);
        }
      }
      // one chunk's splits live at a time (keeps the NTN = 3 kernel at 3 waves/SIMD)
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int q = 0; q < NTK; ++q) {
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) {
#pragma unroll
        for (int I = 0; I < NTN; ++I) {
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const int t = tile_index(I, J);
            acc[t] = M::mma(zr[I][q][comp], zr[J][q][comp], acc[t]);
          }
        }
      }
    }
  }
  double xb = 0.0;  // xᵀb of the row (= x'ᵀ Zₛᵀc)
  T ul[NTN];        // u of signal 16I + cl
  if (!hasQ) {
    // Every real signal is in P.  S = W⁻¹ + K on all 16·NTN slots: padding slots have
    // K = 0 (zero rows) and take W⁻¹ = 1, so S is the identity there and u = 0.
    const T iw = isP ? fast_rcp(wl) : T(1);
    const T rhs = isP ? cwl * iw : T(0);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const T iwd = __shfl(iw, 16 * I + cl, 64);  // diagonal (e, e), e = 16I + cl
      const int t = tile_index(I, I);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] += M::crow(lane, r) == cl ? iwd : T(0);
    }
    if (lane < 16 * NTN) S.bw[lane] = rhs;
    __syncthreads();
    if (TRACE) tr[2] = __builtin_amdgcn_s_memtime();
    chol_solve<T, NTN>(acc, S, lane, bad);
    if (TRACE) tr[3] = __builtin_amdgcn_s_memtime();
    // xᵀb = uᵀK c = cᵀ(r − W⁻¹u) = Σ_e (c_e/w_e)(c_e − u_e)   (S u = r, r = W⁻¹c)
    const T ue = lane < 16 * NTN ? S.xs[lane] : T(0);
    xb = wave_sum(isP ? (double)(rhs * (cwl - ue)) : 0.0);
#pragma unroll
    for (int I = 0; I < NTN; ++I) ul[I] = S.xs[16 * I + cl];
  } else {
    // General row (some signals with v = 0: c = 1, w = 0, the set Q):
    // (W_P⁻¹ + K_PP) u_P = W_P⁻¹ c_P − K_PQ 1_Q,  u_Q = 1,  kq_e = z_eᵀ Σ_{f∈Q} z_f
    T rhs = isP ? cwl * fast_rcp(wl) : T(0);
    {
      T gpart[NTK][4];
#pragma unroll
      for (int q = 0; q < NTK; ++q)
#pragma unroll
        for (int comp = 0; comp < 4; ++comp) gpart[q][comp] = T(0);
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        const bool qe = (mQ >> (16 * I + cl)) & 1;
#pragma unroll
        for (int q = 0; q < NTK; ++q)
#pragma unroll
          for (int comp = 0; comp < 4; ++comp)
            if (qe) gpart[q][comp] += zr[I][q][comp];
      }
#pragma unroll
      for (int q = 0; q < NTK; ++q) row16_sum4(gpart[q]);
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        T sq = T(0);
#pragma unroll
        for (int q = 0; q < NTK; ++q)
#pragma unroll
          for (int comp = 0; comp < 4; ++comp) sq += zr[I][q][comp] * gpart[q][comp];
        sq += shfl_xor(sq, 16);
        sq += shfl_xor(sq, 32);
        if (kk == 0) gq[16 * I + cl] = sq;
      }
      __syncthreads();
      const T kqv = lane < 16 * NTN ? gq[lane] : T(0);
      if (isP) rhs -= kqv;
    }
    // S = W_P⁻¹ + K_PP on P×P, identity elsewhere (Q rows and padding)
    const T iw = isP ? fast_rcp(wl) : T(0);
    const uint64_t mP = __ballot(isP);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      // the diagonal element (e, e), e = 16I + cl, sits in this lane's column cl
      const T iwd = __shfl(iw, 16 * I + cl, 64);
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        const int f = 16 * J + cl;
        const bool pf = (mP >> f) & 1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 16 * I + M::crow(lane, r);
          const bool pe = (mP >> e) & 1;
          T v = acc[t][r];
          if (pe && pf) v += (e == f) ? iwd : T(0);
          else v = (e == f) ? T(1) : T(0);
          acc[t][r] = v;
        }
      }
    }
    if (lane < 16 * NTN) S.bw[lane] = rhs;
    __syncthreads();
    if (TRACE) tr[2] = __builtin_amdgcn_s_memtime();
    chol_solve<T, NTN>(acc, S, lane, bad);
    if (TRACE) tr[3] = __builtin_amdgcn_s_memtime();
    // u_e: solved for P, 1 for Q (c = 1), 0 for padding
    T cv[NTN];
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const int e = 16 * I + cl;
      const bool pe = (mP >> e) & 1;
      const bool qe = (mQ >> e) & 1;
      ul[I] = pe ? S.xs[e] : (qe ? T(1) : T(0));
      cv[I] = __shfl(cwl, e, 64);
    }
    // xᵀb = x'ᵀ(Zₛᵀc)
#pragma unroll
    for (int q = 0; q < NTK; ++q) {
      T sx[4], sb[4];
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) {
        sx[comp] = T(0);
        sb[comp] = T(0);
#pragma unroll
        for (int I = 0; I < NTN; ++I) {
          sx[comp] += zr[I][q][comp] * ul[I];
          sb[comp] += zr[I][q][comp] * cv[I];
        }
      }
      row16_sum4(sx);
      row16_sum4(sb);
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) xb += (double)sx[comp] * (double)sb[comp];
    }
    xb = wave_sum(cl == 0 ? xb : 0.0);
  }
  // x' = Zₛᵀ u, column j = 16q + 4kk + comp; lane cl == q of each group stores its 4
  // columns (a failed row stores x' = 0, so x = 0 and its loss term is 0; the host
  // re-solves it)
#pragma unroll
  for (int q = 0; q < NTK; ++q) {
    T xq[4];
#pragma unroll
    for (int comp = 0; comp < 4; ++comp) {
      T sx = T(0);
#pragma unroll
      for (int I = 0; I < NTN; ++I) sx += zr[I][q][comp] * ul[I];
      xq[comp] = sx;
    }
    row16_sum4(xq);
    if (cl == q) {
      v4 o = {xq[0], xq[1], xq[2], xq[3]};
      if (bad) o = v4{};
      reinterpret_cast<v4*>(a.X + row * KP)[4 * q + kk] = o;
    }
  }
  const double csum = wave_sum((double)cwl);
  if (lane == 0) {
    a.rowloss[row] = bad ? 0.0 : csum - xb;  // −λ‖x‖² added after unwhitening
    if (bad && a.status) a.status[row] = 1;
  }
  if (TRACE && lane == 0) {
    tr[4] = __builtin_amdgcn_s_memtime();
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* o = a.trace + 8 * (a.row_begin + i);
#pragma unroll
    for (int j = 0; j < 5; ++j) o[j] = tr[j];
    o[5] = hw | ((uint64_t)xcc << 32);
    o[6] = (uint64_t)n;
    o[7] = (uint64_t)row;
  }
}

// ---------------------------------------------------------------------------------------
// Whitened row kernel, multi-wave: the same n×n solve as wals_woodbury_kernel for factor
// counts whose whitened rows do not fit one wave's registers (fp64 k > 64, fp32 k = 256).
// One workgroup of NWK waves per row; wave w holds the column blocks q = w·KW .. w·KW+KW-1
// of the row's whitened rows Zₛ (same per-lane MFMA operand order as the one-wave kernel),
// so each wave gathers 1/NWK of every signal's row and computes K = Zₛ Zₛᵀ over its columns.
// The partial K tiles are summed in fixed order ((w0 + w2) + (w1 + w3)) through LDS into
// wave 0, which solves the n×n system alone (chol_solve with wave-local LDS ordering); u
// goes back through LDS and every wave forms x' = Zₛᵀu for its own columns.
// ---------------------------------------------------------------------------------------
#ifndef QMFX_MW_F64_NTN4_DEFAULT
#define QMFX_MW_F64_NTN4_DEFAULT 2
#endif
#ifndef QMFX_MW_NWK
// waves per row of the multi-wave whitened kernel (2 beats 4 at fp64 k = 128, 421 -> 314 ms
// per C3 user half, and the one-wave kernel at fp32 k = 256, 193 -> 167 ms per C5 user half:
// twice the rows in flight per CU, one idle wave during the n×n solve instead of three)
#define QMFX_MW_NWK 2
#endif
template <typename T, int NTK, int NTN, int NWK>
struct MwCfg {
  static constexpr int KW = (NTK + NWK - 1) / NWK;  // column blocks of 16 per wave
  static constexpr int NTT = NTN * (NTN + 1) / 2;
};

template <typename T, int NTK, int NTN, int NWK>
__global__ __launch_bounds__(64 * NWK, 2) void wals_woodbury_mw_kernel(SolveArgs<T> a) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  using v4 = typename M::acc_t;
  using C = MwCfg<T, NTK, NTN, NWK>;
  constexpr int KP = 16 * NTK;
  constexpr int KW = C::KW;
  constexpr int NTT = C::NTT;
  static_assert(NWK == 2 || NWK == 4, "wave count");  // the K reduction tree
  __shared__ __attribute__((aligned(16))) CholShared<T, NTN> S;
  __shared__ __attribute__((aligned(16))) acc_t red[NWK / 2][NTT][64];
  __shared__ T gq[NWK][16 * NTN];
  __shared__ double xbp[NWK];
  __shared__ int sbad;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const RowDesc dn = a.desc[a.row_begin + blockIdx.x];
  const int64_t row = dn.row;
  const int n = dn.n;  // ≤ 16·NTN by bucketing

  // signal e = lane (every wave holds the same copy)
  const bool mine = lane < n;
  const int cr = mine ? a.col[dn.beg + lane] : a.zrow;
  const T vr = mine ? a.val[dn.beg + lane] : T(0);
  const T wl = mine ? a.alpha * vr : T(0);
  const T cwl = mine ? T(1) + a.alpha * vr : T(0);
  const bool isP = mine && wl > T(0);
  const bool isQ = mine && wl == T(0);
  const uint64_t mQ = __ballot(isQ);
  const uint64_t mP = __ballot(isP);
  const bool hasQ = mQ != 0;

  // this wave's column blocks of Zₛ: zr[I][j] = z_{16I+cl}[16q + 4kk .. +3], q = wv·KW + j
  v4 zr[NTN][KW];
#pragma unroll
  for (int I = 0; I < NTN; ++I) {
    const int ce = __shfl(cr, 16 * I + cl, 64);
    const v4* zrow = reinterpret_cast<const v4*>(a.Y + (uint64_t)(uint32_t)ce * KP) + kk;
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const int q = wv * KW + j;
      zr[I][j] = q < NTK ? zrow[4 * q] : v4{};
    }
  }
  // partial K over this wave's columns
  acc_t acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0, 0, 0, 0};
  if constexpr (sizeof(T) == 4) {
    constexpr int NS = (KW + 1) / 2;
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      Split3 sp[NTN];
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        float x[8];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          x[c4] = zr[I][2 * s2][c4];
          x[4 + c4] = (2 * s2 + 1 < KW) ? zr[I][(2 * s2 + 1) % KW][c4] : 0.f;
        }
        split3(x, sp[I]);
      }
#pragma unroll
      for (int I = 0; I < NTN; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J) acc[tile_index(I, J)] = mma_split6(sp[I], sp[J], acc[tile_index(I, J)]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < KW; ++j)
#pragma unroll
      for (int comp = 0; comp < 4; ++comp)
#pragma unroll
        for (int I = 0; I < NTN; ++I)
#pragma unroll
          for (int J = 0; J <= I; ++J)
            acc[tile_index(I, J)] = M::mma(zr[I][j][comp], zr[J][j][comp], acc[tile_index(I, J)]);
  }
  // kq_e = z_eᵀ Σ_{f∈Q} z_f over this wave's columns (general rows only)
  if (hasQ) {
    T gpart[KW][4];
#pragma unroll
    for (int j = 0; j < KW; ++j)
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) gpart[j][comp] = T(0);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const bool qe = (mQ >> (16 * I + cl)) & 1;
#pragma unroll
      for (int j = 0; j < KW; ++j)
#pragma unroll
        for (int comp = 0; comp < 4; ++comp)
          if (qe) gpart[j][comp] += zr[I][j][comp];
    }
#pragma unroll
    for (int j = 0; j < KW; ++j) row16_sum4(gpart[j]);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      T sq = T(0);
#pragma unroll
      for (int j = 0; j < KW; ++j)
#pragma unroll
        for (int comp = 0; comp < 4; ++comp) sq += zr[I][j][comp] * gpart[j][comp];
      sq += shfl_xor(sq, 16);
      sq += shfl_xor(sq, 32);
      if (kk == 0) gq[wv][16 * I + cl] = sq;
    }
  }
  // fixed-order reduction of the K partials into wave 0: ((w0 + w2) + (w1 + w3))
#pragma unroll
  for (int h = NWK / 2; h >= 1; h /= 2) {
    if (wv >= h && wv < 2 * h) {
#pragma unroll
      for (int t = 0; t < NTT; ++t) red[wv - h][t][lane] = acc[t];
    }
    __syncthreads();
    if (wv < h) {
#pragma unroll
      for (int t = 0; t < NTT; ++t) acc[t] += red[wv][t][lane];
    }
    __syncthreads();
  }

  double xb = 0.0;
  if (wv == 0) {
    int bad = __any(mine && wl < T(0)) ? 1 : 0;  // negative confidence: not SPD in this form
    T rhs;
    if (!hasQ) {
      // every real signal in P: S = W⁻¹ + K, identity on padding slots
      const T iw = isP ? fast_rcp(wl) : T(1);
      rhs = isP ? cwl * iw : T(0);
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        const T iwd = __shfl(iw, 16 * I + cl, 64);
        const int t = tile_index(I, I);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] += M::crow(lane, r) == cl ? iwd : T(0);
      }
    } else {
      // (W_P⁻¹ + K_PP) u_P = W_P⁻¹ c_P − K_PQ 1_Q,  u_Q = 1
      rhs = isP ? cwl * fast_rcp(wl) : T(0);
      if (lane < 16 * NTN) {
        T kq = T(0);
#pragma unroll
        for (int w = 0; w < NWK; ++w) kq += gq[w][lane];
        if (isP) rhs -= kq;
      }
      const T iw = isP ? fast_rcp(wl) : T(0);
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        const T iwd = __shfl(iw, 16 * I + cl, 64);
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          const int t = tile_index(I, J);
          const int f = 16 * J + cl;
          const bool pf = (mP >> f) & 1;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int e = 16 * I + M::crow(lane, r);
            const bool pe = (mP >> e) & 1;
            T v = acc[t][r];
            if (pe && pf) v += (e == f) ? iwd : T(0);
            else v = (e == f) ? T(1) : T(0);
            acc[t][r] = v;
          }
        }
      }
    }
    if (lane < 16 * NTN) S.bw[lane] = rhs;
    csync<true>();
    chol_solve<T, NTN, true>(acc, S, lane, bad);
    if (!hasQ) {
      // xᵀb = Σ_e (c_e/w_e)(c_e − u_e)
      const T ue = lane < 16 * NTN ? S.xs[lane] : T(0);
      xb = wave_sum(isP ? (double)(rhs * (cwl - ue)) : 0.0);
    }
    if (lane == 0) sbad = bad;
  }
  __syncthreads();
  // every wave: u of its lane's signals, x' = Zₛᵀu over its columns
  T ul[NTN], cv[NTN];
#pragma unroll
  for (int I = 0; I < NTN; ++I) {
    const int e = 16 * I + cl;
    const bool pe = (mP >> e) & 1;
    const bool qe = (mQ >> e) & 1;
    ul[I] = hasQ ? (pe ? S.xs[e] : (qe ? T(1) : T(0))) : S.xs[e];
    cv[I] = __shfl(cwl, e, 64);
  }
  const bool bad = sbad != 0;
  double xbw = 0.0;
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int q = wv * KW + j;
    T xq[4], sb[4];
#pragma unroll
    for (int comp = 0; comp < 4; ++comp) {
      xq[comp] = T(0);
      sb[comp] = T(0);
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        xq[comp] += zr[I][j][comp] * ul[I];
        if (hasQ) sb[comp] += zr[I][j][comp] * cv[I];
      }
    }
    row16_sum4(xq);
    if (hasQ) {
      row16_sum4(sb);
#pragma unroll
      for (int comp = 0; comp < 4; ++comp) xbw += (double)xq[comp] * (double)sb[comp];
    }
    if (q < NTK && cl == j % 16) {
      v4 o = {xq[0], xq[1], xq[2], xq[3]};
      if (bad) o = v4{};
      reinterpret_cast<v4*>(a.X + row * KP)[4 * q + kk] = o;
    }
  }
  if (hasQ) {
    // xᵀb = x'ᵀ(Zₛᵀc): per-wave partials (one copy per 16-lane row), fixed-order total
    xbw = wave_sum(cl == 0 ? xbw : 0.0);
    if (lane == 0) xbp[wv] = xbw;
    __syncthreads();
    if (tid == 0) {
      xb = 0.0;
#pragma unroll
      for (int w = 0; w < NWK; ++w) xb += xbp[w];
    }
  }
  if (wv == 0) {
    const double csum = wave_sum((double)cwl);
    if (lane == 0) {
      a.rowloss[row] = bad ? 0.0 : csum - xb;  // −λ‖x‖² added after unwhitening
      if (bad && a.status) a.status[row] = 1;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Whitening / unwhitening GEMMs with the inverse Cholesky factor Linv = L⁻¹ (lower, KP×KP).
//   whiten:   Z[r] = Linv · Y[r]     (z = L⁻¹ y)            rows 0..n-1, 16 per wave
//   unwhiten: X[r] = Linvᵀ · X'[r]   (x = L⁻ᵀ x') in place, rows from `order`; also
//             rowloss[r] −= λ‖x‖².
// One wave computes a 16-row × KP block with NT accumulator tiles; the zero upper
// triangle of Linv is skipped.
// ---------------------------------------------------------------------------------------
template <typename T, int NT, bool UNWHITEN>
__global__ __launch_bounds__(256) void whiten_kernel(const T* in, T* out, const int64_t* order,
                                                     int64_t nrows, const T* __restrict__ Linv,
                                                     double* rowloss, double lambda) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NT;
  const int lane = threadIdx.x & 63;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (r0 >= nrows) return;
  const int64_t ra = r0 + cl < nrows ? r0 + cl : nrows - 1;
  const int64_t rowa = UNWHITEN ? order[ra] : ra;
  acc_t acc[NT];
#pragma unroll
  for (int J = 0; J < NT; ++J) acc[J] = acc_t{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < KP / 4; ++s) {
    const int m = 4 * s + kk;
    const T av = in[rowa * KP + m];
#pragma unroll
    for (int J = 0; J < NT; ++J) {
      const int j = 16 * J + cl;
      if (UNWHITEN) {
        // x_j = Σ_m x'_m Linv[m][j]: nonzero only for m ≥ j
        if (4 * s + 3 >= 16 * J) acc[J] = M::mma(av, Linv[m * KP + j], acc[J]);
      } else {
        // z_j = Σ_m Linv[j][m] y_m: nonzero only for m ≤ j
        if (4 * s <= 16 * J + 15) acc[J] = M::mma(av, Linv[j * KP + m], acc[J]);
      }
    }
  }
  // all reads of this wave's rows are done before any write (in-place unwhitening)
  T ss[4] = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t ro = r0 + M::crow(lane, r);
    if (ro < nrows) {
      const int64_t rowo = UNWHITEN ? order[ro] : ro;
#pragma unroll
      for (int J = 0; J < NT; ++J) {
        out[rowo * KP + 16 * J + cl] = acc[J][r];
        ss[r] += acc[J][r] * acc[J][r];
      }
    }
  }
  if (UNWHITEN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const T tot = row16_sum(ss[r]);
      const int64_t ro = r0 + M::crow(lane, r);
      if (cl == 0 && ro < nrows) rowloss[order[ro]] -= lambda * (double)tot;
    }
  }
}

// ---------------------------------------------------------------------------------------
// M = G + λI (padding: 1) → L (Cholesky, fp64, in LDS) → Linv = L⁻¹ written in T.
// One 256-thread workgroup; run once per half when whitened rows exist.
// ---------------------------------------------------------------------------------------
template <typename T, int NT>
__global__ __launch_bounds__(256) void chol_inv_kernel(const T* G, int k, double lambda,
                                                       T* Linv, int32_t* status) {
  constexpr int KP = 16 * NT;
  constexpr int LD = KP + 1;
  __shared__ double A[KP * LD];
  __shared__ double dinv[KP];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < KP * KP; idx += 256) {
    const int i = idx / KP, j = idx % KP;
    double v = (double)G[idx];
    if (i == j) v += i < k ? lambda : 1.0;
    A[i * LD + j] = v;
  }
  __syncthreads();
  for (int j = 0; j < KP; ++j) {
    if (tid == 0) {
      const double d = A[j * LD + j];
      if (!(d > 0.0)) *status = 1;
      const double l = sqrt(d > 0.0 ? d : 1.0);
      A[j * LD + j] = l;
      dinv[j] = 1.0 / l;
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < KP; i += 256) A[i * LD + j] *= dinv[j];
    __syncthreads();
    const int m = KP - j - 1;  // trailing size
    for (int idx = tid; idx < m * m; idx += 256) {
      const int ii = j + 1 + idx / m, mm = j + 1 + idx % m;
      if (mm <= ii) A[ii * LD + mm] -= A[ii * LD + j] * A[mm * LD + j];
    }
    __syncthreads();
  }
  // Linv column c (thread c): Linv[c][c] = 1/L[c][c];
  // Linv[i][c] = −(Σ_{m=c}^{i−1} L[i][m] Linv[m][c]) / L[i][i], kept in A's upper triangle
  // at A[c][i] (row c is private to thread c)
  if (tid < KP) {
    const int c = tid;
    for (int i = c + 1; i < KP; ++i) {
      double s = A[i * LD + c] * dinv[c];
      for (int m = c + 1; m < i; ++m) s += A[i * LD + m] * A[c * LD + m];
      A[c * LD + i] = -s * dinv[i];
    }
  }
  __syncthreads();
  for (int idx = tid; idx < KP * KP; idx += 256) {
    const int i = idx / KP, c = idx % KP;
    double v = 0.0;
    if (i == c) v = dinv[c];
    else if (i > c) v = A[c * LD + i];
    Linv[idx] = (T)v;
  }
}

// ---------------------------------------------------------------------------------------
// YᵀY (WALSEngine.cpp:246-264, without its OpenMP race): each wave accumulates a block of
// rows into all lower tiles with MFMA and writes its partial; a second kernel adds the
// partials in fixed order (deterministic) in fp64 and mirrors the upper triangle.
// ---------------------------------------------------------------------------------------
template <typename T, int NT>
__global__ __launch_bounds__(64) void gram_partial_kernel(const T* Y, int64_t n,
                                                          int64_t rows_per_block,
                                                          double* partial) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  acc_t acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0, 0, 0, 0};
  for (int64_t e0 = r0; e0 < r1; e0 += 4) {
    const int64_t e = e0 + kk;
    const bool valid = e < r1;
    const T* yrow = Y + (valid ? e : r0) * KP + cl;
    T yv[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) yv[q] = valid ? yrow[16 * q] : T(0);
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        acc[t] = M::mma(yv[I], yv[J], acc[t]);
      }
    }
  }
  double* out = partial + (int64_t)blockIdx.x * NTT * 256;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) out[t * 256 + M::crow(lane, r) * 16 + cl] = (double)acc[t][r];
  }
}

// Fixed-order sum of the partials: 16 outputs per 256-thread block, each summed as 16
// consecutive chunks of blocks (thread (chunk, output)), then the chunk sums in order —
// deterministic, and 16× the parallelism of one thread per output (C2: 0.32 → ~0.03 ms).
__device__ __forceinline__ double gram_reduce_one(const double* partial, int nblocks,
                                                  int64_t stride, int off, double (*red)[16],
                                                  int o, int ch) {
  const int cs = (nblocks + 15) / 16;
  const int b0 = ch * cs, b1 = b0 + cs < nblocks ? b0 + cs : nblocks;
  double s = 0.0;
  for (int b = b0; b < b1; ++b) s += partial[(int64_t)b * stride + off];
  red[ch][o] = s;
  __syncthreads();
  double t = 0.0;
  if (ch == 0)
    for (int c = 0; c < 16; ++c) t += red[c][o];
  return t;
}

template <typename T, int NT>
__global__ __launch_bounds__(256) void gram_reduce_kernel(const double* partial, int nblocks, T* G) {
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  __shared__ double red[16][16];
  const int o = threadIdx.x & 15, ch = threadIdx.x >> 4;
  const int idx = blockIdx.x * 16 + o;  // KP² is a multiple of 16
  const int i = idx / KP, j = idx % KP;
  const int ii = i >= j ? i : j, jj = i >= j ? j : i;  // lower-triangle element
  const int t = tile_index(ii >> 4, jj >> 4);
  const int off = t * 256 + (ii & 15) * 16 + (jj & 15);
  const double s = gram_reduce_one(partial, nblocks, (int64_t)NTT * 256, off, red, o, ch);
  if (ch == 0) G[idx] = (T)s;
}

// Fixed-order sum of the per-row losses: per-block partials in fixed slots, then one
// block adds them in order (deterministic; the value is a reporting quantity only).
constexpr int kSumBlocks = 512;
__global__ __launch_bounds__(256) void sum_f64_partial_kernel(const double* x, int64_t n,
                                                              double* partial) {
  __shared__ double red[4];
  const int64_t chunk = (n + kSumBlocks - 1) / kSumBlocks;
  const int64_t b = (int64_t)blockIdx.x * chunk;
  const int64_t e = b + chunk < n ? b + chunk : n;
  double s = 0.0;
  for (int64_t i = b + threadIdx.x; i < e; i += 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ __launch_bounds__(256) void sum_f64_final_kernel(const double* partial, double* out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < kSumBlocks; i += 256) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = red[0] + red[1] + red[2] + red[3];
}

// MFMA layout self-test: C(16×16) = A(16×4) · B(4×16) written row-major via crow().
template <typename T>
__global__ void mfma_selftest_kernel(const T* A, const T* B, T* C) {
  using M = Mfma<T>;
  const int lane = threadIdx.x;
  typename M::acc_t acc = {0, 0, 0, 0};
  acc = M::mma(A[(lane & 15) * 4 + (lane >> 4)], B[(lane >> 4) * 16 + (lane & 15)], acc);
  for (int r = 0; r < 4; ++r) C[M::crow(lane, r) * 16 + (lane & 15)] = acc[r];
}

// ---------------------------------------------------------------------------------------
// Host launchers.  (QMFX_KERNELS_ONLY: kernel-only builds for ISA inspection, tools/isa_one.sh)
// ---------------------------------------------------------------------------------------
#ifndef QMFX_KERNELS_ONLY
template <typename T, int NT>
static hipError_t launch_direct_nt(const SolveArgs<T>& a, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc || !a.Gimg) return hipErrorInvalidValue;
  return launch_row_chunks(a, 64, [&](const SolveArgs<T>& c) {
    if (c.trace)
      hipLaunchKernelGGL((wals_direct_kernel<T, NT, true>), dim3((unsigned)c.nrows), dim3(64), 0, s, c);
    else
      hipLaunchKernelGGL((wals_direct_kernel<T, NT, false>), dim3((unsigned)c.nrows), dim3(64), 0, s, c);
  });
}

template <typename T, int NT>
static hipError_t launch_gimg_nt(const T* G, int k, double lambda, T* img, hipStream_t s) {
  constexpr int NTT = NT * (NT + 1) / 2;
  hipLaunchKernelGGL((gimg_kernel<T, NT>), dim3(NTT), dim3(256), 0, s, G, k, lambda, img);
  return hipGetLastError();
}

template <typename T, int NTK>
static hipError_t launch_woodbury_ntk(const SolveArgs<T>& a, int ntn, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc) return hipErrorInvalidValue;
  const dim3 b(64);
#define QMFX_WB(N)                                                                            \
  return launch_row_chunks(a, 64, [&](const SolveArgs<T>& c) {                                \
    if (c.trace)                                                                              \
      hipLaunchKernelGGL((wals_woodbury_kernel<T, NTK, N, true>), dim3((unsigned)c.nrows), b, 0, s, c); \
    else                                                                                      \
      hipLaunchKernelGGL((wals_woodbury_kernel<T, NTK, N, false>), dim3((unsigned)c.nrows), b, 0, s, c); \
  })
  if (ntn == 1) {
    QMFX_WB(1);
  } else if (ntn == 2) {
    if constexpr (NTK >= 4) QMFX_WB(2);
    else return hipErrorInvalidValue;
  } else if (ntn == 3) {
    if constexpr (NTK >= 6) QMFX_WB(3);
    else return hipErrorInvalidValue;
  } else if (ntn == 4) {
    if constexpr (NTK >= 8) QMFX_WB(4);
    else return hipErrorInvalidValue;
#undef QMFX_WB
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// multi-wave whitened kernel: 4 waves per row
// fp64 n×n bucket 4 at k = 128: 2 waves per row spill 76 VGPRs, 4 waves do not
// (QMFX_MW_F64_NTN4 = 2 or 4 picks one for comparisons)
static int mw_f64_ntn4_waves() {
  const char* e = std::getenv("QMFX_MW_F64_NTN4");
  return e ? std::atoi(e) : QMFX_MW_F64_NTN4_DEFAULT;
}

template <typename T, int NTK>
static hipError_t launch_woodbury_mw_ntk(const SolveArgs<T>& a, int ntn, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc) return hipErrorInvalidValue;
  constexpr int NWK = QMFX_MW_NWK;
  if constexpr (sizeof(T) == 8 && NTK >= 8) {
    if (ntn == 4 && mw_f64_ntn4_waves() == 4)
      return launch_row_chunks(a, 256, [&](const SolveArgs<T>& c) {
        hipLaunchKernelGGL((wals_woodbury_mw_kernel<T, NTK, 4, 4>), dim3((unsigned)c.nrows),
                           dim3(256), 0, s, c);
      });
  }
#define QMFX_WBMW(N)                                                                   \
  return launch_row_chunks(a, 64 * NWK, [&](const SolveArgs<T>& c) {                   \
    hipLaunchKernelGGL((wals_woodbury_mw_kernel<T, NTK, N, NWK>), dim3((unsigned)c.nrows), \
                       dim3(64 * NWK), 0, s, c);                                       \
  })
  switch (ntn) {
    case 1: QMFX_WBMW(1);
    case 2: QMFX_WBMW(2);
    case 3:
      if constexpr (NTK >= 6) QMFX_WBMW(3);
      return hipErrorInvalidValue;
    case 4:
      if constexpr (NTK >= 8) QMFX_WBMW(4);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
#undef QMFX_WBMW
}

// fp32 k = 256: the multi-wave kernel, or the one-wave one with QMFX_WB_MW=0
static bool wb_mw_fp32() {
  const char* e = std::getenv("QMFX_WB_MW");
  return !e || std::atoi(e) != 0;
}

template <typename T, int NT>
static hipError_t launch_whiten_nt(const T* in, T* out, const int64_t* order, int64_t nrows,
                                   const T* Linv, double* rowloss, double lambda, bool unwhiten,
                                   hipStream_t s) {
  if (nrows <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((nrows + 63) / 64);
  if (unwhiten)
    hipLaunchKernelGGL((whiten_kernel<T, NT, true>), dim3(blocks), dim3(256), 0, s, in, out, order,
                       nrows, Linv, rowloss, lambda);
  else
    hipLaunchKernelGGL((whiten_kernel<T, NT, false>), dim3(blocks), dim3(256), 0, s, in, out,
                       order, nrows, Linv, rowloss, lambda);
  return hipGetLastError();
}

// The same factorization for KP > 128 (the fp64 matrix exceeds LDS): one 1024-thread
// workgroup on a global fp64 scratch of KP·(KP+1) doubles (L2-resident; __syncthreads
// orders the block's global accesses).  Once per half; ≈ms at KP = 256.
template <typename T, int NT>
__global__ __launch_bounds__(1024) void chol_inv_global_kernel(const T* G, int k, double lambda,
                                                               T* Linv, int32_t* status,
                                                               double* A) {
  constexpr int KP = 16 * NT;
  constexpr int LD = KP + 1;
  __shared__ double dinv[KP];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < KP * KP; idx += 1024) {
    const int i = idx / KP, j = idx % KP;
    double v = (double)G[idx];
    if (i == j) v += i < k ? lambda : 1.0;
    A[i * LD + j] = v;
  }
  __syncthreads();
  for (int j = 0; j < KP; ++j) {
    if (tid == 0) {
      const double d = A[j * LD + j];
      if (!(d > 0.0)) *status = 1;
      const double l = sqrt(d > 0.0 ? d : 1.0);
      A[j * LD + j] = l;
      dinv[j] = 1.0 / l;
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < KP; i += 1024) A[i * LD + j] *= dinv[j];
    __syncthreads();
    const int m = KP - j - 1;
    for (int idx = tid; idx < m * m; idx += 1024) {
      const int ii = j + 1 + idx / m, mm = j + 1 + idx % m;
      if (mm <= ii) A[ii * LD + mm] -= A[ii * LD + j] * A[mm * LD + j];
    }
    __syncthreads();
  }
  if (tid < KP) {
    const int c = tid;
    for (int i = c + 1; i < KP; ++i) {
      double sm = A[i * LD + c] * dinv[c];
      for (int mm = c + 1; mm < i; ++mm) sm += A[i * LD + mm] * A[c * LD + mm];
      A[c * LD + i] = -sm * dinv[i];
    }
  }
  __syncthreads();
  for (int idx = tid; idx < KP * KP; idx += 1024) {
    const int i = idx / KP, c = idx % KP;
    double v = 0.0;
    if (i == c) v = dinv[c];
    else if (i > c) v = A[c * LD + i];
    Linv[idx] = (T)v;
  }
}

template <typename T, int NT>
static hipError_t launch_chol_inv_nt(const T* G, int k, double lambda, T* Linv, int32_t* status,
                                     double* scratch, hipStream_t s) {
  if constexpr (NT > 8) {
    if (!scratch) return hipErrorInvalidValue;
    hipLaunchKernelGGL((chol_inv_global_kernel<T, NT>), dim3(1), dim3(1024), 0, s, G, k, lambda,
                       Linv, status, scratch);
    return hipGetLastError();
  } else {
    (void)scratch;
    hipLaunchKernelGGL((chol_inv_kernel<T, NT>), dim3(1), dim3(256), 0, s, G, k, lambda, Linv,
                       status);
    return hipGetLastError();
  }
}

template <typename T, int NT>
static hipError_t launch_gram_nt(const T* Y, int64_t n, T* G, double* partial,
                                 int max_blocks, hipStream_t s) {
  int64_t rpb = (n + max_blocks - 1) / max_blocks;
  rpb = ((rpb + 3) / 4) * 4;
  if (rpb < 64) rpb = 64;
  const int nblocks = (int)((n + rpb - 1) / rpb);
  if (nblocks > 0) {
    hipLaunchKernelGGL((gram_partial_kernel<T, NT>), dim3(nblocks), dim3(64), 0, s, Y, n, rpb,
                       partial);
  }
  constexpr int KP = 16 * NT;
  hipLaunchKernelGGL((gram_reduce_kernel<T, NT>), dim3(KP * KP / 16), dim3(256), 0, s,
                     partial, nblocks, G);
  return hipGetLastError();
}

#define QMFX_NT_SWITCH(NTV, CALL)         \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    case 5: return CALL(5);               \
    case 6: return CALL(6);               \
    case 7: return CALL(7);               \
    case 8: return CALL(8);               \
    default: return hipErrorInvalidValue; \
  }
// fp32 whitened path: every one-wave tiling plus k = 256 (NT = 16, beside the multi-wave
// direct kernel)
#define QMFX_NT_SWITCH_W(NTV, CALL)       \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    case 5: return CALL(5);               \
    case 6: return CALL(6);               \
    case 7: return CALL(7);               \
    case 8: return CALL(8);               \
    case 16: return CALL(16);             \
    default: return hipErrorInvalidValue; \
  }
#define QMFX_NT_SWITCH64(NTV, CALL)       \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_gimg(const float* G, int nt, int k, double lambda, float* img, hipStream_t s) {
#define CALL(N) launch_gimg_nt<float, N>(G, k, lambda, img, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_gimg(const double* G, int nt, int k, double lambda, double* img,
                       hipStream_t s) {
#define CALL(N) launch_gimg_nt<double, N>(G, k, lambda, img, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_wals_direct(const SolveArgs<float>& a, int nt, hipStream_t s) {
#define CALL(N) launch_direct_nt<float, N>(a, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_wals_direct(const SolveArgs<double>& a, int nt, hipStream_t s) {
#define CALL(N) launch_direct_nt<double, N>(a, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_wals_woodbury(const SolveArgs<float>& a, int nt, int ntn, hipStream_t s) {
  if (nt == 16 && wb_mw_fp32()) return launch_woodbury_mw_ntk<float, 16>(a, ntn, s);
#define CALL(N) launch_woodbury_ntk<float, N>(a, ntn, s)
  QMFX_NT_SWITCH_W(nt, CALL)
#undef CALL
}
hipError_t launch_wals_woodbury(const SolveArgs<double>& a, int nt, int ntn, hipStream_t s) {
  // one wave up to k = 64; k = 80..128 on the multi-wave kernel
  switch (nt) {
    case 5: return launch_woodbury_mw_ntk<double, 5>(a, ntn, s);
    case 6: return launch_woodbury_mw_ntk<double, 6>(a, ntn, s);
    case 7: return launch_woodbury_mw_ntk<double, 7>(a, ntn, s);
    case 8: return launch_woodbury_mw_ntk<double, 8>(a, ntn, s);
    default: break;
  }
#define CALL(N) launch_woodbury_ntk<double, N>(a, ntn, s)
  QMFX_NT_SWITCH64(nt, CALL)
#undef CALL
}
hipError_t launch_whiten(const float* in, float* out, const int64_t* order, int64_t nrows,
                         int nt, const float* Linv, double* rowloss, double lambda,
                         bool unwhiten, hipStream_t s) {
#define CALL(N) launch_whiten_nt<float, N>(in, out, order, nrows, Linv, rowloss, lambda, unwhiten, s)
  QMFX_NT_SWITCH_W(nt, CALL)
#undef CALL
}
hipError_t launch_whiten(const double* in, double* out, const int64_t* order, int64_t nrows,
                         int nt, const double* Linv, double* rowloss, double lambda,
                         bool unwhiten, hipStream_t s) {
#define CALL(N) launch_whiten_nt<double, N>(in, out, order, nrows, Linv, rowloss, lambda, unwhiten, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_chol_inv(const float* G, int nt, int k, double lambda, float* Linv,
                           int32_t* status, double* scratch, hipStream_t s) {
#define CALL(N) launch_chol_inv_nt<float, N>(G, k, lambda, Linv, status, scratch, s)
  QMFX_NT_SWITCH_W(nt, CALL)
#undef CALL
}
hipError_t launch_chol_inv(const double* G, int nt, int k, double lambda, double* Linv,
                           int32_t* status, double* scratch, hipStream_t s) {
#define CALL(N) launch_chol_inv_nt<double, N>(G, k, lambda, Linv, status, scratch, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_gram(const float* Y, int64_t n, int nt, float* G, double* partial,
                       int max_blocks, hipStream_t s) {
#define CALL(N) launch_gram_nt<float, N>(Y, n, G, partial, max_blocks, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_gram(const double* Y, int64_t n, int nt, double* G, double* partial,
                       int max_blocks, hipStream_t s) {
#define CALL(N) launch_gram_nt<double, N>(Y, n, G, partial, max_blocks, s)
  QMFX_NT_SWITCH64(nt, CALL)
#undef CALL
}

// `out` must have room for kSumBlocks + 1 doubles: out[0] = sum, out[1..] = partials.
hipError_t launch_sum_f64(const double* x, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_f64_partial_kernel, dim3(kSumBlocks), dim3(256), 0, s, x, n, out + 1);
  hipLaunchKernelGGL(sum_f64_final_kernel, dim3(1), dim3(256), 0, s, out + 1, out);
  return hipGetLastError();
}

hipError_t launch_mfma_selftest_f32(const float* A, const float* B, float* C, hipStream_t s) {
  hipLaunchKernelGGL(mfma_selftest_kernel<float>, dim3(1), dim3(64), 0, s, A, B, C);
  return hipGetLastError();
}
hipError_t launch_mfma_selftest_f64(const double* A, const double* B, double* C,
                                    hipStream_t s) {
  hipLaunchKernelGGL(mfma_selftest_kernel<double>, dim3(1), dim3(64), 0, s, A, B, C);
  return hipGetLastError();
}
#endif  // QMFX_KERNELS_ONLY

}  // namespace qmfx
