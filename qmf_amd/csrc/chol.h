// Register-tile Cholesky + solve of one SPD system per wave64 (shared by the direct and
// the whitened row kernels).
#pragma once
#include "common.h"
#include "rowsolve.h"

namespace qmfx {

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
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T>
struct CholLd {
  // padded LDS row of a panel: fp32 rows are 16-B aligned and conflict-free for the
  // b128 row accesses and the MFMA-layout tile accesses used here
  static constexpr int PLD = sizeof(T) == 4 ? 20 : 17;
};

// LTP = true keeps the diagonal L blocks (Lt) in the panel array instead of an array of their
// own: panel p stages rows [0, 16·(NT−p)), so the rows past them are free, and block p goes
// to rows [16·(NT−p−1), 16·(NT−p)) once panel p's last tile has been read back.  Half the LDS
// (the whitened fp64 kernel at n ≤ 64: 19.5 → 10.8 KB per row, three rows per SIMD).
template <typename T, int NT, bool LTP = false>
struct CholShared {
  static constexpr int PLD = CholLd<T>::PLD;
  static constexpr bool kLtInPanel = LTP;
  T panel[16 * NT * PLD];
  T Lt[LTP ? 1 : NT * 16 * PLD];
  T bw[16 * NT];
  T xs[16 * NT];
  T invd[16 * NT];
  // row r of the transposed, column-scaled diagonal L blocks
  __device__ __forceinline__ T* lt_row(int r) {
    if constexpr (LTP)
      return &panel[(16 * (NT - 1 - (r >> 4)) + (r & 15)) * PLD];
    else
      return &Lt[r * PLD];
  }
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

template <typename T, int NT, bool WS = false, bool LTP = false>
__device__ __forceinline__ void chol_solve(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                           CholShared<T, NT, LTP>& S, int lane, int& bad) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr int SLOTS = (KP + 63) / 64;
  constexpr int PLD = CholShared<T, NT, LTP>::PLD;
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
            } else {
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
    T ltv[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = lane + 64 * it;
      const int r = idx >> 4, c = idx & 15;
      ltv[it] = c < r ? S.panel[r * PLD + c] * S.invd[16 * p + c] : T(0);
    }
    if constexpr (!LTP) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = lane + 64 * it;
        S.lt_row(p * 16 + (idx & 15))[idx >> 4] = ltv[it];
      }
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
    }
    if constexpr (LTP) {
      // block p lands on the panel's last 16 rows (tile (NT−1, p), or at p = NT−1 the
      // diagonal block itself): the reads of them above have returned first (the asm
      // fence also keeps the compiler's order; one wave reads and writes these rows)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = lane + 64 * it;
        S.lt_row(p * 16 + (idx & 15))[idx >> 4] = ltv[it];
      }
    }
#pragma unroll
    for (int I = p + 1; I < NT; ++I) {
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
    lds_row_load(S.lt_row(16 * I + cl), lt);
#pragma unroll
    for (int c = 15; c >= 0; --c) vm -= lt[c] * readlane(vm, c);
    if (lane < 16) S.xs[16 * I + lane] = vm;
    csync<WS>();
  }
}

// The row kernels' factorization (the 4-column-panel form measured slower in round 4 is kept
// under tools/exp/chol4.h)
template <typename T, int NT, bool LTP>
__device__ __forceinline__ void row_chol(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                         CholShared<T, NT, LTP>& S, int lane, int& bad) {
  chol_solve<T, NT, false, LTP>(acc, S, lane, bad);
}

}  // namespace qmfx
