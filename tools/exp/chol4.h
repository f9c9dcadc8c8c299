// Cholesky + solve of one SPD system per wave64 by 4-column panels (shared by the fp64
// whitened and direct row kernels; same contract as chol_solve in chol.h).
//
// The register-tile Cholesky of chol.h factors 16-column panels: per column it broadcasts
// the diagonal block's column with 30 readlanes and runs the pivot's dependent chain, so a
// 64×64 fp64 system costs ≈48K cycles per wave (profiles/r04: removing the factorization
// from the C3 fp64 whitened class saves 38 of its 184 ms).  Here a panel is 4 columns wide,
// the K depth of one v_mfma_f64_16x16x4: the panel's rows move to one row per lane through
// LDS (a 48-byte row each), its 4 pivots run there with at most 6 readlanes per column, the
// finished L columns go back to the tiles and, in MFMA operand order, feed ONE MFMA per
// trailing tile (a rank-4 update).  The tile column the next panel reads is updated first.
//
// Reference: linearSymmetricSolve → dsysv_ (qmf/Matrix.cpp:81-96); the systems here are SPD
// (the callers flag a non-positive pivot and the row is re-solved by the pivoted fallback,
// fallback.hip, as dsysv_'s role).
#pragma once
#include <utility>

#include "chol.h"

namespace qmfx {

template <typename T, int NT, bool WS = false>
__device__ __forceinline__ void chol4_solve(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                            CholShared<T, NT>& S, int lane, int& bad) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr int SLOTS = (KP + 63) / 64;
  constexpr int PLD = CholShared<T, NT>::PLD;
  // panel staging rows of 6 values (48 B at fp64): 16-B aligned row reads, and the MFMA
  // operand reads (lane (x, k) → row 16X + x, value k) hit 64 distinct banks
  constexpr int PS = 6;
  // rows past KP (the last slot's idle lanes) read and write P too, unconditionally (a
  // divergent branch there cost the NT = 5 tiling 222 spilled VGPRs): S.panel holds them
  static_assert(64 * SLOTS * PS <= 16 * NT * PLD, "panel staging must fit S.panel");
  T* P = S.panel;
  const int cl = lane & 15;
  const int kk = lane >> 4;

  // forward-substitution right-hand side, one row per lane (row lane + 64s)
  T bv[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) bv[s] = lane + 64 * s < KP ? S.bw[lane + 64 * s] : T(0);

  // the panels as a fold over compile-time indices (a `#pragma unroll` loop stays rolled past
  // the unroller's size limit at NT = 8, and a runtime tile index puts acc in scratch)
  auto panel = [&](auto pc) {
    constexpr int p = decltype(pc)::value;
    constexpr int J = p >> 2;       // tile column of the panel
    constexpr int q0 = 4 * (p & 3); // its first column inside the tile
    constexpr int c0 = 16 * J + q0; // its first global column
    // lanes cl = q0..q0+3 hold the panel's columns in the tiles; their panel column is
    // cl & 3, so every P address below is a per-lane base plus a compile-time offset (no
    // per-panel address registers)
    const bool own = (cl >> 2) == (q0 >> 2);
    const int qc = cl & 3;
    // (A) columns c0..c0+3 of the tiles (I, J), I ≥ J → P[row][0..3]
#pragma unroll
    for (int I = J; I < NT; ++I) {
      const int t = tile_index(I, J);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (own) P[(16 * I + M::crow(lane, r)) * PS + qc] = acc[t][r];
    }
    csync<WS>();
    T a[SLOTS][4];
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int row = lane + 64 * s;
      const bool in = 64 * s + 63 < KP || row < KP;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const T v = P[row * PS + q];
        a[s][q] = in ? v : T(0);
      }
    }
    // (B) the panel's 4 columns, right-looking inside the panel; rows above a pivot only
    // change their dead upper part, and the forward solve rides along in bv
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + q;
      const T d = readlane(a[c >> 6][q], c & 63);
      const T bc = readlane(bv[c >> 6], c & 63);
      T ljj, inv;
      pivot_sqrt(d, ljj, inv);
      (void)ljj;
      // a pivot that is not positive (or not finite) leaves 1/√d outside (0, ∞); the flag is
      // pinned here (left to the compiler, all the pivots stayed live to the end: +128 VGPRs)
      if (!(inv > T(0) && inv < __builtin_huge_val())) bad = 1;
      asm volatile("" : "+v"(bad));
      const T yc = bc * inv;
      if (lane == (c & 63)) {
        S.invd[c] = inv;
        S.bw[c] = yc;
      }
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        const T lq = a[s][q] * inv;
        a[s][q] = lq;
        bv[s] -= lq * yc;
      }
#pragma unroll
      for (int q2 = q + 1; q2 < 4; ++q2) {
        const int c2 = c0 + q2;
        const T lm = readlane(a[c2 >> 6][q], c2 & 63);  // L[c2][c]
#pragma unroll
        for (int s = 0; s < SLOTS; ++s) a[s][q2] -= a[s][q] * lm;
      }
      // pin the updates of the rows past the first 64 to this column (chol_solve's fence):
      // left free, the compiler defers them to the panel's end with every broadcast live
#pragma unroll
      for (int s = 1; s < SLOTS; ++s) {
#pragma unroll
        for (int q2 = q; q2 < 4; ++q2) asm volatile("" : "+v"(a[s][q2]));
        asm volatile("" : "+v"(bv[s]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    csync<WS>();
    // (C) the finished L columns back to P; rows above the panel are zero there (they are
    // the upper part, and as MFMA operands of block J they must contribute nothing)
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int row = lane + 64 * s;
      const bool live = row >= c0 && (64 * s + 63 < KP || row < KP);
#pragma unroll
      for (int q = 0; q < 4; ++q) P[row * PS + q] = live ? a[s][q] : T(0);
    }
    csync<WS>();
    // (D) L into the tiles' columns c0..c0+3 (the backward solve and later panels read them)
#pragma unroll
    for (int I = J; I < NT; ++I) {
      const int t = tile_index(I, J);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const T v = P[(16 * I + M::crow(lane, r)) * PS + qc];
        if (own) acc[t][r] = v;
      }
    }
    // (E) MFMA operands: lane (x, k) holds L[16X + x][c0 + k] for the blocks X ≥ J
    T F[NT];
#pragma unroll
    for (int X = J; X < NT; ++X) F[X] = P[(16 * X + cl) * PS + kk];
    // block J as the column side: its columns up to c0+3 are final, so their B rows are 0
    const T FJ = cl >= q0 + 4 ? F[J] : T(0);
    // (F) rank-4 trailing update, the next panel's tile column first
    if constexpr ((p & 3) < 3) {
#pragma unroll
      for (int I = J; I < NT; ++I) {
        const int t = tile_index(I, J);
        acc[t] = M::mma(-F[I], FJ, acc[t]);
      }
    }
#pragma unroll
    for (int J2 = J + 1; J2 < NT; ++J2) {
#pragma unroll
      for (int I = J2; I < NT; ++I) {
        const int t = tile_index(I, J2);
        acc[t] = M::mma(-F[I], F[J2], acc[t]);
      }
    }
    csync<WS>();  // the next panel overwrites P
    // one panel per scheduling window: interleaved panels keep every panel's LDS reads and
    // operands live at once
    __builtin_amdgcn_sched_barrier(0);
  };
  [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
    (panel(std::integral_constant<int, Ps>{}), ...);
  }(std::make_integer_sequence<int, 4 * NT>{});

  // diagonal L blocks → Lt (transposed, scaled by the column's 1/L[q][q], zero on and above
  // the diagonal), as chol_solve leaves them for its backward solve
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    const int t = tile_index(J, J);
    const T dc = S.invd[16 * J + cl];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = M::crow(lane, r);
      S.Lt[(16 * J + cl) * PLD + row] = cl < row ? acc[t][r] * dc : T(0);
    }
  }
  csync<WS>();
  // backward solve Lᵀ x = y by 16-blocks from the bottom (chol_solve's): lane cl carries row
  // cl of the block scaled by its own 1/L[cl][cl]; column c then finishes x_c (readlane) and
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

// The row kernels' factorization: chol_solve; QMFX_CHOL4=1 puts fp64 systems of 32 rows and
// more on the 4-column panels (one 16×16 tile stays on chol_solve: its panel staging would
// not fit S.panel).  Measured (profiles/r04/ab_chol4_c3_f64.txt, same box): SLOWER — C3 fp64
// whitened class 187 → 198 ms, direct item half 188 → 210 ms; traces: the 64×64 factorization
// 48K → 59K cycles, the 128×128 one 83K → 110K.  In one wave the rank-4 trailing MFMAs (70
// instead of 40 at NT = 4, 444 instead of 336 at NT = 8) issue in order on the critical path,
// and each 4-column panel pays two LDS round trips, where chol_solve pays one per 16 columns.
#ifndef QMFX_CHOL4
#define QMFX_CHOL4 0
#endif
template <typename T, int NT, bool LTP>
__device__ __forceinline__ void row_chol(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                         CholShared<T, NT, LTP>& S, int lane, int& bad) {
  if constexpr (sizeof(T) == 8 && NT >= 2 && QMFX_CHOL4 && !LTP)
    chol4_solve<T, NT>(acc, S, lane, bad);
  else
    chol_solve<T, NT>(acc, S, lane, bad);
}

}  // namespace qmfx
