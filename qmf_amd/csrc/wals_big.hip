// WALS row solve for large factor counts (fp32 k > 128, fp64 k > 64; up to k = 256).
//
// Reference path: WALSEngine::updateFactorsForOne (qmf/wals/WALSEngine.cpp:266-310) and
// linearSymmetricSolve → dsysv_ (qmf/Matrix.cpp:81-96), as in wals.hip.  At large k one
// wave cannot hold the k×k system in registers, so one WORKGROUP of NW waves solves a row:
//
//   * the NT(NT+1)/2 lower 16×16 tiles of A are distributed round-robin over the waves and
//     stay in their registers for the whole solve;
//   * Gram: the row's fixed-side rows are staged into LDS SIG signals at a time (double
//     buffer, register-staged loads of the next stage in flight during the MFMAs); every
//     wave reads its tiles' operands from LDS, so the tile→wave map is a runtime table;
//   * Cholesky, right-looking over 16-column panels: owners write panel column p to LDS,
//     wave 0 factors its diagonal block and the next 48 rows, the waves solve the remaining
//     rows 64 at a time in parallel (with the forward solve of b), then every wave applies
//     the rank-16 trailing update to its own tiles with MFMA (operands from the LDS panel);
//   * backward solve by 16-blocks: owners of L(J, I) tiles add their part of Lᵀx in LDS,
//     wave 0 finishes the block with the diagonal triangle.
// Same results contract as the single-wave kernels: status[row] = 1 on a non-positive pivot.
#include <type_traits>
#include <utility>

#include "common.h"

// `#pragma unroll 2` on the Gram step loops is not honoured for every tiling (those keep a
// rolled loop); dropping the hint costs the fp32 NT = 16 kernels 24-44 VGPRs, so it stays
#pragma clang diagnostic ignored "-Wpass-failed"
#include "kernels.h"
#include "rowsolve.h"
#include "chol.h"

#ifndef QMFX_BIG_SIG32
#define QMFX_BIG_SIG32 32
#endif
#ifndef QMFX_BIG_NW32
#define QMFX_BIG_NW32 8  // waves per row at fp32 k > 160
#endif
#ifndef QMFX_BIG_SIG64
#define QMFX_BIG_SIG64 16
#endif
#ifndef QMFX_BIG_SPLIT
#define QMFX_BIG_SPLIT 1  // fp32 k = 256: the split-bf16 Gram from LDS (QMFX_BIG_SPLIT=0: f32 MFMA)
#endif
#ifndef QMFX_BIG_STREAM
#define QMFX_BIG_STREAM 1  // fp64: per-wave streamed Gram (0: the LDS-staged Gram)
#endif
#ifndef QMFX_BIG_LDL32
#define QMFX_BIG_LDL32 1  // fp32 k = 256: wave-specialised rows with the LDLᵀ (0: the Cholesky)
#endif
#ifndef QMFX_BIG_PAIR64
#define QMFX_BIG_PAIR64 1  // fp64 k = 256: row-pair tile map (0: round-robin)
#endif

namespace qmfx {

template <typename T, int NT>
struct BigCfg {
  static constexpr int KP = 16 * NT;
  static constexpr int NTT = NT * (NT + 1) / 2;
  // waves per row: ≤ 17 fp32 / ≤ 10 fp64 accumulator tiles per wave (fp64 NT ≤ 8: the tiled
  // YᵀY only; those rows run the one-wave direct kernel)
  static constexpr int NW = sizeof(T) == 4 ? (NT <= 10 ? 4 : QMFX_BIG_NW32) : (NT <= 8 ? 4 : 8);
  // split-bf16 Gram (fp32, NT = 2·NW): the loader threads split each staged element once
  // into bf16 hi/mid/lo planes ([column][signal], 32 signals = one 16x16x32 MFMA K step)
  // and wave W owns block rows W and NT−1−W (NT + 1 tiles), reading each column block's
  // planes once per stage for both rows
  static constexpr bool SPLIT = sizeof(T) == 4 && NT == 2 * NW && QMFX_BIG_SPLIT;
  // fp64: every wave gathers its own operand fragments of the row's signals (big_gram_stream),
  // with no LDS staging and no barrier in the Gram
  static constexpr bool STREAM = sizeof(T) == 8 && QMFX_BIG_STREAM;
  // row-pair tile map (wave W owns block rows W and NT−1−W: NT + 1 tiles)
  static constexpr bool PAIR = SPLIT || (STREAM && NT == 2 * NW && QMFX_BIG_PAIR64);
  // one wave-specialised copy of the row solve per wave (compile-time tile map) and the LDLᵀ
  // factorization (big_ldl_solve): the streamed fp64 rows and the split fp32 rows
  static constexpr bool WSPEC = STREAM || (SPLIT && QMFX_BIG_LDL32);
  // waves per SIMD the row kernel is compiled for (512-thread workgroups: two)
  static constexpr int WPE = (64 * NW + 255) / 256;
  // LDLᵀ panel buffers: two (no barrier between a panel's readers and the next panel's
  // stores), or one when more than two workgroups share a CU's LDS
  static constexpr bool PANEL2 = WSPEC && (NT > 8 || WPE <= 2);
  static constexpr int TPW = PAIR ? NT + 1 : (NTT + NW - 1) / NW;
  static constexpr int SPAD = 40;  // bf16 per plane column (32 signals + 16 B pad: no bank conflicts)
  static constexpr int NTHR = 64 * NW;
  static constexpr int SIG = sizeof(T) == 4 ? QMFX_BIG_SIG32 : QMFX_BIG_SIG64;  // signals per LDS stage
  static constexpr int VEC = 16 / sizeof(T);             // elements per 16-B load
  static constexpr int CPR = KP / VEC;                   // 16-B chunks per row
  static constexpr int TRIPS = (SIG * CPR + NTHR - 1) / NTHR;
  // padded LDS row of a panel (fp32: 16-B aligned rows for the b128 row accesses)
  static constexpr int PLD = sizeof(T) == 4 ? 20 : 17;
  // compile-time tile map with LDS fragments reused across a wave's tiles (Gram and
  // trailing update); the fp64 tilings above NT = 11 lack the registers for it
  static constexpr bool REUSE = sizeof(T) == 4 || NT <= 11;
};

// tile s of wave W: round-robin t = W + NW·s, or (split map) rows W and NT−1−W
template <typename C>
__host__ __device__ constexpr void big_tile(int W, int s, int& I, int& J) {
  if constexpr (C::PAIR) {
    constexpr int NT = C::KP / 16;
    if (s <= W) {
      I = W;
      J = s;
    } else {
      I = NT - 1 - W;
      J = s - W - 1;
    }
  } else {
    const int t = W + C::NW * s;
    if (t < C::NTT) {
      int i = 0;
      while ((i + 1) * (i + 2) / 2 <= t) ++i;
      I = i;
      J = t - i * (i + 1) / 2;
    } else {
      I = J = -1;
    }
  }
}

template <typename T, int NT>
struct BigShared {
  using C = BigCfg<T, NT>;
  // the Gram staging and the Cholesky panels are never live together
  union {
    T stage[2][C::STREAM ? 1 : C::SIG * C::KP];
    uint16_t planes[2][3][C::SPLIT ? C::KP * C::SPAD : 1];  // split Gram: bf16 hi/mid/lo, [column][signal]
    float bred[8][C::KP];                    // split Gram: per-wave b partials (after the Gram)
    struct {
      T panel[C::KP * C::PLD];
      T Ldiag[NT * 16 * C::PLD];
      T panel2[C::PANEL2 ? C::KP * C::PLD : 1];  // LDLᵀ factorization: odd panels
    };
  };
  T w[2][C::SIG];   // α·v of the staged signals (0 past the row end)
  T c[2][C::SIG];   // 1 + α·v (0 past the row end)
  double cred[8];   // split Gram: per-wave Σc
  int negw;         // split Gram: some signal has a negative weight (row goes to the re-solve)
  T bw[C::KP];
  T borig[C::KP];
  T xs[C::KP];
  T invd[C::KP];
  T yd[C::KP];  // forward-solve y of each diagonal block (read by the backward solve)
  T part[C::NW * 16];
  double red[C::NW];
  int bad;  // wave 0's pivot flag, for every wave's output stores
};

// Calls f(integral_constant<W>) for the wave-uniform wave index wv (compile-time tile maps).
template <int NW, int W = 0, typename F>
__device__ __forceinline__ void dispatch_wave(int wv, F&& f) {
  if constexpr (W < NW) {
    if (wv == W)
      f(std::integral_constant<int, W>{});
    else
      dispatch_wave<NW, W + 1>(wv, f);
  }
}

// Panel p on every wave at once: lanes 0..15 of each wave hold the diagonal block (factored
// redundantly, as in the head), lanes 16..63 rows 48W + 16 .. 48W + 63 of the panel; each
// wave runs the head's column loop on its own rows, so the serial head and the slot phase
// behind it (and one barrier) become one step.  Wave 0 writes the diagonal block.
template <typename T, int NT>
__device__ void big_panel_all(BigShared<T, NT>& S, int p, int wv, int lane, int& bad) {
  constexpr int KP = 16 * NT;
  constexpr int PLD = BigCfg<T, NT>::PLD;
  const int R = KP - 16 * p;
  static_assert(48 * BigCfg<T, NT>::NW + 16 >= KP, "panel rows beyond the waves' lanes");
  if (wv > 0 && 48 * wv + 16 >= R) return;  // no rows below the diagonal block for this wave
  const int q = lane < 16 ? lane : 48 * wv + lane;
  const bool live = q < R;
  T pa[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) pa[c] = live ? S.panel[q * PLD + c] : T(0);
  T pb = live ? S.bw[16 * p + q] : T(0);
  T invv = T(0), yv = T(0);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    T am[16];
#pragma unroll
    for (int m = 1; m < 16; ++m)
      if (m > c) am[m] = readlane(pa[c], m);
    const T d = readlane(pa[c], c);
    const T bc = readlane(pb, c);
    T ljj, inv;
    pivot_sqrt(d, ljj, inv);
    (void)ljj;
    bad |= !(d > T(0));
    const bool me = lane == c;
    invv = me ? inv : invv;
    yv = me ? bc * inv : yv;
    const T lq = pa[c] * inv;
    const T lqs = lq * inv;
    pa[c] = lq;
    pb -= lqs * bc;
#pragma unroll
    for (int m = 1; m < 16; ++m)
      if (m > c) pa[m] -= lqs * am[m];
    __builtin_amdgcn_sched_barrier(0);
  }
  // every wave read the diagonal block before wave 0 overwrites it: the caller's barrier
  // after the panel orders the stores of other waves; rows ≥ 16 are disjoint per wave
  if (lane >= 16 && live) {
#pragma unroll
    for (int c = 0; c < 16; ++c) S.panel[q * PLD + c] = pa[c];
    S.bw[16 * p + q] = pb;
  }
  if (wv == 0 && lane < 16) {
    // y of the diagonal block goes to S.yd: other waves may still be reading S.bw[16p..]
    S.invd[16 * p + lane] = invv;
    S.yd[16 * p + lane] = yv;
#pragma unroll
    for (int c = 0; c < 16; ++c) S.Ldiag[(p * 16 + lane) * PLD + c] = c <= lane ? pa[c] : T(0);
  }
}

// One 4-signal step of the Gram for the tiles of wave W (t = W + NW·s, compile-time map):
// the wave reads each 16-row fragment of the staged signals once (NT LDS reads instead of
// two per tile) and reuses it for every tile in its tile row or column.
template <typename T, int NT, int W>
__device__ __forceinline__ void big_gram_step(typename Mfma<T>::acc_t* acc, const T* yk, T wk) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  T y[NT], wy[NT];
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    y[J] = yk[16 * J];
    wy[J] = wk * y[J];
  }
#pragma unroll
  for (int s = 0; s < C::TPW; ++s) {
    int I = -1, J = -1;
    big_tile<C>(W, s, I, J);
    if (I >= 0) acc[s] = M::mma(y[I], wy[J], acc[s]);
  }
}

// Rank-16 trailing update of panel p for the tiles of wave W (compile-time map): the panel
// rows of every block I > p are read from LDS once (4 fragments each) and reused by all of
// the wave's tiles in block row or column I.
template <typename T, int NT, int W>
__device__ __forceinline__ void big_trailing(typename Mfma<T>::acc_t* acc, const T* panel, int p,
                                             int cl, int kk) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  T fr[NT][4];
#pragma unroll
  for (int I = 0; I < NT; ++I) {
    if (I > p) {
      const T* src = panel + (16 * (I - p) + cl) * C::PLD + kk;
#pragma unroll
      for (int q = 0; q < 4; ++q) fr[I][q] = src[4 * q];
    }
  }
#pragma unroll
  for (int s = 0; s < C::TPW; ++s) {
    int I = -1, J = -1;
    big_tile<C>(W, s, I, J);
    if (I >= 0 && J > p) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[s] = M::mma(-fr[I][q], fr[J][q], acc[s]);
    }
  }
}

// Streamed Gram (fp64): the blocks wave W needs — its tiles' block rows and columns and the
// blocks of b it owns (big_b_owner) — as bit masks, fixed at compile time.
template <typename C>
__host__ __device__ constexpr int big_b_owner(int X) {
  constexpr int NT = C::KP / 16;
  if constexpr (C::PAIR) return X < NT - 1 - X ? X : NT - 1 - X;
  return X % C::NW;
}
template <typename C, int W>
constexpr uint32_t big_rows_mask() {
  uint32_t m = 0;
  for (int s = 0; s < C::TPW; ++s) {
    int I = -1, J = -1;
    big_tile<C>(W, s, I, J);
    if (I >= 0) m |= 1u << I;
  }
  return m;
}
template <typename C, int W>
constexpr uint32_t big_need_mask() {
  uint32_t m = big_rows_mask<C, W>();
  for (int s = 0; s < C::TPW; ++s) {
    int I = -1, J = -1;
    big_tile<C>(W, s, I, J);
    if (I >= 0) m |= 1u << J;
  }
  for (int X = 0; X < C::KP / 16; ++X)
    if (big_b_owner<C>(X) == W) m |= 1u << X;
  return m;
}

// The streamed Gram's block order within a step: the wave's tile-row blocks first (their w·y
// start the next step, so they are gathered again first), then the other blocks ascending.
template <typename C, int W>
constexpr int big_jorder(int q) {
  constexpr uint32_t rows = big_rows_mask<C, W>();
  for (int pass = 0; pass < 2; ++pass)
    for (int X = 0; X < C::KP / 16; ++X)
      if ((((rows >> X) & 1) != 0) == (pass == 0) && q-- == 0) return X;
  return 0;
}

// Streamed Gram of wave W (fp64 multi-wave rows): A_tiles += Σ w y yᵀ over the row's signals
// for the wave's own tiles, and b_X = Σ c y_X for the blocks it owns.  Step t takes signals
// 4t..4t+3, one per 16-lane group (the MFMA's K index): lane (cl, g) gathers element
// 16X + cl of signal 4t + g for each block X the wave needs (one 8-B load per block, the
// same base address with an immediate offset), scales its tile-row blocks by w and issues one
// 16x16x4 MFMA per tile.  No LDS and no barrier: every wave runs ahead on its own, the other
// waves of the row read the same rows from L2.  (column, value) pairs are loaded CD steps
// ahead into a ring, the rows of step t + 2 while step t's MFMAs run (2 buffers).  Loads are
// unconditional (a clamped address past the end; the all-zero row a.zrow with w = 0 at use).
template <typename T, int NT, int W>
__device__ __forceinline__ void big_gram_stream(const SolveArgs<T>& a, int64_t beg, int n,
                                                typename Mfma<T>::acc_t (&acc)[BigCfg<T, NT>::TPW],
                                                T (&bq)[NT], int lane) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  constexpr int KP = C::KP, TPW = C::TPW;
  constexpr uint32_t ROWS = big_rows_mask<C, W>();
  constexpr uint32_t NEED = big_need_mask<C, W>();
  // column ring: loaded CD steps ahead, used for the gather two steps ahead
  constexpr int CD = 4;
  const int cl = lane & 15, g = lane >> 4;
  const int nsteps = (n + 3) >> 2;
  if (nsteps == 0) return;
  int cr[CD];
  T yb[2][NT];
  T vb[2];
  auto ldcol = [&](int t, int& c) {
    const int e = 4 * t + g;
    c = a.col[beg + (e < n ? e : 0)];
  };
  // the row base and the value of step t (value loaded with the rows: consumed a step later)
  auto rowbase = [&](int t, int c, int b) -> const T* {
    const int e = 4 * t + g;
    const bool ok = e < n;
    const uint32_t col = ok ? (uint32_t)c : (uint32_t)a.zrow;
    vb[b] = a.val[beg + (ok ? e : 0)];
    return a.Y + (uint64_t)col * KP + cl;
  };
  auto gather = [&](int t, int c, int b) {
    const T* yr = rowbase(t, c, b);
#pragma unroll
    for (int X = 0; X < NT; ++X)
      if ((NEED >> X) & 1) yb[b][X] = yr[16 * X];
  };
  // step u from buffer b, and the gathers of step u + 2 into b: block J's fragment is loaded
  // again right after the step's last MFMA that reads it (tiles (I, J) in J order), so each
  // gather is in flight for about two steps instead of one
  auto step = [&](int b, int tn, int cn) {
    // (past the end: the zero row, whatever the value; it adds nothing to the tiles or b)
    const T w = a.alpha * vb[b];
    const T cw = T(1) + w;
    T wy[NT];
#pragma unroll
    for (int X = 0; X < NT; ++X) {
      if ((ROWS >> X) & 1) wy[X] = w * yb[b][X];
      if (big_b_owner<C>(X) == W) bq[X] += cw * yb[b][X];
    }
    const T* yr = rowbase(tn, cn, b);
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int J = big_jorder<C, W>(q);
      if (!((NEED >> J) & 1)) continue;
#pragma unroll
      for (int s = 0; s < TPW; ++s) {
        int I = -1, J2 = -1;
        big_tile<C>(W, s, I, J2);
        if (I >= 0 && J2 == J) acc[s] = M::mma(wy[I], yb[b][J], acc[s]);
      }
      yb[b][J] = yr[16 * J];
    }
  };
  // (the prologue issues its loads in the loop's order — columns, then rows — so the
  // vmcnt waits the loop entry merges from both paths are the loop's own)
#pragma unroll
  for (int j = 0; j < CD; ++j) ldcol(j, cr[j]);
  __builtin_amdgcn_sched_barrier(0);
  gather(0, cr[0], 0);
  __builtin_amdgcn_sched_barrier(0);
  gather(1, cr[1], 1);
  for (int t = 0; t < nsteps; t += CD) {
#pragma unroll
    for (int j = 0; j < CD; ++j) {
      const int u = t + j;
      __builtin_amdgcn_sched_barrier(0);
      ldcol(u + CD, cr[j]);  // slot j held step u, gathered two steps ago
      step(j & 1, u + 2, cr[(j + 2) % CD]);
      // keep the loads beside the MFMAs that free their registers
      [&]<int... Js>(std::integer_sequence<int, Js...>) {
        auto grp = [&](auto Qc) {
          constexpr int J = big_jorder<C, W>(decltype(Qc)::value);
          if constexpr ((NEED >> J) & 1) {
            constexpr int nm = [] {
              int m = 0;
              for (int s2 = 0; s2 < TPW; ++s2) {
                int I = -1, J2 = -1;
                big_tile<C>(W, s2, I, J2);
                m += (I >= 0 && J2 == J);
              }
              return m;
            }();
            if constexpr (nm > 0) __builtin_amdgcn_sched_group_barrier(0x8, nm, 0);
            __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
          }
        };
        (grp(std::integral_constant<int, Js>{}), ...);
      }(std::make_integer_sequence<int, NT>{});
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

// Split Gram, MFMA side, for wave W (rows A = W, B = NT−1−W): each column block's planes
// are read once per stage (three 16-B LDS reads per lane) and used for both rows.
template <int NT, int W>
__device__ __forceinline__ void big_split_mfma(f32x4* acc, const uint16_t* pl, int cl, int kk) {
  using C = BigCfg<float, NT>;
  constexpr int A = W, B = NT - 1 - W;
  constexpr int PS = C::KP * C::SPAD;  // one plane
  auto rd = [&](int X, Split3& sp) {
    const int off = (16 * X + cl) * C::SPAD + 8 * kk;
    sp.h = *reinterpret_cast<const u32x4*>(pl + off);
    sp.m = *reinterpret_cast<const u32x4*>(pl + PS + off);
    sp.l = *reinterpret_cast<const u32x4*>(pl + 2 * PS + off);
  };
  Split3 sa, sb;
  rd(A, sa);
  rd(B, sb);
#pragma unroll
  for (int J = 0; J <= B; ++J) {
    Split3 sj;
    if (J == A) {
      sj = sa;
    } else if (J == B) {
      sj = sb;
    } else {
      rd(J, sj);
    }
    acc[W + 1 + J] = mma_split6(sb, sj, acc[W + 1 + J]);  // tile (B, J)
    if (J <= A) acc[J] = mma_split6(sa, sj, acc[J]);      // tile (A, J)
  }
}

// 4 fp32 values → their exact bf16 hi/mid/lo parts, packed 2 per word (value 0 in the low
// half, as split3 packs)
__device__ __forceinline__ void split3x4(const float (&x)[4], uint2& h, uint2& m, uint2& l) {
  float r[4], lo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = x[j] - trunc_bf16(x[j]);
    lo[j] = r[j] - trunc_bf16(r[j]);
  }
  h = uint2{pack_hi16(x[0], x[1]), pack_hi16(x[2], x[3])};
  m = uint2{pack_hi16(r[0], r[1]), pack_hi16(r[2], r[3])};
  l = uint2{pack_hi16(lo[0], lo[1]), pack_hi16(lo[2], lo[3])};
}

// fp32 twin of chol.h's bcast16 (lane J of every 16-lane row)
template <int J>
__device__ __forceinline__ float bcast16(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + J, 0xf, 0xf, true));
}
// Column C of a panel in the replicated-diagonal layout (chol.h dg_column, for either precision):
// the pivot d = U[C][C] and z_C = b_C broadcast from lane C of every 16-lane row, the
// right-hand sides' update, and the trailing columns m > C of the diagonal block and of the
// lane's panel row, each element one v_fmac_dpp row_newbcast of column C's entry U[m][C].
template <int C, typename T>
__device__ __forceinline__ void big_dg_column(T (&dg)[16], T& bdg, T (&pa)[16], T& pb, int cl,
                                              T& invv, T& zv) {
  const T d = bcast16<C>(dg[C]);
  const T bc = bcast16<C>(bdg);
  const T invd = pivot_rcp(d);
  const bool me = cl == C;
  invv = me ? invd : invv;
  zv = me ? bc : zv;
  const T nl = -(dg[C] * invd);
  const T nls = -(pa[C] * invd);
  bdg = __builtin_fma(nl, bc, bdg);
  pb = __builtin_fma(nls, bc, pb);
  [&]<int... Ms>(std::integer_sequence<int, Ms...>) {
    auto upd = [&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      if constexpr (m > C) {
        fmac_bcast16<m, (m == C + 1) ? 1 : 0>(dg[m], dg[C], nl);
        fmac_bcast16<m>(pa[m], dg[C], nls);
      }
    };
    (upd(std::integral_constant<int, Ms>{}), ...);
  }(std::make_integer_sequence<int, 16>{});
  __builtin_amdgcn_sched_barrier(0);
}

// LDLᵀ factorization and solves of the streamed (fp64) rows, for wave W (compile-time tile
// map): chol.h's method (A = U D⁻¹ Uᵀ, U the unnormalised columns, one reciprocal per pivot,
// the forward solve folded into the panel) spread over the workgroup.  Per 16-column panel p:
//   (a) the owners of the panel's tiles store them to the panel buffer (two buffers in turn, so
//       the next panel's stores need no barrier behind this panel's readers);
//   (b) the waves with panel rows below the diagonal block (at most 4, one per SIMD; wave 0
//       always) factor the panel column by column: the diagonal block sits in every 16-lane row
//       of the wave, so column c's entries arrive by one v_fmac_f64_dpp row_newbcast per
//       element (no readlane); lane q holds panel row 16 + 64W + q and its b entry.  Wave 0
//       keeps 1/d, z and the transposed, scaled diagonal block for the backward solve;
//   (c) the owners take U(I, p) back into their tiles and apply the rank-16 trailing update
//       A(I, J) −= U(I, p) D⁻¹ U(J, p)ᵀ to their tiles with MFMA (operands from the buffer).
// Then the backward solve by 16-blocks: the owners of tiles (J, I), J > I, add their part of
// Uᵀx in LDS, and wave 0 finishes the block with one DPP FMA per column.
// In: acc = lower tiles of A; S.bw = b.  Out: S.xs = x; `bad` (wave 0) on a pivot ∉ (0, ∞).
template <typename T, int NT, int WI>
__device__ __forceinline__ void big_ldl_solve(BigShared<T, NT>& S,
                                              typename Mfma<T>::acc_t (&acc)[BigCfg<T, NT>::TPW],
                                              int lane, int& bad, uint64_t* sub = nullptr) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  constexpr int KP = C::KP, TPW = C::TPW, PLD = C::PLD;
  const int cl = lane & 15, kk = lane >> 4;
  // (QMFX_BIG_SUBTRACE diagnostics builds: cycles of (a), (b), (c) and the backward solve)
  uint64_t t0 = 0, ta = 0, tb = 0, tc = 0;
  auto stamp = [&]() -> uint64_t { return sub ? __builtin_amdgcn_s_memtime() : 0; };
  t0 = stamp();
  for (int p = 0; p < NT; ++p) {
    T* P = (C::PANEL2 && (p & 1)) ? S.panel2 : S.panel;
    const int R = KP - 16 * p;
    // (a)
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      int I = -1, J = -1;
      big_tile<C>(WI, s, I, J);
      if (I >= 0 && J == p) {
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(16 * (I - p) + M::crow(lane, r)) * PLD + cl] = acc[s][r];
      }
    }
    __syncthreads();
    if (sub) {
      const uint64_t t = stamp();
      ta += t - t0;
      t0 = t;
    }
    // (b)
    if (WI == 0 || 16 + 64 * WI < R) {
      const int q = 16 + 64 * WI + lane;
      const bool live = q < R;
      const int qq = live ? q : 0;
      T dg[16], pa[16];
      lds_row_load(&P[cl * PLD], dg);
      T bdg = S.bw[16 * p + cl];
      lds_row_load(&P[qq * PLD], pa);
      T pb = S.bw[16 * p + qq];
      T invv = T(0), zv = T(0);
      [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        (big_dg_column<Cs>(dg, bdg, pa, pb, cl, invv, zv), ...);
      }(std::make_integer_sequence<int, 16>{});
      if (live) {
        lds_row_store(&P[q * PLD], pa);
        S.bw[16 * p + q] = pb;
      }
      if (WI == 0) {
        bad |= __any(lane < 16 && !(invv > T(0) && invv < __builtin_huge_val())) ? 1 : 0;
        if (lane < 16) {
          lds_row_store(&P[lane * PLD], dg);  // U of the diagonal block (for Lt below)
          S.invd[16 * p + lane] = invv;
          S.bw[16 * p + lane] = zv;
        }
      }
    }
    __syncthreads();
    if (sub) {
      const uint64_t t = stamp();
      tb += t - t0;
      t0 = t;
    }
    if (WI == C::NW - 1) {
      // the diagonal block → Lt, transposed and scaled by 1/d of its row, negated:
      // Lt[q][c] = −U[c][q]/d_q for c > q (the backward solve's DPP FMAs)
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = lane + 64 * it;
        const int r = idx >> 4, c = idx & 15;
        S.Ldiag[(16 * p + c) * PLD + r] = c < r ? -(P[r * PLD + c] * S.invd[16 * p + c]) : T(0);
      }
    }
    // (c)
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      int I = -1, J = -1;
      big_tile<C>(WI, s, I, J);
      if (I >= 0 && J == p && I > p) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[s][r] = P[(16 * (I - p) + M::crow(lane, r)) * PLD + cl];
      }
    }
    T dcol[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) dcol[s4] = S.invd[16 * p + 4 * s4 + kk];
#pragma unroll
    for (int J = 1; J < NT; ++J) {
      bool any = false;
#pragma unroll
      for (int s = 0; s < TPW; ++s) {
        int I = -1, J2 = -1;
        big_tile<C>(WI, s, I, J2);
        any |= I >= 0 && J2 == J;
      }
      if (!any || J <= p) continue;
      T sj[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) sj[s4] = P[(16 * (J - p) + cl) * PLD + 4 * s4 + kk] * dcol[s4];
#pragma unroll
      for (int s = 0; s < TPW; ++s) {
        int I = -1, J2 = -1;
        big_tile<C>(WI, s, I, J2);
        if (I >= 0 && J2 == J) {
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc[s] = M::mma(-P[(16 * (I - p) + cl) * PLD + 4 * s4 + kk], sj[s4], acc[s]);
        }
      }
    }
    // one panel buffer: its readers finish before the next panel's stores
    if constexpr (!C::PANEL2) __syncthreads();
    if (sub) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint64_t t = stamp();
      tc += t - t0;
      t0 = t;
    }
  }
  // backward solve, Uᵀ x = D z by 16-blocks from the bottom
  for (int I = NT - 1; I >= 0; --I) {
    T part = T(0);
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      int I2 = -1, J = -1;
      big_tile<C>(WI, s, I2, J);
      if (I2 >= 0 && J == I && I2 > I) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part += acc[s][r] * S.xs[16 * I2 + M::crow(lane, r)];
      }
    }
    part += shfl_xor(part, 16);
    part += shfl_xor(part, 32);
    if (kk == 0) S.part[WI * 16 + cl] = part;
    __syncthreads();
    if (WI == 0) {
      T vm = S.bw[16 * I + cl];
#pragma unroll
      for (int w = 0; w < C::NW; ++w) vm -= S.part[w * 16 + cl];
      vm *= S.invd[16 * I + cl];
      T lt[16];
      lds_row_load(&S.Ldiag[(16 * I + cl) * PLD], lt);
      // x_c is lane c's vm in every 16-lane row: one DPP FMA per column (chol.h), two wait
      // states first (vm was just written by a VALU the hazard recognizer sees, read by asm)
      asm volatile("s_nop 1" : "+v"(vm));
      [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        (fmac_bcast16<15 - Cs, 1>(vm, vm, lt[15 - Cs]), ...);
      }(std::make_integer_sequence<int, 16>{});
      if (lane < 16) S.xs[16 * I + lane] = vm;
    }
    __syncthreads();
  }
  if (sub) {
    sub[0] = ta;
    sub[1] = tb;
    sub[2] = tc;
    sub[3] = stamp() - t0;
  }
}

// MODE (compile time, as in the one-wave direct kernel): 0 = row solve; 1 = split-K segment
// Gram (slot = segment of a.desc: the Gram of its signals from zero, written as tile images
// + rhs + Σc + flag to the segment's part/partb/partc slot, no solve); 2 = split-K heavy-row
// solve (slot = heavy row of a.desc: the reduced image of the row's first segment in place of
// G + λI and the Gram).  The reference loops a heavy row inside one thread
// (WALSEngine.cpp:277-287); SURVEY.md §5 "long rows".
// WV ≥ 0: the body of wave WV alone, with its tile map at compile time (the streamed fp64
// Gram: one wave-specialised copy of the whole row solve per wave, so no accumulator values
// merge across the waves' code paths); WV = −1: one body for every wave (runtime tile map).
template <typename T, int NT, int MODE, int WV>
__device__ __forceinline__ void big_row_body(const SolveArgs<T>& a, BigShared<T, NT>& S) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  using vec_t = T __attribute__((ext_vector_type(C::VEC)));
  constexpr int KP = C::KP, NW = C::NW, TPW = C::TPW, SIG = C::SIG;
  constexpr int CPR = C::CPR, TRIPS = C::TRIPS, PLD = C::PLD;

  const int tid = threadIdx.x;
  const int wv = WV >= 0 ? WV : __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t slot = a.row_begin + blockIdx.x;
  // QMFX_TRACE phase stamps (thread 0, row solves only): start, G + λI loaded, Gram done,
  // factorization done, backward solve done (direct-kernel record layout, tools/trace_analyze.py)
  const bool trace = MODE == 0 && a.trace != nullptr && tid == 0;
  uint64_t tr[5] = {0, 0, 0, 0, 0};
  if (trace) tr[0] = __builtin_amdgcn_s_memtime();
  int64_t row, beg, end, seg0 = 0;
  if constexpr (MODE == 0) {
    row = a.order ? a.order[slot] : slot;
    beg = a.rowptr[row];
    end = a.rowptr[row + 1];
  } else {
    const RowDesc d = a.desc[slot];
    row = MODE == 2 ? (int64_t)d.row : -1;
    seg0 = d.beg;                        // mode 2: the row's first segment slot
    beg = MODE == 1 ? d.beg : 0;         // mode 1: the segment's signals
    end = MODE == 1 ? d.beg + d.n : 0;   // mode 2: no signals
  }
  constexpr int NTT = C::NTT;

  // this wave's tiles (big_tile)
  int TI[TPW], TJ[TPW];
#pragma unroll
  for (int s = 0; s < TPW; ++s) big_tile<C>(wv, s, TI[s], TJ[s]);
  acc_t acc[TPW];
#pragma unroll
  for (int s = 0; s < TPW; ++s) {
    if constexpr (MODE == 1) {
      acc[s] = acc_t{0, 0, 0, 0};
    } else if constexpr (MODE == 2) {
      // the reduced image: [tile][lane][4] (the direct kernel's accumulator-image layout)
      const T* img = a.part + seg0 * (NTT * 256);
      const int t = TI[s] >= 0 ? tile_index(TI[s], TJ[s]) : 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[s][r] = TI[s] >= 0 ? img[(t * 64 + lane) * 4 + r] : T(0);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * TI[s] + M::crow(lane, r), j = 16 * TJ[s] + cl;
        T g = TI[s] >= 0 ? a.G[(int64_t)i * KP + j] : T(0);
        if (TI[s] >= 0 && i == j) g += (i < a.k) ? a.lambda : T(1);
        acc[s][r] = g;
      }
    }
  }

  if (trace) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[1] = __builtin_amdgcn_s_memtime();
  }
  // ---- Gram: A += Σ w y yᵀ, b = Σ c y, Σc -------------------------------------------------
  T bp = T(0);        // b[tid] for tid < KP
  double cs = 0.0;    // Σc (thread 0)
  int negw = 0;       // split Gram: a negative weight (the split needs √w)
  if constexpr (C::SPLIT) {
    // loader thread: column group g (columns 4g..4g+3), signals 4q..4q+3 of each stage
    // (KP/4 groups × 8 quads = 32·NT = the workgroup's threads when NT = 2·NW)
    constexpr int NG4 = KP / 4;
    static_assert(NG4 * 8 == C::NTHR, "split loader: one (column group, quad) per thread");
    const int g = tid % NG4, q = tid / NG4;
    int colq[4];
    float valq[4];
    int nval = 0;
    f32x4 y4[4];
    float bpart[4] = {0.f, 0.f, 0.f, 0.f};
    double csl = 0.0;
    auto load_meta = [&](int64_t sb) {
      const int64_t e0 = sb + 4 * q;
      nval = (int)(end - e0 < 0 ? 0 : (end - e0 > 4 ? 4 : end - e0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        colq[j] = j < nval ? a.col[e0 + j] : a.zrow;
        valq[j] = j < nval ? (float)a.val[e0 + j] : 0.f;
      }
    };
    auto load_rows = [&]() {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        y4[j] = *(reinterpret_cast<const f32x4*>(a.Y + (int64_t)(uint32_t)colq[j] * KP) + g);
    };
    auto store_split = [&](int buf) {
      float sw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float w = (float)a.alpha * valq[j];
        const float cw = j < nval ? 1.f + w : 0.f;
        negw |= w < 0.f;
        sw[j] = fast_sqrt(fabsf(w));
        if (g == 0) csl += (double)cw;
#pragma unroll
        for (int m = 0; m < 4; ++m) bpart[m] += cw * y4[j][m];
      }
      uint16_t* pl = S.planes[buf][0];
      constexpr int PS = KP * C::SPAD;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = sw[j] * y4[j][m];
        uint2 h, mi, l;
        split3x4(x, h, mi, l);
        const int off = (4 * g + m) * C::SPAD + 4 * q;
        *reinterpret_cast<uint2*>(pl + off) = h;
        *reinterpret_cast<uint2*>(pl + PS + off) = mi;
        *reinterpret_cast<uint2*>(pl + 2 * PS + off) = l;
      }
    };
    const int nstages = (int)((end - beg + SIG - 1) / SIG);
    if (nstages > 0) {
      load_meta(beg);
      load_rows();
      store_split(0);
      if (nstages > 1) load_meta(beg + SIG);
      __syncthreads();
      for (int st = 0; st < nstages; ++st) {
        const int buf = st & 1;
        const bool more = st + 1 < nstages;
        if (more) load_rows();  // stage st+1 (meta already in registers)
        auto mf = [&](auto wtag) {
          big_split_mfma<NT, decltype(wtag)::value>(acc, S.planes[buf][0], cl, kk);
        };
        dispatch_wave<NW>(wv, mf);
        if (more) {
          store_split(buf ^ 1);
          if (st + 2 < nstages) load_meta(beg + (int64_t)(st + 2) * SIG);
        }
        __syncthreads();
      }
    }
    // b and Σc: per-wave partials in fixed order
#pragma unroll
    for (int m = 0; m < 4; ++m) S.bred[q][4 * g + m] = bpart[m];
    if (g == 0) S.cred[q] = csl;
    negw = __syncthreads_or(negw);
    if (tid < KP) {
      float b = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) b += S.bred[w][tid];
      bp = b;
    }
    if (tid == 0)
      for (int w = 0; w < 8; ++w) cs += S.cred[w];
    __syncthreads();
  } else if constexpr (C::STREAM) {
    const int n = (int)(end - beg);
    auto gs = [&](auto wtag) {
      constexpr int W = decltype(wtag)::value;
      T bq[NT];
#pragma unroll
      for (int X = 0; X < NT; ++X) bq[X] = T(0);
      big_gram_stream<T, NT, W>(a, beg, n, acc, bq, lane);
      // the wave's blocks of b, summed over the four signal groups
#pragma unroll
      for (int X = 0; X < NT; ++X) {
        if (big_b_owner<C>(X) == W) {
          T v = bq[X];
          v += shfl_xor(v, 16);
          v += shfl_xor(v, 32);
          if (kk == 0) S.bw[16 * X + cl] = v;
        }
      }
      if constexpr (W == NW - 1) {  // Σc over the row's signals
        double c = 0.0;
        for (int e = lane; e < n; e += 64) c += (double)(T(1) + a.alpha * a.val[beg + e]);
        c = wave_sum(c);
        if (lane == 0) S.cred[0] = c;
      }
    };
    dispatch_wave<NW>(wv, gs);
    __syncthreads();
    if (tid < KP) bp = S.bw[tid];
    if (tid == 0) cs = S.cred[0];
  } else {
  int cols[TRIPS];
  vec_t stg[TRIPS];
  T wmeta = T(0), cmeta = T(0);
  auto load_cols = [&](int64_t sb) {
#pragma unroll
    for (int t = 0; t < TRIPS; ++t) {
      const int ch = tid + C::NTHR * t;
      const int64_t e = sb + ch / CPR;
      cols[t] = (ch < SIG * CPR && e < end) ? a.col[e] : -1;
    }
  };
  auto load_rows = [&]() {
#pragma unroll
    for (int t = 0; t < TRIPS; ++t) {
      const int ch = tid + C::NTHR * t;
      const vec_t* src = reinterpret_cast<const vec_t*>(a.Y + (int64_t)(cols[t] < 0 ? 0 : cols[t]) * KP) + ch % CPR;
      const vec_t v = *src;
      stg[t] = cols[t] >= 0 ? v : vec_t{};
    }
  };
  auto load_meta = [&](int64_t sb) {
    const int64_t e = sb + tid;
    const bool ok = tid < SIG && e < end;
    const T v = ok ? a.val[e] : T(0);
    wmeta = ok ? a.alpha * v : T(0);
    cmeta = ok ? T(1) + a.alpha * v : T(0);
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int t = 0; t < TRIPS; ++t) {
      const int ch = tid + C::NTHR * t;
      if (ch < SIG * CPR) reinterpret_cast<vec_t*>(S.stage[buf])[ch] = stg[t];
    }
    if (tid < SIG) {
      S.w[buf][tid] = wmeta;
      S.c[buf][tid] = cmeta;
    }
  };

  const int nstages = (int)((end - beg + SIG - 1) / SIG);
  if (nstages > 0) {
    load_cols(beg);
    load_rows();
    load_meta(beg);
    store_stage(0);
    if (nstages > 1) load_cols(beg + SIG);
    __syncthreads();
    for (int st = 0; st < nstages; ++st) {
      const int buf = st & 1;
      const bool more = st + 1 < nstages;
      if (more) {
        load_rows();  // rows of stage st+1 (columns already in registers)
        load_meta(beg + (int64_t)(st + 1) * SIG);
      }
      // MFMAs of stage st: 4 signals per step, operands straight from LDS
      const T* sg = S.stage[buf];
      auto gram_stage = [&](auto wtag) {
        constexpr int W = decltype(wtag)::value;
#pragma unroll 2
        for (int k4 = 0; k4 < SIG; k4 += 4)
          big_gram_step<T, NT, W>(acc, sg + (k4 + kk) * KP + cl, S.w[buf][k4 + kk]);
      };
      static_assert(NW == 2 || NW == 4 || NW == 8 || NW == 16, "wave count");
      if constexpr (C::REUSE) {
        dispatch_wave<NW>(wv, gram_stage);
      } else {
#pragma unroll 2
        for (int k4 = 0; k4 < SIG; k4 += 4) {
          const T* yk = sg + (k4 + kk) * KP + cl;
          const T wk = S.w[buf][k4 + kk];
#pragma unroll
          for (int s = 0; s < TPW; ++s) {
            if (TI[s] >= 0) acc[s] = M::mma(yk[16 * TI[s]], wk * yk[16 * TJ[s]], acc[s]);
          }
        }
      }
      if (tid < KP) {
#pragma unroll 4
        for (int k = 0; k < SIG; ++k) bp += S.c[buf][k] * sg[k * KP + tid];
      }
      if (tid == 0) {
        for (int k = 0; k < SIG; ++k) cs += (double)S.c[buf][k];
      }
      if (more) {
        store_stage(buf ^ 1);
        if (st + 2 < nstages) load_cols(beg + (int64_t)(st + 2) * SIG);
      }
      __syncthreads();
    }
  }
  }  // plain Gram
  if constexpr (MODE == 1) {
    // one segment of a heavy row: its partial tiles (image layout), rhs, Σc and flag
    T* img = a.part + slot * (NTT * 256);
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      if (TI[s] >= 0) {
        const int t = tile_index(TI[s], TJ[s]);
#pragma unroll
        for (int r = 0; r < 4; ++r) img[(t * 64 + lane) * 4 + r] = acc[s][r];
      }
    }
    if (tid < KP) a.partb[slot * KP + tid] = bp;
    if (tid == 0) {
      a.partc[2 * slot] = cs;
      a.partc[2 * slot + 1] = negw ? 1.0 : 0.0;
    }
    return;
  }
  if constexpr (MODE == 2) {
    if (tid < KP) bp = a.partb[seg0 * KP + tid];
    if (tid == 0) {
      cs = a.partc[2 * seg0];
      negw = a.partc[2 * seg0 + 1] != 0.0;
    }
  }
  if (tid < KP) {
    S.bw[tid] = bp;
    S.borig[tid] = bp;
  }
  __syncthreads();

  if (trace) tr[2] = __builtin_amdgcn_s_memtime();
  // ---- Cholesky A = L Lᵀ with the forward solve of b folded in --------------------------
  int bad = negw ? 1 : 0;  // a negative weight: flagged for the pivoted re-solve
#ifdef QMFX_BIG_SUBTRACE
  uint64_t sub[4] = {0, 0, 0, 0};
#endif
  if constexpr (C::WSPEC && WV >= 0) {
#ifdef QMFX_BIG_SUBTRACE
    big_ldl_solve<T, NT, WV>(S, acc, lane, bad, trace ? sub : nullptr);
#else
    big_ldl_solve<T, NT, WV>(S, acc, lane, bad);
#endif
    if (tid == 0) S.bad = bad;
    __syncthreads();
    if (trace) tr[3] = __builtin_amdgcn_s_memtime();
  } else {
  for (int p = 0; p < NT; ++p) {
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      if (TJ[s] == p) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          S.panel[(16 * (TI[s] - p) + M::crow(lane, r)) * PLD + cl] = acc[s][r];
      }
    }
    __syncthreads();
    big_panel_all<T, NT>(S, p, wv, lane, bad);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      if (TJ[s] == p && TI[s] > p) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[s][r] = S.panel[(16 * (TI[s] - p) + M::crow(lane, r)) * PLD + cl];
      }
    }
    if constexpr (!C::REUSE) {
#pragma unroll
      for (int s = 0; s < TPW; ++s) {
        if (TJ[s] > p) {
          const T* li = S.panel + (16 * (TI[s] - p) + cl) * PLD + kk;
          const T* lj = S.panel + (16 * (TJ[s] - p) + cl) * PLD + kk;
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[s] = M::mma(-li[4 * q], lj[4 * q], acc[s]);
        }
      }
    } else if (p + 1 < NT) {
      auto trailing = [&](auto wtag) {
        big_trailing<T, NT, decltype(wtag)::value>(acc, S.panel, p, cl, kk);
      };
      dispatch_wave<NW>(wv, trailing);
    }
    __syncthreads();
  }

  if (tid == 0) S.bad = bad;
  __syncthreads();

  if (trace) tr[3] = __builtin_amdgcn_s_memtime();
  // ---- backward solve Lᵀ x = y ----------------------------------------------------------
  for (int I = NT - 1; I >= 0; --I) {
    T part = T(0);
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      if (TJ[s] == I && TI[s] > I) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part += acc[s][r] * S.xs[16 * TI[s] + M::crow(lane, r)];
      }
    }
    part += shfl_xor(part, 16);
    part += shfl_xor(part, 32);
    if (kk == 0) S.part[wv * 16 + cl] = part;
    __syncthreads();
    if (wv == 0) {
      T vm = S.yd[16 * I + cl];
#pragma unroll
      for (int w = 0; w < NW; ++w) vm -= S.part[w * 16 + cl];
      // row cl scaled by its own 1/L[cl][cl] (x_c is then row c's value itself): each step
      // is one readlane and one FMA
      const T dcl = S.invd[16 * I + cl];
      T lc[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) lc[c] = S.Ldiag[(I * 16 + c) * PLD + cl] * dcl;
      vm *= dcl;
      T xv = T(0);
#pragma unroll
      for (int c = 15; c >= 0; --c) {
        const T xc = readlane(vm, c);
        xv = lane == c ? xc : xv;
        if (cl < c) vm -= lc[c] * xc;
      }
      if (lane < 16) S.xs[16 * I + lane] = xv;
    }
    __syncthreads();
  }
  }  // LDLᵀ / Cholesky

  // ---- output: x, row loss = Σc − xᵀb − λ‖x‖² ----------------------------------------------
  double xb = 0.0, xx = 0.0;
  if (tid < KP) {
    const T xi = S.bad ? T(0) : S.xs[tid];  // a failed row stores x = 0 (re-solved by the caller)
    a.X[row * KP + tid] = xi;
    xb = (double)xi * (double)S.borig[tid];
    xx = (double)xi * (double)xi;
  }
  const double contrib = wave_sum(xb + (double)a.lambda * xx);
  if (lane == 0) S.red[wv] = contrib;
  __syncthreads();
  if (tid == 0) {  // wave 0 owns `bad` (set by its panel factorizations) and Σc
    double t = 0.0;
    for (int w = 0; w < NW; ++w) t += S.red[w];
    a.rowloss[row] = bad ? 0.0 : cs - t;
    if (bad && a.status) a.status[row] = 1;
  }
  if constexpr (MODE == 0) {
    if (trace) {
      tr[4] = __builtin_amdgcn_s_memtime();
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* o = a.trace + 8 * slot;
#pragma unroll
      for (int j = 0; j < 5; ++j) o[j] = tr[j];
      o[5] = hw | ((uint64_t)xcc << 32);
#ifdef QMFX_BIG_SUBTRACE
      if constexpr (C::WSPEC && WV >= 0) {
        // diagnostics record: start, (a), (b), (c), backward, Gram cycles, n, row
        o[1] = sub[0];
        o[2] = sub[1];
        o[3] = sub[2];
        o[4] = sub[3];
        o[5] = tr[2] - tr[1];
      }
#endif
      o[6] = (uint64_t)(end - beg);
      o[7] = (uint64_t)row;
    }
  }
}

template <typename T, int NT, int MODE = 0>
__global__ __launch_bounds__((BigCfg<T, NT>::NTHR), (BigCfg<T, NT>::WPE)) void wals_big_kernel(SolveArgs<T> a) {
  using C = BigCfg<T, NT>;
  __shared__ __attribute__((aligned(16))) BigShared<T, NT> S;
  if constexpr (C::WSPEC) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dispatch_wave<C::NW>(wv, [&](auto w) { big_row_body<T, NT, MODE, decltype(w)::value>(a, S); });
  } else {
    big_row_body<T, NT, MODE, -1>(a, S);
  }
}

// ---- YᵀY for large NT, every tile per workgroup: the block's rows are staged through LDS
// SIG at a time with coalesced 16-B loads, so Y is read from HBM once (a strip per block
// row read it NT times: 42 -> 4 ms per launch at C5), and the waves split the NT(NT+1)/2
// tiles as in the row kernel's Gram (big_gram_step, weight 1).
template <typename T, int NT>
__global__ __launch_bounds__((BigCfg<T, NT>::NTHR)) void gram_tiles_kernel(
    const T* Y, int64_t n, int64_t rows_per_block, double* partial) {
  using C = BigCfg<T, NT>;
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  using vec_t = T __attribute__((ext_vector_type(C::VEC)));
  constexpr int KP = C::KP, NW = C::NW, TPW = C::TPW, NTT = C::NTT, SIG = C::SIG;
  constexpr int CPR = C::CPR, TRIPS = C::TRIPS;
  __shared__ __attribute__((aligned(16))) T stage[SIG * KP];

  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;

  int TI[TPW], TJ[TPW];
  acc_t acc[TPW];
#pragma unroll
  for (int s = 0; s < TPW; ++s) {
    big_tile<C>(wv, s, TI[s], TJ[s]);
    acc[s] = acc_t{0, 0, 0, 0};
  }

  // the next stage's rows are loaded into registers while this stage's MFMAs run (the
  // same rows in the same order: the partials are bit-identical to a load-then-compute loop)
  vec_t nx[TRIPS];
  auto fetch = [&](int64_t e0) {
#pragma unroll
    for (int t = 0; t < TRIPS; ++t) {
      const int ch = tid + C::NTHR * t;
      const int64_t e = e0 + ch / CPR;
      nx[t] = (ch < SIG * CPR && e < r1)
                  ? *(reinterpret_cast<const vec_t*>(Y + e * KP) + ch % CPR)
                  : vec_t{};
    }
  };
  if (r0 < r1) fetch(r0);
  for (int64_t e0 = r0; e0 < r1; e0 += SIG) {
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TRIPS; ++t) {
      const int ch = tid + C::NTHR * t;
      if (ch < SIG * CPR) reinterpret_cast<vec_t*>(stage)[ch] = nx[t];
    }
    __syncthreads();
    if (e0 + SIG < r1) fetch(e0 + SIG);
    if constexpr (C::REUSE) {
      auto step = [&](auto wtag) {
#pragma unroll 2
        for (int k4 = 0; k4 < SIG; k4 += 4)
          big_gram_step<T, NT, decltype(wtag)::value>(acc, stage + (k4 + kk) * KP + cl, T(1));
      };
      dispatch_wave<NW>(wv, step);
    } else {
      for (int k4 = 0; k4 < SIG; k4 += 4) {
        const T* yk = stage + (k4 + kk) * KP + cl;
#pragma unroll
        for (int s = 0; s < TPW; ++s)
          if (TI[s] >= 0) acc[s] = M::mma(yk[16 * TI[s]], yk[16 * TJ[s]], acc[s]);
      }
    }
  }
  double* out = partial + (int64_t)blockIdx.x * NTT * 256;
#pragma unroll
  for (int s = 0; s < TPW; ++s) {
    if (TI[s] >= 0) {
      const int t = tile_index(TI[s], TJ[s]);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[t * 256 + M::crow(lane, r) * 16 + cl] = (double)acc[s][r];
    }
  }
}

// fixed-order fp64 sum of the per-block partials + mirror (runtime NT): 16 outputs per
// block, 16 chunk sums each, then the chunks in order (as gram_reduce_kernel in wals.hip)
template <typename T>
__global__ __launch_bounds__(256) void gram_reduce_rt_kernel(const double* partial, int nblocks,
                                                             int nt, T* G) {
  __shared__ double red[16][16];
  const int KP = 16 * nt;
  const int NTT = nt * (nt + 1) / 2;
  const int o = threadIdx.x & 15, ch = threadIdx.x >> 4;
  const int idx = blockIdx.x * 16 + o;
  const int i = idx / KP, j = idx % KP;
  const int ii = i >= j ? i : j, jj = i >= j ? j : i;
  const int t = tile_index(ii >> 4, jj >> 4);
  const int off = t * 256 + (ii & 15) * 16 + (jj & 15);
  const int cs = (nblocks + 15) / 16;
  const int b0 = ch * cs, b1 = b0 + cs < nblocks ? b0 + cs : nblocks;
  double sum = 0.0;
  for (int b = b0; b < b1; ++b) sum += partial[(int64_t)b * NTT * 256 + off];
  red[ch][o] = sum;
  __syncthreads();
  if (ch == 0) {
    double tot = 0.0;
    for (int c = 0; c < 16; ++c) tot += red[c][o];
    G[idx] = (T)tot;
  }
}

template <typename T, int NT, int MODE>
static hipError_t launch_big_mode(const SolveArgs<T>& a, hipStream_t s) {
  return launch_row_chunks(a, BigCfg<T, NT>::NTHR, [&](const SolveArgs<T>& c) {
    hipLaunchKernelGGL((wals_big_kernel<T, NT, MODE>), dim3((unsigned)c.nrows),
                       dim3(BigCfg<T, NT>::NTHR), 0, s, c);
  });
}
template <typename T, int NT>
static hipError_t launch_big_nt(const SolveArgs<T>& a, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (a.seg_mode == 1) return launch_big_mode<T, NT, 1>(a, s);
  if (a.seg_mode == 2) return launch_big_mode<T, NT, 2>(a, s);
  return launch_big_mode<T, NT, 0>(a, s);
}

template <typename T, int NT>
static hipError_t launch_gram_tiles_nt(const T* Y, int64_t n, double* partial, int nblocks,
                                       int64_t rows_per_block, hipStream_t s) {
  if (nblocks > 0)
    hipLaunchKernelGGL((gram_tiles_kernel<T, NT>), dim3(nblocks), dim3(BigCfg<T, NT>::NTHR), 0,
                       s, Y, n, rows_per_block, partial);
  return hipGetLastError();
}

// G + λI (padding diagonal 1) as the big kernel's tile image [tile][lane][4] (no column
// permutation: the big kernel's tiles are canonical), for the split-K reduction
template <typename T>
__global__ void gimg_big_kernel(const T* G, int nt, int k, double lambda, T* img) {
  using M = Mfma<T>;
  const int KP = 16 * nt, NTT = nt * (nt + 1) / 2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NTT * 256) return;
  const int r = idx & 3, lane = (idx >> 2) & 63, t = idx >> 8;
  int I = 0;
  while (tile_index(I + 1, 0) <= t) ++I;
  const int J = t - tile_index(I, 0);
  const int i = 16 * I + M::crow(lane, r), j = 16 * J + (lane & 15);
  double g = (double)G[(int64_t)i * KP + j];
  if (i == j) g += (i < k) ? lambda : 1.0;
  img[idx] = (T)g;
}

// Split-K second pass for the big tilings (runtime tile count; heavy_reduce_kernel's contract,
// wals_heavy.hip): one workgroup of 256 threads per (heavy row, tile) sums the row's segments
// in segment order in fp64 with G + λI, rounds once and writes over the first segment's
// slot; tile index NTT takes the rhs, Σc and the flag.
template <typename T>
__global__ __launch_bounds__(256) void heavy_reduce_big_kernel(T* part, T* partb, double* partc,
                                                               const int64_t* hseg, int64_t h0,
                                                               const T* Gimg, int nt) {
  const int KP = 16 * nt, NTT = nt * (nt + 1) / 2;
  const int t = blockIdx.y;
  const int64_t h = h0 + blockIdx.x;
  const int64_t s0 = hseg[h], s1 = hseg[h + 1];
  const int tid = threadIdx.x;
  if (t < NTT) {
    const int64_t off = (int64_t)t * 256 + tid;
    double v = (double)Gimg[off];
    for (int64_t s = s0; s < s1; ++s) v += (double)part[s * ((int64_t)NTT * 256) + off];
    part[s0 * ((int64_t)NTT * 256) + off] = (T)v;
  } else {
    for (int j = tid; j < KP; j += 256) {
      double b = 0.0;
      for (int64_t s = s0; s < s1; ++s) b += (double)partb[s * KP + j];
      partb[s0 * KP + j] = (T)b;
    }
    if (tid == 0) {
      double c = 0.0, f = 0.0;
      for (int64_t s = s0; s < s1; ++s) {
        c += partc[2 * s];
        f = fmax(f, partc[2 * s + 1]);
      }
      partc[2 * s0] = c;
      partc[2 * s0 + 1] = f;
    }
  }
}

template <typename T>
static hipError_t heavy_reduce_big(T* part, T* partb, double* partc, const int64_t* hseg,
                                   int64_t h0, int64_t nh, const T* G, T* Gimg, int nt, int k,
                                   double lambda, hipStream_t s) {
  const int NTT = nt * (nt + 1) / 2;
  hipLaunchKernelGGL((gimg_big_kernel<T>), dim3(NTT), dim3(256), 0, s, G, nt, k, lambda, Gimg);
  for (int64_t done = 0; done < nh; done += 65535) {
    const int64_t cnt = nh - done < 65535 ? nh - done : 65535;
    hipLaunchKernelGGL((heavy_reduce_big_kernel<T>), dim3((unsigned)cnt, NTT + 1), dim3(256), 0,
                       s, part, partb, partc, hseg, h0 + done, (const T*)Gimg, nt);
  }
  return hipGetLastError();
}
hipError_t launch_heavy_reduce_big(float* part, float* partb, double* partc, const int64_t* hseg,
                                   int64_t h0, int64_t nh, const float* G, float* Gimg, int nt,
                                   int k, double lambda, hipStream_t s) {
  return heavy_reduce_big(part, partb, partc, hseg, h0, nh, G, Gimg, nt, k, lambda, s);
}
hipError_t launch_heavy_reduce_big(double* part, double* partb, double* partc, const int64_t* hseg,
                                   int64_t h0, int64_t nh, const double* G, double* Gimg, int nt,
                                   int k, double lambda, hipStream_t s) {
  return heavy_reduce_big(part, partb, partc, hseg, h0, nh, G, Gimg, nt, k, lambda, s);
}

#define QMFX_BIG_SWITCH(NTV, CALL)        \
  switch (NTV) {                          \
    case 5: return CALL(5);               \
    case 6: return CALL(6);               \
    case 7: return CALL(7);               \
    case 8: return CALL(8);               \
    case 9: return CALL(9);               \
    case 10: return CALL(10);             \
    case 11: return CALL(11);             \
    case 12: return CALL(12);             \
    case 13: return CALL(13);             \
    case 14: return CALL(14);             \
    case 15: return CALL(15);             \
    case 16: return CALL(16);             \
    default: return hipErrorInvalidValue; \
  }

#ifdef QMFX_BIG_DEV16
// (register / ISA inspection builds only: the k = 256 instances alone)
#undef QMFX_BIG_SWITCH
#define QMFX_BIG_SWITCH(NTV, CALL) return NTV == 16 ? CALL(16) : hipErrorInvalidValue;
#define QMFX_BIG_ROW_SWITCH(NTV, CALL) return NTV == 16 ? CALL(16) : hipErrorInvalidValue;
#else
// the row kernel takes k > 128 only (qmfx.cpp use_big_rows); the tiled YᵀY also fp64 k = 80..128
#define QMFX_BIG_ROW_SWITCH(NTV, CALL)    \
  switch (NTV) {                          \
    case 9: return CALL(9);               \
    case 10: return CALL(10);             \
    case 11: return CALL(11);             \
    case 12: return CALL(12);             \
    case 13: return CALL(13);             \
    case 14: return CALL(14);             \
    case 15: return CALL(15);             \
    case 16: return CALL(16);             \
    default: return hipErrorInvalidValue; \
  }
#endif
hipError_t launch_wals_big(const SolveArgs<float>& a, int nt, hipStream_t s) {
#define CALL(N) launch_big_nt<float, N>(a, s)
  QMFX_BIG_ROW_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_wals_big(const SolveArgs<double>& a, int nt, hipStream_t s) {
#define CALL(N) launch_big_nt<double, N>(a, s)
  QMFX_BIG_ROW_SWITCH(nt, CALL)
#undef CALL
}
template <typename T>
static hipError_t gram_big(const T* Y, int64_t n, int nt, T* G, double* partial, int max_blocks,
                           hipStream_t s) {
  int64_t rpb = (n + max_blocks - 1) / max_blocks;
  rpb = ((rpb + 3) / 4) * 4;
  if (rpb < 64) rpb = 64;
  const int nblocks = (int)((n + rpb - 1) / rpb);
  hipError_t e = hipSuccess;
#define CALL(N) launch_gram_tiles_nt<T, N>(Y, n, partial, nblocks, rpb, s)
  e = [&]() -> hipError_t { QMFX_BIG_SWITCH(nt, CALL) }();
#undef CALL
  if (e != hipSuccess) return e;
  const int KP = 16 * nt;
  hipLaunchKernelGGL((gram_reduce_rt_kernel<T>), dim3(KP * KP / 16), dim3(256), 0, s,
                     partial, nblocks, nt, G);
  return hipGetLastError();
}
hipError_t launch_gram_big(const float* Y, int64_t n, int nt, float* G, double* partial,
                           int max_blocks, hipStream_t s) {
  return gram_big(Y, n, nt, G, partial, max_blocks, s);
}
hipError_t launch_gram_big(const double* Y, int64_t n, int nt, double* G, double* partial,
                           int max_blocks, hipStream_t s) {
  return gram_big(Y, n, nt, G, partial, max_blocks, s);
}

}  // namespace qmfx
