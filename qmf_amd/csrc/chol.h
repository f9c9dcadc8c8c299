// Register-tile Cholesky + solve of one SPD system per wave64 (shared by the direct and
// the whitened row kernels).
#pragma once
#include "common.h"
#include "rowsolve.h"

#include <utility>

namespace qmfx {

// ---------------------------------------------------------------------------------------
// Register-tile LDLᵀ factorization + solves of one SPD system per wave64, shared by the
// direct and the whitened row kernels (the method: chol_solve's comment below).
//   In:  acc = lower 16×16 tiles of an SPD matrix of size 16·NT (diagonal tiles full);
//        S.bw = right-hand side (written and synchronised by the caller).
//   Out: S.xs = solution.  `bad` set on a non-positive pivot.
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

// LDS ordering inside chol_solve.  chol_solve REQUIRES a single-wave workgroup: LDS accesses
// of one wave execute in order, so draining them and pinning the compiler's order is enough
// (no s_barrier; the same speed as a plain compiler fence in the micro-benchmark,
// tools/exp/chol_bench.hip).  Both WS values behave the same — there is no workgroup barrier
// here — and a multi-wave caller would race on S.panel and S.bw (debug builds trap on one,
// chol_solve below).
template <bool WS>
__device__ __forceinline__ void csync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// fp64 broadcast of lane J of every 16-lane row (one v_mov_b64_dpp row_newbcast)
template <int J>
__device__ __forceinline__ double bcast16(double v) {
  long long b = __builtin_bit_cast(long long, v);
  long long r = __builtin_amdgcn_update_dpp(b, b, 0x150 + J, 0xf, 0xf, true);
  return __builtin_bit_cast(double, r);
}
// acc += (lane J of src's 16-lane row) · m: one v_fmac_f64_dpp row_newbcast, the broadcast
// fused into the FMA (the compiler does not form the 64-bit DPP FMA itself).  NOP = 1 pads
// two wait states after it: the hazard recognizer does not see this asm's VGPR write, and the
// next column broadcasts the register it writes.
template <int J, int NOP = 0>
__device__ __forceinline__ void fmac_bcast16(double& acc, double src, double m) {
  if constexpr (NOP)
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf\n\ts_nop 1"
                 : "+v"(acc) : "v"(src), "v"(m), "n"(J));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(m), "n"(J));
}
template <int J, int NOP = 0>
__device__ __forceinline__ void fmac_bcast16(float& acc, float src, float m) {
  if constexpr (NOP)
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf\n\ts_nop 1"
                 : "+v"(acc) : "v"(src), "v"(m), "n"(J));
  else
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(m), "n"(J));
}
// 1/d for the LDLᵀ pivots: fp32 v_rcp_f32 (1 ulp); fp64 v_rcp_f64 + two Newton steps (an ulp
// or so; a non-positive or NaN d leaves the result outside (0, ∞), which the caller flags)
__device__ __forceinline__ float pivot_rcp(float d) { return __builtin_amdgcn_rcpf(d); }
#ifndef QMFX_RCP_NEWTON
#define QMFX_RCP_NEWTON 2
#endif
__device__ __forceinline__ double pivot_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
#pragma unroll
  for (int i = 0; i < QMFX_RCP_NEWTON; ++i) {
    const double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
  }
  return r;
}

// Column C of an fp64 panel in the replicated-diagonal layout (chol_solve below): the pivot
// d = U[C][C] and z_C = b_C broadcast from lane C of every 16-lane row, l = U[q][C]/d, the
// right-hand sides' update, and the trailing columns m > C of the diagonal block and of the
// first slot of rows below it (`has0`), each element one v_fmac_f64_dpp of column C's
// broadcast entry U[m][C].
template <int C>
__device__ __forceinline__ void dg_column(double (&dg)[16], double& bdg, double (&pa)[16],
                                          double& pb, bool has0, int cl, double& invv,
                                          double& zv) {
  const double d = bcast16<C>(dg[C]);
  const double bc = bcast16<C>(bdg);
  const double invd = pivot_rcp(d);
  const bool me = cl == C;
  invv = me ? invd : invv;
  zv = me ? bc : zv;
  // rows at or above the pivot only change their dead upper part (and their b, read no more)
  const double nl = -(dg[C] * invd);
  const double nls = -(pa[C] * invd);
  bdg = __builtin_fma(nl, bc, bdg);
  if (has0) pb = __builtin_fma(nls, bc, pb);
  // the next column first (the chain: the next pivot broadcasts it), padded for the DPP read
  // that follows
  [&]<int... Ms>(std::integer_sequence<int, Ms...>) {
    auto upd = [&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      if constexpr (m > C) {
        fmac_bcast16<m, (m == C + 1) ? 1 : 0>(dg[m], dg[C], nl);
        if (has0) fmac_bcast16<m>(pa[m], dg[C], nls);
      }
    };
    (upd(std::integral_constant<int, Ms>{}), ...);
  }(std::make_integer_sequence<int, 16>{});
  __builtin_amdgcn_sched_barrier(0);
}
// Column C for a further slot of rows, after the diagonal block is factored: its final
// column C is what column C broadcast, and lane C holds 1/d_C and z_C.
template <int C>
__device__ __forceinline__ void slot_column(const double (&dg)[16], double invv, double zv,
                                            double (&pa)[16], double& pb) {
  const double invd = bcast16<C>(invv);
  const double bc = bcast16<C>(zv);
  const double nls = -(pa[C] * invd);
  pb = __builtin_fma(nls, bc, pb);
  [&]<int... Ms>(std::integer_sequence<int, Ms...>) {
    auto upd = [&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      if constexpr (m > C) fmac_bcast16<m>(pa[m], dg[C], nls);
    };
    (upd(std::integral_constant<int, Ms>{}), ...);
  }(std::make_integer_sequence<int, 16>{});
  __builtin_amdgcn_sched_barrier(0);
}

// ---------------------------------------------------------------------------------------
// LDLᵀ of one SPD system per wave64 with the forward and backward solves (A = U D⁻¹ Uᵀ,
// U = the unnormalised columns: U[q][c] = the trailing matrix's A[q][c] when column c is
// eliminated, D = diag(U[c][c])).  Right-looking over 16-column panels, as a Cholesky, but
// the pivots take one reciprocal instead of a reciprocal square root, the panel keeps U
// (nothing is rescaled), and the forward solve's z_c = b_c needs no multiply.
//   Panel, fp32: lane q holds row q of the panel (two slots at KP > 64); column c's entries
//   U[m][c] of the diagonal block are broadcast by readlane and the update is packed FMAs.
//   Panel, fp64: the diagonal block's 16 rows are held in EVERY 16-lane row of the wave
//   (`dg`, lane 16g + i holds row i), and the rows below it in `pa` (lane q, slot s: row 16 +
//   q + 64s).  Column c's entries then sit in lane c of every 16-lane row, so each update
//   element is one v_fmac_f64_dpp row_newbcast (measured 4.9 cycles for one wave, as a plain
//   FMA) instead of two v_readlane_b32 (6.4 each) + an FMA; the copy costs one FMA per
//   element of the diagonal block.
//   The trailing update A(I,J) −= U(I,p) D⁻¹ U(J,p)ᵀ is 4 MFMAs per tile with operands from
//   the LDS panel (the J operand scaled by 1/d of its column); the diagonal blocks go to LDS
//   transposed and scaled, Lt[q][c] = U[c][q]/d_q (c > q), for the backward substitution
//   (one v_fmac_dpp row_newbcast per column instead of a readlane + an FMA).
// In: acc = lower 16×16 tiles of the SPD matrix; S.bw = right-hand side.  Out: S.xs = x.
// `bad` is set on a pivot that is not positive (or not finite).
// ---------------------------------------------------------------------------------------
template <typename T, int NT, bool WS = false, bool LTP = false>
__device__ __forceinline__ void chol_solve(typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                           CholShared<T, NT, LTP>& S, int lane, int& bad) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr bool DG = sizeof(T) == 8;  // fp64: replicated diagonal block + DPP FMAs
  // row slots per lane: fp32 every panel row; fp64 the rows below the diagonal block
  // (at KP = 16 the fp64 slot holds nothing: every guard below is false)
  constexpr int SLOTS = DG ? ((KP - 16 + 63) / 64 > 0 ? (KP - 16 + 63) / 64 : 1) : (KP + 63) / 64;
  constexpr int PLD = CholShared<T, NT, LTP>::PLD;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int q0 = DG ? 16 : 0;  // first panel row held by slot 0
#ifdef QMFX_DEBUG
  if (blockDim.x * blockDim.y * blockDim.z != 64) __builtin_trap();  // single-wave callers only
#endif
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
    // lanes c (fp32) / lanes 16g + c (fp64) collect 1/d_c and z_c, stored once per panel
    T invv = T(0), zv = T(0);
    T pa[SLOTS][16];
    T pb[SLOTS];
    if constexpr (DG) {
      // the diagonal block in every 16-lane row and the first slot of rows below it, factored
      // column by column together; further slots (k = 96..128) after it, one at a time
      T dg[16];
      lds_row_load(&S.panel[cl * PLD], dg);
      T bdg = S.bw[16 * p + cl];
      const bool has0 = 16 < R;
      {
        const int q = 16 + lane;
        const int qq = q < R ? q : 0;
        lds_row_load(&S.panel[qq * PLD], pa[0]);
        pb[0] = S.bw[16 * p + qq];
      }
      [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        (dg_column<Cs>(dg, bdg, pa[0], pb[0], has0, cl, invv, zv), ...);
      }(std::make_integer_sequence<int, 16>{});
#pragma unroll
      for (int s = 1; s < SLOTS; ++s) {
        if (16 + 64 * s < R) {
          const int q = 16 + lane + 64 * s;
          const int qq = q < R ? q : 0;
          lds_row_load(&S.panel[qq * PLD], pa[s]);
          pb[s] = S.bw[16 * p + qq];
          [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
            (slot_column<Cs>(dg, invv, zv, pa[s], pb[s]), ...);
          }(std::make_integer_sequence<int, 16>{});
          if (q < R) {
            lds_row_store(&S.panel[q * PLD], pa[s]);
            S.bw[16 * p + q] = pb[s];
          }
        }
      }
      if (lane < 16) lds_row_store(&S.panel[lane * PLD], dg);
    } else {
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        const int q = lane + 64 * s;
        const int qq = q < R ? q : 0;
        lds_row_load(&S.panel[qq * PLD], pa[s]);
        pb[s] = S.bw[16 * p + qq];
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const bool me = cl == c;
        // A[m][c] of the diagonal block's rows, broadcast (readlane) before the pivot is
        // known; constant trip counts with a predicate (the loops must unroll fully before c
        // is known, or the compiler falls back to indexed register access)
        T am[16];
#pragma unroll
        for (int m = 1; m < 16; ++m)
          if (m > c) am[m] = readlane(pa[0][c], m);
        const T d = readlane(pa[0][c], c);
        const T bc = readlane(pb[0], c);
        const T invd = pivot_rcp(d);
        invv = me ? invd : invv;
        zv = me ? bc : zv;
#pragma unroll
        for (int s = 0; s < SLOTS; ++s) {
          if (64 * s < R) {
            const T lqs = pa[s][c] * invd;
            pb[s] -= lqs * bc;
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
          }
        }
        // one column per scheduling window: readlanes hoisted across columns exhaust the
        // SGPRs.  The fence pins every slot's updates inside the window; without it the
        // compiler defers the slots past the first to the end of the panel.
#pragma unroll
        for (int s = 1; s < SLOTS; ++s) {
          if (64 * s < R) {
#pragma unroll
            for (int m = 0; m < 16; ++m)
              if (m > c) asm volatile("" : "+v"(pa[s][m]));
            asm volatile("" : "+v"(pb[s]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // a pivot that is not positive (or not finite) leaves 1/d outside (0, ∞)
    bad |= __any(lane < 16 && !(invv > T(0) && invv < __builtin_huge_val())) ? 1 : 0;
    if (lane < 16) {
      S.invd[16 * p + lane] = invv;
      S.bw[16 * p + lane] = zv;
    }
    // (fp64: the slots after the first were stored by their own pass)
#pragma unroll
    for (int s = 0; s < (DG ? 1 : SLOTS); ++s) {
      const int q = q0 + lane + 64 * s;
      if (q < R) lds_row_store(&S.panel[q * PLD], pa[s]);
      if (q >= 16 && q < R) S.bw[16 * p + q] = pb[s];
    }
    csync<WS>();
    // diagonal block → Lt (transposed, scaled by the row's 1/d, zero on and above the
    // diagonal)
    T ltv[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = lane + 64 * it;
      const int r = idx >> 4, c = idx & 15;
      ltv[it] = c < r ? -(S.panel[r * PLD + c] * S.invd[16 * p + c]) : T(0);
    }
    if constexpr (!LTP) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = lane + 64 * it;
        S.lt_row(p * 16 + (idx & 15))[idx >> 4] = ltv[it];
      }
    }
    // trailing operands: U(I, p) fragments (the J side is scaled by 1/d of its column below)
    T fr[NT][4];
    T dcol[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) dcol[s] = S.invd[16 * p + 4 * s + kk];
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
    for (int J = p + 1; J < NT; ++J) {
      T sj[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) sj[s] = fr[J][s] * dcol[s];
#pragma unroll
      for (int I = J; I < NT; ++I) {
        const int tj = tile_index(I, J);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[tj] = M::mma(-fr[I][s], sj[s], acc[tj]);
      }
    }
    csync<WS>();
  }
  // backward solve Uᵀ-form by 16-blocks from the bottom: x_q = (z_q − Σ_{c>q} U[c][q] x_c)/d_q.
  // Lane cl carries row cl of the block scaled by its own 1/d; column c then finishes x_c
  // (readlane) and removes it from the rows above with the scaled Lt (one FMA)
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
    // x_c is lane c's vm in every 16-lane row: one DPP FMA per column (Lt stored negated),
    // padded for the next column's DPP read of the register it writes
    // (vm was just written by the compiler's VALU, which does not see this asm's DPP read:
    // two wait states first)
    asm volatile("s_nop 1" : "+v"(vm));
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
      (fmac_bcast16<15 - Cs, 1>(vm, vm, lt[15 - Cs]), ...);
    }(std::make_integer_sequence<int, 16>{});
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
