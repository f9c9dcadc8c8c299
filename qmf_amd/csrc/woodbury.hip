// WALS whitened (n×n Woodbury) row kernels on MI355X (gfx950), the whitening GEMMs and the
// fp64 inverse Cholesky factor of G + λI.  See wals.hip for the per-row algebra.
//
// Reference path (taozhijiang/qmf): WALSEngine::updateFactorsForOne
// qmf/wals/WALSEngine.cpp:266-310 and linearSymmetricSolve qmf/Matrix.cpp:81-96 (the same
// solution by the push-through identity).
#include <algorithm>
#include <cstdlib>

#include "chol.h"
#include "common.h"
#include "kernels.h"
#include "ntswitch.h"
#include "rowsolve.h"

namespace qmfx {

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
#ifndef QMFX_WB3_MIN_WAVES
#define QMFX_WB3_MIN_WAVES 2
#endif
template <typename T, int NTK, int NTN, bool TRACE>
__global__ __launch_bounds__(64, NTK > 8 ? 1 : (NTN == 4 ? QMFX_WB4_MIN_WAVES : (NTN == 3 ? QMFX_WB3_MIN_WAVES : 2)))
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
  {
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
// Whitened row kernel, streamed (fp32, k ≤ 128): the n×n solve of wals_woodbury_kernel
// without holding Zₛ in registers.  K = Zₛ Zₛᵀ accumulates over 32-column chunks of the
// gathered rows — each chunk split into bf16 parts as it arrives, the next chunk in flight —
// and x' = Zₛᵀu gathers the rows a second time after the solve, from the L2 / MALL (the same
// rows were read a few µs earlier).  Lane (i, g) holds columns 32s + 8g .. +7 of signal
// 16I + i in chunk s.  ≈150 VGPRs instead of 256 at NTN = 4: three waves per SIMD.
// ---------------------------------------------------------------------------------------
#ifndef QMFX_WB_ST_WAVES
#define QMFX_WB_ST_WAVES 3
#endif
// K on the bf16 matrix cores from split3 parts (the exact f32 MFMA path measured slower at
// k = 64 and 128: profiles/r06/ab_c2_f32_kpass.txt)
// n×n buckets beyond 64 signals (NTN = 5..8, k = 256): each lane carries H = 2 signals (e
// = lane and lane + 64); the registers of the wider tiles leave two or one waves per SIMD.
template <int NTN>
constexpr int wb_st_waves() {
  return NTN <= 4 ? QMFX_WB_ST_WAVES : (NTN == 5 ? 2 : 1);
}
// chunks in flight ahead of the one being consumed, K pass and x' pass (n ≤ 64 buckets)
#ifndef QMFX_WBS_KD
#define QMFX_WBS_KD 1
#endif
#ifndef QMFX_WBS_XD
#define QMFX_WBS_XD 1
#endif
template <int NTN>
constexpr int wbs_kdepth() {
  return NTN <= 4 ? QMFX_WBS_KD : 1;
}
template <int NTN>
constexpr int wbs_xdepth() {
  return NTN <= 4 ? QMFX_WBS_XD : 1;
}
template <int NTK, int NTN>
__global__ __launch_bounds__(64, wb_st_waves<NTN>()) void wals_woodbury_st_kernel(SolveArgs<float> a) {
  using M = Mfma<float>;
  using acc_t = f32x4;
  constexpr int KP = 16 * NTK;
  constexpr int NTT = NTN * (NTN + 1) / 2;
  constexpr int NS = (KP + 31) / 32;
  __shared__ __attribute__((aligned(16))) CholShared<float, NTN> S;
  __shared__ __attribute__((aligned(16))) float gq[16 * NTN];

  constexpr int H = NTN > 4 ? 2 : 1;  // signals per lane: e = lane + 64h
  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const RowDesc dn = a.desc[a.row_begin + blockIdx.x];
  const int64_t row = dn.row;
  const int n = dn.n;  // ≤ 16·NTN by bucketing
  bool mine[H], isP[H], isQ[H];
  int cr[H];
  float wl[H], cwl[H];
  uint64_t mQ[H];
  int bad = 0;
  bool hasQ = false;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const int e = lane + 64 * h;
    mine[h] = e < n;
    cr[h] = mine[h] ? a.col[dn.beg + e] : a.zrow;
    const float vr = mine[h] ? a.val[dn.beg + e] : 0.f;
    wl[h] = mine[h] ? a.alpha * vr : 0.f;
    cwl[h] = mine[h] ? 1.f + a.alpha * vr : 0.f;
    isP[h] = mine[h] && wl[h] > 0.f;
    isQ[h] = mine[h] && wl[h] == 0.f;
    bad |= __any(mine[h] && wl[h] < 0.f) ? 1 : 0;
    mQ[h] = __ballot(isQ[h]);
    hasQ |= mQ[h] != 0;
  }
  // bit e of a per-signal mask held as H 64-bit words
  auto bit = [](const uint64_t (&m)[H], int e) -> bool { return (m[e >> 6] >> (e & 63)) & 1; };

  // this lane's signals 16I + cl (padding signals read the all-zero row a.zrow)
  const f32x4* zp[NTN];
#pragma unroll
  for (int I = 0; I < NTN; ++I) {
    const int ce = __shfl(cr[I >> 2], (16 * I + cl) & 63, 64);
    zp[I] = reinterpret_cast<const f32x4*>(a.Y + (uint64_t)(uint32_t)ce * KP);
  }
  auto load_chunk = [&](int s, f32x4 (&buf)[NTN][2]) {
    const int c4 = 8 * s + 2 * kk;  // f32x4 index of column 32s + 8kk
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      if (32 * s + 32 <= KP || 32 * s + 8 * kk < KP) {
        buf[I][0] = zp[I][c4];
        buf[I][1] = zp[I][c4 + 1];
      } else {
        buf[I][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        buf[I][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  acc_t acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0.f, 0.f, 0.f, 0.f};
  float sq[NTN];  // z_eᵀ Σ_{f∈Q} z_f over this lane's columns (rows with Q signals)
#pragma unroll
  for (int I = 0; I < NTN; ++I) sq[I] = 0.f;
  {
    // a ring of KD + 1 chunk buffers: chunk s + KD is in flight while chunk s is consumed
    constexpr int KD = wbs_kdepth<NTN>();
    f32x4 buf[KD + 1][NTN][2];
#pragma unroll
    for (int s = 0; s < KD && s < NS; ++s) load_chunk(s, buf[s]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + KD < NS) load_chunk(s + KD, buf[(s + KD) % (KD + 1)]);
      f32x4 (&cur)[NTN][2] = buf[s % (KD + 1)];
      Split3 sp[NTN];
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
        float x[8];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          x[c] = cur[I][0][c];
          x[4 + c] = cur[I][1][c];
        }
        split3(x, sp[I]);
      }
      if (hasQ) {
        float g[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float v = 0.f;
#pragma unroll
            for (int I = 0; I < NTN; ++I)
              if (bit(mQ, 16 * I + cl)) v += cur[I][h][c];
            g[h][c] = v;
          }
        row16_sum4(g[0]);
        row16_sum4(g[1]);
#pragma unroll
        for (int I = 0; I < NTN; ++I)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 4; ++c) sq[I] += cur[I][h][c] * g[h][c];
      }
#pragma unroll
      for (int I = 0; I < NTN; ++I) {
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          const int t = tile_index(I, J);
          acc[t] = mma_split6(sp[I], sp[J], acc[t]);
        }
      }
      // one chunk's splits and the next chunks' loads live at a time
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  double xb = 0.0;
  float ul[NTN], cv[NTN];
  if (!hasQ) {
    float iw[H], rhs[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      iw[h] = isP[h] ? fast_rcp(wl[h]) : 1.f;
      rhs[h] = isP[h] ? cwl[h] * iw[h] : 0.f;
    }
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const float iwd = __shfl(iw[I >> 2], (16 * I + cl) & 63, 64);
      const int t = tile_index(I, I);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] += M::crow(lane, r) == cl ? iwd : 0.f;
    }
#pragma unroll
    for (int h = 0; h < H; ++h)
      if (lane + 64 * h < 16 * NTN) S.bw[lane + 64 * h] = rhs[h];
    __syncthreads();
    chol_solve<float, NTN>(acc, S, lane, bad);
    double xbl = 0.0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float ue = lane + 64 * h < 16 * NTN ? S.xs[lane + 64 * h] : 0.f;
      xbl += isP[h] ? (double)(rhs[h] * (cwl[h] - ue)) : 0.0;
    }
    xb = wave_sum(xbl);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      ul[I] = S.xs[16 * I + cl];
      cv[I] = 0.f;
    }
  } else {
    float rhs[H], iw[H];
#pragma unroll
    for (int h = 0; h < H; ++h) rhs[h] = isP[h] ? cwl[h] * fast_rcp(wl[h]) : 0.f;
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      float v = sq[I];
      v += shfl_xor(v, 16);
      v += shfl_xor(v, 32);
      if (kk == 0) gq[16 * I + cl] = v;
    }
    __syncthreads();
    uint64_t mP[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float kqv = lane + 64 * h < 16 * NTN ? gq[lane + 64 * h] : 0.f;
      if (isP[h]) rhs[h] -= kqv;
      iw[h] = isP[h] ? fast_rcp(wl[h]) : 0.f;
      mP[h] = __ballot(isP[h]);
    }
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const float iwd = __shfl(iw[I >> 2], (16 * I + cl) & 63, 64);
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        const int f = 16 * J + cl;
        const bool pf = bit(mP, f);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 16 * I + M::crow(lane, r);
          const bool pe = bit(mP, e);
          float v = acc[t][r];
          if (pe && pf) v += (e == f) ? iwd : 0.f;
          else v = (e == f) ? 1.f : 0.f;
          acc[t][r] = v;
        }
      }
    }
#pragma unroll
    for (int h = 0; h < H; ++h)
      if (lane + 64 * h < 16 * NTN) S.bw[lane + 64 * h] = rhs[h];
    __syncthreads();
    chol_solve<float, NTN>(acc, S, lane, bad);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const int e = 16 * I + cl;
      const bool pe = bit(mP, e);
      const bool qe = bit(mQ, e);
      ul[I] = pe ? S.xs[e] : (qe ? 1.f : 0.f);
      cv[I] = __shfl(cwl[I >> 2], e & 63, 64);
    }
  }

  // x' = Zₛᵀu (and for rows with Q signals xᵀb = x'ᵀ(Zₛᵀc)), the rows gathered again
  {
    // XD chunks in flight (the accumulators are dead after the solve)
    constexpr int XD = wbs_xdepth<NTN>();
    f32x4 buf[XD + 1][NTN][2];
#pragma unroll
    for (int s = 0; s < XD && s < NS; ++s) load_chunk(s, buf[s]);
    double xbq = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + XD < NS) load_chunk(s + XD, buf[(s + XD) % (XD + 1)]);
      f32x4 (&cur)[NTN][2] = buf[s % (XD + 1)];
      float sx[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float v = 0.f;
#pragma unroll
          for (int I = 0; I < NTN; ++I) v += cur[I][h][c] * ul[I];
          sx[h][c] = v;
        }
      // column 32s + 8kk + row16_sum8_column(cl) of x' in the lanes with cl & 2 == 0 (and
      // their neighbours)
      const float sxc = row16_sum8_split(sx, cl);
      if (hasQ) {
        float sb[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float v = 0.f;
#pragma unroll
            for (int I = 0; I < NTN; ++I) v += cur[I][h][c] * cv[I];
            sb[h][c] = v;
          }
        const float sbc = row16_sum8_split(sb, cl);
        xbq += (cl & 2) == 0 ? (double)sxc * (double)sbc : 0.0;
      }
      if ((cl & 2) == 0 && 32 * s + 8 * kk < KP)
        a.X[row * KP + 32 * s + 8 * kk + row16_sum8_column(cl)] = bad ? 0.f : sxc;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (hasQ) xb = wave_sum(xbq);
  }
  double cs = 0.0;
#pragma unroll
  for (int h = 0; h < H; ++h) cs += (double)cwl[h];
  const double csum = wave_sum(cs);
  if (lane == 0) {
    a.rowloss[row] = bad ? 0.0 : csum - xb;  // −λ‖x‖² added after unwhitening
    if (bad && a.status) a.status[row] = 1;
  }
}

// ---------------------------------------------------------------------------------------
// Whitened row kernel, streamed, fp64 (k = 80..128 and 256): the fp32 streamed kernel's plan on the
// fp64 matrix path.  K = Zₛ Zₛᵀ accumulates over 16-column chunks of the gathered rows with
// the next chunk in flight: lane (i, g) holds columns 16s + 4g .. +3 of signal 16I + i, and
// its j-th value is the K index of 16x16x4 f64 MFMA j (exact fp64 products, no split).
// x' = Zₛᵀu gathers the rows a second time after the solve.  Replaces the multi-wave kernel
// whose register-resident Zₛ (half a row of doubles per lane) spilled.
// ---------------------------------------------------------------------------------------
typedef double f64x2 __attribute__((ext_vector_type(2)));

// chunks in flight ahead of the one being consumed: K pass (beside the NTT accumulator
// tiles) and x' pass (after the solve, when the accumulators are dead)
#ifndef QMFX_WB64_KD
#define QMFX_WB64_KD 1
#endif
// (x' pass: 2 since round 6, −0.9 ms per C3 fp64 user half same box, profiles/r06/
// ab_whiten_lds.txt; round 3 had measured no gain with more chunks kept on chip)
#ifndef QMFX_WB64_XD
#define QMFX_WB64_XD 2
#endif
#ifndef QMFX_WB64_LTP
#define QMFX_WB64_LTP 1
#endif
// waves per SIMD the streamed fp64 kernel is compiled for, by n×n tile count (n ≤ 16·NTN)
#ifndef QMFX_WB64_WAVES
#define QMFX_WB64_WAVES 2
#endif
#ifndef QMFX_WB64_WAVES3
#define QMFX_WB64_WAVES3 2
#endif
#ifndef QMFX_WB64_WAVES2
#define QMFX_WB64_WAVES2 2
#endif
template <int NTN>
constexpr int wb64_waves() {
  return NTN <= 2 ? QMFX_WB64_WAVES2 : NTN == 3 ? QMFX_WB64_WAVES3 : NTN == 4 ? QMFX_WB64_WAVES : 1;
}
template <int NTN>
constexpr int wb64_kdepth() {
  return NTN <= 4 ? QMFX_WB64_KD : 1;
}
// 16-column chunks of Zₛ kept in registers from the K pass to the x' pass (the first KEEP;
// the rest are gathered again): the registers the n×n Cholesky leaves free at two waves per
// SIMD (fp64 whitened rows are bound by the fabric's random-row rate, so every chunk not
// re-gathered is 1/NTK of the second pass's bytes)
// fp64 k = 64 whitened rows on the streamed kernel (round 5: C2 fp64 18.5 -> 17.6 ms/epoch
// with n ≤ 48 whitened; the register-resident kernel measured slower there)
#ifndef QMFX_WB64_KEEP2
#define QMFX_WB64_KEEP2 6
#endif
#ifndef QMFX_WB64_KEEP3
#define QMFX_WB64_KEEP3 2
#endif
#ifndef QMFX_WB64_KEEP4
#define QMFX_WB64_KEEP4 1
#endif
template <int NTK, int NTN>
constexpr int wb64_keep() {
  constexpr int k = NTN <= 2 ? QMFX_WB64_KEEP2 : NTN == 3 ? QMFX_WB64_KEEP3 : NTN == 4 ? QMFX_WB64_KEEP4 : 0;
  return k < NTK ? k : NTK;
}
// and the next QMFX_WB64_KL{3,4,5} chunks kept in LDS (the room left under the per-CU LDS
// at the kernel's waves per SIMD: ≤ 20 KB per row at n ≤ 64, ≤ 40 KB at n ≤ 80)
#ifndef QMFX_WB64_KL3
#define QMFX_WB64_KL3 1
#endif
#ifndef QMFX_WB64_KL4
#define QMFX_WB64_KL4 1
#endif
#ifndef QMFX_WB64_KL5
#define QMFX_WB64_KL5 2
#endif
template <int NTK, int NTN>
constexpr int wb64_keep_lds() {
  constexpr int k = NTN == 3 ? QMFX_WB64_KL3 : NTN == 4 ? QMFX_WB64_KL4 : NTN == 5 ? QMFX_WB64_KL5 : 0;
  constexpr int room = NTK - wb64_keep<NTK, NTN>();
  return k < room ? k : room;
}
template <int NTN>
constexpr int wb64_xdepth() {
  return NTN <= 4 ? QMFX_WB64_XD : 1;
}
template <int NTK, int NTN, bool TRACE = false>
__global__ __launch_bounds__(64, wb64_waves<NTN>()) void wals_woodbury_st64_kernel(SolveArgs<double> a) {
  using M = Mfma<double>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NTK;
  constexpr int NTT = NTN * (NTN + 1) / 2;
  constexpr int NS = NTK;  // 16-column chunks
  // the diagonal L blocks ride in the panel array (chol.h, LTP): 10.8 KB per row at n ≤ 64
  __shared__ __attribute__((aligned(16))) CholShared<double, NTN, QMFX_WB64_LTP != 0> S;
  __shared__ __attribute__((aligned(16))) double gq[16 * NTN];
  // Zₛ chunks kept in LDS for the x' pass: [chunk][I·4 + c][lane]
  constexpr int KL = wb64_keep_lds<NTK, NTN>();
  __shared__ __attribute__((aligned(16))) double kl[KL > 0 ? KL : 1][NTN * 4][64];

  constexpr int H = NTN > 4 ? 2 : 1;  // signals per lane: e = lane + 64h
  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  uint64_t tr[5] = {0, 0, 0, 0, 0};
  if (TRACE) tr[0] = __builtin_amdgcn_s_memtime();
  const RowDesc dn = a.desc[a.row_begin + blockIdx.x];
  const int64_t row = dn.row;
  const int n = dn.n;  // ≤ 16·NTN by bucketing
  bool mine[H], isP[H], isQ[H];
  int cr[H];
  double wl[H], cwl[H];
  uint64_t mQ[H];
  int bad = 0;
  bool hasQ = false;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const int e = lane + 64 * h;
    mine[h] = e < n;
    cr[h] = mine[h] ? a.col[dn.beg + e] : a.zrow;
    const double vr = mine[h] ? a.val[dn.beg + e] : 0.0;
    wl[h] = mine[h] ? a.alpha * vr : 0.0;
    cwl[h] = mine[h] ? 1.0 + a.alpha * vr : 0.0;
    isP[h] = mine[h] && wl[h] > 0.0;
    isQ[h] = mine[h] && wl[h] == 0.0;
    bad |= __any(mine[h] && wl[h] < 0.0) ? 1 : 0;
    mQ[h] = __ballot(isQ[h]);
    hasQ |= mQ[h] != 0;
  }
  auto bit = [](const uint64_t (&m)[H], int e) -> bool { return (m[e >> 6] >> (e & 63)) & 1; };

  if (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[1] = __builtin_amdgcn_s_memtime();
  }
  // this lane's signals 16I + cl (padding signals read the all-zero row a.zrow)
  const f64x2* zp[NTN];
#pragma unroll
  for (int I = 0; I < NTN; ++I) {
    const int ce = __shfl(cr[I >> 2], (16 * I + cl) & 63, 64);
    zp[I] = reinterpret_cast<const f64x2*>(a.Y + (uint64_t)(uint32_t)ce * KP);
  }
  auto load_chunk = [&](int s, double (&buf)[NTN][4]) {
    const int c2 = 8 * s + 2 * kk;  // f64x2 index of column 16s + 4kk
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const f64x2 u = zp[I][c2], v = zp[I][c2 + 1];
      buf[I][0] = u[0], buf[I][1] = u[1], buf[I][2] = v[0], buf[I][3] = v[1];
    }
  };
  auto load_chunk_x = load_chunk;

  acc_t acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0.0, 0.0, 0.0, 0.0};
  double sq[NTN];  // z_eᵀ Σ_{f∈Q} z_f over this lane's columns (rows with Q signals)
#pragma unroll
  for (int I = 0; I < NTN; ++I) sq[I] = 0.0;
  constexpr int KEEP = wb64_keep<NTK, NTN>();
  double keep[KEEP > 0 ? KEEP : 1][NTN][4];
  {
    // a ring of KD + 1 chunk buffers: chunk s + KD is in flight while chunk s is consumed
    // (the loop unrolls fully, so every ring index is a compile-time constant)
    constexpr int KD = wb64_kdepth<NTN>();
    double buf[KD + 1][NTN][4];
#pragma unroll
    for (int s = 0; s < KD && s < NS; ++s) load_chunk(s, buf[s]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + KD < NS) load_chunk(s + KD, buf[(s + KD) % (KD + 1)]);
      double (&cur)[NTN][4] = buf[s % (KD + 1)];
      if (s < KEEP) {
#pragma unroll
        for (int I = 0; I < NTN; ++I)
#pragma unroll
          for (int c = 0; c < 4; ++c) keep[s < KEEP ? s : 0][I][c] = cur[I][c];
      } else if (s < KEEP + KL) {
#pragma unroll
        for (int I = 0; I < NTN; ++I)
#pragma unroll
          for (int c = 0; c < 4; ++c) kl[s - KEEP < KL ? s - KEEP : 0][4 * I + c][lane] = cur[I][c];
      }
      if (hasQ) {
        double g[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double v = 0.0;
#pragma unroll
          for (int I = 0; I < NTN; ++I)
            if (bit(mQ, 16 * I + cl)) v += cur[I][c];
          g[c] = v;
        }
        row16_sum4(g);
#pragma unroll
        for (int I = 0; I < NTN; ++I)
#pragma unroll
          for (int c = 0; c < 4; ++c) sq[I] += cur[I][c] * g[c];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int I = 0; I < NTN; ++I) {
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const int t = tile_index(I, J);
            acc[t] = M::mma(cur[I][j], cur[J][j], acc[t]);
          }
        }
      }
      // one chunk and the next chunks' loads live at a time
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  double xb = 0.0;
  double ul[NTN], cv[NTN];
  // the n×n system: one factorization for both forms (a copy per form pushed the n = 64
  // instance past three waves' registers)
  double iw[H], rhs[H];
  uint64_t mP[H];
#pragma unroll
  for (int h = 0; h < H; ++h) mP[h] = __ballot(isP[h]);
  if (!hasQ) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      iw[h] = isP[h] ? 1.0 / wl[h] : 1.0;
      rhs[h] = isP[h] ? cwl[h] * iw[h] : 0.0;
    }
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const double iwd = __shfl(iw[I >> 2], (16 * I + cl) & 63, 64);
      const int t = tile_index(I, I);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] += M::crow(lane, r) == cl ? iwd : 0.0;
    }
  } else {
    // Q signals (w = 0): u_Q = 1 moves to the right-hand side, the Q rows/columns become
    // identity
#pragma unroll
    for (int h = 0; h < H; ++h) rhs[h] = isP[h] ? cwl[h] / wl[h] : 0.0;
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      double v = sq[I];
      v += shfl_xor(v, 16);
      v += shfl_xor(v, 32);
      if (kk == 0) gq[16 * I + cl] = v;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const double kqv = lane + 64 * h < 16 * NTN ? gq[lane + 64 * h] : 0.0;
      if (isP[h]) rhs[h] -= kqv;
      iw[h] = isP[h] ? 1.0 / wl[h] : 0.0;
    }
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const double iwd = __shfl(iw[I >> 2], (16 * I + cl) & 63, 64);
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        const int f = 16 * J + cl;
        const bool pf = bit(mP, f);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 16 * I + M::crow(lane, r);
          const bool pe = bit(mP, e);
          double v = acc[t][r];
          if (pe && pf) v += (e == f) ? iwd : 0.0;
          else v = (e == f) ? 1.0 : 0.0;
          acc[t][r] = v;
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h)
    if (lane + 64 * h < 16 * NTN) S.bw[lane + 64 * h] = rhs[h];
  __syncthreads();
  if (TRACE) tr[2] = __builtin_amdgcn_s_memtime();
  row_chol<double, NTN>(acc, S, lane, bad);
  if (TRACE) tr[3] = __builtin_amdgcn_s_memtime();
  if (!hasQ) {
    double xbl = 0.0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const double ue = lane + 64 * h < 16 * NTN ? S.xs[lane + 64 * h] : 0.0;
      xbl += isP[h] ? rhs[h] * (cwl[h] - ue) : 0.0;
    }
    xb = wave_sum(xbl);
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      ul[I] = S.xs[16 * I + cl];
      cv[I] = 0.0;
    }
  } else {
#pragma unroll
    for (int I = 0; I < NTN; ++I) {
      const int e = 16 * I + cl;
      const bool pe = bit(mP, e);
      const bool qe = bit(mQ, e);
      ul[I] = pe ? S.xs[e] : (qe ? 1.0 : 0.0);
      cv[I] = __shfl(cwl[I >> 2], e & 63, 64);
    }
  }

  // x' = Zₛᵀu (and for rows with Q signals xᵀb = x'ᵀ(Zₛᵀc)), the rows gathered again
  {
    // XD chunks in flight: the Gram's accumulators are dead here, so the x' pass can hold
    // a deeper ring than the K pass (each chunk costs little compute: its loads would
    // otherwise be waited for one after the other)
    constexpr int XD = wb64_xdepth<NTN>();
    constexpr int KT = KEEP + KL;  // chunks kept on chip (registers, then LDS)
    constexpr int NG = NS - KT;    // chunks gathered again
    double buf[XD + 1][NTN][4];
#pragma unroll
    for (int q = 0; q < XD && q < NG; ++q) load_chunk_x(KT + q, buf[q]);
    double xbq = 0.0;
    auto xchunk = [&](int s, const double (&cur)[NTN][4]) {
      double sx[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = 0.0;
#pragma unroll
        for (int I = 0; I < NTN; ++I) v += cur[I][c] * ul[I];
        sx[c] = v;
      }
      // column 16s + 4kk + (cl >> 2) of x' in lanes cl = 0, 4, 8, 12 (and their neighbours)
      const double sxc = row16_sum4_split(sx, cl);
      if (hasQ) {
        double sb[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double v = 0.0;
#pragma unroll
          for (int I = 0; I < NTN; ++I) v += cur[I][c] * cv[I];
          sb[c] = v;
        }
        const double sbc = row16_sum4_split(sb, cl);
        xbq += (cl & 3) == 0 ? sxc * sbc : 0.0;
      }
      if ((cl & 3) == 0) a.X[row * KP + 16 * s + 4 * kk + (cl >> 2)] = bad ? 0.0 : sxc;
      __builtin_amdgcn_sched_barrier(0);
    };
    // the kept chunks while the first gathers are in flight, then the gathered ring
#pragma unroll
    for (int s = 0; s < KEEP; ++s) xchunk(s, keep[s]);
#pragma unroll
    for (int s = 0; s < KL; ++s) {
      double cur[NTN][4];
#pragma unroll
      for (int I = 0; I < NTN; ++I)
#pragma unroll
        for (int c = 0; c < 4; ++c) cur[I][c] = kl[s][4 * I + c][lane];
      xchunk(KEEP + s, cur);
    }
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      if (q + XD < NG) load_chunk_x(KT + q + XD, buf[(q + XD) % (XD + 1)]);
      xchunk(KT + q, buf[q % (XD + 1)]);
    }
    if (hasQ) xb = wave_sum(xbq);
  }
  double cs = 0.0;
#pragma unroll
  for (int h = 0; h < H; ++h) cs += cwl[h];
  const double csum = wave_sum(cs);
  if (lane == 0) {
    a.rowloss[row] = bad ? 0.0 : csum - xb;  // −λ‖x‖² added after unwhitening
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
    o[6] = (uint64_t)n;
    o[7] = (uint64_t)row;
  }
}

// ---------------------------------------------------------------------------------------
// Whitening / unwhitening GEMMs with the inverse Cholesky factor Linv = L⁻¹ (lower, KP×KP).
//   whiten:   Z[r] = Linv · Y[r]     (z = L⁻¹ y)            rows 0..n-1, 16 per wave
//   unwhiten: X[r] = Linvᵀ · X'[r]   (x = L⁻ᵀ x') in place, rows from `order`; also
//             rowloss[r] −= λ‖x‖².
// One wave computes QMFX_WHITEN_RG 16-row × KP blocks with NT accumulator tiles each (two: each
// L⁻¹ fragment serves two MFMAs; C3 fp64 382.9 → 381.5 ms/epoch); the zero upper
// triangle of Linv is skipped.
// ---------------------------------------------------------------------------------------
// row groups of 16 per wave in the whitening GEMMs: each L⁻¹ operand fragment is loaded once
// and used for RG groups' MFMAs
#ifndef QMFX_WHITEN_RG
#define QMFX_WHITEN_RG 2
#endif
template <typename T, int NT, bool UNWHITEN>
__global__ __launch_bounds__(256) void whiten_kernel(const T* in, T* out, const int64_t* order,
                                                     int64_t nrows, const T* __restrict__ Linv,
                                                     double* rowloss, double lambda) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NT;
  constexpr int RG = QMFX_WHITEN_RG;
  const int lane = threadIdx.x & 63;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t rw = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (16 * RG);
  if (rw >= nrows) return;
  int64_t rowa[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int64_t r = rw + 16 * g + cl;
    const int64_t ra = r < nrows ? r : nrows - 1;
    rowa[g] = UNWHITEN ? order[ra] : ra;
  }
  acc_t acc[RG][NT];
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int J = 0; J < NT; ++J) acc[g][J] = acc_t{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < KP / 4; ++s) {
    const int m = 4 * s + kk;
    T av[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) av[g] = in[rowa[g] * KP + m];
#pragma unroll
    for (int J = 0; J < NT; ++J) {
      const int j = 16 * J + cl;
      if (UNWHITEN) {
        // x_j = Σ_m x'_m Linv[m][j]: nonzero only for m ≥ j
        if (4 * s + 3 >= 16 * J) {
          const T bv = Linv[m * KP + j];
#pragma unroll
          for (int g = 0; g < RG; ++g) acc[g][J] = M::mma(av[g], bv, acc[g][J]);
        }
      } else {
        // z_j = Σ_m Linv[j][m] y_m: nonzero only for m ≤ j
        if (4 * s <= 16 * J + 15) {
          const T bv = Linv[j * KP + m];
#pragma unroll
          for (int g = 0; g < RG; ++g) acc[g][J] = M::mma(av[g], bv, acc[g][J]);
        }
      }
    }
  }
  // all reads of this wave's rows are done before any write (in-place unwhitening)
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int64_t r0 = rw + 16 * g;
    T ss[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t ro = r0 + M::crow(lane, r);
      if (ro < nrows) {
        const int64_t rowo = UNWHITEN ? order[ro] : ro;
#pragma unroll
        for (int J = 0; J < NT; ++J) {
          out[rowo * KP + 16 * J + cl] = acc[g][J][r];
          ss[r] += acc[g][J][r] * acc[g][J][r];
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
}

// The same GEMMs for KP ≤ 128 with L⁻¹ staged once per workgroup in LDS (round 6).  The
// global-operand kernel above keeps its L⁻¹ fragments in the same VMEM queue as the row
// gathers: of the ~18 loads a wave has in flight, two in seven are row bytes, so the rows
// (the kernel's HBM traffic) arrive at ~3 TB/s (C3 fp64 unwhiten: 21.6 GB in 6.7 ms, PMC).
// Here the B operand is an LDS read, every VMEM load in flight is a row load, and the grid
// is persistent (one or two 512-thread workgroups per CU, each wave striding over 32-row
// blocks), so L⁻¹ crosses the fabric once per workgroup instead of once per 32 rows.
//   LDS layout: B[m][j] (= Linv[m][j] to unwhiten, Linv[j][m] to whiten) with a row pitch of
//   KP + 16 elements (fp64: + 128 B), so the four K rows of one fragment read (lanes kk =
//   0..3) fall on two disjoint halves of the banks.
// ---------------------------------------------------------------------------------------
#ifndef QMFX_WHITEN_LDS_D
#define QMFX_WHITEN_LDS_D 4
#endif
#ifndef QMFX_WHITEN_LDS32
#define QMFX_WHITEN_LDS32 0
#endif
#ifndef QMFX_WHITEN_LDS_RG
#define QMFX_WHITEN_LDS_RG 2
#endif
template <typename T, int NT>
struct WhitenLds {
  static constexpr int KP = 16 * NT;
  // row pitch KP + 16 elements: fp64 KP + 128 B (a fragment read's four K rows of 128 B on
  // two bank halves), fp32 KP + 64 B (four 64-B rows on four bank quarters; 72 KB at k = 128,
  // two workgroups per CU)
  static constexpr int LDL = KP + 16;
  static constexpr int BYTES = KP * LDL * (int)sizeof(T);
  // fp64 only by default: at fp32 (C3) the kernel measured slower with one workgroup per CU
  // (profiles/r06/ab_whiten_lds.txt); QMFX_WHITEN_LDS32 = 1 enables the two-per-CU form
  static constexpr bool FITS =
      (sizeof(T) == 8 || QMFX_WHITEN_LDS32) && NT <= 8 && BYTES <= 150 * 1024;
  // workgroups per CU the LDS allows (at most 2: 16 waves)
  static constexpr int PER_CU = BYTES <= 75 * 1024 ? 2 : 1;
};
template <typename T, int NT, bool UNWHITEN>
__global__ __launch_bounds__(512) void whiten_lds_kernel(const T* in, T* out,
                                                         const int64_t* order, int64_t nrows,
                                                         const T* __restrict__ Linv,
                                                         double* rowloss, double lambda) {
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  using W = WhitenLds<T, NT>;
  constexpr int KP = W::KP;
  constexpr int LDL = W::LDL;
  constexpr int RG = QMFX_WHITEN_LDS_RG;
  __shared__ __attribute__((aligned(16))) T B[KP * LDL];
  for (int i = threadIdx.x; i < KP * KP; i += 512) {
    const int r = i / KP, c = i % KP;
    const T v = Linv[i];
    if (UNWHITEN)
      B[r * LDL + c] = v;
    else
      B[c * LDL + r] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const int64_t stride = (int64_t)gridDim.x * 8 * (16 * RG);
  for (int64_t rw = ((int64_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * (16 * RG); rw < nrows;
       rw += stride) {
    int64_t rowa[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const int64_t r = rw + 16 * g + cl;
      const int64_t ra = r < nrows ? r : nrows - 1;
      rowa[g] = UNWHITEN ? order[ra] : ra;
    }
    acc_t acc[RG][NT];
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int J = 0; J < NT; ++J) acc[g][J] = acc_t{0, 0, 0, 0};
    // the row values of step s + D are in flight while step s's MFMAs run (each step is its
    // own scheduling region, or the compiler hoists every step's LDS reads and spills)
    constexpr int NS = KP / 4;
    constexpr int D = QMFX_WHITEN_LDS_D < NS ? QMFX_WHITEN_LDS_D : NS;
    T ring[D][RG];
#pragma unroll
    for (int s = 0; s < D; ++s)
#pragma unroll
      for (int g = 0; g < RG; ++g) ring[s][g] = in[rowa[g] * KP + 4 * s + kk];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int m = 4 * s + kk;
      T av[RG];
#pragma unroll
      for (int g = 0; g < RG; ++g) av[g] = ring[s % D][g];
      if (s + D < NS) {
#pragma unroll
        for (int g = 0; g < RG; ++g) ring[s % D][g] = in[rowa[g] * KP + 4 * (s + D) + kk];
      }
#pragma unroll
      for (int J = 0; J < NT; ++J) {
        // unwhiten: x_j = Σ_{m ≥ j} Linv[m][j] x'_m; whiten: z_j = Σ_{m ≤ j} Linv[j][m] y_m
        const bool live = UNWHITEN ? (4 * s + 3 >= 16 * J) : (4 * s <= 16 * J + 15);
        if (live) {
          const T bv = B[m * LDL + 16 * J + cl];
#pragma unroll
          for (int g = 0; g < RG; ++g) acc[g][J] = M::mma(av[g], bv, acc[g][J]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // all reads of this block's rows are done before any write (in-place unwhitening)
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const int64_t r0 = rw + 16 * g;
      T ss[4] = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t ro = r0 + M::crow(lane, r);
        if (ro < nrows) {
          const int64_t rowo = UNWHITEN ? order[ro] : ro;
#pragma unroll
          for (int J = 0; J < NT; ++J) {
            out[rowo * KP + 16 * J + cl] = acc[g][J][r];
            ss[r] += acc[g][J][r] * acc[g][J][r];
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


#ifndef QMFX_KERNELS_ONLY
template <typename T, int NTK>
static hipError_t launch_woodbury_ntk(const SolveArgs<T>& a, int ntn, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc) return hipErrorInvalidValue;
  const dim3 b(64);
  // fp32: the streamed kernel (every bucket); fp64 k ≤ 64: the register-resident one
  if constexpr (sizeof(T) == 4) {
    {
#define QMFX_WBS(N)                                                                        \
  return launch_row_chunks(a, 64, [&](const SolveArgs<T>& c) {                             \
    hipLaunchKernelGGL((wals_woodbury_st_kernel<NTK, N>), dim3((unsigned)c.nrows), b, 0, s, c); \
  })
      switch (ntn) {
        case 1: QMFX_WBS(1);
        case 2:
          if constexpr (NTK >= 4) QMFX_WBS(2);
          return hipErrorInvalidValue;
        case 3:
          if constexpr (NTK >= 4) QMFX_WBS(3);
          return hipErrorInvalidValue;
        case 4:
          if constexpr (NTK >= 4) QMFX_WBS(4);
          return hipErrorInvalidValue;
        // n = 65..128 (two signals per lane): fp32 k = 128 and 256
        case 5:
          if constexpr (NTK == 16 || NTK == 8) QMFX_WBS(5);
          return hipErrorInvalidValue;
        case 6:
          if constexpr (NTK == 16 || NTK == 8) QMFX_WBS(6);
          return hipErrorInvalidValue;
        case 7:
          if constexpr (NTK == 16 || NTK == 8) QMFX_WBS(7);
          return hipErrorInvalidValue;
        case 8:
          if constexpr (NTK == 16 || NTK == 8) QMFX_WBS(8);
          return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
      }
#undef QMFX_WBS
    }
  } else {
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
    if constexpr (NTK >= 4) QMFX_WB(3);
    else return hipErrorInvalidValue;
  } else if (ntn == 4) {
    if constexpr (NTK >= 8) QMFX_WB(4);
    else return hipErrorInvalidValue;
#undef QMFX_WB
  } else {
    return hipErrorInvalidValue;
  }
  }
}

template <int NTK>
static hipError_t launch_woodbury_st64_ntk(const SolveArgs<double>& a, int ntn, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc) return hipErrorInvalidValue;
#define QMFX_WBS64(N)                                                                      \
  return launch_row_chunks(a, 64, [&](const SolveArgs<double>& c) {                        \
    if (c.trace)                                                                           \
      hipLaunchKernelGGL((wals_woodbury_st64_kernel<NTK, N, true>), dim3((unsigned)c.nrows), \
                         dim3(64), 0, s, c);                                               \
    else                                                                                   \
      hipLaunchKernelGGL((wals_woodbury_st64_kernel<NTK, N>), dim3((unsigned)c.nrows),     \
                         dim3(64), 0, s, c);                                               \
  })
  switch (ntn) {
    case 1: QMFX_WBS64(1);
    case 2: QMFX_WBS64(2);
    case 3:
      if constexpr (NTK >= 4) QMFX_WBS64(3);
      return hipErrorInvalidValue;
    case 4:
      if constexpr (NTK >= 4) QMFX_WBS64(4);
      return hipErrorInvalidValue;
    // n = 65..80 (two signals per lane) at k = 128 and 256 (n > 80 spills: direct)
    case 5:
      if constexpr (NTK == 8 || NTK == 16) QMFX_WBS64(5);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
#undef QMFX_WBS64
}

template <typename T, int NT>
static hipError_t launch_whiten_nt(const T* in, T* out, const int64_t* order, int64_t nrows,
                                   const T* Linv, double* rowloss, double lambda, bool unwhiten,
                                   hipStream_t s) {
  if (nrows <= 0) return hipSuccess;
  if constexpr (WhitenLds<T, NT>::FITS) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const int64_t need = (nrows + 8 * 16 * QMFX_WHITEN_LDS_RG - 1) / (8 * 16 * QMFX_WHITEN_LDS_RG);
    int64_t cap = (int64_t)cus * WhitenLds<T, NT>::PER_CU;
    // test hook (read per launch): fewer workgroups, so that every wave strides over several
    // 32-row blocks at test sizes
    if (const char* g = std::getenv("QMFX_WHITEN_GRID")) {
      const long v = std::strtol(g, nullptr, 10);
      if (v > 0 && v < cap) cap = v;
    }
    const unsigned grid = (unsigned)(need < cap ? need : cap);
    if (unwhiten)
      hipLaunchKernelGGL((whiten_lds_kernel<T, NT, true>), dim3(grid), dim3(512), 0, s, in, out,
                         order, nrows, Linv, rowloss, lambda);
    else
      hipLaunchKernelGGL((whiten_lds_kernel<T, NT, false>), dim3(grid), dim3(512), 0, s, in,
                         out, order, nrows, Linv, rowloss, lambda);
    return hipGetLastError();
  }
  const unsigned blocks = (unsigned)((nrows + 64 * QMFX_WHITEN_RG - 1) / (64 * QMFX_WHITEN_RG));
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
  // L⁻¹ column c by forward substitution on four threads (lanes 4c .. 4c + 3 of one wave):
  // thread q sums the terms mm ≡ q (mod 4), two shuffles combine them, and entry i is stored
  // by the thread that will read it again (q = i mod 4), so each thread only re-reads its own
  // writes.  One thread per column left the k = 256 launch at 6.2 ms, the column chains
  // (up to 32K dependent-address FMAs) being the whole of it.
  {
    const int c = tid >> 2, q = tid & 3;
    if (c < KP) {
      for (int i = c + 1; i < KP; ++i) {
        double sm = q == 0 ? A[i * LD + c] * dinv[c] : 0.0;
        int mm = c + 1 + ((q - (c + 1)) & 3);
        for (; mm < i; mm += 4) sm += A[i * LD + mm] * A[c * LD + mm];
        sm += __shfl_xor(sm, 1, 64);
        sm += __shfl_xor(sm, 2, 64);
        if ((i & 3) == q) A[c * LD + i] = -sm * dinv[i];
      }
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

hipError_t launch_wals_woodbury(const SolveArgs<float>& a, int nt, int ntn, hipStream_t s) {
#define CALL(N) launch_woodbury_ntk<float, N>(a, ntn, s)
  QMFX_NT_SWITCH_W(nt, CALL)
#undef CALL
}
hipError_t launch_wals_woodbury(const SolveArgs<double>& a, int nt, int ntn, hipStream_t s) {
  // k = 64 .. 128 and 256 on the streamed fp64 kernel; the register-resident one below
  switch (nt) {
    case 4: return launch_woodbury_st64_ntk<4>(a, ntn, s);
    case 5: return launch_woodbury_st64_ntk<5>(a, ntn, s);
    case 6: return launch_woodbury_st64_ntk<6>(a, ntn, s);
    case 7: return launch_woodbury_st64_ntk<7>(a, ntn, s);
    case 8: return launch_woodbury_st64_ntk<8>(a, ntn, s);
    case 16: return launch_woodbury_st64_ntk<16>(a, ntn, s);
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
  QMFX_NT_SWITCH_W(nt, CALL)
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
  QMFX_NT_SWITCH_W(nt, CALL)
#undef CALL
}
#endif  // QMFX_KERNELS_ONLY

}  // namespace qmfx
