// Direct row solve for fp64 k = 80..128 with TWO waves per row (gfx950).
//
// Reference path: WALSEngine::updateFactorsForOne (qmf/wals/WALSEngine.cpp:266-310) and
// linearSymmetricSolve → dsysv_ (qmf/Matrix.cpp:81-96), as the one-wave direct kernel
// (direct.h), which holds all NT(NT+1)/2 accumulator tiles of a row in one wave: 288
// registers at k = 128, so one wave per SIMD, nothing to cover the step boundary of its Gram
// loop (the next rows' shuffle and its LDS round trip, the loads' issue, the moves of the
// landed rows: ≈550 of ≈2900 cycles per 36-MFMA step, profiles/r04) nor its 83K-cycle
// Cholesky.  Here the tiles are split over the two waves of a 128-thread workgroup by block
// row (wave 0: rows I with I mod 4 ∈ {0, 3}; wave 1: the others; 18 tiles each at NT = 8), so
// a wave needs ≈144 accumulator registers and two workgroups share each SIMD: one row's step
// boundary and Cholesky run beside another row's MFMAs.
//
//   Gram: both waves walk the row's signals (4 per step, one gathered row per lane group) and
//         accumulate their own tiles; wave 0 also forms b = Σ c·y and Σc.  The second wave's
//         gathers of the same rows hit L2.
//   Cholesky, right-looking over 16-column panels: the owners write panel p's tiles to LDS,
//         wave 0 factors the panel (chol.h's column loop, rows in 1 or 2 slots per lane) with
//         the forward solve, both waves read their L tiles back and apply the rank-16
//         trailing update to their own tiles (4 MFMAs per tile, operands from the LDS panel).
//   Backward solve by 16-blocks: both waves add their tiles' part of Lᵀx in LDS, wave 0
//         finishes each block with the transposed diagonal block (chol.h's scheme).
// Results contract of the direct kernel: status[row] = 1 and x = 0 on a non-positive pivot.
#include <utility>

#include "chol.h"
#include "common.h"
#include "kernels.h"
#include "rowsolve.h"

#ifndef QMFX_EXP_GRAM_MASK
#define QMFX_EXP_GRAM_MASK 0xffffffffu  // timing experiments only: fold the gathers onto few rows
#endif

namespace qmfx {

// owner wave of block row I
__host__ __device__ constexpr int d2_owner(int I) { return ((I & 3) == 0 || (I & 3) == 3) ? 0 : 1; }

template <int NT, int W>
struct D2Tiles {
  struct L {
    int n;
    int I[64];
    int J[64];
  };
  static constexpr L make() {
    L l{};
    for (int I = 0; I < NT; ++I)
      if (d2_owner(I) == W)
        for (int J = 0; J <= I; ++J) {
          l.I[l.n] = I;
          l.J[l.n] = J;
          ++l.n;
        }
    return l;
  }
  static constexpr L list = make();
  static constexpr int n = list.n;
};
template <int NT>
constexpr int d2_max_tiles() {
  return D2Tiles<NT, 0>::n > D2Tiles<NT, 1>::n ? D2Tiles<NT, 0>::n : D2Tiles<NT, 1>::n;
}

template <int NT>
struct D2Shared {
  static constexpr int KP = 16 * NT;
  static constexpr int PLD = CholLd<double>::PLD;
  double panel[KP * PLD];       // panel p's rows (16(I−p) + r) · PLD + c
  double Lt[NT * 16 * PLD];     // diagonal L blocks, transposed and column-scaled
  double bw[KP];                // rhs, then the forward-solved y
  double xs[KP];                // solution
  double invd[KP];              // 1 / L[c][c]
  double borig[KP];             // b (for the row loss)
  double part[2][16];           // backward solve: each wave's part of Lᵀx
  double red[2];                // loss partials
  int bad;
  unsigned hw1;                 // QMFX_TRACE: wave 1's HW_ID
};

// Panel p of the right-looking Cholesky on ONE wave (chol.h's chol_solve panel, with the
// forward solve; rows lane + 64 s of the panel, s < SLOTS): L into S.panel, 1/L[c][c] and y
// into S.invd / S.bw, the diagonal block transposed and scaled into S.Lt.
template <int NT, int P>
__device__ __forceinline__ void d2_panel(D2Shared<NT>& S, int lane, int& bad) {
  constexpr int KP = 16 * NT;
  constexpr int R = KP - 16 * P;
  constexpr int SLOTS = (R + 63) / 64;
  constexpr int PLD = D2Shared<NT>::PLD;
  double pa[SLOTS][16];
  double pb[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int q = lane + 64 * s;
    const int qq = q < R ? q : 0;
    lds_row_load(&S.panel[qq * PLD], pa[s]);
    pb[s] = S.bw[16 * P + qq];
  }
  double invv = 0.0, yv = 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double am[16];
#pragma unroll
    for (int m = 1; m < 16; ++m)
      if (m > c) am[m] = readlane(pa[0][c], m);
    const double d = readlane(pa[0][c], c);
    const double bc = readlane(pb[0], c);
    double ljj, inv;
    pivot_sqrt(d, ljj, inv);
    (void)ljj;
    const bool me = lane == c;
    invv = me ? inv : invv;
    yv = me ? bc * inv : yv;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const double lq = pa[s][c] * inv;
      const double lqs = lq * inv;
      pa[s][c] = lq;
      pb[s] -= lqs * bc;
#pragma unroll
      for (int m = 1; m < 16; ++m)
        if (m > c) pa[s][m] -= lqs * am[m];
    }
    // the second slot's updates stay in this column's window (chol.h: deferred, they spill)
#pragma unroll
    for (int s = 1; s < SLOTS; ++s) {
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m >= c) asm volatile("" : "+v"(pa[s][m]));
      asm volatile("" : "+v"(pb[s]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  bad |= __any(lane < 16 && !(invv > 0.0 && invv < __builtin_huge_val())) ? 1 : 0;
  if (lane < 16) {
    S.invd[16 * P + lane] = invv;
    S.bw[16 * P + lane] = yv;
  }
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int q = lane + 64 * s;
    if (q < R) lds_row_store(&S.panel[q * PLD], pa[s]);
    if (q >= 16 && q < R) S.bw[16 * P + q] = pb[s];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = lane + 64 * it;
    const int r = idx >> 4, c = idx & 15;
    S.Lt[(P * 16 + c) * PLD + r] = c < r ? S.panel[r * PLD + c] * S.invd[16 * P + c] : 0.0;
  }
}

template <int NT, int W>
__device__ __forceinline__ void d2_row(const SolveArgs<double>& a, D2Shared<NT>& S, int lane) {
  using M = Mfma<double>;
  using acc_t = f64x4;
  using TL = D2Tiles<NT, W>;
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  constexpr int TW = TL::n;
  constexpr int PLD = D2Shared<NT>::PLD;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  const RowDesc d = a.desc[a.row_begin + blockIdx.x];
  const int64_t row = d.row;
  const int64_t beg = d.beg;
  const int64_t end = beg + d.n;
  // phase stamps (QMFX_TRACE, wave 0): start, G image loaded, Gram done, Cholesky done, end
  uint64_t tr[5] = {0, 0, 0, 0, 0};
  if (W == 0 && a.trace) tr[0] = __builtin_amdgcn_s_memtime();

  // this wave's tiles from the image of G + λI (gimg_kernel: [tile][lane][4])
  acc_t acc[TW];
  {
    constexpr int AB = (int)sizeof(acc_t);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.Gimg, (short)0, NTT * 64 * AB, 0x00020000);
#pragma unroll
    for (int s = 0; s < TW; ++s) {
      const int t = tile_index(TL::list.I[s], TL::list.J[s]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * AB + 16 * h, t * 64 * AB, 0);
        acc[s][2 * h] = __builtin_bit_cast(double, (unsigned long long)v[0] | ((unsigned long long)v[1] << 32));
        acc[s][2 * h + 1] = __builtin_bit_cast(double, (unsigned long long)v[2] | ((unsigned long long)v[3] << 32));
      }
    }
  }

  if (W == 0 && a.trace) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[1] = __builtin_amdgcn_s_memtime();
  }
  // ---- Gram: A += Σ w y yᵀ (this wave's tiles); wave 0: b = Σ c y, Σc --------------------
  double bpart[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) bpart[q] = 0.0;
  double csum = 0.0;
  // signals past the row's end gather the all-zero row a.zrow with v = 0 (no selects)
  for (int64_t base = beg; base < end; base += 64) {
    const int nst = (int)(end - base < 64 ? end - base : 64);
    const int cr = lane < nst ? (int)(a.col[base + lane] & QMFX_EXP_GRAM_MASK) : a.zrow;
    const double vr = lane < nst ? a.val[base + lane] : 0.0;
    bool valid = kk < nst;
    double v = __shfl(vr, kk, 64);
    double yn[NT];
    {
      const double* yrow = a.Y + (uint64_t)(uint32_t)__shfl(cr, kk, 64) * KP + cl;
#pragma unroll
      for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
    }
    for (int s = 0; 4 * s < nst; ++s) {
      double yv[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) yv[q] = yn[q];
      const double w = a.alpha * v;
      const double cw = valid ? 1.0 + w : 0.0;
      const int jn = 4 * (s + 1) + kk;
      const bool vn = jn < nst;
      if (4 * (s + 1) < nst) {
        const int cn = __shfl(cr, jn < 64 ? jn : 63, 64);
        v = __shfl(vr, jn < 64 ? jn : 63, 64);
        const double* yrow = a.Y + (uint64_t)(uint32_t)cn * KP + cl;
#pragma unroll
        for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
      }
      valid = vn;
      if constexpr (W == 0) {
#pragma unroll
        for (int q = 0; q < NT; ++q) bpart[q] += cw * yv[q];
        csum += cw;
      }
      double wy[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) wy[q] = w * yv[q];
#pragma unroll
      for (int t = 0; t < TW; ++t) acc[t] = M::mma(yv[TL::list.I[t]], wy[TL::list.J[t]], acc[t]);
    }
  }
  if constexpr (W == 0) {
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      bpart[q] += shfl_xor(bpart[q], 16);
      bpart[q] += shfl_xor(bpart[q], 32);
      if (kk == 0) {
        S.borig[16 * q + cl] = bpart[q];
        S.bw[16 * q + cl] = bpart[q];
      }
    }
    csum = wave_sum(cl == 0 ? csum : 0.0);  // each k-slot row counted once
  }
  int bad = 0;
  if (W == 0 && a.trace) tr[2] = __builtin_amdgcn_s_memtime();

  // ---- Cholesky with the forward solve --------------------------------------------------
  [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
    auto panel = [&](auto pc) {
      constexpr int P = decltype(pc)::value;
      // owners stage panel P's tiles (I, P), I ≥ P
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        if constexpr (true) {
          const int I = TL::list.I[t], J = TL::list.J[t];
          if (J == P) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              S.panel[(16 * (I - P) + M::crow(lane, r)) * PLD + cl] = acc[t][r];
          }
        }
      }
      __syncthreads();
      if constexpr (W == 0) d2_panel<NT, P>(S, lane, bad);
      __syncthreads();
      // L tiles back, then the rank-16 trailing update of this wave's tiles (I, J), J > P
      double fr[NT][4];
#pragma unroll
      for (int I = P + 1; I < NT; ++I) {
#pragma unroll
        for (int q = 0; q < 4; ++q) fr[I][q] = S.panel[(16 * (I - P) + cl) * PLD + 4 * q + kk];
      }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int I = TL::list.I[t], J = TL::list.J[t];
        if (J == P && I > P) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][r] = S.panel[(16 * (I - P) + M::crow(lane, r)) * PLD + cl];
        }
        if (J > P) {
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[t] = M::mma(-fr[I][q], fr[J][q], acc[t]);
        }
      }
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
    };
    (panel(std::integral_constant<int, Ps>{}), ...);
  }(std::make_integer_sequence<int, NT>{});

  if (W == 0 && a.trace) tr[3] = __builtin_amdgcn_s_memtime();
  // ---- backward solve Lᵀ x = y by 16-blocks from the bottom ----------------------------
#pragma unroll
  for (int I = NT - 1; I >= 0; --I) {
    double part = 0.0;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      if (TL::list.J[t] == I && TL::list.I[t] > I) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part += acc[t][r] * S.xs[16 * TL::list.I[t] + M::crow(lane, r)];
      }
    }
    part += shfl_xor(part, 16);
    part += shfl_xor(part, 32);
    if (kk == 0) S.part[W][cl] = part;
    __syncthreads();
    if constexpr (W == 0) {
      double vm = (S.bw[16 * I + cl] - S.part[0][cl] - S.part[1][cl]) * S.invd[16 * I + cl];
      double lt[16];
      lds_row_load(&S.Lt[(16 * I + cl) * PLD], lt);
#pragma unroll
      for (int c = 15; c >= 0; --c) vm -= lt[c] * readlane(vm, c);
      if (lane < 16) S.xs[16 * I + lane] = vm;
    }
    __syncthreads();
  }
  if constexpr (W == 0) {
    if (lane == 0) S.bad = bad;
  }
  __syncthreads();

  // ---- output: x, row loss = Σc − xᵀb − λ‖x‖² ---------------------------------------------
  const int bad_all = S.bad;
  const int j = lane + 64 * W;
  double xb = 0.0, xx = 0.0;
  for (int jj = j; jj < KP; jj += 128) {
    const double xj = S.xs[jj];
    a.X[row * KP + jj] = bad_all ? 0.0 : xj;
    xb += xj * S.borig[jj];
    xx += xj * xj;
  }
  const double contrib = wave_sum(xb + a.lambda * xx);
  if (lane == 0) S.red[W] = contrib;
  if (W == 1 && a.trace && lane == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    S.hw1 = hw;
  }
  __syncthreads();
  if constexpr (W == 0) {
    if (lane == 0) {
      a.rowloss[row] = bad_all ? 0.0 : csum - (S.red[0] + S.red[1]);
      if (bad_all && a.status) a.status[row] = 1;
      if (a.trace) {
        tr[4] = __builtin_amdgcn_s_memtime();
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t* o = a.trace + 8 * (a.row_begin + blockIdx.x);
#pragma unroll
        for (int j = 0; j < 5; ++j) o[j] = tr[j];
        // wave 1's HW_ID (its SIMD) in bits 40..55
        o[5] = hw | ((uint64_t)xcc << 32) | ((uint64_t)(S.hw1 & 0xffff) << 40);
        o[6] = (uint64_t)d.n;
        o[7] = (uint64_t)row;
      }
    }
  }
}

template <int NT>
__global__ __launch_bounds__(128, 2) void wals_direct2_kernel(SolveArgs<double> a) {
  __shared__ __attribute__((aligned(16))) D2Shared<NT> S;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  if (wv == 0)
    d2_row<NT, 0>(a, S, lane);
  else
    d2_row<NT, 1>(a, S, lane);
}

#ifndef QMFX_KERNELS_ONLY
template <int NT>
static hipError_t launch_direct2_nt(const SolveArgs<double>& a, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc || !a.Gimg) return hipErrorInvalidValue;
  return launch_row_chunks(a, 128, [&](const SolveArgs<double>& c) {
    hipLaunchKernelGGL((wals_direct2_kernel<NT>), dim3((unsigned)c.nrows), dim3(128), 0, s, c);
  });
}
hipError_t launch_wals_direct2(const SolveArgs<double>& a, int nt, hipStream_t s) {
  switch (nt) {
    case 5: return launch_direct2_nt<5>(a, s);
    case 6: return launch_direct2_nt<6>(a, s);
    case 7: return launch_direct2_nt<7>(a, s);
    case 8: return launch_direct2_nt<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}
#endif  // QMFX_KERNELS_ONLY

}  // namespace qmfx
