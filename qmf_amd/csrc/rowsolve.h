// Helpers shared by the WALS row-solve kernels (wals.hip, wals_big.hip).
#pragma once
#include "common.h"

namespace qmfx {

__host__ __device__ constexpr int tile_index(int I, int J) { return I * (I + 1) / 2 + J; }
// the block row I of lower tile t (tile_index(I, J) = t)
__host__ __device__ constexpr int tile_row(int t) {
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  return I;
}

// Square root / reciprocal inside the factorizations.  fp32: hardware v_sqrt_f32 /
// v_rcp_f32 (1 ulp; the IEEE-exact expansions cost ~27 instructions each, on the critical
// path twice per column).  fp64: correctly rounded (the tight-parity path).
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double fast_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double fast_rcp(double x) { return 1.0 / x; }
// Pivot of a Cholesky column: l = √d and 1/l.  fp32: one v_rsq_f32 on the critical path
// (l = d·(1/√d)); fp64: below.
__device__ __forceinline__ void pivot_sqrt(float d, float& l, float& inv) {
  inv = __builtin_amdgcn_rsqf(d);
  l = d * inv;
}
// fp64 pivot: v_rsq_f64 and two coupled Newton steps (8 instructions, within an ulp or two
// of 1/√d) instead of the correctly rounded √d and division (≈25 dependent fp64 operations
// on the column loop's critical path: ≈30% of the k = 128 Cholesky).  A non-positive or
// NaN pivot still yields NaN or ∞, which the callers' (0, ∞) test flags.
__device__ __forceinline__ void pivot_sqrt(double d, double& l, double& inv) {
  const double y = __builtin_amdgcn_rsq(d);
  double g = d * y, h = 0.5 * y;
  double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  r = __builtin_fma(-g, h, 0.5);
  h = __builtin_fma(h, r, h);
  l = __builtin_fma(g, r, g);
  inv = 2.0 * h;
}

// Sum over the 16 lanes of a DPP row (lanes 16g..16g+15); every lane receives the sum.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, true));
  return v;
}
// DPP moves for the lane patterns in which every lane has a source (row_ror, row_mirror,
// row_half_mirror, quad_perm): no "old" operand, so no zero-initialising v_mov in front of
// each DPP move (update_dpp(0, …) cost one per 32-bit move: 32 per row16_sum4 at fp64)
template <int CTL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTL, 0xf, 0xf, true);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_mov_f64<0x128>(v);
  v += dpp_mov_f64<0x124>(v);
  v += dpp_mov_f64<0x122>(v);
  v += dpp_mov_f64<0x121>(v);
  return v;
}

template <int CTL>
__device__ __forceinline__ float dpp_mov_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTL, 0xf, 0xf, true));
}
// Four independent 16-lane row sums in lockstep: each DPP step reads a value written three
// instructions earlier, so no hazard padding (s_nop) separates the steps of one chain.
template <int CTL, typename T>
__device__ __forceinline__ T dpp_step(T v) {
  if constexpr (sizeof(T) == 4) return dpp_mov_f32<CTL>(v);
  else return dpp_mov_f64<CTL>(v);
}
template <typename T>
__device__ __forceinline__ void row16_sum4(T (&v)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += dpp_step<0x128>(v[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += dpp_step<0x124>(v[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += dpp_step<0x122>(v[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += dpp_step<0x121>(v[i]);
}

// The same four row sums when each lane needs only one of them: a transposing butterfly over
// the lane pairs i^8 (row_ror:8), i^7 (row_half_mirror), i^1 and i^2 (quad_perm), which span
// the 16 lanes.  Each of the first two steps keeps half of the lane's columns and adds the
// partner's copy of them, so the exchanges shrink 2 → 1 → 1 → 1 values instead of 4 per step.
// Afterwards lane 16g + i holds the row's full sum of v[i >> 2] (each sum in four lanes).
// fp64: 27 VALU instructions against 64 for row16_sum4.
template <typename T>
__device__ __forceinline__ T row16_sum4_split(const T (&v)[4], int cl) {
  const bool b3 = (cl & 8) != 0, b2 = (cl & 4) != 0;
  T k0 = b3 ? v[2] : v[0], k1 = b3 ? v[3] : v[1];
  const T s0 = b3 ? v[0] : v[2], s1 = b3 ? v[1] : v[3];
  k0 += dpp_step<0x128>(s0);
  k1 += dpp_step<0x128>(s1);
  T k = b2 ? k1 : k0;
  k += dpp_step<0x141>(b2 ? k0 : k1);
  k += dpp_step<0xB1>(k);
  k += dpp_step<0x4E>(k);
  return k;
}
// Eight row sums (v[h][c], column 4h + c), one per lane pair: lane 16g + i holds the full sum
// of column 4·b3 + 2·b2 + b0 (bits of i).  30 VALU instructions against 64 at fp32.
template <typename T>
__device__ __forceinline__ T row16_sum8_split(const T (&v)[2][4], int cl) {
  const bool b3 = (cl & 8) != 0, b2 = (cl & 4) != 0, b0 = (cl & 1) != 0;
  T k[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    k[c] = b3 ? v[1][c] : v[0][c];
    k[c] += dpp_step<0x128>(b3 ? v[0][c] : v[1][c]);
  }
  T m0 = b2 ? k[2] : k[0], m1 = b2 ? k[3] : k[1];
  m0 += dpp_step<0x141>(b2 ? k[0] : k[2]);
  m1 += dpp_step<0x141>(b2 ? k[1] : k[3]);
  T r = b0 ? m1 : m0;
  r += dpp_step<0xB1>(b0 ? m0 : m1);
  r += dpp_step<0x4E>(r);
  return r;
}
// the column row16_sum8_split leaves in lane i of a 16-lane row
__device__ __forceinline__ int row16_sum8_column(int cl) {
  return 4 * ((cl >> 3) & 1) + 2 * ((cl >> 2) & 1) + (cl & 1);
}

// ---------------------------------------------------------------------------------------
// fp32-accurate Gram on the bf16 matrix cores.  gfx950's f32-input MFMA runs at the f32
// vector rate (64 flop/clk/SIMD); v_mfma_f32_16x16x32_bf16 does 16× that.  Each fp32 value
// is split EXACTLY into three bf16 parts by truncation, x = hi + mid + lo (8 + 8 + 8
// significand bits), and a product x·y is summed from the six parts of order ≤ 2:
//   hi·hi + hi·mid + mid·hi + mid·mid + hi·lo + lo·hi
// (each part product is exact in the fp32 accumulator; the dropped mid·lo + lo·mid + lo·lo
// are ≤ 2⁻²³ relative — the size of fp32 rounding).  Six 16-cycle MFMAs per 16×16 tile and
// 32 signals replace eight 32-cycle f32 MFMAs: 2.7× fewer matrix-core cycles.
// Measured on gfx950 (tools/exp/bf16_layout.hip): Gram error 4.7e-7 of Σ|xᵢxⱼ| vs 2.5e-7
// for an fp32 FMA chain.
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float trunc_bf16(float x) {
  return __uint_as_float(__float_as_uint(x) & 0xffff0000u);
}
// upper halves of (a, b) packed as two bf16: a in the low half, b in the high half
__device__ __forceinline__ unsigned pack_hi16(float a, float b) {
  return (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xffff0000u);
}
struct Split3 {
  u32x4 h, m, l;
};
// 8 values (x[0..7]) → three bf16x8 operands with x = h + m + l exactly
__device__ __forceinline__ void split3(const float (&x)[8], Split3& s) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x0 = x[2 * p], x1 = x[2 * p + 1];
    const float r0 = x0 - trunc_bf16(x0), r1 = x1 - trunc_bf16(x1);
    const float l0 = r0 - trunc_bf16(r0), l1 = r1 - trunc_bf16(r1);
    s.h[p] = pack_hi16(x0, x1);
    s.m[p] = pack_hi16(r0, r1);
    s.l[p] = pack_hi16(l0, l1);
  }
}
__device__ __forceinline__ f32x4 mma_bf16(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// acc += Xᵢ Xⱼᵀ to fp32 accuracy from the splits of the two row blocks
__device__ __forceinline__ f32x4 mma_split6(const Split3& a, const Split3& b, f32x4 c) {
  c = mma_bf16(a.h, b.h, c);
  c = mma_bf16(a.h, b.m, c);
  c = mma_bf16(a.m, b.h, c);
  c = mma_bf16(a.m, b.m, c);
  c = mma_bf16(a.h, b.l, c);
  c = mma_bf16(a.l, b.h, c);
  return c;
}

}  // namespace qmfx
