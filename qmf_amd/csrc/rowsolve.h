// Helpers shared by the WALS row-solve kernels (wals.hip, wals_big.hip).
#pragma once
#include "common.h"

namespace qmfx {

__host__ __device__ constexpr int tile_index(int I, int J) { return I * (I + 1) / 2 + J; }

// Square root / reciprocal inside the factorizations.  fp32: hardware v_sqrt_f32 /
// v_rcp_f32 (1 ulp; the IEEE-exact expansions cost ~27 instructions each, on the critical
// path twice per column).  fp64: correctly rounded (the tight-parity path).
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double fast_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double fast_rcp(double x) { return 1.0 / x; }
// Pivot of a Cholesky column: l = √d and 1/l.  fp32: one v_rsq_f32 on the critical path
// (l = d·(1/√d)); fp64: correctly rounded √d and an exact division.
__device__ __forceinline__ void pivot_sqrt(float d, float& l, float& inv) {
  inv = __builtin_amdgcn_rsqf(d);
  l = d * inv;
}
__device__ __forceinline__ void pivot_sqrt(double d, double& l, double& inv) {
  l = sqrt(d);
  inv = 1.0 / l;
}

// Sum over the 16 lanes of a DPP row (lanes 16g..16g+15); every lane receives the sum.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}
template <int CTL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTL, 0xf, 0xf, false);
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
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTL, 0xf, 0xf, false));
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

}  // namespace qmfx
