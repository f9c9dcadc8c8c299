// Shared device helpers for the qmf MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qmfx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// MFMA 16x16x4 in the factor precision.  Operand maps (both dtypes): lane l supplies
// A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15].  Accumulator maps differ:
//   f32: lane l, reg r  ->  row 4*(l>>4) + r, col l&15
//   f64: lane l, reg r  ->  row (l>>4) + 4*r, col l&15
template <typename T>
struct Mfma;

template <>
struct Mfma<float> {
  using acc_t = f32x4;
  __device__ static __forceinline__ acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int crow(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

template <>
struct Mfma<double> {
  using acc_t = f64x4;
  __device__ static __forceinline__ acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int crow(int lane, int r) { return (lane >> 4) + (r << 2); }
};

__device__ __forceinline__ float readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

template <typename T>
__device__ __forceinline__ T shfl_xor(T v, int m) {
  return __shfl_xor(v, m, 64);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Counter-based hash (splitmix64 finaliser) for synthetic data and BPR sampling.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

}  // namespace qmfx
