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
//
// This file: YᵀY, the G + λI tile image of the direct kernel, the fixed-order loss sum and
// the MFMA layout self-test.  The direct row kernel is csrc/direct.h (instantiated by
// wals_direct_f32.hip / wals_direct_f64.hip / wals_heavy.hip), the whitened kernels
// woodbury.hip, the multi-wave k > 128 kernels wals_big.hip.
#include "direct.h"

namespace qmfx {

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
static hipError_t launch_gimg_nt(const T* G, int k, double lambda, T* img, hipStream_t s) {
  constexpr int NTT = NT * (NT + 1) / 2;
  hipLaunchKernelGGL((gimg_kernel<T, NT>), dim3(NTT), dim3(256), 0, s, G, k, lambda, img);
  return hipGetLastError();
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
