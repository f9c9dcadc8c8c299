// Micro-benchmark: f64 16x16x4 MFMA issue rate in the direct Gram's shape — 36 lower-tile
// accumulators, per 4-signal step A = y[I] (8 registers), B = w·y[J] (8 registers), one wave
// per SIMD (512 registers) or 18 tiles per wave at two waves per SIMD.  Prints cycles per
// MFMA per wave (s_memtime) and the chip's f64 MFMA TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 [-mllvm -amdgpu-mfma-vgpr-form] tools/exp/mfma_f64_gram.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NT, int WPS, int VALU>
__global__ __launch_bounds__(64, WPS) void gram(const double* in, double* out, long long* cyc, int steps) {
  constexpr int NTT = NT * (NT + 1) / 2;
  const int lane = threadIdx.x;
  f64x4 acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = f64x4{0, 0, 0, 0};
  double y[NT], wy[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    y[q] = in[lane + 64 * q];
    wy[q] = in[lane + 64 * q + 512];
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
        acc[I * (I + 1) / 2 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(y[I], wy[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
    if constexpr (VALU) {
      // the step boundary's VALU: next rows' w·y and the rhs
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        wy[q] = wy[q] * 1.0000001;
        y[q] = __builtin_fma(y[q], 0.9999999, 1e-30);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double sum = 0;
#pragma unroll
  for (int t = 0; t < NTT; ++t) sum += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 64 + lane] = sum;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NT, int WPS, int VALU>
void run(const char* name) {
  constexpr int NTT = NT * (NT + 1) / 2;
  double *din, *dout;
  long long* dc;
  const int blocks = 1024 * WPS;
  hipMalloc(&din, 2048 * sizeof(double));
  hipMalloc(&dout, blocks * 64 * sizeof(double));
  hipMalloc(&dc, blocks * sizeof(long long));
  hipMemset(din, 0, 2048 * sizeof(double));
  const int steps = 400;
  hipLaunchKernelGGL((gram<NT, WPS, VALU>), dim3(blocks), dim3(64), 0, 0, din, dout, dc, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((gram<NT, WPS, VALU>), dim3(blocks), dim3(64), 0, 0, din, dout, dc, steps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  static long long c[8192];
  hipMemcpy(c, dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)c[i];
  avg /= blocks;
  const double n = (double)steps * NTT;
  std::printf("%-26s tiles %2d waves/SIMD %d: %6.1f cyc/MFMA per wave, %5.1f TF/s\n", name, NTT, WPS,
              avg / n, n * 2048.0 * blocks / (ms * 1e-3) / 1e12);
}

int main() {
  run<8, 1, 0>("gram k=128 no VALU");
  run<8, 1, 1>("gram k=128 + step VALU");
  run<6, 1, 0>("gram k=96 no VALU");
  run<6, 2, 0>("gram k=96 no VALU");
  run<5, 2, 0>("gram k=80 no VALU");
  run<4, 2, 0>("gram k=64 no VALU");
  run<4, 4, 0>("gram k=64 no VALU");
  return 0;
}
