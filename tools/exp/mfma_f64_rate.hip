// Micro-benchmark: cycles per v_mfma_f64_16x16x4_f64 on one wave per SIMD, with NV
// independent fp64 VALU FMAs issued per MFMA (the direct kernel's Gram issues ≈1-2).
// Build: hipcc --offload-arch=gfx950 -O3 tools/exp/mfma_f64_rate.hip -o /tmp/mfma_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC, int NV, int WPS = 1>
__global__ __launch_bounds__(64, WPS) void bench(const double* in, double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[lane + 64];
  f64x4 acc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) acc[t] = f64x4{0, 0, 0, 0};
  double v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = in[lane + 128 + j];
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < NACC; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = __builtin_fma(v[j], a, b);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int t = 0; t < NACC; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC, int NV, int WPS = 1>
void run(const double* din, double* dout, long long* dcyc) {
  const int iters = 2000, blocks = 1024 * WPS;
  hipLaunchKernelGGL((bench<NACC, NV, WPS>), dim3(blocks), dim3(64), 0, 0, din, dout, dcyc, 10);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((bench<NACC, NV, WPS>), dim3(blocks), dim3(64), 0, 0, din, dout, dcyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  static long long c[4096];
  hipMemcpy(c, dcyc, sizeof(c), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)c[i];
  avg /= blocks;
  const double n = (double)iters * NACC;
  printf("acc %2d valu/mfma %d waves/SIMD %d: %.1f cyc/mfma per wave (s_memtime), %.1f TF/s f64 MFMA (wall, %d waves)\n",
         NACC, NV, WPS, avg / n, n * 2048.0 * blocks / (ms * 1e-3) / 1e12, blocks);
}

int main() {
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, 256 * sizeof(double));
  hipMalloc(&dout, 4096 * 64 * sizeof(double));
  hipMalloc(&dcyc, 4096 * sizeof(long long));
  double h[256];
  for (int i = 0; i < 256; ++i) h[i] = 1.0 + 1e-3 * i;
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  run<8, 0>(din, dout, dcyc);
  run<36, 0>(din, dout, dcyc);
  run<36, 1>(din, dout, dcyc);
  run<36, 2>(din, dout, dcyc);
  run<36, 4>(din, dout, dcyc);
  run<36, 8>(din, dout, dcyc);
  run<18, 0, 2>(din, dout, dcyc);
  run<18, 1, 2>(din, dout, dcyc);
  run<18, 2, 2>(din, dout, dcyc);
  run<10, 0, 2>(din, dout, dcyc);
  run<10, 0, 4>(din, dout, dcyc);
  return 0;
}
