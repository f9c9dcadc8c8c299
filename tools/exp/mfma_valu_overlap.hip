// Micro-benchmark: does one wave's (or a SIMD's) f64 VALU work overlap its f64 MFMAs?
// Per iteration: M independent v_mfma_f64_16x16x4 (8 accumulators) and V independent
// v_fma_f64 (8 chains, not feeding the MFMAs), in one wave; and the same with v_fma_f32 or
// v_pk_fma_f32.  If the FP64 VALU shares the matrix core's datapath the mixed time is the sum
// of the parts, else their max.  Prints cycles per iteration (s_memtime), one wave per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/exp/mfma_valu_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int M, int V, int KIND>  // KIND 0: v_fma_f64, 1: v_fma_f32, 2: v_pk_fma_f32
__global__ __launch_bounds__(64, 1) void mix(const double* in, double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  f64x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f64x4{0, 0, 0, 0};
  const double a = in[lane], b = in[lane + 64];
  double d[8];
  float f[8];
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 p[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    d[j] = in[lane + 128 + j];
    f[j] = (float)d[j];
    p[j] = f32x2{f[j], f[j]};
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < (M > V / 8 ? M : V / 8); ++s) {
      if (s < M) acc[s & 7] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s & 7], 0, 0, 0);
      if (s < V / 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (KIND == 0) d[j] = __builtin_fma(d[j], 0.999999, 1e-9);
          else if constexpr (KIND == 1) f[j] = __builtin_fmaf(f[j], 0.9999f, 1e-7f);
          else p[j] = __builtin_elementwise_fma(p[j], f32x2{0.9999f, 0.9999f}, f32x2{1e-7f, 1e-7f});
        }
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
#pragma unroll
  for (int j = 0; j < 8; ++j) s += d[j] + f[j] + p[j][0] + p[j][1];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int M, int V, int KIND>
void run(const char* name) {
  double *din, *dout;
  long long* dc;
  const int blocks = 1024;
  hipMalloc(&din, 1024 * sizeof(double));
  hipMalloc(&dout, blocks * 64 * sizeof(double));
  hipMalloc(&dc, blocks * sizeof(long long));
  hipMemset(din, 0, 1024 * sizeof(double));
  const int iters = 2000;
  hipLaunchKernelGGL((mix<M, V, KIND>), dim3(blocks), dim3(64), 0, 0, din, dout, dc, 10);
  hipLaunchKernelGGL((mix<M, V, KIND>), dim3(blocks), dim3(64), 0, 0, din, dout, dc, iters);
  hipDeviceSynchronize();
  static long long c[1024];
  hipMemcpy(c, dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)c[i];
  avg /= blocks;
  std::printf("%-34s M=%2d V=%3d: %8.1f cyc/iter\n", name, M, V, avg / iters);
  hipFree(din);
  hipFree(dout);
  hipFree(dc);
}

int main() {
  run<8, 0, 0>("f64 MFMA only");
  run<0, 64, 0>("v_fma_f64 only");
  run<8, 64, 0>("f64 MFMA + v_fma_f64");
  run<0, 64, 1>("v_fma_f32 only");
  run<8, 64, 1>("f64 MFMA + v_fma_f32");
  run<0, 64, 2>("v_pk_fma_f32 only");
  run<8, 64, 2>("f64 MFMA + v_pk_fma_f32");
  run<8, 32, 0>("f64 MFMA + v_fma_f64 (half)");
  return 0;
}
