// Micro-benchmark for the whitened fp64 class's next step: two waves per SIMD
// sharing a fixed amount of work per "row" — 16 f64 MFMAs and 224 f64 VALU FMAs — either
// each wave doing its own rows as an MFMA phase then a VALU phase (ALTERNATE, today's
// kernel), or one wave doing every row's MFMAs and its neighbour every row's VALU (SPECIAL,
// wave specialisation).  2048 one-wave workgroups, blocks i and i + grid/2 share a SIMD.
// Prints the SIMD's cycles per row (the slower wave's time over the rows both finished).
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/exp/wave_specialize.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma_phase(f64x4 (&acc)[8], double a, double b, int n8) {
  for (int i = 0; i < n8; ++i)
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s], 0, 0, 0);
}
__device__ __forceinline__ void valu_phase(double (&d)[8], int n112) {
  for (int i = 0; i < n112; ++i)
#pragma unroll
    for (int s = 0; s < 14; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = __builtin_fma(d[j], 0.999999, 1e-9);
}

template <bool SPECIAL>
__global__ __launch_bounds__(64, 2) void rows(const double* in, double* out, long long* rec, int nrows) {
  const int lane = threadIdx.x;
  const int role = (int)(2 * blockIdx.x >= gridDim.x);
  f64x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f64x4{0, 0, 0, 0};
  const double a = in[lane], b = in[lane + 64];
  double d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = in[lane + 128 + j];
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (SPECIAL) {
    // the pair's 2·nrows rows: one wave all MFMA phases, the other all VALU phases
    if (role == 0) mfma_phase(acc, a, b, 2 * 2 * nrows);
    else valu_phase(d, 2 * 2 * nrows);
  } else {
    for (int r = 0; r < nrows; ++r) {
      mfma_phase(acc, a, b, 2);
      valu_phase(d, 2);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
#pragma unroll
  for (int j = 0; j < 8; ++j) s += d[j];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    rec[2 * blockIdx.x] = t1 - t0;
    rec[2 * blockIdx.x + 1] = ((long long)xcc << 32) | (hw & 0xfff0);
  }
}

template <bool SPECIAL>
void run(const char* name) {
  const int blocks = 2048, nrows = 200;
  double *din, *dout;
  long long* dr;
  hipMalloc(&din, 1024 * sizeof(double));
  hipMalloc(&dout, blocks * 64 * sizeof(double));
  hipMalloc(&dr, 2 * blocks * sizeof(long long));
  hipMemset(din, 0, 1024 * sizeof(double));
  hipLaunchKernelGGL((rows<SPECIAL>), dim3(blocks), dim3(64), 0, 0, din, dout, dr, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((rows<SPECIAL>), dim3(blocks), dim3(64), 0, 0, din, dout, dr, nrows);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> r(2 * blocks);
  hipMemcpy(r.data(), dr, r.size() * sizeof(long long), hipMemcpyDeviceToHost);
  std::map<long long, long long> simd_max;  // the slower wave of each SIMD
  for (int i = 0; i < blocks; ++i) {
    long long& m = simd_max[r[2 * i + 1]];
    if (r[2 * i] > m) m = r[2 * i];
  }
  double avg = 0;
  for (auto& kv : simd_max) avg += (double)kv.second;
  avg /= simd_max.size();
  // rows per SIMD: two waves × nrows each
  std::printf("%-12s SIMDs %4zu: %8.1f SIMD cycles per row, kernel %.3f ms\n", name, simd_max.size(),
              avg / (2.0 * nrows), ms);
  hipFree(din);
  hipFree(dout);
  hipFree(dr);
}

int main() {
  run<false>("alternate");
  run<true>("specialised");
  run<false>("alternate");
  run<true>("specialised");
  return 0;
}
