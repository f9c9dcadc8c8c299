// Micro-benchmark: two waves on one SIMD, one issuing f64 MFMAs, the other f64 VALU FMAs
// (the whitened kernel's situation: one row in its K pass, the other in its factorization).
// 2048 one-wave workgroups (two per SIMD); wave role by block half (blocks i and i + grid/2
// share a SIMD); each wave records its HW_ID and its cycles (s_memtime).  The host groups waves by SIMD and reports, for SIMDs
// holding one wave of each role, each role's cycles per iteration against SIMDs holding two
// waves of the same role and against one wave alone.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/exp/mfma_valu_2wave.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int ROLES>  // 0: every wave MFMA, 1: every wave VALU, 2: by block half
__global__ __launch_bounds__(64, 2) void two(const double* in, double* out, long long* rec, int iters) {
  const int lane = threadIdx.x;
  const int role = ROLES == 2 ? (int)(2 * blockIdx.x >= gridDim.x) : ROLES;
  f64x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f64x4{0, 0, 0, 0};
  const double a = in[lane], b = in[lane + 64];
  double d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = in[lane + 128 + j];
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (role == 0) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int s = 0; s < 8; ++s) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s], 0, 0, 0);
  } else {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int s = 0; s < 14; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = __builtin_fma(d[j], 0.999999, 1e-9);
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
    rec[3 * blockIdx.x] = t1 - t0;
    rec[3 * blockIdx.x + 1] = ((long long)xcc << 32) | (hw & 0xfff0);  // drop wave slot bits
    rec[3 * blockIdx.x + 2] = role;
  }
}

template <int ROLES>
void run(const char* name, int blocks) {
  double *din, *dout;
  long long* dr;
  hipMalloc(&din, 1024 * sizeof(double));
  hipMalloc(&dout, blocks * 64 * sizeof(double));
  hipMalloc(&dr, 3 * blocks * sizeof(long long));
  hipMemset(din, 0, 1024 * sizeof(double));
  const int iters = 2000;
  hipLaunchKernelGGL((two<ROLES>), dim3(blocks), dim3(64), 0, 0, din, dout, dr, 10);
  hipLaunchKernelGGL((two<ROLES>), dim3(blocks), dim3(64), 0, 0, din, dout, dr, iters);
  hipDeviceSynchronize();
  std::vector<long long> r(3 * blocks);
  hipMemcpy(r.data(), dr, r.size() * sizeof(long long), hipMemcpyDeviceToHost);
  // per SIMD key: the roles and cycles of its waves
  std::map<long long, std::vector<int>> bysimd;
  for (int i = 0; i < blocks; ++i) bysimd[r[3 * i + 1]].push_back(i);
  double sum[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // [pairing: 0 alone, 1 same role, 2 mixed][role]
  int cnt[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  for (auto& kv : bysimd) {
    const auto& w = kv.second;
    for (int i : w) {
      const int role = (int)r[3 * i + 2];
      int pairing = 0;
      if (w.size() >= 2) {
        bool mixed = false;
        for (int j : w)
          if (j != i && r[3 * j + 2] != role) mixed = true;
        pairing = mixed ? 2 : 1;
      }
      sum[pairing][role] += (double)r[3 * i];
      cnt[pairing][role]++;
    }
  }
  const char* pn[3] = {"alone", "same-role pair", "mixed pair"};
  for (int p = 0; p < 3; ++p)
    for (int role = 0; role < 2; ++role)
      if (cnt[p][role])
        std::printf("%-20s %-15s %s waves %5d: %8.1f cyc/iter\n", name, pn[p], role ? "VALU" : "MFMA",
                    cnt[p][role], sum[p][role] / cnt[p][role] / iters);
  hipFree(din);
  hipFree(dout);
  hipFree(dr);
}

int main() {
  run<0>("all MFMA", 2048);
  run<1>("all VALU", 2048);
  run<2>("half/half", 2048);
  run<0>("all MFMA, 1/SIMD", 1024);
  run<1>("all VALU, 1/SIMD", 1024);
  return 0;
}
