// Micro-benchmark: issue cost (cycles per instruction, s_memtime) of the instructions the
// row kernels' factorizations are made of, in long independent streams, at 1 and 2 waves
// per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 tools/exp/issue_cost.hip -o /tmp/ic
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(x) x x x x x x x x x x x x x x x x
template <int OP, int W>
__global__ __launch_bounds__(64, W) void ic(double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  double a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3, a4 = lane + 4, a5 = lane + 5,
         a6 = lane + 6, a7 = lane + 7, m = 1.0000001, s = 0.5;
  float f0 = lane, f1 = lane + 1, f2 = lane + 2, f3 = lane + 3;
  int i0 = lane, i1 = lane * 3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) {  // v_fma_f64, 8 independent chains
      REP16(asm volatile("v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %3, %1, %2, %3\n v_fma_f64 %4, %1, %2, %4\n v_fma_f64 %5, %1, %2, %5\n v_fma_f64 %6, %1, %2, %6\n v_fma_f64 %7, %1, %2, %7\n v_fma_f64 %8, %1, %2, %8\n v_fma_f64 %9, %1, %2, %9"
                         : "+v"(a0), "+v"(m), "+v"(s), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (OP == 1) {  // v_readlane_b32 (8 per asm)
      int r;
      REP16(asm volatile("v_readlane_b32 s20, %1, 1\n v_readlane_b32 s21, %1, 2\n v_readlane_b32 s22, %1, 3\n v_readlane_b32 s23, %1, 4\n v_readlane_b32 s24, %1, 5\n v_readlane_b32 s25, %1, 6\n v_readlane_b32 s26, %1, 7\n v_readlane_b32 s27, %1, 8\n s_mov_b32 %0, s20"
                         : "=s"(r) : "v"(i0) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");)
      i1 += r;
    } else if constexpr (OP == 2) {  // v_fmac_f64_dpp row_newbcast
      REP16(asm volatile("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m), "v"(s));)
    } else if constexpr (OP == 3) {  // v_fma_f64 with an SGPR operand (the readlane form's FMA)
      REP16(asm volatile("v_fma_f64 %0, %8, s[20:21], %0\n v_fma_f64 %1, %8, s[20:21], %1\n v_fma_f64 %2, %8, s[20:21], %2\n v_fma_f64 %3, %8, s[20:21], %3\n v_fma_f64 %4, %8, s[20:21], %4\n v_fma_f64 %5, %8, s[20:21], %5\n v_fma_f64 %6, %8, s[20:21], %6\n v_fma_f64 %7, %8, s[20:21], %7"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m) : "s20", "s21");)
    } else if constexpr (OP == 4) {  // v_pk_fma_f32
      REP16(asm volatile("v_pk_fma_f32 %0, %2, %3, %0\n v_pk_fma_f32 %1, %2, %3, %1\n v_pk_fma_f32 %0, %2, %3, %0\n v_pk_fma_f32 %1, %2, %3, %1\n v_pk_fma_f32 %0, %2, %3, %0\n v_pk_fma_f32 %1, %2, %3, %1\n v_pk_fma_f32 %0, %2, %3, %0\n v_pk_fma_f32 %1, %2, %3, %1"
                         : "+v"(a0), "+v"(a1) : "v"(a2), "v"(a3));)
    } else if constexpr (OP == 5) {  // v_fma_f32
      REP16(asm volatile("v_fma_f32 %0, %4, %5, %0\n v_fma_f32 %1, %4, %5, %1\n v_fma_f32 %2, %4, %5, %2\n v_fma_f32 %3, %4, %5, %3\n v_fma_f32 %0, %4, %5, %0\n v_fma_f32 %1, %4, %5, %1\n v_fma_f32 %2, %4, %5, %2\n v_fma_f32 %3, %4, %5, %3"
                         : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(1.0001f), "v"(0.5f));)
    } else if constexpr (OP == 6) {  // dependent v_fma_f64 chain (latency)
      REP16(asm volatile("v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0"
                         : "+v"(a0) : "v"(m), "v"(s));)
    } else if constexpr (OP == 7) {  // readlane -> dependent VALU using that SGPR (the chain's hop)
      REP16(asm volatile("v_readlane_b32 s20, %0, 3\n v_add_u32 %0, s20, %0\n v_readlane_b32 s20, %0, 5\n v_add_u32 %0, s20, %0\n v_readlane_b32 s20, %0, 7\n v_add_u32 %0, s20, %0\n v_readlane_b32 s20, %0, 9\n v_add_u32 %0, s20, %0"
                         : "+v"(i0) : : "s20");)
    } else if constexpr (OP == 8) {  // v_rsq_f64
      REP16(asm volatile("v_rsq_f64 %0, %4\n v_rsq_f64 %1, %4\n v_rsq_f64 %2, %4\n v_rsq_f64 %3, %4\n v_rsq_f64 %0, %4\n v_rsq_f64 %1, %4\n v_rsq_f64 %2, %4\n v_rsq_f64 %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(m));)
    } else if constexpr (OP == 9) {  // v_rcp_f64
      REP16(asm volatile("v_rcp_f64 %0, %4\n v_rcp_f64 %1, %4\n v_rcp_f64 %2, %4\n v_rcp_f64 %3, %4\n v_rcp_f64 %0, %4\n v_rcp_f64 %1, %4\n v_rcp_f64 %2, %4\n v_rcp_f64 %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(m));)
    } else if constexpr (OP == 10) {  // v_mov_b64_dpp row_newbcast
      REP16(asm volatile("v_mov_b64_dpp %0, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %1, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %3, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %4, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %5, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %6, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %7, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                         : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) : "v"(m));)
    } else if constexpr (OP == 11) {  // dependent fmac_f64_dpp chain (latency through DPP)
      REP16(asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                         : "+v"(a0) : "v"(m));)
    } else if constexpr (OP == 12) {  // v_permlane32_swap
      REP16(asm volatile("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3"
                         : "+v"(i0), "+v"(i1), "+v"(f0), "+v"(f1));)
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 + f3 + i0 + i1;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, int W>
void run(const char* name, int per_iter) {
  double* d;
  long long* c;
  const int blocks = 1024 * W;
  hipMalloc(&d, blocks * 64 * sizeof(double));
  hipMalloc(&c, blocks * sizeof(long long));
  const int iters = 200;
  hipLaunchKernelGGL((ic<OP, W>), dim3(blocks), dim3(64), 0, 0, d, c, 2);
  hipLaunchKernelGGL((ic<OP, W>), dim3(blocks), dim3(64), 0, 0, d, c, iters);
  hipDeviceSynchronize();
  static long long h[8192];
  hipMemcpy(h, c, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  std::printf("%-34s W=%d: %6.2f cyc/instr per wave (%6.2f per SIMD)\n", name, W, avg / ((double)iters * per_iter),
              avg / ((double)iters * per_iter) / W);
  hipFree(d);
  hipFree(c);
}

int main() {
  run<0, 1>("v_fma_f64 (8 chains)", 128);
  run<0, 2>("v_fma_f64 (8 chains)", 128);
  run<3, 1>("v_fma_f64 sgpr operand", 128);
  run<3, 2>("v_fma_f64 sgpr operand", 128);
  run<2, 1>("v_fmac_f64_dpp row_newbcast", 128);
  run<2, 2>("v_fmac_f64_dpp row_newbcast", 128);
  run<10, 1>("v_mov_b64_dpp row_newbcast", 128);
  run<10, 2>("v_mov_b64_dpp row_newbcast", 128);
  run<1, 1>("v_readlane_b32", 144);
  run<1, 2>("v_readlane_b32", 144);
  run<4, 1>("v_pk_fma_f32", 128);
  run<4, 2>("v_pk_fma_f32", 128);
  run<5, 1>("v_fma_f32", 128);
  run<5, 2>("v_fma_f32", 128);
  run<8, 1>("v_rsq_f64", 128);
  run<9, 1>("v_rcp_f64", 128);
  run<12, 1>("v_permlane32_swap_b32", 128);
  run<6, 1>("dependent v_fma_f64 (latency)", 128);
  run<11, 1>("dependent v_fmac_f64_dpp (latency)", 128);
  run<7, 1>("readlane -> dependent v_add (hop, per pair)", 64);
  return 0;
}
