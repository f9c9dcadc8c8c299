// Does SQ_INSTS_VALU count MFMA instructions on gfx950?  Two kernels, one wave each per
// workgroup, with instruction counts fixed by inline asm:
//   kmix: per iteration 4 v_mfma_f64_16x16x4_f64 + 8 v_add_f64;
//   kval: per iteration 8 v_add_f64 only.
// Under rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES the per-wave VALU count of kmix
// is 8·ITERS (+ a few) if MFMAs are not counted as VALU and 12·ITERS if they are.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 1000;

__global__ __launch_bounds__(64) void kmix(double* out, double a0, double b0) {
  f64x4 acc = {0, 0, 0, 0};
  double a = a0 + threadIdx.x, b = b0, s = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mfma_f64_16x16x4_f64 %0, %1, %2, %0\n\t"
        "v_mfma_f64_16x16x4_f64 %0, %1, %2, %0\n\t"
        "v_mfma_f64_16x16x4_f64 %0, %1, %2, %0\n\t"
        "v_mfma_f64_16x16x4_f64 %0, %1, %2, %0\n\t"
        "s_nop 15\n\t"
        "v_add_f64 %3, %3, %1\n\t"
        "v_add_f64 %3, %3, %2\n\t"
        "v_add_f64 %3, %3, %1\n\t"
        "v_add_f64 %3, %3, %2\n\t"
        "v_add_f64 %3, %3, %1\n\t"
        "v_add_f64 %3, %3, %2\n\t"
        "v_add_f64 %3, %3, %1\n\t"
        "v_add_f64 %3, %3, %2"
        : "+v"(acc), "+v"(a), "+v"(b), "+v"(s));
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3] + s;
}

__global__ __launch_bounds__(64) void kval(double* out, double a0, double b0) {
  double a = a0 + threadIdx.x, b = b0, s = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_f64 %0, %0, %1\n\t"
        "v_add_f64 %0, %0, %2\n\t"
        "v_add_f64 %0, %0, %1\n\t"
        "v_add_f64 %0, %0, %2\n\t"
        "v_add_f64 %0, %0, %1\n\t"
        "v_add_f64 %0, %0, %2\n\t"
        "v_add_f64 %0, %0, %1\n\t"
        "v_add_f64 %0, %0, %2"
        : "+v"(s), "+v"(a), "+v"(b));
  }
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main() {
  const int blocks = 1024;
  double* out;
  if (hipMalloc(&out, blocks * 64 * sizeof(double)) != hipSuccess) return 1;
  hipLaunchKernelGGL(kmix, dim3(blocks), dim3(64), 0, 0, out, 1.0, 2.0);
  hipLaunchKernelGGL(kval, dim3(blocks), dim3(64), 0, 0, out, 1.0, 2.0);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("%d waves per kernel, %d iterations: kmix 4 MFMA + 8 VALU, kval 8 VALU per iteration\n",
              blocks, ITERS);
  return 0;
}
