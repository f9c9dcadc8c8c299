// FETCH_SIZE calibration for 8-B-per-lane gathers (MI355X_MICROARCH.md: only 16-B-per-lane
// streaming reads are calibrated, at half their bytes).  Three kernels read the same 2 GiB
// buffer once each (it is far beyond the 256 MiB Infinity Cache):
//   k16: 16 B per lane, contiguous (the calibrated case);
//   k8:  8 B per lane, contiguous;
//   kg:  the streamed Gram's pattern — lane (c, g) reads bytes 8c.. of a 128-B segment of
//        row g, four 2-KiB rows per instruction, every segment of a row by successive loads.
// Run under rocprofv3 --pmc FETCH_SIZE; each kernel reads 2 GiB.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k16(const double2* __restrict__ p, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = p[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;
}
__global__ void k8(const double* __restrict__ p, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += p[i];
  if (s == 1.2345) out[0] = s;
}
// rows of 256 doubles (2 KiB, k = 256 fp64); a wave takes 4 rows per step, 16 segments each
__global__ void kg(const double* __restrict__ p, size_t nrows, double* out) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  double s = 0;
  for (size_t r0 = 4 * wave; r0 < nrows; r0 += 4 * nw) {
    const double* row = p + (r0 + g) * 256 + c;
#pragma unroll
    for (int X = 0; X < 16; ++X) s += row[16 * X];
  }
  if (s == 1.2345) out[0] = s;
}

int main() {
  const size_t bytes = (size_t)2 << 30;
  double* p;
  double* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
  if (hipMemset(p, 0, bytes) != hipSuccess) return 1;
  hipLaunchKernelGGL(k16, dim3(4096), dim3(256), 0, 0, (const double2*)p, bytes / 16, out);
  hipLaunchKernelGGL(k8, dim3(4096), dim3(256), 0, 0, (const double*)p, bytes / 8, out);
  hipLaunchKernelGGL(kg, dim3(4096), dim3(256), 0, 0, (const double*)p, bytes / 2048, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("each kernel read %zu bytes\n", bytes);
  return 0;
}
