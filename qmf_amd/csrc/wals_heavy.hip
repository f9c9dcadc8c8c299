// Split-K heavy rows (SURVEY.md §5 "long rows"; the reference loops such a row inside one
// thread, WALSEngine.cpp:277-287): rows with more than QMFX_HEAVY_MIN signals are cut into
// QMFX_SEG_LEN-signal segments.  Pass 1: the direct kernel in mode 1, one wave per segment,
// writes the segment's partial Gram tiles, rhs, Σc and negative-weight flag.  Pass 2:
// heavy_reduce_kernel sums a row's segments in fixed order in fp64 with G + λI.  Pass 3: the
// direct kernel in mode 2 solves the row from that image (no signals).
#include "direct.h"

namespace qmfx {

// ---------------------------------------------------------------------------------------
// Split-K heavy rows, second pass: one wave per (heavy row h, tile t).  Tile t < NTT: the
// row's segments' partial tiles summed in fp64 in segment order, plus G + λI (the direct
// kernel's tile image), rounded once to T and written over the first segment's tile t
// (only this wave reads that tile, and it reads it first).  t = NTT: the rhs, Σc and the
// negative-weight flag.  Deterministic: the segment order is fixed.
// ---------------------------------------------------------------------------------------
template <typename T, int NT>
__global__ __launch_bounds__(64) void heavy_reduce_kernel(T* part, T* partb, double* partc,
                                                          const int64_t* hseg, int64_t h0,
                                                          const T* Gimg) {
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  const int lane = threadIdx.x;
  const int t = blockIdx.y;
  const int64_t h = h0 + blockIdx.x;
  const int64_t s0 = hseg[h], s1 = hseg[h + 1];
  if (t < NTT) {
    const int64_t off = (int64_t)(t * 64 + lane) * 4;
    double v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (double)Gimg[off + r];
    for (int64_t s = s0; s < s1; ++s) {
      const T* p = part + s * (NTT * 256) + off;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (double)p[r];
    }
    T* o = part + s0 * (NTT * 256) + off;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (T)v[r];
  } else {
    for (int j = lane; j < KP; j += 64) {
      double b = 0.0;
      for (int64_t s = s0; s < s1; ++s) b += (double)partb[s * KP + j];
      partb[s0 * KP + j] = (T)b;
    }
    if (lane == 0) {
      double c = 0.0, f = 0.0;
      for (int64_t s = s0; s < s1; ++s) {
        c += partc[2 * s];
        f = fmax(f, partc[2 * s + 1]);
      }
      partc[2 * s0] = c;
      partc[2 * s0 + 1] = f;
    }
  }
}

#ifndef QMFX_KERNELS_ONLY
template <typename T, int NT>
static hipError_t launch_heavy_reduce_nt(T* part, T* partb, double* partc, const int64_t* hseg,
                                         int64_t h0, int64_t nh, const T* Gimg, hipStream_t s) {
  constexpr int NTT = NT * (NT + 1) / 2;
  for (int64_t done = 0; done < nh; done += 65535) {
    const int64_t cnt = nh - done < 65535 ? nh - done : 65535;
    hipLaunchKernelGGL((heavy_reduce_kernel<T, NT>), dim3((unsigned)cnt, NTT + 1), dim3(64), 0, s,
                       part, partb, partc, hseg, h0 + done, Gimg);
  }
  return hipGetLastError();
}
hipError_t launch_heavy_reduce(float* part, float* partb, double* partc, const int64_t* hseg,
                               int64_t h0, int64_t nh, const float* Gimg, int nt, hipStream_t s) {
#define CALL(N) launch_heavy_reduce_nt<float, N>(part, partb, partc, hseg, h0, nh, Gimg, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}
hipError_t launch_heavy_reduce(double* part, double* partb, double* partc, const int64_t* hseg,
                               int64_t h0, int64_t nh, const double* Gimg, int nt, hipStream_t s) {
#define CALL(N) launch_heavy_reduce_nt<double, N>(part, partb, partc, hseg, h0, nh, Gimg, s)
  QMFX_NT_SWITCH(nt, CALL)
#undef CALL
}

template <typename T>
static hipError_t heavy_seg(const SolveArgs<T>& a, int nt, hipStream_t s) {
#define CALL1(N) launch_direct_mode<T, N, 1>(a, s)
#define CALL2(N) launch_direct_mode<T, N, 2>(a, s)
  if (a.seg_mode == 1) {
    QMFX_NT_SWITCH(nt, CALL1)
  }
  if (a.seg_mode == 2) {
    QMFX_NT_SWITCH(nt, CALL2)
  }
#undef CALL1
#undef CALL2
  return hipErrorInvalidValue;
}
hipError_t launch_wals_heavy(const SolveArgs<float>& a, int nt, hipStream_t s) {
  return heavy_seg(a, nt, s);
}
hipError_t launch_wals_heavy(const SolveArgs<double>& a, int nt, hipStream_t s) {
  return heavy_seg(a, nt, s);
}
#endif  // QMFX_KERNELS_ONLY

}  // namespace qmfx
