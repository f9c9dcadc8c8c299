// Micro-benchmark of the row kernels' register-tile Cholesky + solve (qmf_amd/csrc/chol.h)
// in isolation: every wave loads the same SPD system (accumulator-tile image, L2-resident),
// factors and solves it REPS times, and stamps s_memtime around each chol_solve.  Occupancy
// is pinned with dynamic LDS (W waves per SIMD).  Prints cycles per solve (mean over waves)
// and solves/s over the whole GPU, and checks x against a host fp64 solve.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Iqmf_amd/csrc
//        [-DQMFX_CHOL_LA=0] tools/exp/chol_bench.hip -o /tmp/chol_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "chol.h"
using namespace qmfx;

template <typename T, int NT, int W, bool LTP>
__global__ __launch_bounds__(64, W) void chol_bench(const T* img, const T* b, T* x,
                                                     long long* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) CholShared<T, NT, LTP> S;
  extern __shared__ char pad[];
  using acc_t = typename Mfma<T>::acc_t;
  constexpr int NTT = NT * (NT + 1) / 2;
  const int lane = threadIdx.x;
  long long tot = 0;
  if (lane == 0) pad[0] = 0;
  for (int r = 0; r < reps; ++r) {
    acc_t acc[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[t][q] = img[(t * 64 + lane) * 4 + q];
    for (int i = lane; i < 16 * NT; i += 64) S.bw[i] = b[i];
    __syncthreads();
    int bad = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    chol_solve<T, NT, false, LTP>(acc, S, lane, bad);
    const long long t1 = __builtin_amdgcn_s_memtime();
    tot += t1 - t0;
    if (blockIdx.x == 0)
      for (int i = lane; i < 16 * NT; i += 64) x[i] = bad ? T(-1e30) : S.xs[i];
    __syncthreads();
  }
  if (lane == 0) cyc[blockIdx.x] = tot;
}

template <typename T, int NT, int W, bool LTP>
void run(const char* tag) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT, NTT = NT * (NT + 1) / 2;
  std::mt19937 g(7);
  std::normal_distribution<double> nd(0.0, 0.01);
  // A = Zᵀ Z + D (an SPD matrix with the whitened rows' scale)
  std::vector<double> Z(KP * 200), A(KP * KP), bv(KP);
  for (auto& z : Z) z = nd(g);
  for (int i = 0; i < KP; ++i)
    for (int j = 0; j < KP; ++j) {
      double s = 0;
      for (int r = 0; r < 200; ++r) s += Z[r * KP + i] * Z[r * KP + j];
      A[i * KP + j] = s + (i == j ? 0.005 + 0.02 * (i % 7) / 7.0 : 0.0);
    }
  for (int i = 0; i < KP; ++i) bv[i] = 1.0 + 0.1 * (i % 5);
  std::vector<T> img(NTT * 256), hb(KP);
  for (int I = 0; I < NT; ++I)
    for (int J = 0; J <= I; ++J)
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
          const int t = tile_index(I, J);
          const int row = 16 * I + (sizeof(T) == 4 ? ((l >> 4) << 2) + r : (l >> 4) + (r << 2));
          img[(t * 64 + l) * 4 + r] = (T)A[row * KP + 16 * J + (l & 15)];
        }
  for (int i = 0; i < KP; ++i) hb[i] = (T)bv[i];
  // host solve (Cholesky in double) for the check
  std::vector<double> L(A), y(bv);
  for (int j = 0; j < KP; ++j) {
    double d = L[j * KP + j];
    for (int k = 0; k < j; ++k) d -= L[j * KP + k] * L[j * KP + k];
    d = std::sqrt(d);
    L[j * KP + j] = d;
    for (int i = j + 1; i < KP; ++i) {
      double s = L[i * KP + j];
      for (int k = 0; k < j; ++k) s -= L[i * KP + k] * L[j * KP + k];
      L[i * KP + j] = s / d;
    }
  }
  for (int i = 0; i < KP; ++i) {
    double s = y[i];
    for (int k = 0; k < i; ++k) s -= L[i * KP + k] * y[k];
    y[i] = s / L[i * KP + i];
  }
  for (int i = KP - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < KP; ++k) s -= L[k * KP + i] * y[k];
    y[i] = s / L[i * KP + i];
  }
  T *dimg, *db, *dx;
  long long* dc;
  const int blocks = 1024 * W * 8;
  hipMalloc(&dimg, img.size() * sizeof(T));
  hipMalloc(&db, KP * sizeof(T));
  hipMalloc(&dx, KP * sizeof(T));
  hipMalloc(&dc, blocks * sizeof(long long));
  hipMemcpy(dimg, img.data(), img.size() * sizeof(T), hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), KP * sizeof(T), hipMemcpyHostToDevice);
  const size_t stat = sizeof(CholShared<T, NT, LTP>);
  const size_t per_wave = 160 * 1024 / (4 * W);
  const size_t dyn = per_wave > stat + 256 ? per_wave - stat - 256 : 0;
  const int reps = 8;
  hipLaunchKernelGGL((chol_bench<T, NT, W, LTP>), dim3(blocks), dim3(64), dyn, 0, dimg, db, dx, dc, 1);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((chol_bench<T, NT, W, LTP>), dim3(blocks), dim3(64), dyn, 0, dimg, db, dx, dc, reps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(blocks);
  std::vector<T> hx(KP);
  hipMemcpy(c.data(), dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  hipMemcpy(hx.data(), dx, KP * sizeof(T), hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : c) avg += (double)v;
  avg /= (double)blocks * reps;
  double err = 0, nrm = 0;
  for (int i = 0; i < KP; ++i) {
    err = std::max(err, std::fabs((double)hx[i] - y[i]));
    nrm = std::max(nrm, std::fabs(y[i]));
  }
  std::printf("%-28s %s NT=%d W=%d: %8.0f cyc/solve (s_memtime), %7.2f M solves/s, rel err %.2e\n",
              tag, sizeof(T) == 4 ? "f32" : "f64", NT, W, avg, (double)blocks * reps / (ms * 1e-3) / 1e6,
              err / nrm);
  hipFree(dimg);
  hipFree(db);
  hipFree(dx);
  hipFree(dc);
}

int main(int argc, char** argv) {
  const char* tag = argc > 1 ? argv[1] : "chol";
  run<double, 4, 2, true>(tag);   // whitened fp64 n ≤ 64 (LTP form), 2 waves/SIMD
  run<double, 3, 2, true>(tag);   // whitened fp64 n ≤ 48
  run<double, 4, 1, true>(tag);
  run<double, 8, 1, false>(tag);  // direct fp64 k = 128, one wave/SIMD
  run<float, 4, 4, false>(tag);   // direct fp32 k = 64 (C2), 4 waves/SIMD
  run<float, 4, 2, false>(tag);
  run<float, 8, 1, false>(tag);   // fp32 k = 128
  return 0;
}
