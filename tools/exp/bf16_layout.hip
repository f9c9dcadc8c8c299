// Experiment: operand / accumulator layout of v_mfma_f32_16x16x32_bf16 on gfx950, and the
// exactness of the truncation 3-way split (x = hi + mid + lo) with 6 bf16 products.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout(const float* A, const float* B, float* C) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[(l & 15) * 32 + 8 * (l >> 4) + j];   // A[i][k], i = l&15, k = 8g + j
    b[j] = (__bf16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];  // B[k][n], n = l&15
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__device__ inline unsigned hi16(float x) { return __float_as_uint(x) >> 16; }
__device__ inline float trunc16(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// Gram of 32 signals × 16 columns via the split: G[i][j] = Σ_k x_k[i] x_k[j]
__global__ void split_gram(const float* X, float* G) {
  const int l = threadIdx.x;
  bf16x8 h, m, o;
  for (int j = 0; j < 8; ++j) {
    const float x = X[(8 * (l >> 4) + j) * 16 + (l & 15)];  // signal k = 8g+j, column l&15
    const float xh = trunc16(x), r = x - xh, xm = trunc16(r), xl = r - xm;
    h[j] = __builtin_bit_cast(__bf16, (unsigned short)hi16(xh));
    m[j] = __builtin_bit_cast(__bf16, (unsigned short)hi16(xm));
    o[j] = __builtin_bit_cast(__bf16, (unsigned short)hi16(xl));
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, o, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o, h, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) G[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  std::mt19937 g(1);
  std::uniform_int_distribution<int> d(-8, 8);
  std::vector<float> A(16 * 32), B(32 * 16), C(256);
  for (auto& x : A) x = (float)d(g);
  for (auto& x : B) x = (float)d(g);
  float *dA, *dB, *dC;
  (void)hipMalloc(&dA, A.size() * 4);
  (void)hipMalloc(&dB, B.size() * 4);
  (void)hipMalloc(&dC, 256 * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(C.data(), dC, 256 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0;
      for (int k = 0; k < 32; ++k) s += A[i * 32 + k] * B[k * 16 + j];
      bad += s != C[i * 16 + j];
    }
  std::printf("layout mismatches: %d / 256\n", bad);
  // split accuracy on random normal data
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> X(32 * 16);
  double maxrel_split = 0, maxrel_f32 = 0;
  for (int trial = 0; trial < 20; ++trial) {
    for (auto& x : X) x = nd(g) * std::pow(10.f, (float)(trial % 5) - 2);
    (void)hipMemcpy(dA, X.data(), X.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(split_gram, dim3(1), dim3(64), 0, 0, dA, dC);
    (void)hipMemcpy(C.data(), dC, 256 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double ref = 0, scale = 0;
        float f32 = 0;
        for (int k = 0; k < 32; ++k) {
          ref += (double)X[k * 16 + i] * X[k * 16 + j];
          scale += std::fabs((double)X[k * 16 + i] * X[k * 16 + j]);
          f32 = std::fmaf(X[k * 16 + i], X[k * 16 + j], f32);
        }
        maxrel_split = std::fmax(maxrel_split, std::fabs(C[i * 16 + j] - ref) / scale);
        maxrel_f32 = std::fmax(maxrel_f32, std::fabs(f32 - ref) / scale);
      }
  }
  std::printf("max |err|/Σ|x_i x_j|: split-bf16x6 %.3e   fp32 fma chain %.3e\n", maxrel_split, maxrel_f32);
  return 0;
}
