// Probe: accuracy of the split-fp16 (hi·hi + hi·lo + lo·hi) MFMA product vs fp64, one 16x16 tile, K = 32*NK.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void tile(const float* U, int NK, float* out, int mode) {
  // U: [K][16] values; C[i][j] = sum_k U[k][i] U[k][j]
  const int l = threadIdx.x, i16 = l & 15, g = l >> 4;
  f32x4 acc = {0, 0, 0, 0};
  for (int kb = 0; kb < NK; ++kb) {
    f16x8 h, lo;
    for (int j = 0; j < 8; ++j) {
      const float v = U[(kb * 32 + 8 * g + j) * 16 + i16];
      const _Float16 hh = (_Float16)v;
      h[j] = hh;
      lo[j] = (_Float16)(v - (float)hh);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(h, h, acc, 0, 0, 0);
    if (mode >= 1) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(h, lo, acc, 0, 0, 0);
    if (mode >= 1) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, h, acc, 0, 0, 0);
    if (mode >= 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, lo, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) out[(4 * g + r) * 16 + i16] = acc[r];
}
int main() {
  const int NK = 8, K = 32 * NK;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> U(K * 16);
  for (auto& v : U) v = nd(rng) * 4096.f;
  float *dU, *dO;
  hipMalloc(&dU, U.size() * 4); hipMalloc(&dO, 256 * 4);
  hipMemcpy(dU, U.data(), U.size() * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    tile<<<1, 64>>>(dU, NK, dO, mode);
    std::vector<float> C(256);
    hipMemcpy(C.data(), dO, 1024, hipMemcpyDeviceToHost);
    double maxe = 0, maxv = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double s = 0; for (int k = 0; k < K; ++k) s += (double)U[k * 16 + i] * U[k * 16 + j];
      maxe = fmax(maxe, fabs(C[i * 16 + j] - s)); maxv = fmax(maxv, fabs(s));
    }
    printf("mode %d (0: hi*hi, 1: +hi*lo+lo*hi, 2: +lo*lo): max abs err / max |C| = %.3e\n", mode, maxe / maxv);
  }
  return 0;
}
