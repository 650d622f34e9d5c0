// Probe: v_mfma_f32_16x16x32_f16 accumulation error, started from C = 0 vs C = -x (then + x), against
// the fp64 sum of the same fp16 products.  Random fp16 operands scaled like the top-k scan (|v| < 2^13).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <random>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int KP = 128, NQ = KP / 32;
// A: [16][KP], B: [16][KP] fp16; x: [16] offsets (per A row); out0/out1: [16][16]
__global__ void probe(const _Float16* A, const _Float16* B, const float* x, float* out0, float* out1) {
  const int lane = threadIdx.x, g = lane >> 4, i16 = lane & 15;
  f32x4 c0 = {0, 0, 0, 0}, c1;
  for (int r = 0; r < 4; ++r) c1[r] = -x[4 * g + r];
  for (int q = 0; q < NQ; ++q) {
    f16x8 a, b;
    for (int e = 0; e < 8; ++e) { a[e] = A[i16 * KP + 32 * q + 8 * g + e]; b[e] = B[i16 * KP + 32 * q + 8 * g + e]; }
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) {
    out0[(4 * g + r) * 16 + i16] = c0[r];
    out1[(4 * g + r) * 16 + i16] = c1[r] + x[4 * g + r];
  }
}
int main() {
  std::mt19937_64 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  double worst0 = 0, worst1 = 0, worst01 = 0;
  _Float16 *dA, *dB; float *dx, *d0, *d1;
  hipMalloc(&dA, 16 * KP * 2); hipMalloc(&dB, 16 * KP * 2); hipMalloc(&dx, 64); hipMalloc(&d0, 1024); hipMalloc(&d1, 1024);
  for (int trial = 0; trial < 2000; ++trial) {
    std::vector<_Float16> A(16 * KP), B(16 * KP);
    const float sa = std::ldexp(1.f, 9), sb = std::ldexp(1.f, 9);
    for (auto& v : A) v = (_Float16)(nd(rng) * sa);
    for (auto& v : B) v = (_Float16)(nd(rng) * sb * (trial % 3 == 0 ? 1.f : 0.25f));
    // align B rows with A rows sometimes (large scores)
    if (trial % 2) for (int j = 0; j < 16; ++j) for (int c = 0; c < KP; ++c) B[j * KP + c] = (_Float16)((float)A[j * KP + c] * 0.9f);
    std::vector<double> ex(256);
    std::vector<float> x(16);
    double nrmA[16], nrmB[16];
    for (int i = 0; i < 16; ++i) { nrmA[i] = 0; nrmB[i] = 0; for (int c = 0; c < KP; ++c) { nrmA[i] += (double)A[i*KP+c]*(double)A[i*KP+c]; nrmB[i] += (double)B[i*KP+c]*(double)B[i*KP+c]; } }
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int c = 0; c < KP; ++c) s += (double)A[i*KP+c]*(double)B[j*KP+c]; ex[i*16+j] = s; }
    for (int i = 0; i < 16; ++i) x[i] = (float)(ex[i * 16 + (trial % 16)] * (1.0 + 1e-3 * nd(rng)));
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), 64, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(dA, dB, dx, d0, d1);
    std::vector<float> o0(256), o1(256);
    hipMemcpy(o0.data(), d0, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(o1.data(), d1, 1024, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i) {
      double bmax = 0; for (int j = 0; j < 16; ++j) bmax = std::max(bmax, std::sqrt(nrmB[j]));
      const double scale = std::sqrt(nrmA[i]) * bmax;
      for (int j = 0; j < 16; ++j) {
        worst0 = std::max(worst0, std::fabs(o0[i*16+j] - ex[i*16+j]) / scale);
        worst1 = std::max(worst1, std::fabs(o1[i*16+j] - ex[i*16+j]) / scale);
        worst01 = std::max(worst01, std::fabs((double)o1[i*16+j] - (double)o0[i*16+j]) / scale);
      }
    }
  }
  std::printf("max |C=0 - exact| / (|a||b|max) = %.3e (2^-24 = 5.96e-08)\n", worst0);
  std::printf("max |C=-x, +x - exact| / (|a||b|max) = %.3e\n", worst1);
  std::printf("max |C=-x,+x - C=0| / (|a||b|max) = %.3e\n", worst01);
  return 0;
}
