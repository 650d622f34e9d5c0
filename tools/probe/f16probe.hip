// Probe: (1) does v_mfma_f32_16x16x32_f16 keep fp16 denormal inputs?  (2) colscale on a known Z.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../albedo_amd/csrc/kernels.h"
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void mf(float* out, float av, float bv) {
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)0.f; b[j] = (_Float16)0.f; }
  if (threadIdx.x == 0) { a[0] = (_Float16)av; }   // A[0][k=0]
  if (threadIdx.x == 0) { b[0] = (_Float16)bv; }   // B[k=0][0]
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  if (threadIdx.x == 0) { out[0] = c[0]; out[1] = (float)(_Float16)av; }
}
int main() {
  float* d; hipMalloc(&d, 64);
  float h[2];
  const float tests[3] = {1.0f, 1e-5f, 3e-7f};
  for (float t : tests) {
    mf<<<1, 64>>>(d, t, 1.0f);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("mfma f16: a=%g (as f16 %g) * 1 -> %g\n", t, h[1], h[0]);
  }
  const int KP = 64; const int n = 1000;
  std::vector<float> Z((size_t)n * KP);
  for (int r = 0; r < n; ++r) for (int c = 0; c < KP; ++c) Z[(size_t)r * KP + c] = (c + 1) * 0.01f * ((r % 7) - 3);
  float* dZ; unsigned* tmp; float* cs;
  hipMalloc(&dZ, Z.size() * 4); hipMalloc(&tmp, KP * 4); hipMalloc(&cs, 2 * KP * 4);
  hipMemcpy(dZ, Z.data(), Z.size() * 4, hipMemcpyHostToDevice);
  hipError_t e = albedo::launch_colscale(KP, dZ, n, 40.f, tmp, cs, 0);
  std::vector<float> hc(2 * KP); std::vector<unsigned> ht(KP);
  hipDeviceSynchronize();
  hipMemcpy(hc.data(), cs, 2 * KP * 4, hipMemcpyDeviceToHost);
  hipMemcpy(ht.data(), tmp, KP * 4, hipMemcpyDeviceToHost);
  printf("launch %d; col 0: max %g scale %g inv %g; col 63: max %g scale %g\n", (int)e, *(float*)&ht[0], hc[0], hc[KP],
         *(float*)&ht[63], hc[63]);
  return 0;
}
