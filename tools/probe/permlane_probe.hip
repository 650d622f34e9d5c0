// Probe (not a test): semantics of v_permlane16_swap / v_permlane32_swap as the builtins return them,
// and the lane-group broadcast built from them in wave_chol.h (grp_bcast).  ./permlane_probe
#include "../../albedo_amd/csrc/wave_chol.h"
#include <cstdio>
using namespace albedo;
__global__ void k(float* out) {
  const int lane = threadIdx.x;
  const float x = 100.f * (lane >> 4) + (lane & 15);
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  out[lane] = __uint_as_float(a[0]);
  out[64 + lane] = __uint_as_float(a[1]);
  out[128 + lane] = __uint_as_float(b[0]);
  out[192 + lane] = __uint_as_float(b[1]);
  out[256 + lane] = grp_bcast<0>(x);
  out[320 + lane] = grp_bcast<1>(x);
  out[384 + lane] = grp_bcast<2>(x);
  out[448 + lane] = grp_bcast<3>(x);
}
int main() {
  float* d;
  (void)hipMalloc(&d, 512 * 4);
  k<<<1, 64>>>(d);
  float h[512];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[8] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "bcast0", "bcast1", "bcast2", "bcast3"};
  for (int v = 0; v < 8; ++v) {
    printf("%-7s", nm[v]);
    for (int g = 0; g < 4; ++g) printf("  row%d: %4.0f %4.0f", g, h[64 * v + 16 * g], h[64 * v + 16 * g + 5]);
    printf("\n");
  }
  return 0;
}
