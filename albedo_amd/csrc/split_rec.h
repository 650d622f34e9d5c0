// Split-K record layout (kernels.h SplitArgs), shared by the workgroup build (als_kernels.hip
// heavy_partial_kernel) and the wave build (heavy_wave.hip wave_partial_kernel): the packed lower
// 16x16 tiles of A' with 17-float rows (tile (I, J), I >= J, at (I(I+1)/2 + J)·HT_SZ), then b', then
// the positive-rating count (int bits).
#pragma once
#include <hip/hip_runtime.h>

namespace albedo {

constexpr int HT_LD = 17, HT_SZ = 16 * HT_LD;
__host__ __device__ __forceinline__ constexpr int htile(int I, int J) { return (I * (I + 1) / 2 + J) * HT_SZ; }
__host__ __device__ __forceinline__ constexpr int hel(int r, int c) {
  return htile(r >> 4, c >> 4) + (r & 15) * HT_LD + (c & 15);
}

template <int KP>
struct SplitRec {
  static constexpr int NQ = KP / 16, NTL = NQ * (NQ + 1) / 2;
  static constexpr int TILES = NTL * HT_SZ;
  static constexpr int OFF_B = TILES, OFF_N = OFF_B + KP;
  static constexpr int FLOATS = (OFF_N + 1 + 3) & ~3;  // 16-B aligned records
};

}  // namespace albedo
