// Wave-level helpers of the NNLS loops (als_kernels.hip: the 1024-thread per-row kernel; nnls_row.hip:
// the 512-thread one): DPP / permlane reductions of fp32 and fp64 values and Spark's stopping rule
// (mllib/optimization/NNLS.scala, `stop`).
#pragma once
#include <hip/hip_runtime.h>
#include "device_common.h"

namespace albedo {

template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}

__device__ __forceinline__ bool nnls_stop(double step, double ndir, double nx) {
  return isnan(step) || step < 1e-7 || step > 1e40 || ndir < 1e-12 * nx || ndir < 1e-32;
}

__device__ __forceinline__ double rdlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// a wave-uniform double into scalar registers (the VALU results of uniform math stay in VGPRs otherwise)
__device__ __forceinline__ double uni(double v) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)), __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
__device__ __forceinline__ double vmin_f64(double a, double b) {  // no NaN canonicalisation (none occur)
  double r;
  asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// DPP move of a double with bound_ctrl (lanes without a source read 0)
template <int CTRL>
__device__ __forceinline__ double dpp64z(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// sum over each 16-lane row (row_shr prefix), the result in the row's lane 15
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp64z<0x111>(x);
  x += dpp64z<0x112>(x);
  x += dpp64z<0x114>(x);
  x += dpp64z<0x118>(x);
  return x;
}
// sum or min over each 16-lane row, the result in every lane of the row: butterfly over the lane
// partners i^15, i^7, i^3, i^1 (row_mirror, row_half_mirror, quad perms) -- every lane has a source,
// so no fill values and no bound_ctrl; partners combine the same operands (bit-identical results)
template <int CTRL>
__device__ __forceinline__ double dpp64f(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <bool MIN>
__device__ __forceinline__ double row16_all(double x) {
  auto op = [](double a, double b) { return MIN ? vmin_f64(a, b) : a + b; };
  x = op(x, dpp64f<0x140>(x));
  x = op(x, dpp64f<0x141>(x));
  x = op(x, dpp64f<0x1B>(x));
  x = op(x, dpp64f<0xB1>(x));
  return x;
}
// (u, w) -> lanes of one half / row set hold u's pair sum, the others w's: v_permlane32_swap (halves)
// or v_permlane16_swap (odd rows of u with even rows of w)
template <bool R32, bool MIN>
__device__ __forceinline__ double halve64(double u, double w) {
  const auto lo = R32 ? __builtin_amdgcn_permlane32_swap(__double2loint(u), __double2loint(w), false, false)
                      : __builtin_amdgcn_permlane16_swap(__double2loint(u), __double2loint(w), false, false);
  const auto hi = R32 ? __builtin_amdgcn_permlane32_swap(__double2hiint(u), __double2hiint(w), false, false)
                      : __builtin_amdgcn_permlane16_swap(__double2hiint(u), __double2hiint(w), false, false);
  const double a = __hiloint2double((int)hi[0], (int)lo[0]), b = __hiloint2double((int)hi[1], (int)lo[1]);
  return MIN ? vmin_f64(a, b) : a + b;
}
// Wave reduction of 4 sums (x[0..3]) and 4 minima (x[4..7]): halves by permlane32 (k, k+2), rows by
// permlane16 (k, k+1), then a row butterfly.  Sum k ends in every lane of row
// r = 2 (k >> 1) + (k & 1) of s, minimum k in the same row of m.
__device__ __forceinline__ void wave_reduce8(const double (&x)[8], double& s, double& m) {
  const double y0 = halve64<true, false>(x[0], x[2]), y1 = halve64<true, false>(x[1], x[3]);
  const double z0 = halve64<true, true>(x[4], x[6]), z1 = halve64<true, true>(x[5], x[7]);
  s = row16_all<false>(halve64<false, false>(y0, y1));
  m = row16_all<true>(halve64<false, true>(z0, z1));
}

}  // namespace albedo
