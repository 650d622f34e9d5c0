// Device helpers shared by the HIP kernels of libalbedo_als.so (gfx950 only): vector types, MFMA
// wrappers, DPP broadcasts / row reductions, the register 16x16 Cholesky and Spark's implicit
// rating weights.  MFMA operand layout: cdna_hip_programming.md §3 (A[i][k] from lane i+16k,
// B[k][j] from lane j+16k, C/D lane l holds rows 4(l>>4)+r, column l&15).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include <utility>

namespace albedo {

#define WAVE_LDS_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
// Compiler-only barrier for lanes of ONE wave exchanging data through LDS: a wave's LDS operations
// execute in order, so no wait is needed, but without it the compiler may forward a lane's own
// (possibly conditional) store to a later load of the same address that another lane wrote, or
// move the load above the store (r06: a y store under `if (i16 == 0)` folded into the back
// substitution's load of it)
#define WAVE_LDS_FENCE() asm volatile("" ::: "memory")

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ int rdlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// Broadcast of lane M of every 16-lane row to the whole row (DPP row_newbcast, gfx90a+): the
// diagonal-block kernels below keep one 16x16 problem per 16-lane row (rows replicated), so a
// broadcast is one v_mov_dpp instead of a v_readlane + SGPR hazard.
template <int M>
__device__ __forceinline__ float bc16(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + M, 0xF, 0xF, true));
}

// acc -= (v of lane M of the 16-lane row) * w in ONE instruction (v_fmac_f32 with a DPP
// row_newbcast source; the compiler keeps the broadcast as a separate v_mov_b32_dpp).  Same single
// rounding as fmaf(-w, bc16<M>(v), acc).  NOP: v may have been written by the previous VALU
// instruction (a DPP source needs 2 wait states, which the compiler does not insert around asm);
// volatile keeps these in program order, so only the first use after a write needs it.
template <int M, bool NOP>
__device__ __forceinline__ void fnmac_bc16(float& acc, float v, float w) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(acc) : "v"(v), "v"(w), "n"(M));
  else
    asm volatile("v_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(acc) : "v"(v), "v"(w), "n"(M));
}
// bc16 for a source written by asm (fnmac_bc16): the wait states are explicit
template <int M>
__device__ __forceinline__ float bc16_after_asm(float v) {
  float r;
  asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
               : "=v"(r) : "v"(v), "n"(M));
  return r;
}

// Sum over each 16-lane row, result in the row's lane 15: DPP row_shr prefix sums (VALU only; a
// __shfl_xor butterfly goes through the LDS crossbar instead).
__device__ __forceinline__ float sum16_last(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x111, 0xF, 0xF, true));  // row_shr:1
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x112, 0xF, 0xF, true));  // row_shr:2
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x114, 0xF, 0xF, true));  // row_shr:4
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x118, 0xF, 0xF, true));  // row_shr:8
  return x;
}

// Sum over the four 16-lane rows of the wave (lanes l, l^16, l^32, l^48), every lane getting the same
// value: v_permlane16_swap pairs rows (0,1) and (2,3), v_permlane32_swap the two halves -- VALU only,
// no LDS round trip (a __shfl_xor is one).  Partners add in the same order: bit-identical results.
__device__ __forceinline__ float rows4_sum(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// max over the wave of a non-negative value, in every lane: DPP row_shr prefix maxima within the
// 16-lane rows, row_bcast:15 / :31 across rows (lane 63 ends with the maximum), then readlane -- VALU
// only (a __shfl_xor butterfly is six dependent LDS round trips)
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xF, 0xF, false)));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// v_rsq_f32 / v_rcp_f32 / v_sqrt_f32: single instructions (~1 ulp) instead of the IEEE-exact
// multi-instruction expansions; the solve tolerance is 1e-4 relative (tests state it)
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// launches of one workgroup per row are split so that rows x threads stays below 2^31 (AQL grid size)
inline int64_t max_rows_per_launch(int threads) { return (int64_t(1) << 31) / threads; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma_h(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// F2J sdot (netlib sdot.f via F2J: float products added left to right, no FMA contraction)
__device__ __forceinline__ float f2j_dot(const float* __restrict__ x, const float* __restrict__ y, int k) {
#pragma clang fp contract(off)
  float acc = 0.f;
  for (int c = 0; c < k; ++c) {
    const float p = x[c] * y[c];
    acc = acc + p;
  }
  return acc;
}

// the same F2J sum with 16-B loads (x, y 16-B aligned): identical products and addition order
__device__ __forceinline__ float f2j_dot_v4(const float* __restrict__ x, const float* __restrict__ y, int k) {
#pragma clang fp contract(off)
  float acc = 0.f;
  int c = 0;
  for (; c + 4 <= k; c += 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(x + c), b = *reinterpret_cast<const f32x4*>(y + c);
    const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
    acc = acc + p0;
    acc = acc + p1;
    acc = acc + p2;
    acc = acc + p3;
  }
  for (; c < k; ++c) {
    const float p = x[c] * y[c];
    acc = acc + p;
  }
  return acc;
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// Dynamic LDS beyond 64 KiB needs the per-kernel attribute (set once per instantiation).
template <typename K>
hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

struct TilePair { int a, b; };
// t-th tile of the upper triangle (a <= b) of an nq x nq block grid, row-major.
__host__ __device__ constexpr TilePair upper_tile(int t, int nq) {
  int a = 0;
  while (t >= nq - a) { t -= nq - a; ++a; }
  return TilePair{a, a + t};
}
// Column of local index i in permuted 16-column block q (q = 4h + m): 64h + 4i + m.
__host__ __device__ constexpr int pcol(int q, int i) { return 64 * (q >> 2) + 4 * i + (q & 3); }

// Spark NormalEquation weights of one rating (implicit: c = alpha|r|, w = (r > 0)(1 + c);
// explicit: c = 1, w = r).
__device__ __forceinline__ void rating_weights(float r, int implicit, float alpha, float& c, float& w) {
  if (implicit) {
    c = alpha * fabsf(r);
    w = r > 0.f ? 1.f + c : 0.f;
  } else {
    c = 1.f;
    w = r;
  }
}

// 16x16 Cholesky of a diagonal tile in registers: lane i (of each 16-lane row) holds row i (rr[m],
// m <= i meaningful).  On return rr[m] = L[i][m] (m <= i), dg = 1/L[i][i].  A pivot that collapses
// below 2^-21 of its start value is numerically singular in fp32 (Spark's fp64 dppsv reports
// info > 0 on such systems): reported as not positive definite (return value, wave-uniform).
__device__ __forceinline__ bool chol16(float (&rr)[16], float& dg, int i) {
  bool notpd = false;
  float d0 = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) d0 = (i == c) ? rr[c] : d0;
  static_for<0, 16>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (i == c && !(rr[c] > d0 * 4.76837158e-07f)) notpd = true;
    const float piv = bc16_after_asm<c>(rr[c]);
    const float inv = frsq(piv), sq = piv * inv;
    rr[c] = (i == c) ? sq : rr[c] * inv;
    dg = (i == c) ? inv : dg;
    static_for<c + 1, 16>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      fnmac_bc16<m, m == c + 1>(rr[m], rr[c], rr[c]);
    });
  });
  return __any(notpd);
}

// NNLS layout: packed lower 16x16 tiles with 16-float rows (1 KiB per tile, 16-B aligned rows for
// ds_read_b128), diagonal tiles stored full (both triangles)
__host__ __device__ __forceinline__ constexpr int ntile(int I, int J) { return (I * (I + 1) / 2 + J) * 256; }
__host__ __device__ __forceinline__ constexpr int nel(int r, int c) {
  return ntile(r >> 4, c >> 4) + (r & 15) * 16 + (c & 15);
}

}  // namespace albedo
