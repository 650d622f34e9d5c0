// HIP/CDNA4 (gfx950) kernels of the implicit-ALS half-sweep and the scoring path.
//
// Hot path per half-sweep (Spark MLlib 2.2.0 ALS.computeFactors):
//   gram_partial/gram_reduce   G = YᵀY (Spark computeYtY), fp32 MFMA flushed to fp64 every 64 rows
//   rotate                     Z = Y·P  (P = eigenvectors of G, host fp64): G becomes diagonal (Λ)
//   solve_light<KP,D>          rows with degree <= D: push-through / Woodbury form of the SAME
//                              normal equation, x = D⁻¹Zᵀv, (C⁻¹ + Z D⁻¹ Zᵀ) v = C⁻¹w, a d×d
//                              Cholesky in registers (one wave per row)
//   solve_heavy<KP>            other rows: A' = diag(Λ+λn) + Zᵀ C Z built with MFMA, blocked
//                              Cholesky + forward/back substitution in LDS (one workgroup per row)
// The normal equation is Spark's (NormalEquation.add/merge + CholeskySolver):
//   (G + λ·n_j·I + Σ_i c_i y_i y_iᵀ) x_j = Σ_i w_i y_i,  c = α|r|, w = (r>0)(1+c), n = #(r>0)
// expressed in the eigenbasis of G; x_j comes out in that basis (the host tracks the basis).
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain, 64 FLOP/clk/SIMD).  Operand layout
// (cdna_hip_programming.md §3): A[i][k] from lane i+16k, B[k][j] from lane j+16k, C/D lane l holds
// rows 4(l>>4)+r, column l&15.  Contractions over a 16-wide chunk use a permuted k order so every
// lane issues one float4 (16-B) load: sub-step m of chunk c0 contracts column c0 + 4(l>>4) + m.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <type_traits>
#include <algorithm>
#include <utility>
#include "kernels.h"
#include "device_common.h"
#include "wave_chol.h"
#include "nnls_common.h"
#include "split_rec.h"

namespace albedo {

// Workgroup-per-row launches are issued in pieces: an AQL dispatch carries the grid size as a 32-bit
// count of work-items, so rows x threads must stay below 2^32 (kept at 2^31).
inline SolveArgs chunk_args(const SolveArgs& a, int64_t r0, int threads, int rec_floats) {
  SolveArgs b = a;
  b.rows = a.rows + r0;
  b.n_rows = std::min<int64_t>(a.n_rows - r0, max_rows_per_launch(threads));
  if (a.prebuilt) b.prebuilt = a.prebuilt + (size_t)r0 * rec_floats;
  return b;
}

#ifdef ALBEDO_HEAVY_TIMING  // probes only: per-phase clock64 stamps of the first 64 heavy workgroups
__device__ unsigned long long albedo_heavy_ts[64][48];
#define HEAVY_TS(k) \
  if (threadIdx.x == 0 && blockIdx.x < 64) albedo_heavy_ts[blockIdx.x][k] = clock64()
#else
#define HEAVY_TS(k)
#endif
#ifdef ALBEDO_NNLS_TIMING  // probes only: NNLS loop phase cycles summed over iterations (thread 0)
__device__ unsigned long long albedo_nnls_ph[64][8];
#define NNLS_T0() unsigned long long nt_t = clock64(), nt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define NNLS_PH(k) { const unsigned long long nt_n = clock64(); nt_acc[k] += nt_n - nt_t; nt_t = nt_n; }
#define NNLS_OUT() \
  if (threadIdx.x == 0 && blockIdx.x < 64) for (int q = 0; q < 8; ++q) albedo_nnls_ph[blockIdx.x][q] = nt_acc[q]
#else
#define NNLS_T0()
#define NNLS_PH(k)
#define NNLS_OUT()
#endif

int padded_rank(int rank) {
  if (rank <= 0) return 0;
  if (rank <= 64) return 64;
  if (rank <= 128) return 128;
  if (rank <= 256) return 256;
  return 0;
}

// =============================================================================================
// Gram: G = Σ_rows x xᵀ  (Spark ALS.computeYtY: NormalEquation.add(y, 0.0) per src row, fp64)
// =============================================================================================
template <int KP> constexpr int gram_waves() { return KP >= 256 ? 16 : 4; }  // tile owners per row range

template <int KP, int W>
__device__ __forceinline__ void gram_body(const float* __restrict__ X, int64_t rb, int64_t re,
                                          double* __restrict__ out) {
  constexpr int NWV = gram_waves<KP>();
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2, NTW = (NT + NWV - 1) / NWV, NH = KP / 64;
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  f32x4 acc[NTW];
  double acc64[NTW][4];
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    acc[s] = zero4();
    for (int r = 0; r < 4; ++r) acc64[s][r] = 0.0;
  }
  // 16 rows per trip: the four 4-row groups' loads are all in flight before the first MFMA
  for (int64_t r0 = rb; r0 < re; r0 += 64) {
    const int64_t r1 = r0 + 64 < re ? r0 + 64 : re;
    for (int64_t q0 = r0; q0 < r1; q0 += 16) {
      f32x4 v[4][NH];
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          const int64_t row = q0 + 4 * d + g;
          v[d][h] = row < r1 ? ld4(X + row * KP + 64 * h + 4 * i16) : zero4();
        }
#pragma unroll
      for (int d = 0; d < 4; ++d)
        static_for<0, NTW>([&](auto s) {
          constexpr int t = W + NWV * decltype(s)::value;
          if constexpr (t < NT) {
            constexpr TilePair p = upper_tile(t, NQ);
            acc[s] = mfma4(v[d][p.a >> 2][p.a & 3], v[d][p.b >> 2][p.b & 3], acc[s]);
          }
        });
    }
    // 64 rows per fp32 partial, then fp64 (Spark accumulates in fp64)
#pragma unroll
    for (int s = 0; s < NTW; ++s) {
      for (int r = 0; r < 4; ++r) acc64[s][r] += (double)acc[s][r];
      acc[s] = zero4();
    }
  }
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    const int t = W + NWV * s;
    if (t < NT)
      for (int r = 0; r < 4; ++r) out[((size_t)t * 64 + lane) * 4 + r] = acc64[s][r];
  }
}

template <int KP>
__global__ __launch_bounds__(256) void gram_partial_kernel(const float* __restrict__ X, int64_t n,
                                                           int64_t per_blk, double* __restrict__ slab) {
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2;
  const int64_t rb = (int64_t)blockIdx.x * per_blk;
  const int64_t re = rb + per_blk < n ? rb + per_blk : n;
  double* out = slab + (size_t)blockIdx.x * NT * 256;
  const int wg = blockIdx.y * 4 + (threadIdx.x >> 6);  // blockIdx.y: group of 4 tile owners
  static_for<0, gram_waves<KP>()>([&](auto w) {
    if (wg == decltype(w)::value) gram_body<KP, decltype(w)::value>(X, rb, re, out);
  });
}

template <int KP>
__global__ void gram_reduce_kernel(const double* __restrict__ slab, int nblk, double* __restrict__ G) {
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (t, lane, r)
  if (e >= NT * 256) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += slab[(size_t)b * NT * 256 + e];
  const int t = e >> 8, lane = (e >> 2) & 63, r = e & 3;
  const TilePair p = upper_tile(t, NQ);
  const int c1 = pcol(p.a, 4 * (lane >> 4) + r), c2 = pcol(p.b, lane & 15);
  G[c1 * KP + c2] = s;
  G[c2 * KP + c1] = s;
}

// ---- Gram on bf16 MFMA (KP = 128) -----------------------------------------------------------
// Each fp32 x = h + m + l (three bf16 parts, exact to 2^-24), products hh, hm, mh, hl, lh, mm on
// v_mfma_f32_16x16x32_bf16 (32 rows per instruction) instead of fp32 16x16x4 (4 rows): the fp32
// form ran the Gram MFMA-bound (55 % busy, r03 c4 counters).  The block stages 32 rows at a time in
// LDS as three bf16 planes (row r: plane p at bytes 256p.., 16-B chunks xor-swizzled by gram_pre_f(r)
// so the transposed reads below are conflict-free), and every wave reads the MFMA operands of the
// 8 column blocks with ds_read_b64_tr_b16: lane i + 16q gets column 16A + i of rows 8q .. 8q+7.
// Wave w owns the upper tiles (a, b) with a ∈ {w, 7 - w} (9 tiles each); fp32 partials go to fp64
// every 64 rows, like gram_body.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma_b(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int gram_pre_f(int r) { return 2 * ((r & 3) | ((r & 8) >> 1)); }
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef short i16x4_vs __attribute__((__vector_size__(8)));
__device__ __forceinline__ bf16x4v gram_tr_read(const char* p) {
  const i16x4_vs v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_vs*)(p));
  return __builtin_bit_cast(bf16x4v, v);
}
constexpr int GBF_RB = 768;  // LDS bytes per staged row: three 256-B bf16 planes

template <int W>
__device__ __forceinline__ void gram_bf_body(const float* __restrict__ X, int64_t rb, int64_t re, double* __restrict__ out,
                                             char* st) {
  constexpr int KP = 128, NQ = 8, A0 = W, A1 = NQ - 1 - W, NTW = 9;
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, q = lane >> 4;
  f32x4 acc[NTW];
  double acc64[NTW][4];
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    acc[s] = zero4();
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[s][r] = 0.0;
  }
  // staging map: thread t holds float4 (row (t + 256m) >> 5, column 4((t + 256m) & 31)), m = 0..3
  auto xload = [&](int64_t r0, f32x4 (&xv)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int idx = tid + 256 * m;
      const int64_t row = r0 + (idx >> 5);
      xv[m] = row < re ? ld4(X + row * KP + 4 * (idx & 31)) : zero4();
    }
  };
  // two 32-row chunks in flight: buffers xa / xb alternate, each reloaded (two chunks ahead) right
  // after it has been staged
  auto step = [&](f32x4 (&xn)[4], int64_t r0, bool flush) {
    // stage: split into three bf16 planes
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int idx = tid + 256 * m, r = idx >> 5, c = 4 * (idx & 31);
      bf16x4v ph, pm, pl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = xn[m][e];
        const __bf16 h = (__bf16)v;
        const float r1 = v - (float)h;
        const __bf16 mm = (__bf16)r1;
        ph[e] = h;
        pm[e] = mm;
        pl[e] = (__bf16)(r1 - (float)mm);
      }
      char* rowp = st + r * GBF_RB + 2 * (c & 7) + 16 * ((c >> 3) ^ gram_pre_f(r));
      *reinterpret_cast<bf16x4v*>(rowp) = ph;
      *reinterpret_cast<bf16x4v*>(rowp + 256) = pm;
      *reinterpret_cast<bf16x4v*>(rowp + 512) = pl;
    }
    __syncthreads();
    if (r0 + 64 < re) xload(r0 + 64, xn);
    // operands of the column blocks this wave touches (A >= W): lane i + 16q = column 16A + i of
    // rows 8q .. 8q+7, per plane
    bf16x8 fr[NQ][3];
    {
      const int qq = i16 >> 2, p = i16 & 3;
      static_for<W, NQ>([&](auto AA) {
        constexpr int A = decltype(AA)::value;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 8 * q + 4 * h + qq;
          const char* row = st + r * GBF_RB + 8 * (p & 1) + 16 * ((2 * A + (p >> 1)) ^ gram_pre_f(r));
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const bf16x4v v = gram_tr_read(row + 256 * pl);
#pragma unroll
            for (int e = 0; e < 4; ++e) fr[A][pl][4 * h + e] = v[e];
          }
        }
      });
    }
    __syncthreads();  // the stage is free for the next chunk
    auto tile = [&](auto SS, auto AA, auto BB) {
      constexpr int s = decltype(SS)::value, a = decltype(AA)::value, b = decltype(BB)::value;
      f32x4 c = acc[s];
      c = mfma_b(fr[a][2], fr[b][0], c);  // the small terms first
      c = mfma_b(fr[a][0], fr[b][2], c);
      c = mfma_b(fr[a][1], fr[b][1], c);
      c = mfma_b(fr[a][1], fr[b][0], c);
      c = mfma_b(fr[a][0], fr[b][1], c);
      c = mfma_b(fr[a][0], fr[b][0], c);
      acc[s] = c;
    };
    static_for<0, NQ - A0>([&](auto BB) {
      tile(BB, std::integral_constant<int, A0>{}, std::integral_constant<int, A0 + decltype(BB)::value>{});
    });
    static_for<0, NQ - A1>([&](auto BB) {
      tile(std::integral_constant<int, NQ - A0 + decltype(BB)::value>{}, std::integral_constant<int, A1>{},
           std::integral_constant<int, A1 + decltype(BB)::value>{});
    });
    if (flush) {  // 64 rows per fp32 partial, then fp64
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc64[t][r] += (double)acc[t][r];
        acc[t] = zero4();
      }
    }
  };
  f32x4 xa[4], xb[4];
  if (rb < re) xload(rb, xa);
  if (rb + 32 < re) xload(rb + 32, xb);
  for (int64_t r0 = rb; r0 < re; r0 += 64) {
    step(xa, r0, false);
    if (r0 + 32 < re) step(xb, r0 + 32, true);
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[t][r] += (double)acc[t][r];
  // slab: tile (a, b) at its upper_tile index, lane-major like gram_body (natural column blocks)
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    const int a = s < NQ - A0 ? A0 : A1;
    const int b = s < NQ - A0 ? A0 + s : A1 + (s - (NQ - A0));
    const int t = a * NQ - a * (a - 1) / 2 + (b - a);
#pragma unroll
    for (int r = 0; r < 4; ++r) out[((size_t)t * 64 + lane) * 4 + r] = acc64[s][r];
  }
}

__global__ __launch_bounds__(256, 2) void gram_bf_kernel(const float* __restrict__ X, int64_t n, int64_t per_blk,
                                                        double* __restrict__ slab) {
  constexpr int NT = 36;
  __shared__ __attribute__((aligned(16))) char st[32 * GBF_RB];
  const int64_t rb = (int64_t)blockIdx.x * per_blk;
  const int64_t re = rb + per_blk < n ? rb + per_blk : n;
  double* out = slab + (size_t)blockIdx.x * NT * 256;
  const int wave = threadIdx.x >> 6;
  static_for<0, 4>([&](auto w) {
    if (wave == decltype(w)::value) gram_bf_body<decltype(w)::value>(X, rb, re, out, st);
  });
}

// natural column blocks (gram_bf_kernel): tile t = (a, b), lane l, r -> G[16a + 4(l >> 4) + r][16b + (l & 15)]
__global__ void gram_reduce_nat_kernel(const double* __restrict__ slab, int nblk, double* __restrict__ G, int KP) {
  const int NQ = KP / 16, NT = NQ * (NQ + 1) / 2;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= NT * 256) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += slab[(size_t)b * NT * 256 + e];
  const int t = e >> 8, lane = (e >> 2) & 63, r = e & 3;
  const TilePair p = upper_tile(t, NQ);
  const int c1 = 16 * p.a + 4 * (lane >> 4) + r, c2 = 16 * p.b + (lane & 15);
  // a diagonal tile holds (i, j) and (j, i) separately: the split products reach them in different
  // accumulation orders, so they can differ in the last bit; (i <= j) writes both (deterministic)
  if (c1 > c2) return;
  G[c1 * KP + c2] = s;
  G[c2 * KP + c1] = s;
}

int gram_slab_blocks(int KP, int64_t n) {
  (void)KP;
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 1024) b = 1024;
  return (int)b;
}
size_t gram_slab_doubles(int KP, int slab_blocks) {
  const int nq = KP / 16, nt = nq * (nq + 1) / 2;
  return (size_t)slab_blocks * nt * 256;
}

hipError_t launch_gram(int KP, const float* X, int64_t n, double* slab, int nblk, double* G, hipStream_t s) {
  int64_t per = (n + nblk - 1) / nblk;
  per = (per + 3) & ~int64_t(3);
  const int nq = KP / 16, nt = nq * (nq + 1) / 2;
  if (KP == 64) {
    gram_partial_kernel<64><<<nblk, 256, 0, s>>>(X, n, per, slab);
    gram_reduce_kernel<64><<<(nt * 256 + 255) / 256, 256, 0, s>>>(slab, nblk, G);
  } else if (KP == 128) {
    // bf16 MFMA form (three-part split, gram_bf_kernel)
    gram_bf_kernel<<<nblk, 256, 0, s>>>(X, n, (per + 63) & ~int64_t(63), slab);
    gram_reduce_nat_kernel<<<(nt * 256 + 255) / 256, 256, 0, s>>>(slab, nblk, G, 128);
  } else if (KP == 256) {
    gram_partial_kernel<256><<<dim3(nblk, gram_waves<256>() / 4), 256, 0, s>>>(X, n, per, slab);
    gram_reduce_kernel<256><<<(nt * 256 + 255) / 256, 256, 0, s>>>(slab, nblk, G);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// =============================================================================================
// Rotation: Z = X · M   ([n][KP] x [KP][KP]); M staged in LDS, 64 rows per block iteration.
// =============================================================================================
template <int KP> constexpr int rotate_cols() { return KP >= 256 ? 128 : KP; }  // output columns per block

// 8 waves per block share one LDS copy of M (64+ KB); each wave's
// 16 rows are loaded whole before the first MFMA.
constexpr int ROT_WAVES = 8;
// cmax (or null): bits of max_rows |Z[.][c]| accumulated with atomicMax (zeroed by the caller) -- the
// column maxima the heavy build's fp16 column scales need, without a second pass over Z
template <int KP>
__global__ __launch_bounds__(64 * ROT_WAVES) void rotate_kernel(const float* __restrict__ X,
                                                               const float* __restrict__ M,
                                                               float* __restrict__ Z, int64_t n,
                                                               unsigned* __restrict__ cmax) {
  constexpr int NO = rotate_cols<KP>(), LDM = NO + 4, NJ = NO / 16, NC = KP / 16;
  constexpr int NTH = 64 * ROT_WAVES, RPB = 16 * ROT_WAVES;  // rows per block iteration
  extern __shared__ __attribute__((aligned(16))) float sM[];
  const int co = blockIdx.y * NO;  // this block's output columns co .. co+NO-1
  float cm[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) cm[J] = 0.f;
  for (int e = threadIdx.x; e < KP * NO / 4; e += NTH) {
    const int r = (4 * e) / NO, c = (4 * e) % NO;
    *reinterpret_cast<f32x4*>(sM + r * LDM + c) = ld4(M + r * KP + co + c);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  for (int64_t b = blockIdx.x; b * RPB < n; b += gridDim.x) {
    const int64_t row = b * RPB + wave * 16 + i16;
    constexpr bool PRE = KP <= 128;  // whole-row preload (KP = 256: per slice, registers)
    f32x4 a4[PRE ? NC : 1];
    if constexpr (PRE) {
#pragma unroll
      for (int c = 0; c < NC; ++c) a4[c] = row < n ? ld4(X + row * KP + 16 * c + 4 * g) : zero4();
    }
    f32x4 acc[NJ];
#pragma unroll
    for (int J = 0; J < NJ; ++J) acc[J] = zero4();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x4 av;
      if constexpr (PRE) av = a4[c];
      else av = row < n ? ld4(X + row * KP + 16 * c + 4 * g) : zero4();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float* mr = sM + (16 * c + 4 * g + m) * LDM + i16;
#pragma unroll
        for (int J = 0; J < NJ; ++J) acc[J] = mfma4(av[m], mr[16 * J], acc[J]);
      }
      __builtin_amdgcn_sched_barrier(0);  // one 16-column slice of M in registers at a time
    }
#pragma unroll
    for (int J = 0; J < NJ; ++J)
      for (int r = 0; r < 4; ++r) {
        const int64_t rr = b * RPB + wave * 16 + 4 * g + r;
        if (rr < n) Z[rr * KP + co + 16 * J + i16] = acc[J][r];
        cm[J] = fmaxf(cm[J], fabsf(acc[J][r]));  // rows past n are zero (zero loads)
      }
  }
  if (cmax) {  // column maxima: the wave's four lane groups, the block's waves (LDS), one atomic each
    __syncthreads();  // M's LDS image is dead
    float* red = sM;  // [ROT_WAVES][NO]
#pragma unroll
    for (int J = 0; J < NJ; ++J) {
      float v = cm[J];
      v = fmaxf(v, __shfl_xor(v, 16));
      v = fmaxf(v, __shfl_xor(v, 32));
      if (g == 0) red[wave * NO + 16 * J + i16] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NO; c += NTH) {
      float v = red[c];
      for (int w = 1; w < ROT_WAVES; ++w) v = fmaxf(v, red[w * NO + c]);
      atomicMax(cmax + co + c, __float_as_uint(v));
    }
  }
}

// ---- Rotation on bf16 MFMA (KP = 128) -------------------------------------------------------
// Z = X·P with both operands split into three bf16 parts (x = h + m + l exactly to 2^-24: 8 + 8 + 8
// significant bits, fp32's exponent range, so no scaling) and the six products above 2^-24
// (hh, hm, mh, hl, lh, mm) on v_mfma_f32_16x16x32_bf16: 6 x 16 cycles per 32-deep k-step against
// 8 x 32 for the fp32 16x16x4 form, so the rotation leaves the MFMA bound (74 % busy, r03 c4
// counters) for the HBM one.  One wave per 16 src rows: lane i + 16q loads X[r0 + i][32kc + 8q ..
// +7] (the A operand straight from HBM, 4 lanes per 128-B row segment), P's parts sit in LDS in
// B-fragment order.  With Zhl set the heavy build's operand split is written in the same pass
// (v = z·(sw·cs), hi = fp16(v), lo = fp16(v - hi): presplit_kernel's arithmetic), so Z is not read
// back; cs then comes from a bound on the column maxima known before the rotation (engine).
// P's parts in B-fragment order: element ((J·NK + kc)·3 + part)·512 + l·8 + h holds part `part` of
// P[32 kc + 8 (l >> 4) + h][16 J + (l & 15)]
__global__ void rotate_pfrag_kernel(const float* __restrict__ P, __bf16* __restrict__ Pf, int KP) {
  const int NK = KP / 32;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (J, kc, l, h)
  if (e >= KP * KP) return;
  const int h = e & 7, l = (e >> 3) & 63, kc = (e >> 9) % NK, J = (e >> 9) / NK;
  const float v = P[(32 * kc + 8 * (l >> 4) + h) * KP + 16 * J + (l & 15)];
  const __bf16 ph = (__bf16)v;
  const float r1 = v - (float)ph;
  const __bf16 pm = (__bf16)r1;
  const __bf16 pl = (__bf16)(r1 - (float)pm);
  const int base = ((J * NK + kc) * 3) * 512 + l * 8 + h;
  Pf[base] = ph;
  Pf[base + 512] = pm;
  Pf[base + 1024] = pl;
}

constexpr int RBF_WAVES = 8, RBF_TS = 72;  // waves per block, output image row stride (floats)
constexpr int RBF_JU = 4;                  // column blocks whose accumulator chains interleave
template <int KP>
__global__ __launch_bounds__(64 * RBF_WAVES) void rotate_bf_kernel(const float* __restrict__ X, const __bf16* __restrict__ Pf,
                                                                  float* __restrict__ Z, int64_t n, const float* __restrict__ cs,
                                                                  float sw, _Float16* __restrict__ Zhl, int64_t zrow) {
  constexpr int NK = KP / 32, NJ = KP / 16;
  extern __shared__ __attribute__((aligned(16))) __bf16 sPf[];
  for (int e = threadIdx.x; e < KP * KP * 3 / 8; e += 64 * RBF_WAVES)
    reinterpret_cast<int4*>(sPf)[e] = reinterpret_cast<const int4*>(Pf)[e];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, q = lane >> 4;
  if (Zhl && blockIdx.x == 0)  // the zero row the heavy build's clamped gathers read
    for (int c = threadIdx.x; c < 2 * KP; c += 64 * RBF_WAVES) Zhl[zrow * 2 * KP + c] = (_Float16)0.f;
  if (Zhl)
    for (int c = threadIdx.x; c < KP; c += 64 * RBF_WAVES)
      reinterpret_cast<float*>(sPf + KP * KP * 3)[RBF_WAVES * 16 * RBF_TS + c] = sw * cs[c];
  __syncthreads();
  const int64_t ntile = (n + 15) / 16;
  // this wave's output image (C layout -> 16 consecutive columns of one row per lane), 72-float rows;
  // then sw·cs per column (a global load in the loop would make its vmcnt wait cover the prefetch)
  float* tsc = reinterpret_cast<float*>(sPf + KP * KP * 3) + wave * 16 * RBF_TS;
  float* scs = reinterpret_cast<float*>(sPf + KP * KP * 3) + RBF_WAVES * 16 * RBF_TS;
  // The next tile's X rows are loaded while this one is on MFMA, as ordinary loads: the compiler
  // places the wait for them.  (r03-r05 issued them from asm with a hand-counted vmcnt at the loop
  // head, leaving the tile's stores in flight; but the compiler, which took the asm results as
  // ready, copied the loop-carried registers at the loop head before that wait, and a load still in
  // flight there left a 16-row tile of garbage in Z -- the rare all-paths non-positive pivot of
  // profiles/r05_bench_c4_notpd_twice_diag.err, src Z max 7e34 from finite src X.)
  auto xload = [&](int64_t t, f32x4 (&xv)[NK][2]) {
    const int64_t row = 16 * t + i16;
    const float* src = X + (row < n ? row : n - 1) * KP + 8 * q;  // unconditional, zeroed past n
#pragma unroll
    for (int kc = 0; kc < NK; ++kc) {
      xv[kc][0] = ld4(src + 32 * kc);
      xv[kc][1] = ld4(src + 32 * kc + 4);
    }
  };
  const int64_t tstep = (int64_t)gridDim.x * RBF_WAVES;
  // one 16-row tile: split the A operand, refill its registers with tile tn (two tiles in flight per
  // wave: the one this tile's loads were issued with and tn), then the MFMAs and the stores
  auto tile = [&](int64_t t, f32x4 (&xn)[NK][2], int64_t tn) {
    const int64_t r0 = 16 * t;
    // A operand: row r0 + i16, columns 32kc + 8q .. +7, split into three bf16 parts
    bf16x8 ah[NK], am[NK], al[NK];
    {
      const bool in = r0 + i16 < n;
#pragma unroll
      for (int kc = 0; kc < NK; ++kc)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = in ? xn[kc][e >> 2][e & 3] : 0.f;
          const __bf16 h = (__bf16)v;
          const float r1 = v - (float)h;
          const __bf16 m = (__bf16)r1;
          ah[kc][e] = h;
          am[kc][e] = m;
          al[kc][e] = (__bf16)(r1 - (float)m);
        }
    }
    if (tn < ntile) xload(tn, xn);
    // output: per group of RBF_JU = 4 column blocks (64 columns) the accumulators go through this
    // wave's LDS image [16 rows][RBF_TS], 16-B chunk ch of row r at chunk position ch ^ r (conflict-free
    // b32 stores and b128 reads); lane l then holds row r0 + (l & 15), columns 16q .. 16q + 15 of the
    // group and writes them as 16-B stores only -- 4 for Z, 2 + 2 for the fp16 hi / lo split (r05:
    // 4-column pieces, dwordx2 split stores and two LDS waits per 16 columns)
    const int orow = lane & 15;
    const int64_t rr = r0 + orow;
    for (int J2 = 0; J2 < NJ; J2 += RBF_JU) {
      f32x4 acc2[RBF_JU];
#pragma unroll
      for (int u = 0; u < RBF_JU; ++u) acc2[u] = zero4();
#pragma unroll
      for (int kc = 0; kc < NK; ++kc) {
        bf16x8 bh[RBF_JU], bm[RBF_JU], bl[RBF_JU];
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) {
          const __bf16* pf = sPf + (((J2 + u) * NK + kc) * 3) * 512 + lane * 8;
          bh[u] = *reinterpret_cast<const bf16x8*>(pf);
          bm[u] = *reinterpret_cast<const bf16x8*>(pf + 512);
          bl[u] = *reinterpret_cast<const bf16x8*>(pf + 1024);
        }
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(al[kc], bh[u], acc2[u]);  // the small terms first
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(ah[kc], bl[u], acc2[u]);
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(am[kc], bm[u], acc2[u]);
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(am[kc], bh[u], acc2[u]);
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(ah[kc], bm[u], acc2[u]);
#pragma unroll
        for (int u = 0; u < RBF_JU; ++u) acc2[u] = mfma_b(ah[kc], bh[u], acc2[u]);
      }
      // C layout (lane j + 16q: Z[r0 + 4q + r][16(J2 + u) + j]) -> the image
#pragma unroll
      for (int u = 0; u < RBF_JU; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * q + r, ch = 4 * u + (i16 >> 2);
          tsc[row * RBF_TS + 4 * (ch ^ row) + (i16 & 3)] = acc2[u][r];
        }
      WAVE_LDS_SYNC();
      f32x4 z4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) z4[k] = ld4(tsc + orow * RBF_TS + 4 * ((4 * q + k) ^ orow));
      WAVE_LDS_SYNC();
      const int c0 = 16 * J2 + 16 * q;
      if (rr < n) {
#pragma unroll
        for (int k = 0; k < 4; ++k) *reinterpret_cast<f32x4*>(Z + rr * KP + c0 + 4 * k) = z4[k];
        if (Zhl) {
          f16x8 h8[2], l8[2];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const f32x4 cw4 = ld4(scs + c0 + 4 * k);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float v = z4[k][e] * cw4[e];
              asm("" : "+v"(v));  // one fp32 rounding; hi and lo both from that value (presplit_kernel)
              const _Float16 hv = (_Float16)v;
              h8[k >> 1][4 * (k & 1) + e] = hv;
              l8[k >> 1][4 * (k & 1) + e] = (_Float16)(v - (float)hv);
            }
          }
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            *reinterpret_cast<f16x8*>(Zhl + rr * 2 * KP + c0 + 8 * k) = h8[k];
            *reinterpret_cast<f16x8*>(Zhl + rr * 2 * KP + KP + c0 + 8 * k) = l8[k];
          }
        }
      }
    }
  };
  int64_t t = (int64_t)blockIdx.x * RBF_WAVES + wave;
  f32x4 xa[NK][2], xb[NK][2];
  if (t < ntile) xload(t, xa);
  if (t + tstep < ntile) xload(t + tstep, xb);
  for (; t < ntile; t += 2 * tstep) {
    tile(t, xa, t + 2 * tstep);
    if (t + tstep >= ntile) break;
    tile(t + tstep, xb, t + 3 * tstep);
  }
}

hipError_t launch_rotate_bf(int KP, const float* X, const float* P, void* Pf, float* Z, int64_t n, const float* cs, float sw,
                            void* Zhl, int64_t zrow, int n_cu, hipStream_t s) {
  if (KP != 128) return hipErrorInvalidValue;
  rotate_pfrag_kernel<<<(KP * KP + 255) / 256, 256, 0, s>>>(P, reinterpret_cast<__bf16*>(Pf), KP);
  if (n <= 0) return hipGetLastError();
  const size_t lds = (size_t)KP * KP * 3 * 2 + (size_t)RBF_WAVES * 16 * RBF_TS * 4 + (size_t)KP * 4;
  static const hipError_t attr = allow_lds(rotate_bf_kernel<128>, lds);
  if (attr != hipSuccess) return attr;
  const int64_t tiles = (n + 15) / 16;
  int64_t blocks = (tiles + RBF_WAVES - 1) / RBF_WAVES;
  if (blocks > n_cu) blocks = n_cu;  // one 96-KiB block per CU, grid-stride over the row tiles
  rotate_bf_kernel<128><<<(int)blocks, 64 * RBF_WAVES, lds, s>>>(X, reinterpret_cast<const __bf16*>(Pf), Z, n, cs, sw,
                                                                 reinterpret_cast<_Float16*>(Zhl), zrow);
  return hipGetLastError();
}
int rotate_bf_pfrag_bytes(int KP) { return KP * KP * 3 * 2; }

hipError_t launch_rotate(int KP, const float* X, const float* M, float* Z, int64_t n, hipStream_t s, unsigned* cmax) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 16 * ROT_WAVES - 1) / (16 * ROT_WAVES);
  if (blocks > 1024) blocks = 1024;
  const int nth = 64 * ROT_WAVES;
  if (KP == 64) {
    const size_t lds = (size_t)64 * 68 * 4;
    rotate_kernel<64><<<(int)blocks, nth, lds, s>>>(X, M, Z, n, cmax);
  } else if (KP == 128) {
    const size_t lds = (size_t)128 * 132 * 4;
    static const hipError_t attr = allow_lds(rotate_kernel<128>, lds);
    if (attr != hipSuccess) return attr;
    rotate_kernel<128><<<(int)blocks, nth, lds, s>>>(X, M, Z, n, cmax);
  } else if (KP == 256) {
    const size_t lds = (size_t)256 * (rotate_cols<256>() + 4) * 4;
    static const hipError_t attr = allow_lds(rotate_kernel<256>, lds);
    if (attr != hipSuccess) return attr;
    rotate_kernel<256><<<dim3((int)blocks, 256 / rotate_cols<256>()), nth, lds, s>>>(X, M, Z, n, cmax);
  } else return hipErrorInvalidValue;
  return hipGetLastError();
}

// =============================================================================================
// Light rows: push-through solve, one wave per dst row, degree d <= D.
//   S = (Z_j D^-1/2)(Z_j D^-1/2)ᵀ (d x d, MFMA over the KP columns), K = S + C⁻¹,
//   K v = C⁻¹ w (register Cholesky, lane i = row i), x' = D⁻¹ Z_jᵀ v.
// Entries with c = 0 (implicit zero ratings) contribute nothing to A or b and are masked out.
// =============================================================================================
// LDS floats per wave: D = 16 keeps K and L as packed lower triangles (+ 64: sink); D = 32 / 64 factor
// in the MFMA accumulators (wave_chol.h) and need its scratch (wchol_scratch_floats(NB))
__host__ __device__ constexpr int light_wave_lds(int D) { return D == 16 ? D * (D + 1) / 2 + 64 : wchol_scratch_floats(D / 16); }

// workgroups per CU: D = 32 at KP = 128 keeps its gathered rows in registers (KEEPZ) and spilled 16
// VGPRs at 4 (128 VGPRs); at 3 (168) it does not, and the user light half is 1.9 ms faster (r04 A/B)
template <int KP, int D>
constexpr int light_occupancy() {
  return D > 64 ? 2 : (D == 16 && KP <= 128) ? 6 : (KP == 128 && D == 32) ? 3 : (KP <= 128) ? 4 : 2;
}

// One light row: j, degree d (wave-uniform), lane e < d holds rating r and src row colE of entry e;
// D > 64: lane e also holds entry 64 + e (r2, colE2).
template <int KP, int D>
__device__ __forceinline__ void light_row(const SolveArgs& a, int j, int d, float r, int colE, float r2, int colE2,
                                          float* smem, int wave) {
  constexpr int NB = D / 16, NT = NB * (NB + 1) / 2, TRI = light_wave_lds(D), NHC = KP / 64;
  constexpr bool TWO = D > 64;  // two entries per lane
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  float* Ks = smem + wave * TRI;
  float ce = 0.f, we = 0.f, ce2 = 0.f, we2 = 0.f;
  if (lane < d) rating_weights(r, a.implicit, a.alpha, ce, we);
  if (TWO && 64 + lane < d) rating_weights(r2, a.implicit, a.alpha, ce2, we2);
  const bool valid = lane < d && ce > 0.f;
  const bool valid2 = TWO && 64 + lane < d && ce2 > 0.f;
  const int npos = a.implicit ? __popcll(__ballot(lane < d && r > 0.f)) + (TWO ? __popcll(__ballot(64 + lane < d && r2 > 0.f)) : 0)
                              : d;
  const float lamn = a.reg * (float)npos;

  int colB[NB];
  bool vB[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    colB[I] = __shfl(I < 4 ? colE : colE2, 16 * (I & 3) + i16);
    vB[I] = __shfl((int)(I < 4 ? valid : valid2), 16 * (I & 3) + i16) != 0;
  }
  constexpr int NC = KP / 16;
  constexpr bool KEEPZ = D <= 32 && D * KP <= 4096;  // keep the gathered rows in registers for x' (D = 64 at KP = 128, 2 waves per SIMD: measured slower)
  f32x4 zf[KEEPZ ? NB : 1][KEEPZ ? NC : 1];
  if constexpr (KEEPZ) {  // issue every gather up front: one latency for the whole row
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
      for (int c = 0; c < NC; ++c) zf[I][c] = vB[I] ? ld4(a.Z + (int64_t)colB[I] * KP + 16 * c + 4 * g) : zero4();
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  // D^-1/2 of the row, one rsq per column (lane c, c+64, ...) into this wave's LDS slot
  float* sdl = smem + 4 * TRI + wave * KP;
  bool bad = false;
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    const int cc = lane + 64 * h;
    const float dd = a.lam[cc] + lamn;
    if (cc < a.kreal && !(dd > 0.f)) bad = true;
    sdl[cc] = (cc < a.kreal && dd > 0.f) ? frsq(dd) : 0.f;
  }
  WAVE_LDS_SYNC();
  if constexpr (D >= 64 || KEEPZ) {
    // S on split-fp16 MFMA (hi·hi + hi·lo + lo·hi, 32 columns per instruction: at D = 64 120 instead
    // of 320 fp32 MFMAs, at D = 16 12 x 16 cycles instead of 32 x 32).  One power-of-two scale for the
    // whole row (so S unscales exactly): |Z[.][c]| < 2^(13 - e_c) (colscale), hence
    // |z_c · sd_c| <= max_c sd_c · 2^(13 - e_c).  With the gathered rows in registers (KEEPZ) the
    // 32-deep k-slots of block q take columns 16(2q) + 4g .. +3 and 16(2q+1) + 4g .. +3: both MFMA
    // operands are Zs, so any column-to-slot assignment gives the same S.
    float bnd = 0.f;
#pragma unroll
    for (int h = 0; h < NHC; ++h) {
      const int cc = lane + 64 * h;
      bnd = fmaxf(bnd, sdl[cc] * a.colscale[KP + cc]);
    }
    bnd = wave_max_dpp(bnd);
    int ex = 0;
    frexpf(bnd * 8192.f, &ex);  // bnd·2^13 < 2^ex
    const float sc = ldexpf(1.f, 13 - ex), usc = ldexpf(1.f, 2 * (ex - 13));
    constexpr int NQ = KP / 32;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4 s0 = KEEPZ ? ld4(sdl + 32 * q + 4 * g) : ld4(sdl + 32 * q + 8 * g);
      const f32x4 s1 = KEEPZ ? ld4(sdl + 32 * q + 16 + 4 * g) : ld4(sdl + 32 * q + 8 * g + 4);
      f16x8 zh[NB], zl[NB];
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        f32x4 v0, v1;
        if constexpr (KEEPZ) {
          v0 = zf[I][2 * q];
          v1 = zf[I][2 * q + 1];
        } else {
          const float* zp = a.Z + (int64_t)colB[I] * KP + 32 * q + 8 * g;
          v0 = vB[I] ? ld4(zp) : zero4();
          v1 = vB[I] ? ld4(zp + 4) : zero4();
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = (e < 4 ? v0[e] * s0[e] : v1[e - 4] * s1[e - 4]) * sc;
          asm("" : "+v"(v));  // one fp32 rounding; hi and lo from that value (see lds_put)
          const _Float16 hv = (_Float16)v;
          zh[I][e] = hv;
          zl[I][e] = (_Float16)(v - (float)hv);
        }
      }
      static_for<0, NT>([&](auto t) {
        constexpr TilePair p = upper_tile(decltype(t)::value, NB);
        acc[t] = mfma_h(zh[p.a], zh[p.b], acc[t]);
        acc[t] = mfma_h(zh[p.a], zl[p.b], acc[t]);
        acc[t] = mfma_h(zl[p.a], zh[p.b], acc[t]);
      });
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] *= usc;
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int c0 = 16 * c;
      const f32x4 sd = ld4(sdl + c0 + 4 * g);
      f32x4 z[NB];
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        if constexpr (KEEPZ) z[I] = zf[I][c];
        else z[I] = vB[I] ? ld4(a.Z + (int64_t)colB[I] * KP + c0 + 4 * g) : zero4();
#pragma unroll
        for (int m = 0; m < 4; ++m) z[I][m] *= sd[m];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        static_for<0, NT>([&](auto t) {
          constexpr TilePair p = upper_tile(decltype(t)::value, NB);
          acc[t] = mfma4(z[p.a][m], z[p.b][m], acc[t]);
        });
      }
    }
  }
  if (__any(bad) && lane == 0) atomicOr(a.err, 1);
  const float cinv = valid ? frcp(ce) : 0.f;
  const float cinv2 = valid2 ? frcp(ce2) : 0.f;
  float y, y2 = 0.f;  // lane e < d: v_e on return (y2: v_{64+e})
  if constexpr (D == 16) {  // register Cholesky, lane i = row i, DPP broadcasts
    // S -> LDS (only the lower triangle is read by the Cholesky below)
    static_for<0, NT>([&](auto t) {
      constexpr TilePair p = upper_tile(decltype(t)::value, NB);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * p.a + 4 * g + rr, cl = 16 * p.b + i16;  // p.a <= p.b: cl >= row off the diagonal
        Ks[(p.a < p.b || cl >= row) ? cl * (cl + 1) / 2 + row : TRI - 64 + lane] = acc[t][rr];  // else: sink
      }
    });
    WAVE_LDS_SYNC();
    const int me = lane < D ? lane : 0;
    float kr[D];
#pragma unroll
    for (int m = 0; m < D; ++m) {
      const float v = Ks[me * (me + 1) / 2 + m];  // in bounds for m > me too (unused entries)
      kr[m] = (m == me) ? (valid ? v + cinv : 1.0f) : (valid ? v : 0.0f);
    }
    // Cholesky K = L Lᵀ, lane i holds row i (entries m <= i are L[i][m] when done); then the forward
    // substitution L y = C⁻¹ w; broadcasts of lane c by DPP row_newbcast (rows 0..15 sit in lanes
    // 0..15; the other 16-lane rows broadcast their own unused copies)
    bool notpd = false;
    float dg = 1.f;  // 1 / L[me][me]
    y = valid ? we * cinv : 0.f;
    // rows c >= d are identity rows (and y_c = 0): their steps change nothing and are skipped
    static_for<0, D>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if (c >= d) return;
      const float piv = bc16_after_asm<c>(kr[c]);
      if (!(piv > 0.f)) notpd = true;
      const float inv = frsq(piv), s = piv * inv;
      kr[c] = (me == c) ? s : kr[c] * inv;
      dg = (me == c) ? inv : dg;
      static_for<c + 1, D>([&](auto mm) {
        constexpr int m = decltype(mm)::value;
        fnmac_bc16<m, m == c + 1>(kr[m], kr[c], kr[c]);
      });
    });
    static_for<0, D>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if (c >= d) return;
      const float yc = bc16<c>(y * dg);
      y = (me > c) ? fmaf(-kr[c], yc, y) : ((me == c) ? yc : y);
    });
    if (notpd && lane == 0) atomicOr(a.err, 2 | ALBEDO_EF_LIGHT_REG);
    // transpose L through LDS: lane i gets column i (lt[m] = L[m][i])
    WAVE_LDS_SYNC();
    if (lane < D) {
#pragma unroll
      for (int m = 0; m < D; ++m) Ks[m <= lane ? lane * (lane + 1) / 2 + m : TRI - 64 + lane] = kr[m];
    }
    WAVE_LDS_SYNC();
    float lt[D];
#pragma unroll
    for (int m = 0; m < D; ++m) lt[m] = Ks[m * (m + 1) / 2 + me];  // L[m][me] (m >= me used)
    // backward: Lᵀ v = y
    static_for<0, D>([&](auto cc) {
      constexpr int c = D - 1 - decltype(cc)::value;
      if (c >= d) return;
      const float vc = bc16<c>(y * dg);
      y = (me < c) ? fmaf(-lt[c], vc, y) : ((me == c) ? vc : y);
    });
  } else {
    // K = S + C⁻¹ (identity rows for masked entries), factored in the accumulators (wave_chol.h):
    // the diagonal of tile (A, A) sits in lane i + 16q, slot r with 4q + r == i
    const float dadd = valid ? cinv : 1.0f, rhs = valid ? we * cinv : 0.f;
    const float dadd2 = valid2 ? cinv2 : 1.0f, rhs2 = valid2 ? we2 * cinv2 : 0.f;
    float bacc[NB];
    static_for<0, NB>([&](auto AA) {
      constexpr int A = decltype(AA)::value, t = tix(A, A, NB);
      const float dA = __shfl(A < 4 ? dadd : dadd2, 16 * (A & 3) + i16);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r == i16) acc[t][r] += dA;
      bacc[A] = __shfl(A < 4 ? rhs : rhs2, 16 * (A & 3) + i16);
    });
    float xs[NB];
    const bool notpd = wave_chol_solve<NB>(acc, bacc, Ks, xs);
    if (notpd && lane == 0) atomicOr(a.err, 2 | ALBEDO_EF_LIGHT_ACC);
    y = 0.f;  // lane 16A + i holds v[16A + i] = xs[A] (its own slot A = g); y2: v[64 + 16A + i]
#pragma unroll
    for (int A = 0; A < NB; ++A) {
      if (A < 4) y = g == A ? xs[A] : y;
      else y2 = g == A - 4 ? xs[A] : y2;
    }
  }
  // x' = D⁻¹ Zᵀ v
  if constexpr (KEEPZ) {
    // lane (i16, g) holds Z[entry 16I+i16][16c+4g+m]: scale by v, sum over I in-lane and over the
    // 16 entry lanes of its group by xor-shuffles, lane i16 == 0 of each group stores 4 columns
    float vI[NB];
#pragma unroll
    for (int I = 0; I < NB; ++I) vI[I] = __shfl(y, 16 * I + i16);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x4 pr = zf[0][c] * vI[0];
#pragma unroll
      for (int I = 1; I < NB; ++I) pr += zf[I][c] * vI[I];
#pragma unroll
      for (int m = 0; m < 4; ++m) pr[m] = sum16_last(pr[m]);
      if (i16 == 15) {  // D^-1 = (D^-1/2)^2 (zero on padded / invalid columns)
        const f32x4 sd = ld4(sdl + 16 * c + 4 * g);
        *reinterpret_cast<f32x4*>(a.X + (int64_t)j * KP + 16 * c + 4 * g) = pr * (sd * sd);
      }
    }
  } else {
    // lanes own columns lane + 64h; gathers issued 8 entries at a time
    float xacc[NHC];
#pragma unroll
    for (int h = 0; h < NHC; ++h) xacc[h] = 0.f;
    for (int e0 = 0; e0 < d; e0 += 8) {
      float ve[8], zz[8][NHC];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u < d ? e0 + u : d - 1;  // wave-uniform
        const bool hi = TWO && e >= 64;
        ve[u] = e0 + u < d ? rdlane(hi ? y2 : y, e & 63) : 0.f;
        const float* zr = a.Z + (int64_t)rdlane_i(hi ? colE2 : colE, e & 63) * KP + lane;
#pragma unroll
        for (int h = 0; h < NHC; ++h) zz[u][h] = zr[64 * h];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int h = 0; h < NHC; ++h) xacc[h] = fmaf(ve[u], zz[u][h], xacc[h]);
    }
#pragma unroll
    for (int h = 0; h < NHC; ++h) {
      const int c = lane + 64 * h;
      const float sd = sdl[c];
      a.X[(int64_t)j * KP + c] = xacc[h] * (sd * sd);
    }
  }
}

// One wave per row; the row's descriptor {row, p0, degree} is one scalar load (a.desc) instead of
// the dependent rows -> ptr pair.  (A persistent, prefetching variant of this kernel measured slower
// at c4: its scratch spills and conservative waits serialised the gathers; light16.hip has it.)
template <int KP, int D>
__global__ __launch_bounds__(256, (light_occupancy<KP, D>())) void solve_light_kernel(SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ridx = (int64_t)blockIdx.x * 4 + wave;
  if (ridx >= a.n_rows) return;  // wave-uniform; this kernel has no workgroup barrier
  typedef __attribute__((address_space(4))) const int cint;
  cint* q = (cint*)(a.desc) + 4 * ridx;  // constant address space: s_load_dwordx4
  const int j = q[0], d = q[3];
  const int64_t p0 = (int64_t)(uint32_t)q[1] | ((int64_t)q[2] << 32);
  float r = 0.f, r2 = 0.f;
  int colE = 0, colE2 = 0;
  if (lane < d) {
    r = a.val[p0 + lane];
    colE = a.col[p0 + lane];
  }
  if (D > 64 && 64 + lane < d) {
    r2 = a.val[p0 + 64 + lane];
    colE2 = a.col[p0 + 64 + lane];
  }
  light_row<KP, D>(a, j, d, r, colE, r2, colE2, smem, wave);
}

hipError_t launch_solve_light(int KP, int D, const SolveArgs& a0, hipStream_t s) {
  if (a0.n_rows <= 0) return hipSuccess;
  if (!a0.desc) return hipErrorInvalidValue;
  if (a0.n_rows > max_rows_per_launch(64)) {  // 64 work-items per row: see max_rows_per_launch
    for (int64_t r0 = 0; r0 < a0.n_rows; r0 += max_rows_per_launch(64)) {
      SolveArgs b = chunk_args(a0, r0, 64, 0);
      b.desc = a0.desc + 4 * r0;
      const hipError_t e = launch_solve_light(KP, D, b, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const SolveArgs& a = a0;
  const size_t lds = ((size_t)4 * light_wave_lds(D) + (size_t)4 * KP) * sizeof(float);  // per-wave K / scratch + D^-1/2
  const int blocks = (int)((a.n_rows + 3) / 4);
#define LIGHT(kp, dd) \
  if (KP == kp && D == dd) { solve_light_kernel<kp, dd><<<blocks, 256, lds, s>>>(a); return hipGetLastError(); }
  LIGHT(64, 16) LIGHT(64, 32) LIGHT(64, 64) LIGHT(128, 16) LIGHT(128, 32) LIGHT(128, 64)
  LIGHT(256, 16) LIGHT(256, 32) LIGHT(256, 64) LIGHT(128, 96)
#undef LIGHT
  return hipErrorInvalidValue;
}

// =============================================================================================
// Heavy rows: explicit A' = diag(Λ + λn) + Σ c z zᵀ, b' = Σ w z, then Cholesky + substitutions.
// One workgroup per dst row: 4 waves for KP <= 128 (4 workgroups per CU, <= 40 KiB of LDS each),
// 16 waves for KP = 256 (one workgroup per CU, 150 KiB).
//  build   the row's Z rows are gathered SPS at a time into registers (double-buffered LDS),
//          scaled by √c and a per-column power of two (colscale: max |√c z| < 2^13), split into
//          fp16 hi + lo parts and written COLUMN-major into two LDS images (xor-swizzled 16-B
//          units, conflict-free fragment reads).  Each wave owns the upper 16x16 tiles of one
//          pair of column-block groups and accumulates hi·hi + hi·lo + lo·hi with
//          v_mfma_f32_16x16x32_f16 (32 ratings per MFMA, fp32 accumulation).  The split keeps
//          22 significant bits and the dropped lo·lo term is 2^-22 relative, i.e. fp32-level
//          products at 16/3 = 5.3x the fp32-MFMA rate.  b' = Σ w z is accumulated in fp32 from
//          the raw rows.
//  store   tiles are unscaled (exact powers of two) into packed lower-triangular 16x17 fp32 tiles
//          (the stage is dead by then).
//  factor  right-looking, 16-wide panels, two barriers per panel: the waves that own panel rows
//          factor the 16x16 diagonal tile redundantly in registers and solve their rows against
//          it with wave-uniform (SGPR) broadcasts of L11; the trailing update runs on fp32 MFMA.
//          b' is carried as an extra row, so the forward substitution comes for free.
//  back    Lᵀx = y by one wave, no barriers.
// =============================================================================================


template <int KP>
struct Heavy {
  static constexpr int NW = KP >= 256 ? 16 : 4, NTH = 64 * NW, NQ = KP / 16;
  static constexpr int SPS = KP >= 256 ? 64 : 32;  // ratings per LDS stage
  static constexpr int NU = SPS / 8;                // 16-B units per image column row
  static constexpr int CS = 2 * SPS;                // bytes per image column row
  static constexpr int IMG = KP * CS;               // bytes per image (4 images: 2 buffers x hi/lo)
  static constexpr int NCH = KP / 4, NSG = NTH / NCH, NST = SPS / NSG;  // staging map
  static constexpr bool PERM = KP != 256;           // xor-permuted column order of the image writes
  static constexpr int SWZ = NU == 4 ? 3 : 5;
  static constexpr int GS = KP == 64 ? 2 : 4, NG = NQ / GS;  // column-block groups; wave = group pair
  static constexpr int NTL = NQ * (NQ + 1) / 2;
  static constexpr int TILES = NTL * HT_SZ, STAGE = IMG;      // floats
  static constexpr int BIG = TILES > STAGE ? TILES : STAGE;
  static constexpr int OFF_B = BIG, OFF_DIAG = OFF_B + KP, OFF_FLAG = OFF_DIAG + KP;
  static constexpr int FLOATS = OFF_FLAG + 4;
  static_assert(NG * NG == NW, "one wave per group pair");
  static_assert(NSG * NCH == NTH && NST * NSG == SPS && (NST == 2 || NST == 4), "stage map");
  static_assert(NSG * KP <= STAGE, "b partials fit into the dead stage");
};

// byte offset of (column, byte within the column's SPS ratings) in one image
template <int KP>
__device__ __forceinline__ int img_off(int col, int byteoff) {
  using H = Heavy<KP>;
  const int sw = (col ^ (H::SWZ * (col >> 3))) & (H::NU - 1);
  return col * H::CS + ((((byteoff >> 4) ^ sw) & (H::NU - 1)) << 4) + (byteoff & 15);
}

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  f16x2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, h);
}

// Build of the row's A' tiles owned by this wave: row blocks rb .. rb+NR-1, column blocks
// cb .. cb+GS-1 (DIAG: the same blocks, upper tiles only).
template <int KP, bool DIAG, bool NT = false>
__device__ __forceinline__ void heavy_build(const SolveArgs& a, int64_t p0, int d, float* smem, int rb, int cb) {
  using H = Heavy<KP>;
  constexpr int NR = DIAG ? H::GS : H::GS / 2, NC = H::GS, NST = H::NST;
  constexpr int MT = DIAG ? NR * (NR + 1) / 2 : NR * NC;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i16 = lane & 15;
  char* lds = reinterpret_cast<char*>(smem);
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);
  const int cc = tid % H::NCH, sg = tid / H::NCH;
  const int xr = H::PERM ? (cc & 3) : 0;
  const f32x4 csc = ld4(a.colscale + 4 * cc);
  f32x4 bp = zero4();
  int npos = 0;
  f32x4 zr[NST];
  float sq[NST], wv[NST];
  // loads are unconditional (index clamped to the row's last rating, d >= 1); ratings past the
  // end get zero weight, so they add nothing to A' or b'.  Software pipeline: the (col, val) of
  // stage st+2 are loaded while the Z rows of stage st+1 are in flight and stage st is on MFMA,
  // so each stage waits for one HBM latency, not for the dependent index -> row pair.
  int ci[NST];
  float rv[NST];
  bool in[NST];
  auto iload = [&](int e0) {
#pragma unroll
    for (int m = 0; m < NST; ++m) {
      const int e = e0 + sg * NST + m;
      in[m] = e < d;
      const int64_t pe = p0 + (in[m] ? e : d - 1);
      ci[m] = a.col[pe];
      rv[m] = a.val[pe];
    }
  };
  auto zload = [&]() {
#pragma unroll
    for (int m = 0; m < NST; ++m) zr[m] = ld4(a.Z + (int64_t)ci[m] * KP + 4 * cc);
#pragma unroll
    for (int m = 0; m < NST; ++m) {
      float c = 0.f, w = 0.f;
      rating_weights(rv[m], a.implicit, a.alpha, c, w);
      sq[m] = in[m] ? sqrtf(c) : 0.f;
      wv[m] = in[m] ? w : 0.f;
      npos += (cc == 0 && in[m] && rv[m] > 0.f) ? 1 : 0;
    }
  };
  using PW = typename std::conditional<NST == 4, u32x2, uint32_t>::type;  // NST halves of one column
  auto lds_put = [&](int buf) {
    char* himg = lds + (2 * buf) * H::IMG;
    char* limg = himg + H::IMG;
#pragma unroll
    for (int m = 0; m < NST; ++m) bp += zr[m] * wv[m];
    PW hp0, hp1, hp2, hp3, lp0, lp1, lp2, lp3;
    static_for<0, 4>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      PW hv, lv;
      static_for<0, NST / 2>([&](auto mc) {
        constexpr int m2 = decltype(mc)::value;
        float v0 = zr[2 * m2][q] * (sq[2 * m2] * csc[q]);
        float v1 = zr[2 * m2 + 1][q] * (sq[2 * m2 + 1] * csc[q]);
        // v is rounded to fp32 ONCE and both hi and lo derive from that register: left alone, the
        // compiler folds fp16(a·b) into v_fma_mix (rounding the exact product) for lo's hi while
        // the stored hi rounds the fp32 product; the two disagree at fp16 ties (lo then misses
        // one fp16 ulp of hi, a 2^-11 error on that element)
        asm("" : "+v"(v0), "+v"(v1));
        const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
        const uint32_t hw = pack_h2(h0, h1), lw = pack_h2(v0 - (float)h0, v1 - (float)h1);
        if constexpr (NST == 4) { hv[m2] = hw; lv[m2] = lw; } else { hv = hw; lv = lw; }
      });
      if constexpr (q == 0) { hp0 = hv; lp0 = lv; }
      if constexpr (q == 1) { hp1 = hv; lp1 = lv; }
      if constexpr (q == 2) { hp2 = hv; lp2 = lv; }
      if constexpr (q == 3) { hp3 = hv; lp3 = lv; }
    });
    if constexpr (H::PERM) {  // slot i holds column 4cc + (i ^ xr): spreads the banks of the writes
      const bool b0 = xr & 1, b1 = xr & 2;
      const PW h0 = b0 ? hp1 : hp0, h1 = b0 ? hp0 : hp1, h2 = b0 ? hp3 : hp2, h3 = b0 ? hp2 : hp3;
      const PW l0 = b0 ? lp1 : lp0, l1 = b0 ? lp0 : lp1, l2 = b0 ? lp3 : lp2, l3 = b0 ? lp2 : lp3;
      hp0 = b1 ? h2 : h0; hp1 = b1 ? h3 : h1; hp2 = b1 ? h0 : h2; hp3 = b1 ? h1 : h3;
      lp0 = b1 ? l2 : l0; lp1 = b1 ? l3 : l1; lp2 = b1 ? l0 : l2; lp3 = b1 ? l1 : l3;
    }
    const int boff = 2 * NST * sg;
    *reinterpret_cast<PW*>(himg + img_off<KP>(4 * cc + (0 ^ xr), boff)) = hp0;
    *reinterpret_cast<PW*>(limg + img_off<KP>(4 * cc + (0 ^ xr), boff)) = lp0;
    *reinterpret_cast<PW*>(himg + img_off<KP>(4 * cc + (1 ^ xr), boff)) = hp1;
    *reinterpret_cast<PW*>(limg + img_off<KP>(4 * cc + (1 ^ xr), boff)) = lp1;
    *reinterpret_cast<PW*>(himg + img_off<KP>(4 * cc + (2 ^ xr), boff)) = hp2;
    *reinterpret_cast<PW*>(limg + img_off<KP>(4 * cc + (2 ^ xr), boff)) = lp2;
    *reinterpret_cast<PW*>(himg + img_off<KP>(4 * cc + (3 ^ xr), boff)) = hp3;
    *reinterpret_cast<PW*>(limg + img_off<KP>(4 * cc + (3 ^ xr), boff)) = lp3;
  };
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = zero4();
  const int nst = (d + H::SPS - 1) / H::SPS;
  iload(0);
  zload();
  if (nst > 1) iload(H::SPS);
  lds_put(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) {
      zload();
      if (st + 2 < nst) iload((st + 2) * H::SPS);
    }
    const char* himg = lds + (2 * buf) * H::IMG;
    const char* limg = himg + H::IMG;
#pragma unroll
    for (int ks = 0; ks < H::SPS / 32; ++ks) {
      f16x8 rh[NR], rl[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int off = img_off<KP>(16 * (rb + i) + i16, 64 * ks + 16 * g);
        rh[i] = *reinterpret_cast<const f16x8*>(himg + off);
        rl[i] = *reinterpret_cast<const f16x8*>(limg + off);
      }
      if constexpr (DIAG) {  // column blocks = row blocks
        int t = 0;
#pragma unroll
        for (int i = 0; i < NR; ++i)
#pragma unroll
          for (int j = i; j < NC; ++j, ++t) {
            acc[t] = mfma_h(rh[i], rh[j], acc[t]);
            acc[t] = mfma_h(rh[i], rl[j], acc[t]);
            acc[t] = mfma_h(rl[i], rh[j], acc[t]);
          }
      } else {  // one column block at a time (register pressure)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const int off = img_off<KP>(16 * (cb + j) + i16, 64 * ks + 16 * g);
          const f16x8 ch = *reinterpret_cast<const f16x8*>(himg + off);
          const f16x8 cl = *reinterpret_cast<const f16x8*>(limg + off);
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            const int t = i * NC + j;
            acc[t] = mfma_h(rh[i], ch, acc[t]);
            acc[t] = mfma_h(rh[i], cl, acc[t]);
            acc[t] = mfma_h(rl[i], ch, acc[t]);
          }
        }
      }
    }
    if (st + 1 < nst) lds_put(buf ^ 1);
    __syncthreads();
  }
  // b' partials into the dead stage, reduced in a fixed order by the first KP threads
  *reinterpret_cast<f32x4*>(smem + sg * KP + 4 * cc) = bp;
  if (npos) atomicAdd(&s_flag[0], npos);
  __syncthreads();
  if (tid < KP) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < H::NSG; ++q) s += smem[q * KP + tid];
    smem[H::OFF_B + tid] = s;
  }
  __syncthreads();
  // tiles -> packed lower LDS tiles, unscaled (powers of two: exact)
  const float* isc = a.colscale + KP;
  int t = 0;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const f32x4 ir = ld4(isc + 16 * (rb + i) + 4 * g);
#pragma unroll
    for (int j = DIAG ? i : 0; j < NC; ++j, ++t) {
      const float ic = isc[16 * (cb + j) + i16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c1 = 16 * (rb + i) + 4 * g + r, c2 = 16 * (cb + j) + i16;
        const float v = acc[t][r] * ir[r] * ic;
        if constexpr (NT) {  // NNLS layout: diagonal tiles full
          smem[c1 >= c2 ? nel(c1, c2) : nel(c2, c1)] = v;
          if (DIAG && i == j) smem[nel(c2, c1)] = v;
        } else if (!DIAG || i != j || c1 >= c2) {
          smem[c1 >= c2 ? hel(c1, c2) : hel(c2, c1)] = v;
        }
      }
    }
  }
}

// Dispatch of the build over the waves: waves 0..NG-1 own the diagonal group pairs, the rest
// split each off-diagonal group pair (gi < gj) into two halves of its row blocks.
template <int KP, bool NT = false>
__device__ __forceinline__ void heavy_build_all(const SolveArgs& a, int64_t p0, int d, float* smem) {
  using H = Heavy<KP>;
  const int wave = threadIdx.x >> 6;
  if (wave < H::NG) {
    heavy_build<KP, true, NT>(a, p0, d, smem, wave * H::GS, wave * H::GS);
  } else {
    const int idx = wave - H::NG, pair = idx >> 1, half = idx & 1;
    int gi = 0, gj = 1;
    for (int p = 0; p < pair; ++p)
      if (++gj == H::NG) { ++gi; gj = gi + 1; }
    heavy_build<KP, false, NT>(a, p0, d, smem, gi * H::GS + half * (H::GS / 2), gj * H::GS);
  }
  __syncthreads();
}

// ---- split-K records (kernels.h SplitArgs): packed A' tiles | b' | positive-rating count ------
int split_rec_floats(int KP) {
  return KP == 64 ? SplitRec<64>::FLOATS : KP == 128 ? SplitRec<128>::FLOATS : SplitRec<256>::FLOATS;
}

// Element e of the packed lower tiles holds a matrix entry (not the pad column, not above the
// diagonal of a diagonal tile): only those are written / summed, so stale stage bytes never travel.
__device__ __forceinline__ bool tile_elem_valid(int e) {
  const int t = e / HT_SZ, w = e - t * HT_SZ, r = w / HT_LD, c = w - r * HT_LD;
  int I = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  return c < 16 && (J < I || c <= r);
}

// Reduced record -> the LDS image heavy_build_all leaves behind (tiles at 0, b' at OFF_B, npos).
template <int KP>
__device__ __forceinline__ void heavy_load_record(const float* __restrict__ rec, float* smem) {
  using H = Heavy<KP>;
  using R = SplitRec<KP>;
  for (int e = 4 * (int)threadIdx.x; e < R::TILES; e += 4 * H::NTH)
    *reinterpret_cast<f32x4*>(smem + e) = ld4(rec + e);
  for (int c = threadIdx.x; c < KP; c += H::NTH) smem[H::OFF_B + c] = rec[R::OFF_B + c];
  if (threadIdx.x == 0) reinterpret_cast<int*>(smem + H::OFF_FLAG)[0] = reinterpret_cast<const int*>(rec)[R::OFF_N];
  __syncthreads();
}

// One workgroup per chunk: the heavy build of chunk_len ratings of one row -> fp32 partial record.
template <int KP>
__global__ __launch_bounds__(Heavy<KP>::NTH, 4) void heavy_partial_kernel(SolveArgs a, SplitArgs s) {
  using H = Heavy<KP>;
  using R = SplitRec<KP>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);
  const int tid = threadIdx.x;
  const int64_t slot = blockIdx.x;
  const int j = s.chunk_row[slot];
  const int64_t rp0 = a.ptr[j], off = (int64_t)s.chunk_idx[slot] * s.chunk_len;
  const int64_t rest = a.ptr[j + 1] - rp0 - off;
  const int d = (int)(rest < s.chunk_len ? rest : s.chunk_len);  // >= 1: chunks cover the row
  if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; }
  heavy_build_all<KP>(a, rp0 + off, d, smem);
  float* out = s.partial + slot * R::FLOATS;
  for (int e = tid; e < R::TILES; e += H::NTH) out[e] = tile_elem_valid(e) ? smem[e] : 0.f;
  for (int c = tid; c < KP; c += H::NTH) out[R::OFF_B + c] = smem[H::OFF_B + c];
  if (tid == 0) reinterpret_cast<int*>(out)[R::OFF_N] = s_flag[0];
}

// Reduced record element e of split row r = Σ over the row's chunks (fp64, chunk order).
template <int KP>
__global__ __launch_bounds__(256) void heavy_reduce_kernel(SplitArgs s) {
  using R = SplitRec<KP>;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e > R::OFF_N) return;
  for (int64_t r = blockIdx.y; r < s.n_split; r += gridDim.y) {
    const int q0 = s.slot0[r], q1 = s.slot0[r + 1];
    float* out = s.reduced + r * R::FLOATS;
    if (e == R::OFF_N) {
      int n = 0;
      for (int q = q0; q < q1; ++q) n += reinterpret_cast<const int*>(s.partial + (int64_t)q * R::FLOATS)[R::OFF_N];
      reinterpret_cast<int*>(out)[R::OFF_N] = n;
    } else {
      double acc = 0.0;
      for (int q = q0; q < q1; ++q) acc += (double)s.partial[(int64_t)q * R::FLOATS + e];
      out[e] = (float)acc;
    }
  }
}

template <int KP>
hipError_t launch_split_kp(const SolveArgs& a, const SplitArgs& s, bool wave, hipStream_t st) {
  using R = SplitRec<KP>;
  if (wave && KP <= 128) {
    const hipError_t e = launch_wave_partial(KP, a, s, st);
    if (e != hipSuccess) return e;
  } else {
    const size_t lds = Heavy<KP>::FLOATS * 4;
    static const hipError_t attr = allow_lds(heavy_partial_kernel<KP>, lds);
    if (attr != hipSuccess) return attr;
    heavy_partial_kernel<KP><<<(int)s.n_chunks, Heavy<KP>::NTH, lds, st>>>(a, s);
  }
  const int gy = (int)(s.n_split < 65535 ? s.n_split : 65535);
  heavy_reduce_kernel<KP><<<dim3((R::OFF_N + 1 + 255) / 256, gy), 256, 0, st>>>(s);
  return hipGetLastError();
}

hipError_t launch_heavy_split(int KP, const SolveArgs& a, const SplitArgs& s, bool wave, hipStream_t st) {
  if (s.n_chunks <= 0 || s.n_split <= 0) return hipSuccess;
  if (KP == 64) return launch_split_kp<64>(a, s, wave, st);
  if (KP == 128) return launch_split_kp<128>(a, s, wave, st);
  if (KP == 256) return launch_split_kp<256>(a, s, wave, st);
  return hipErrorInvalidValue;
}

// PH: phase mask for profiling probes (bit 0 build, bit 1 factor + substitution); the engine runs 3.
template <int KP, int PH = 3, bool PRE = false>
__global__ __launch_bounds__(Heavy<KP>::NTH, 4) void solve_heavy_kernel(SolveArgs a) {
  using H = Heavy<KP>;
  constexpr int NB = KP / 16, NTH = H::NTH, NW = H::NW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* bvec = smem + H::OFF_B;
  float* sdiag = smem + H::OFF_DIAG;
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);  // [0] npos, [1] error bits
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, i16 = lane & 15;
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; }
  HEAVY_TS(0);
  if constexpr (PRE) {  // split row: A' / b' / npos reduced from the chunk partials
    heavy_load_record<KP>(a.prebuilt + (size_t)blockIdx.x * SplitRec<KP>::FLOATS, smem);
  } else if constexpr (PH & 1) {
    heavy_build_all<KP>(a, p0, d, smem);
  } else {
    for (int e = tid; e < H::OFF_DIAG; e += NTH) smem[e] = 0.f;
    __syncthreads();
  }
  if constexpr (!(PH & 2)) {
    for (int c = tid; c < KP; c += NTH) a.X[(int64_t)j * KP + c] = smem[H::OFF_B + c] + smem[hel(c, c)];
    return;
  }
  HEAVY_TS(1);
  const float lamn = a.reg * (float)(a.implicit ? s_flag[0] : d);
  for (int c = tid; c < KP; c += NTH) smem[hel(c, c)] += c < a.kreal ? a.lam[c] + lamn : 1.0f;
  __syncthreads();
  // Blocked right-looking Cholesky, 16-wide panels, look-ahead, two barriers per panel:
  //  A  all waves: TRSM of the rows below the panel (and b') against L11, broadcast LDS reads
  //  B  wave 0: update + factor the next diagonal tile (chol16); waves 1..: the rest of the
  //     trailing update on MFMA and the b' update
  // Diagonal tiles are re-laid as L11ᵀ in a 16-float row layout (row c = column c of L11, zero
  // above the diagonal; tile starts are 16-B aligned) for the TRSM and the back substitution.
  auto diag_factor = [&](int jb) {  // wave 0
    float* t = smem + htile(jb, jb);
    float rr[16], dg = 1.f;
#pragma unroll
    for (int m = 0; m < 16; ++m) rr[m] = t[i16 * HT_LD + m];
    const bool np = chol16(rr, dg, i16);
    WAVE_LDS_SYNC();
    if (lane < 16) {
#pragma unroll
      for (int c = 0; c < 16; ++c) t[c * 16 + i16] = c <= i16 ? rr[c] : 0.f;
      sdiag[16 * jb + i16] = dg;
    }
    if (np && lane == 0) s_flag[1] = 2 | ALBEDO_EF_HEAVY;
  };
  // C(I,M) -= L(I,jb) L(M,jb)ᵀ on MFMA (packed lower 16x17 tiles)
  auto tile_update = [&](int jb, int I, int M) {
    float* ct = smem + htile(I, M);
    const float* at = smem + htile(I, jb) + i16 * HT_LD + g;
    const float* bt = smem + htile(M, jb) + i16 * HT_LD + g;
    f32x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = ct[(4 * g + r) * HT_LD + i16];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = mfma4(-at[4 * s4], bt[4 * s4], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) ct[(4 * g + r) * HT_LD + i16] = acc[r];
  };
  if (wave == 0) diag_factor(0);
  __syncthreads();
  HEAVY_TS(2);
  for (int jb = 0; jb < NB; ++jb) {
    const int j0 = 16 * jb, nrem = NB - 1 - jb;
    // ---- A
    {
      const int ridx = tid, nrow = KP - j0 - 16 + 1;  // rows below the panel + the b' row
      if (ridx < nrow) {
        const int i = j0 + 16 + ridx;
        float* src = i < KP ? smem + htile(i >> 4, jb) + (i & 15) * HT_LD : bvec + j0;
        const float* lt = smem + htile(jb, jb);
        float x[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = src[m];
        f32x4 dv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) dv[q] = ld4(sdiag + j0 + 4 * q);
        static_for<0, 16>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          x[c] *= dv[c >> 2][c & 3];
          static_for<(c + 1) / 4, 4>([&](auto qq) {
            constexpr int q = decltype(qq)::value;
            const f32x4 l = ld4(lt + 16 * c + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (4 * q + e > c) x[4 * q + e] = fmaf(-x[c], l[e], x[4 * q + e]);
          });
          if constexpr ((c & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound the hoisted loads
        });
#pragma unroll
        for (int m = 0; m < 16; ++m) src[m] = x[m];
      }
    }
    __syncthreads();
    // ---- B
    if (wave == 0) {
      if (nrem > 0) {
        tile_update(jb, jb + 1, jb + 1);
        WAVE_LDS_SYNC();
        diag_factor(jb + 1);
      }
    } else if (nrem > 0) {
      const int ntr = nrem * (nrem + 1) / 2;
      for (int t = wave; t < ntr; t += NW - 1) {
        int ti = 0, tt = t;  // lower tiles (I >= M) row-major; t = 0 is the next diagonal tile
        while (tt > ti) { tt -= ti + 1; ++ti; }
        tile_update(jb, jb + 1 + ti, jb + 1 + tt);
      }
      for (int m = j0 + 16 + tid - 64; m < KP; m += NTH - 64) {
        float sv = bvec[m];
        const float* lr = smem + htile(m >> 4, jb) + (m & 15) * HT_LD;
#pragma unroll
        for (int c = 0; c < 16; ++c) sv = fmaf(-bvec[j0 + c], lr[c], sv);
        bvec[m] = sv;
      }
    }
    __syncthreads();
    HEAVY_TS(3 + jb);
  }
  if (wave == 0) {  // back substitution Lᵀ x = y, one wave (lane i16 of every 16-lane row: x[j0+i16])
    for (int jb = NB - 1; jb >= 0; --jb) {
      const int j0 = 16 * jb;
      float yv = bvec[j0 + i16];
      const float sdq = sdiag[j0 + i16];
      float lcol[16];  // L11[m][i16] = row i16 of the stored L11ᵀ
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 l = ld4(smem + htile(jb, jb) + 16 * i16 + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) lcol[4 * q + e] = l[e];
      }
      float xb[16];  // x_J[c] on every lane
      static_for<0, 16>([&](auto cc) {
        constexpr int i = 15 - decltype(cc)::value;
        const float xi = bc16<i>(yv * sdq);
        xb[i] = xi;
        yv = (i16 < i) ? fmaf(-lcol[i], xi, yv) : ((i16 == i) ? xi : yv);
      });
      WAVE_LDS_SYNC();
      if (lane < 16) bvec[j0 + i16] = yv;
      for (int m = lane; m < j0; m += 64) {  // y_m -= Σ_c L[j0+c][m] x_J[c]
        float sv = bvec[m];
        const float* lt = smem + htile(jb, m >> 4) + (m & 15);
#pragma unroll
        for (int c = 0; c < 16; ++c) sv = fmaf(-lt[c * HT_LD], xb[c], sv);
        bvec[m] = sv;
      }
      WAVE_LDS_SYNC();
    }
    bool nonfinite = false;
    for (int c = lane; c < KP; c += 64) {
      const float v = c < a.kreal ? bvec[c] : 0.f;
      nonfinite |= !isfinite(v);
      a.X[(int64_t)j * KP + c] = v;
    }
    if (__any(nonfinite)) s_flag[1] |= 2;
    if (lane == 0 && s_flag[1]) atomicOr(a.err, s_flag[1]);
    HEAVY_TS(23);
  }
}

// =============================================================================================
// NNLS rows (nonnegative = true; Spark NNLSSolver -> mllib/optimization/NNLS.scala).  Original basis
// (no rotation: the constraints are coordinate-wise): A = G + λn I + Σ c y yᵀ built exactly like
// the heavy rows (same LDS stage + MFMA + packed tiles) plus the G tiles, then Spark's projected
// gradient with CG acceleration, thread i = coordinate i, fp64 vectors and block reductions.
// =============================================================================================
// Block reductions of the NNLS loop.  Only the NO = KP/64 waves that own coordinates hold nonzero
// terms, so only they reduce (wave-level DPP/shuffle sums, one partial per wave in LDS); after the
// barrier every wave reads the NO partials (uniform control flow needs the result everywhere).
// DPP move of a double (two 32-bit halves); lanes of rows outside ROWMASK, and lanes whose source
// lies outside the row, read `fill`
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp64(double v, double fill) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(fill), __double2loint(v), CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(fill), __double2hiint(v), CTRL, ROWMASK, 0xF, false);
  return __hiloint2double(hi, lo);
}
// Wave-wide fp64 sum / min with the result in lane 63: row_shr 1, 2, 4, 8 within each 16-lane row,
// then row_bcast:15 and row_bcast:31 across rows (VALU only; a shuffle butterfly is six LDS-latency
// round trips per value)
template <bool MIN>
__device__ __forceinline__ double wave_reduce63(double x) {
  const double z = MIN ? INFINITY : 0.0;
  auto op = [](double a, double b) { return MIN ? fmin(a, b) : a + b; };
  x = op(x, dpp64<0x111, 0xF>(x, z));
  x = op(x, dpp64<0x112, 0xF>(x, z));
  x = op(x, dpp64<0x114, 0xF>(x, z));
  x = op(x, dpp64<0x118, 0xF>(x, z));
  x = op(x, dpp64<0x142, 0xA>(x, z));
  x = op(x, dpp64<0x143, 0xC>(x, z));
  return x;
}

template <int NO, int N>
__device__ __forceinline__ void own_sum(double (&v)[N], double* scr, int& phase) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* sp = scr + phase * 16 * 8;
  if (wave < NO) {
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] = wave_reduce63<false>(v[n]);
    if (lane == 63) {
#pragma unroll
      for (int n = 0; n < N; ++n) sp[n * 16 + wave] = v[n];
    }
  }
  __syncthreads();
#pragma unroll
  for (int n = 0; n < N; ++n) {
    double t = sp[n * 16];
#pragma unroll
    for (int w = 1; w < NO; ++w) t += sp[n * 16 + w];
    v[n] = t;
  }
  phase ^= 1;
}

// NSUM sums then NMIN minima in one pass (one barrier)
template <int NO, int NSUM, int NMIN>
__device__ __forceinline__ void own_sum_min(double (&v)[NSUM + NMIN], double* scr, int& phase) {
  constexpr int N = NSUM + NMIN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* sp = scr + phase * 16 * 8;
  if (wave < NO) {
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] = n < NSUM ? wave_reduce63<false>(v[n]) : wave_reduce63<true>(v[n]);
    if (lane == 63) {
#pragma unroll
      for (int n = 0; n < N; ++n) sp[n * 16 + wave] = v[n];
    }
  }
  __syncthreads();
#pragma unroll
  for (int n = 0; n < N; ++n) {
    double t = sp[n * 16];
#pragma unroll
    for (int w = 1; w < NO; ++w) t = n < NSUM ? t + sp[n * 16 + w] : fmin(t, sp[n * 16 + w]);
    v[n] = t;
  }
  phase ^= 1;
}


// y = A·v for NV vectors at once (A symmetric, NNLS layout: packed lower 16x16 tiles, diagonal
// tiles full; v and y fp32 in LDS).  Wave w takes the row blocks I = w, w + NW, ...; lane l reads
// 16 B of tile row r = l >> 2 (columns 4q .. 4q+3, q = l & 3) per tile with ds_read_b128, so one
// pass over a row block streams each of its 16x16 tiles once:
//   J <= I   stored tile (I, J):    y_I[r]      += Σ_s T[r][4q+s] v_J[4q+s]    (sum over q)
//   J >  I   stored tile (J, I)ᵀ:  y_I[4q+s]   += T[r][4q+s] v_J[r]           (sum over r)
// Partial sums combine by DPP (quad_perm, row_ror) plus two cross-row shuffles, fp32 throughout.
// tid: threadIdx.x, passed through an empty asm by the caller every iteration so that the compiler
// recomputes these LDS addresses instead of hoisting dozens of them out of the NNLS loop (which spills
// at the 128 VGPRs a 1024-thread workgroup allows).
template <int KP, int NV>
__device__ __forceinline__ void nt_symv(const float* __restrict__ A, const float* const (&v)[2], float* const (&y)[2],
                                        float* scratch /* per wave: NV x 16 floats */, int tid) {
  constexpr int NB = KP / 16, NW = Heavy<KP>::NW;
  const int lane = tid & 63, wave = tid >> 6, r = lane >> 2, q = lane & 3;
  for (int I = wave; I < NB; I += NW) {
    float yn[NV], yt[NV][4];
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      yn[n] = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) yt[n][e] = 0.f;
    }
#pragma unroll 2
    for (int J = 0; J < NB; ++J) {
      if (J <= I) {
        const f32x4 t = ld4(A + ntile(I, J) + 16 * r + 4 * q);
#pragma unroll
        for (int n = 0; n < NV; ++n) {
          const f32x4 x = ld4(v[n] + 16 * J + 4 * q);
          yn[n] = fmaf(t[0], x[0], fmaf(t[1], x[1], fmaf(t[2], x[2], fmaf(t[3], x[3], yn[n]))));
        }
      } else {
        const f32x4 t = ld4(A + ntile(J, I) + 16 * r + 4 * q);
#pragma unroll
        for (int n = 0; n < NV; ++n) {
          const float x = v[n][16 * J + r];
#pragma unroll
          for (int e = 0; e < 4; ++e) yt[n][e] = fmaf(t[e], x, yt[n][e]);
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      yn[n] += dppf<0xB1>(yn[n]);  // quad_perm [1,0,3,2]: lanes 4r..4r+3 share row r
      yn[n] += dppf<0x4E>(yn[n]);  // quad_perm [2,3,0,1]
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // sum over r: lanes q, q+4, ... of the 16-lane row, then the 4 rows
        float x = yt[n][e];
        x += dppf<0x124>(x);  // row_ror:4
        x += dppf<0x128>(x);  // row_ror:8
        x += __shfl_xor(x, 16);
        x += __shfl_xor(x, 32);
        yt[n][e] = x;
      }
      if (lane < 4) *reinterpret_cast<f32x4*>(scratch + 16 * n + 4 * lane) = f32x4{yt[n][0], yt[n][1], yt[n][2], yt[n][3]};
    }
    WAVE_LDS_SYNC();
    if (q == 0) {
#pragma unroll
      for (int n = 0; n < NV; ++n) y[n][16 * I + r] = yn[n] + scratch[16 * n + r];
    }
    WAVE_LDS_SYNC();
  }
}

template <int KP>
struct NnlsLds {
  static constexpr int NW = Heavy<KP>::NW;
  static constexpr int BASE = Heavy<KP>::FLOATS;           // heavy layout first (tiles, b', flags)
  static constexpr int OFF_V = (BASE + 3) & ~3;            // fp32 vectors: product inputs v0, v1
  static constexpr int OFF_Y = OFF_V + 2 * KP;             // fp32 products y0, y1
  static constexpr int OFF_W = OFF_Y + 2 * KP;             // per-wave product scratch [NW][32]
  static constexpr int OFF_SCR = (OFF_W + 32 * NW + 1) & ~1;  // fp64 reduction scratch [2][8][16]
  static constexpr int FLOATS = OFF_SCR + 2 * 2 * 8 * 16;
  static_assert(ntile(KP / 16, 0) <= Heavy<KP>::OFF_B, "NNLS tiles fit where the heavy build leaves its tiles");
};

// ---- NNLS iteration on a register-resident A (KP = 128 / 256) --------------------------------
// The workgroup's NW waves hold A once per row: wave w = (is, js) keeps the 4 x 4 tiles of row blocks
// 4is .. 4is+3 and column blocks 4js .. 4js+3, lane i + 16q the entries A[16I + 4q + r][16J + i]
// (64 floats, as 32 fp32 pairs for v_pk_fma_f32).  A·g is then 32 packed FMAs on the four g[16J + i]
// a lane needs (one ds_read_b128) and a 15-step recursive-halving sum over the lane's 16-lane DPP row
// (row_mirror, row_half_mirror, quad reversal, quad swap: partners i^15, i^7, i^3, i^1).  Each lane
// stores its 16 row partials in a lane-dependent slot order s -> k = s ^ m(i) (m linear over GF(2),
// m(15) = 8, m(7) = 4, m(3) = 2, m(1) = 1) so that the half a lane keeps and the half its partner sends
// sit in the same registers: no selects.  Lane i ends with row 16(4is + (m(i) >> 2)) + 4q + (m(i) & 3)
// summed over its column-block set; the waves with js = 0 own those rows (x, residual, directions and
// A·dir in fp64).
// Spark's iteration needs A·g and A·dir, dir = g + alpha·lastDir.  By linearity A·dir = A·g +
// alpha·A·lastDir, and A·lastDir is the previous step's A·dir (kept by the owner), so ONE product per
// iteration suffices; the owner forms dir, ‖dir‖², dir·res and the wall ratios in fp64 as Spark does,
// and dir·A·dir = g·A·g + 2 alpha g·(A lastDir) + alpha² lastDir·A·lastDir (the last term is the
// previous step's curvature).  Two barriers per iteration: (B1) the owners publish g (fp32) and the
// sums ‖g‖², g·res, ‖x‖², wall hits, g·A·lastDir; (B2) every wave publishes its row partials of A·g and
// of g·A·g, the owners ‖dir‖², dir·res and the two wall-ratio minima.  Only the owner waves evaluate the
// step and the stopping rule; the others learn a stop at the next pass's first barrier (LDS flag).
__device__ __forceinline__ int nnls_slot_mask(int i) {
  return ((i & 1) ? 1 : 0) ^ ((i & 2) ? 3 : 0) ^ ((i & 4) ? 6 : 0) ^ ((i & 8) ? 12 : 0);
}
template <int KP>
struct NnlsReg {
  static constexpr int NB = KP / 16, NW = Heavy<KP>::NW, IB = 4, JB = 4, NIS = NB / IB, NJS = NB / JB;
  static_assert(NIS * NJS == NW && NW <= 16, "one wave per (row-block set, column-block set)");
  // LDS, inside the tile area once A is in registers (floats)
  static constexpr int OFF_G = 0;                      // fp32 g, element c at (c & 15)·NB + (c >> 4)
  static constexpr int OFF_P = OFF_G + KP;             // row partials of A·g [NJS][KP]
  static constexpr int OFF_R1 = OFF_P + NJS * KP;      // fp64 wave partials of B1 [8][16]
  static constexpr int OFF_R2 = OFF_R1 + 2 * 128;      // fp64 wave partials of B2 [8][16]
  static constexpr int OFF_FLAG = OFF_R2 + 2 * 128;    // stop flag
  static constexpr int FLOATS = OFF_FLAG + 4;
  static_assert(FLOATS <= (KP / 16) * (KP / 16 + 1) / 2 * 256, "fits the dead tile area");
};

__device__ __forceinline__ int nnls_vidx(int c, int NB) { return (c & 15) * NB + (c >> 4); }

template <int KP>
__device__ void nnls_reg_iterate(const SolveArgs& a, float* smem, int j, int iter_max) {
  using R = NnlsReg<KP>;
  using H = Heavy<KP>;
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int NB = R::NB, NIS = R::NIS, NW = R::NW;
  const float* bvec = smem + H::OFF_B;
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, q = lane >> 4;
  const int is = wave % NIS, js = wave / NIS;
  const bool own = js == 0;  // wave-uniform
  const int msk = nnls_slot_mask(i16);
  const int c_own = 16 * (R::IB * is + (msk >> 2)) + 4 * q + (msk & 3);
  // A into registers: slot s (pair s & 7, half s >> 3) holds row k = s ^ msk of the lane's 16
  f2 av[8][4];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int k = s ^ msk;
    const int row = 16 * (R::IB * is + (k >> 2)) + 4 * q + (k & 3);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int col = 16 * (R::JB * js + jj) + i16;
      av[s & 7][jj][s >> 3] = smem[row >= col ? nel(row, col) : nel(col, row)];
    }
  }
  const float bi = own ? bvec[c_own] : 0.f;
  __syncthreads();  // the tile area is free from here on
  float* sG = smem + R::OFF_G;
  float* sP = smem + R::OFF_P;
  double* sR1 = reinterpret_cast<double*>(smem + R::OFF_R1);
  double* sR2 = reinterpret_cast<double*>(smem + R::OFF_R2);
  int* sStop = reinterpret_cast<int*>(smem + R::OFF_FLAG);
  const int vrow = i16 * NB + R::JB * js;  // this lane's product columns in sG
  const int vown = nnls_vidx(c_own, NB);
  // A·v over the lane's columns, summed over the 16-lane row: the partial of row c_own
  // (each pair folds into h[s] as soon as it is done: 8 live floats instead of 16 + 8, so the loop
  // keeps all of A in registers -- no scratch traffic; measured time-neutral)
  auto product = [&](const f32x4 v) -> float {
    float h[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      f2 p = av[s][0] * f2{v[0], v[0]};
      p = av[s][1] * f2{v[1], v[1]} + p;
      p = av[s][2] * f2{v[2], v[2]} + p;
      p = av[s][3] * f2{v[3], v[3]} + p;
      h[s] = p[0] + dppf<0x140>(p[1]);  // row_mirror: lane i^15
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) h[s] += dppf<0x141>(h[s + 4]);  // row_half_mirror: lane i^7
#pragma unroll
    for (int s = 0; s < 2; ++s) h[s] += dppf<0x1B>(h[s + 2]);  // quad_perm [3,2,1,0]: lane i^3
    return h[0] + dppf<0xB1>(h[1]);                             // quad_perm [1,0,3,2]: lane i^1
  };
  // owner state (fp64); uniform: last_norm, the previous step's ‖dir‖² and dir·A·dir
  double xi = 0.0, axi = 0.0, last_dir = 0.0, a_last = 0.0;
  float hit = 0.f;
  double last_norm = 0.0, last_dad = 0.0;
  // owner waves, per pass: B1's totals and the CG direction
  double ngrad = 0.0, gres = 0.0, nx = 0.0, gal = 0.0, alpha = 0.0, dc = 0.0;
  bool cg = false;
  int last_wall = 0, iterno = 0;
  bool stopped = false;  // owner waves only (the others learn it at the next barrier)
  if (tid == 0) sStop[0] = 0;
  NNLS_T0();
  for (; iterno < iter_max; ++iterno) {
    if (iterno > 0 && (iterno & 63) == 0) {  // exact residual refresh: A·x
      if (own && !stopped) sG[vown] = (float)xi;
      if (tid == 0) sStop[0] = stopped;
      __syncthreads();
      if (sStop[0]) break;
      sP[js * KP + c_own] = product(ld4(sG + vrow));
      __syncthreads();
      if (own) {
        float y = sP[c_own];
#pragma unroll
        for (int w = 1; w < R::NJS; ++w) y += sP[w * KP + c_own];
        axi = (double)y;
      }
    }
    // residual = A x - b ; projected gradient
    const double res = own ? axi - (double)bi : 0.0;
    double gi = res;
    if (gi > 0.0 && xi == 0.0) gi = 0.0;
    if (own && !stopped) {
      // sums ‖g‖², g·res, ‖x‖², g·A·lastDir; minimum -hit (the previous step's wall hits)
      const double t[8] = {gi * gi, gi * res, xi * xi, gi * a_last, -(double)hit, INFINITY, INFINITY, INFINITY};
      double s, m;
      wave_reduce8(t, s, m);
      if ((lane & 15) == 0) {  // row r holds sum r and minimum r
        sR1[q * 16 + is] = s;
        sR1[64 + q * 16 + is] = m;
      }
      sG[vown] = (float)gi;
    }
    if (tid == 0) sStop[0] = stopped;
    NNLS_PH(0);
    __syncthreads();  // B1
    NNLS_PH(1);
    if (sStop[0]) break;
    // the product A·g (every wave), its row partial to LDS
    const float gc = sG[vown];
    const float p0 = product(ld4(sG + vrow));
    sP[js * KP + c_own] = p0;
    double t_gag = (double)gc * (double)p0;
    NNLS_PH(2);
    if (own) {
      // r1 totals: lane l reads value l >> 4 (t0) and 4 + (l >> 4) (t1) of wave l & 15; rows 0, 2 of
      // each register are sums, rows 1, 3 minima
      {  // lane l: sum / minimum l >> 4 of owner wave l & 15
        const bool wv = (lane & 15) < NIS;
        const double t0 = row16_all<false>(wv ? sR1[lane] : 0.0);
        const double t1 = row16_all<true>(wv ? sR1[64 + lane] : INFINITY);
        ngrad = rdlane_d(t0, 0);
        gres = rdlane_d(t0, 16);
        nx = rdlane_d(t0, 32);
        gal = rdlane_d(t0, 48);
        if (-rdlane_d(t1, 0) > 0.0) last_wall = iterno - 1;  // the previous step's wall hits
      }
      cg = iterno > last_wall + 1;
      alpha = cg ? uni(ngrad / last_norm) : 0.0;
      dc = cg ? gi + alpha * last_dir : 0.0;
      // sums: g·A·g partials, ‖dir‖², dir·res; minima: wall ratios of g and of dir
      const double t[8] = {t_gag, dc * dc, dc * res, 0.0, gi > 0.0 ? xi / gi : INFINITY,
                           (cg && dc > 0.0) ? xi / dc : INFINITY, INFINITY, INFINITY};
      double s, m;
      wave_reduce8(t, s, m);
      if ((lane & 15) == 0) {
        sR2[q * 16 + wave] = s;
        sR2[64 + q * 16 + wave] = m;
      }
    } else {
      t_gag = row16_sum(t_gag);
      t_gag += dpp64z<0x142>(t_gag);  // row_bcast:15
      t_gag += dpp64z<0x143>(t_gag);  // row_bcast:31 -> lane 63
      if (lane == 63) sR2[wave] = t_gag;
    }
    NNLS_PH(3);
    __syncthreads();  // B2
    NNLS_PH(4);
    if (own) {
      double s0, s1;
      {  // lane l: sum / minimum l >> 4 of wave l & 15 (sum 0 from every wave, the rest from the owners)
        const bool ownv = (lane & 15) < NIS;
        s0 = row16_all<false>(((q == 0 ? (lane & 15) < NW : ownv)) ? sR2[lane] : 0.0);
        s1 = row16_all<true>(ownv ? sR2[64 + lane] : INFINITY);
      }
      const double gag = rdlane_d(s0, 0), ndc = rdlane_d(s0, 16), dres = rdlane_d(s0, 32);
      const double mg = rdlane_d(s1, 0), md = rdlane_d(s1, 16);
      float y0 = sP[c_own];
#pragma unroll
      for (int w = 1; w < R::NJS; ++w) y0 += sP[w * KP + c_own];
      const double agi = (double)y0;
      double step = gres / (gag + 1e-20);
      double di = gi, adi = agi, ndir = ngrad, dad_used = gag;
      bool use_dc = false;
      if (cg) {
        const double dad = gag + 2.0 * alpha * gal + alpha * alpha * last_dad;
        const double dstep = dres / (dad + 1e-20);
        if (!nnls_stop(dstep, ndc, nx)) {  // else: reject the CG direction
          step = dstep;
          di = dc;
          adi = agi + alpha * a_last;
          ndir = ndc;
          dad_used = dad;
          use_dc = true;
        }
      }
      if (nnls_stop(step, ndir, nx)) {
        stopped = true;
      } else {
        // don't run through the walls
        step = fmin(step, use_dc ? md : mg);
        // take the step
        hit = 0.f;
        if (step * di > xi * (1 - 1e-14)) {
          xi = 0.0;
          hit = 1.f;
        } else {
          xi -= step * di;
        }
        axi -= step * adi;
        last_dir = di;
        a_last = adi;
        last_dad = uni(dad_used);
      }
      last_norm = ngrad;
    }
    NNLS_PH(5);
    if (stopped) continue;  // owner waves: on to the next pass's first barrier, which ends the loop
  }
  NNLS_OUT();
  // iterations in Spark's count: the pass whose stopping rule fired (the loop ran one pass further)
  if (stopped) --iterno;
  if (own) a.X[(int64_t)j * KP + c_own] = c_own < a.kreal ? (float)xi : 0.f;
  if (tid == 0 && s_flag[1]) atomicOr(a.err, s_flag[1]);
  if (tid == 0 && a.iters) {
    atomicAdd(&a.iters[0], (unsigned long long)iterno);
    atomicMax(&a.iters[1], (unsigned long long)iterno);
  }
}

// NNLS rows (nonnegative = true; Spark NNLSSolver -> mllib/optimization/NNLS.scala).  Original basis
// (the constraints are coordinate-wise): A = G + λn I + Σ c y yᵀ built like the heavy rows (same LDS
// stage + MFMA) into the NNLS tile layout, then Spark's projected gradient with CG acceleration:
// thread i < KP owns coordinate i (x, residual, directions in fp64 registers), every wave takes part
// in the products.  Per iteration ONE pass over A yields A·grad and A·dir together (dir = grad +
// alpha·lastDir is known once ‖grad‖² is reduced), and the residual follows the steps
// (A·x_new = A·x - step·A·dir, exact refresh every 64 iterations): Spark's three products become one
// pass.  Stopping rules, the wall clamp and the CG restarts are Spark's, unchanged.
template <int KP, bool PRE = false, bool REG = false>
__global__ __launch_bounds__(Heavy<KP>::NTH) void solve_nnls_kernel(SolveArgs a, const float* __restrict__ Gt) {
  using H = Heavy<KP>;
  using NL = NnlsLds<KP>;
  constexpr int NTH = H::NTH, NB = KP / 16, NTT = NB * (NB + 1) / 2 * 256, NO = KP / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* bvec = smem + H::OFF_B;
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);
  float* v0 = smem + NL::OFF_V;
  float* v1 = v0 + KP;
  float* y0 = smem + NL::OFF_Y;
  float* y1 = y0 + KP;
  double* scr = reinterpret_cast<double*>(smem + NL::OFF_SCR);
  const float* const vv[2] = {v0, v1};
  float* const yy[2] = {y0, y1};
  const int tid = threadIdx.x;
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; }
  if constexpr (PRE) {  // split row: the reduced record (heavy tile layout) -> NNLS layout
    const float* rec = a.prebuilt + (size_t)blockIdx.x * SplitRec<KP>::FLOATS;
    for (int e = tid; e < NTT; e += NTH) {
      const int t = e >> 8, w = e & 255, rr = w >> 4, cc = w & 15;
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const bool diag = t == I * (I + 1) / 2 + I;
      smem[e] = (diag && cc > rr) ? rec[t * HT_SZ + cc * HT_LD + rr] : rec[t * HT_SZ + rr * HT_LD + cc];
    }
    for (int c = tid; c < KP; c += NTH) bvec[c] = rec[SplitRec<KP>::OFF_B + c];
    if (tid == 0) s_flag[0] = reinterpret_cast<const int*>(rec)[SplitRec<KP>::OFF_N];
    __syncthreads();
  } else {
    heavy_build_all<KP, true>(a, p0, d, smem);
  }
  const float lamn = a.reg * (float)(a.implicit ? s_flag[0] : d);
  for (int e = tid; e < NTT; e += NTH) smem[e] += Gt[e];  // A = G + Σ c y yᵀ (Gt: the same layout)
  __syncthreads();
  for (int c = tid; c < KP; c += NTH) smem[nel(c, c)] += c < a.kreal ? lamn : 1.0f;
  if constexpr (REG) {
    __syncthreads();
    nnls_reg_iterate<KP>(a, smem, j, 400 > 20 * a.kreal ? 400 : 20 * a.kreal);
    return;
  }
  const bool own = tid < KP;
  const int i = own ? tid : 0;
  const double bi = own ? (double)bvec[i] : 0.0;
  double xi = 0.0, axi = 0.0, last_dir = 0.0, last_norm = 0.0, hit = 0.0;
  __syncthreads();
  int phase = 0, last_wall = 0;
  const int iter_max = 400 > 20 * a.kreal ? 400 : 20 * a.kreal;
  int iterno = 0;
  NNLS_T0();
  for (; iterno < iter_max; ++iterno) {
    int ot = tid;  // opaque copy of threadIdx.x (see nt_symv)
    asm volatile("" : "+v"(ot));
    float* const wsc = smem + NL::OFF_W + 32 * (ot >> 6);
    if (iterno > 0 && (iterno & 63) == 0) {  // exact residual refresh: A·x
      if (own) v0[i] = (float)xi;
      __syncthreads();
      nt_symv<KP, 1>(smem, vv, yy, wsc, ot);
      __syncthreads();
      if (own) axi = (double)y0[i];
    }
    // residual = A x - b ; projected gradient
    const double res = own ? axi - bi : 0.0;
    double gi = res;
    if (gi > 0.0 && xi == 0.0) gi = 0.0;
    double r1[4] = {gi * gi, gi * res, xi * xi, hit};  // + the previous step's wall hits
    NNLS_PH(0);
    own_sum<NO, 4>(r1, scr, phase);
    NNLS_PH(1);
    if (r1[3] > 0.0) last_wall = iterno - 1;
    const double ngrad = r1[0], nx = r1[2];
    const bool cg = iterno > last_wall + 1;
    const double dc = cg ? gi + (ngrad / last_norm) * last_dir : 0.0;
    if (own) {
      v0[i] = (float)gi;
      v1[i] = (float)dc;
    }
    __syncthreads();
    NNLS_PH(2);
    if (cg) nt_symv<KP, 2>(smem, vv, yy, wsc, ot);
    else nt_symv<KP, 1>(smem, vv, yy, wsc, ot);
    NNLS_PH(3);
    __syncthreads();
    NNLS_PH(4);
    const double agi = own ? (double)y0[i] : 0.0;
    const double adc = (own && cg) ? (double)y1[i] : 0.0;
    // + the wall ratios of both candidate directions (min x_i/dir_i over dir_i > 0): clamping the
    // step to the smallest ratio is Spark's sequential clamp, and riding in this reduction saves the
    // third one once the direction is chosen
    double r2[6] = {gi * agi, dc * res, dc * adc, dc * dc, (own && gi > 0.0) ? xi / gi : INFINITY,
                    (own && dc > 0.0) ? xi / dc : INFINITY};
    own_sum_min<NO, 4, 2>(r2, scr, phase);
    NNLS_PH(5);
    double step = r1[1] / (r2[0] + 1e-20);
    double di = gi, adi = agi, ndir = ngrad;
    bool use_dc = false;
    if (cg) {
      const double dstep = r2[1] / (r2[2] + 1e-20);
      if (!nnls_stop(dstep, r2[3], nx)) {  // else: reject the CG direction
        step = dstep;
        di = dc;
        adi = adc;
        ndir = r2[3];
        use_dc = true;
      }
    }
    if (nnls_stop(step, ndir, nx)) break;
    // don't run through the walls
    step = fmin(step, use_dc ? r2[5] : r2[4]);
    NNLS_PH(6);
    // take the step
    hit = 0.0;
    if (own) {
      if (step * di > xi * (1 - 1e-14)) {
        xi = 0.0;
        hit = 1.0;
      } else {
        xi -= step * di;
      }
      axi -= step * adi;
    }
    last_dir = di;
    last_norm = ngrad;
    NNLS_PH(7);
  }
  NNLS_OUT();
  if (own) a.X[(int64_t)j * KP + i] = i < a.kreal ? (float)xi : 0.f;
  if (tid == 0 && s_flag[1]) atomicOr(a.err, s_flag[1]);
  if (tid == 0 && a.iters) {
    atomicAdd(&a.iters[0], (unsigned long long)iterno);
    atomicMax(&a.iters[1], (unsigned long long)iterno);
  }
}

template <int KP>
hipError_t launch_nnls_kp(const SolveArgs& a, const float* Gt, hipStream_t s) {
  const size_t lds = NnlsLds<KP>::FLOATS * 4;
  // KP >= 128: A in registers (nnls_reg_iterate); KP = 64 keeps the LDS-streamed loop
  constexpr bool CAN_REG = KP >= 128;
  constexpr bool reg = CAN_REG;
  static const hipError_t attr = allow_lds(solve_nnls_kernel<KP, false>, lds);
  static const hipError_t attr2 = allow_lds(solve_nnls_kernel<KP, true>, lds);
  static const hipError_t attr3 = allow_lds(solve_nnls_kernel<KP, false, CAN_REG>, lds);
  static const hipError_t attr4 = allow_lds(solve_nnls_kernel<KP, true, CAN_REG>, lds);
  if (attr != hipSuccess) return attr;
  if (attr2 != hipSuccess) return attr2;
  if (attr3 != hipSuccess) return attr3;
  if (attr4 != hipSuccess) return attr4;
  // one workgroup per row, in launches of at most 2^31 work-items (an AQL dispatch's grid size is a
  // 32-bit work-item count: 4.9M rows x 1024 threads would wrap and silently drop rows)
  for (int64_t r0 = 0; r0 < a.n_rows; r0 += max_rows_per_launch(Heavy<KP>::NTH)) {
    SolveArgs b = chunk_args(a, r0, Heavy<KP>::NTH, SplitRec<KP>::FLOATS);
    if (reg && b.prebuilt) solve_nnls_kernel<KP, true, CAN_REG><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b, Gt);
    else if (reg) solve_nnls_kernel<KP, false, CAN_REG><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b, Gt);
    else if (b.prebuilt) solve_nnls_kernel<KP, true><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b, Gt);
    else solve_nnls_kernel<KP, false><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b, Gt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_solve_nnls(int KP, const SolveArgs& a, const float* Gt, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (KP == 64) return launch_nnls_kp<64>(a, Gt, s);
  if (KP == 128) return launch_nnls_kp<128>(a, Gt, s);
  if (KP == 256) {
    const char* e = std::getenv("ALBEDO_NNLS_ROW");  // A/B knob, read per launch
    const bool old_kernel = e && std::atoi(e) == 1024;
    return old_kernel ? launch_nnls_kp<256>(a, Gt, s) : launch_solve_nnls_row256(a, Gt, s);
  }
  return hipErrorInvalidValue;
}
int nnls_gtile_floats(int KP) { const int nb = KP / 16; return nb * (nb + 1) / 2 * 256; }
int nnls_gtile_index(int r, int c) { return nel(r, c); }

template <int KP>
hipError_t launch_heavy_kp(const SolveArgs& a, hipStream_t s) {
  const size_t lds = Heavy<KP>::FLOATS * 4;
  static const hipError_t attr = allow_lds(solve_heavy_kernel<KP>, lds);
  static const hipError_t attr2 = allow_lds(solve_heavy_kernel<KP, 3, true>, lds);
  if (attr != hipSuccess) return attr;
  if (attr2 != hipSuccess) return attr2;
  for (int64_t r0 = 0; r0 < a.n_rows; r0 += max_rows_per_launch(Heavy<KP>::NTH)) {
    SolveArgs b = chunk_args(a, r0, Heavy<KP>::NTH, SplitRec<KP>::FLOATS);
    if (b.prebuilt) solve_heavy_kernel<KP, 3, true><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b);
    else solve_heavy_kernel<KP><<<(int)b.n_rows, Heavy<KP>::NTH, lds, s>>>(b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_solve_heavy(int KP, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (KP == 64) return launch_heavy_kp<64>(a, s);
  if (KP == 128) return launch_heavy_kp<128>(a, s);
  if (KP == 256) return launch_heavy_kp<256>(a, s);
  return hipErrorInvalidValue;
}

// =============================================================================================
// Per-column fp16 scales of the heavy build: colscale[c] = 2^e with max_rows |Z[.][c]|·√cmax < 2^13
// (cmax = the largest confidence c of the dst side), colscale[KP + c] = 2^-e.
// =============================================================================================
template <int KP>
__global__ __launch_bounds__(256) void colmax_kernel(const float* __restrict__ Z, int64_t n, unsigned* __restrict__ out) {
  constexpr int NCQ = KP / 4, RS = 256 / NCQ;  // float4 column chunks per row, rows per block step
  __shared__ f32x4 red[256];
  const int cq = threadIdx.x % NCQ, rsub = threadIdx.x / NCQ;
  f32x4 m = zero4();
  int64_t r = (int64_t)blockIdx.x * RS + rsub;
  const int64_t step = (int64_t)gridDim.x * RS;
  for (; r + 3 * step < n; r += 4 * step) {  // four independent loads in flight
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld4(Z + (r + u * step) * KP + 4 * cq);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], fabsf(v[u][q]));
  }
  for (; r < n; r += step) {
    const f32x4 v = ld4(Z + r * KP + 4 * cq);
#pragma unroll
    for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], fabsf(v[q]));
  }
  red[threadIdx.x] = m;
  __syncthreads();
  if (threadIdx.x < NCQ) {
    for (int s = 1; s < RS; ++s) {
      const f32x4 o = red[s * NCQ + threadIdx.x];
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], o[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = m[q];
      if (!(v <= 3.0e38f)) v = 3.0e38f;  // NaN / inf: saturate (the solve reports the non-finite result)
      atomicMax(out + 4 * threadIdx.x + q, __float_as_uint(v));
    }
  }
}

__global__ void colscale_kernel(const unsigned* __restrict__ cmaxbits, int KP, float csqrt, float* __restrict__ out) {
  const int c = threadIdx.x;
  if (c >= KP) return;
  const float m = __uint_as_float(cmaxbits[c]) * csqrt;
  int e = 0;
  if (m > 0.f && m <= 3.0e38f) {
    int ex;
    frexpf(m, &ex);  // m < 2^ex
    e = 13 - ex;
    e = e < -60 ? -60 : (e > 60 ? 60 : e);
  }
  out[c] = ldexpf(1.f, e);
  out[KP + c] = ldexpf(1.f, -e);
}

__global__ void absmax_kernel(const float* __restrict__ v, int64_t n, unsigned* __restrict__ out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(v[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

hipError_t launch_colscale(int KP, const float* Z, int64_t n, float cmax, unsigned* tmp, float* colscale,
                           hipStream_t s, bool have_max) {
  if (have_max) {  // tmp already holds the column maxima (rotate_kernel)
    colscale_kernel<<<1, KP, 0, s>>>(tmp, KP, sqrtf(cmax > 0.f ? cmax : 1.f), colscale);
    return hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(tmp, 0, KP * sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  if (n > 0) {
    int64_t blocks = (n + 63) / 64;
    if (blocks > 1024) blocks = 1024;
    if (KP == 64) colmax_kernel<64><<<(int)blocks, 256, 0, s>>>(Z, n, tmp);
    else if (KP == 128) colmax_kernel<128><<<(int)blocks, 256, 0, s>>>(Z, n, tmp);
    else if (KP == 256) colmax_kernel<256><<<(int)blocks, 256, 0, s>>>(Z, n, tmp);
    else return hipErrorInvalidValue;
  }
  colscale_kernel<<<1, KP, 0, s>>>(tmp, KP, sqrtf(cmax > 0.f ? cmax : 1.f), colscale);
  return hipGetLastError();
}

__global__ void absmin_kernel(const float* __restrict__ v, int64_t n, unsigned* __restrict__ out) {
  float m = INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fminf(m, fabsf(v[i]));
  for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMin(out, __float_as_uint(m));
}

hipError_t launch_absmin(const float* v, int64_t n, unsigned* out, hipStream_t s) {
  const unsigned inf = 0x7f800000u;
  hipError_t e = hipMemcpyAsync(out, &inf, sizeof inf, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // `inf` is a stack value
  if (e != hipSuccess || n <= 0) return e;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  absmin_kernel<<<(int)blocks, 256, 0, s>>>(v, n, out);
  return hipGetLastError();
}

// The heavy build's operand split, once per src row: v = z·(sw·cs) (the same two roundings as the
// per-rating split in solve_wave_kernel), hi = fp16(v), lo = fp16(v - hi); row n is the zero row.
template <int KP>
__global__ __launch_bounds__(256) void presplit_kernel(const float* __restrict__ Z, int64_t n,
                                                       const float* __restrict__ cs, float sw, _Float16* __restrict__ out) {
  constexpr int CQ = KP / 4;  // float4 chunks per row
  const int64_t tot = (n + 1) * CQ;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / CQ;
    const int c4 = (int)(e % CQ) * 4;
    const f32x4 z = r < n ? ld4(Z + r * KP + c4) : zero4();
    f16x4 h, l;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v = z[m] * (sw * cs[c4 + m]);
      asm("" : "+v"(v));  // one fp32 rounding; hi and lo both from that value
      const _Float16 hv = (_Float16)v;
      h[m] = hv;
      l[m] = (_Float16)(v - (float)hv);
    }
    *reinterpret_cast<f16x4*>(out + r * 2 * KP + c4) = h;
    *reinterpret_cast<f16x4*>(out + r * 2 * KP + KP + c4) = l;
  }
}

hipError_t launch_presplit(int KP, const float* Z, int64_t n, const float* colscale, float sw, void* Zhl, hipStream_t s) {
  const int64_t tot = (n + 1) * (KP / 4);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((tot + 255) / 256, 65536));
  _Float16* o = reinterpret_cast<_Float16*>(Zhl);
  if (KP == 64) presplit_kernel<64><<<blocks, 256, 0, s>>>(Z, n, colscale, sw, o);
  else if (KP == 128) presplit_kernel<128><<<blocks, 256, 0, s>>>(Z, n, colscale, sw, o);
  else if (KP == 256) presplit_kernel<256><<<blocks, 256, 0, s>>>(Z, n, colscale, sw, o);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_absmax(const float* v, int64_t n, unsigned* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(unsigned), s);
  if (e != hipSuccess || n <= 0) return e;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  absmax_kernel<<<(int)blocks, 256, 0, s>>>(v, n, out);
  return hipGetLastError();
}

// =============================================================================================
// Fast seeded init for large workloads (unit-norm Gaussian rows, splitmix64 + Box-Muller).  Row r
// of the side is a pure function of (seed, global row index), independent of the sharding.
// =============================================================================================
__host__ __device__ __forceinline__ uint64_t smix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void init_random_kernel(float* __restrict__ X, int64_t n, int KP, int kreal, uint64_t key, int64_t row0) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float* x = X + r * KP;
  double ss = 0.0;
  for (int c = 0; c < kreal; c += 2) {
    const uint64_t h = smix64(key + (uint64_t)(row0 + r) * (uint64_t)KP + (uint64_t)c);
    const double u1 = ((double)(h >> 40) + 1.0) * (1.0 / 16777217.0);
    const double u2 = (double)(h & 0xFFFFFFull) * (1.0 / 16777216.0);
    const double rad = sqrt(-2.0 * log(u1));
    const float g0 = (float)(rad * cos(6.283185307179586 * u2));
    const float g1 = (float)(rad * sin(6.283185307179586 * u2));
    x[c] = g0;
    ss += (double)g0 * g0;
    if (c + 1 < kreal) {
      x[c + 1] = g1;
      ss += (double)g1 * g1;
    }
  }
  const float inv = (float)(1.0 / sqrt(ss));
  for (int c = 0; c < kreal; ++c) x[c] *= inv;
  for (int c = kreal; c < KP; ++c) x[c] = 0.f;
}
hipError_t launch_init_random(int KP, int kreal, float* X, int64_t n, uint64_t seed, int64_t row0, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  init_random_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(X, n, KP, kreal, smix64(seed), row0);
  return hipGetLastError();
}

// =============================================================================================
// ALSModel.transform: F2J sdot (netlib sdot.f via F2J: float products added left to right, no FMA)
// =============================================================================================

__global__ void predict_kernel(int KP, int kreal, const float* __restrict__ U, const float* __restrict__ V,
                               const int32_t* __restrict__ u, const int32_t* __restrict__ v,
                               float* __restrict__ out, int64_t n) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t a = u[p], b = v[p];
  out[p] = (a < 0 || b < 0) ? __int_as_float(0x7fc00000)
                            : f2j_dot(U + (int64_t)a * KP, V + (int64_t)b * KP, kreal);
}

hipError_t launch_predict(int KP, int kreal, const float* U, const float* V, const int32_t* u,
                          const int32_t* v, float* out, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  predict_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(KP, kreal, U, V, u, v, out, n);
  return hipGetLastError();
}

}  // namespace albedo
