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
#include <cstdint>
#include <utility>
#include "kernels.h"

namespace albedo {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define WAVE_LDS_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ int rdlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// v_rsq_f32 / v_rcp_f32 / v_sqrt_f32: single instructions (~1 ulp) instead of the IEEE-exact
// multi-instruction expansions; the solve tolerance is 1e-4 relative (tests state it)
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
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

int padded_rank(int rank) {
  if (rank <= 0) return 0;
  if (rank <= 64) return 64;
  if (rank <= 128) return 128;
  return 0;
}

// =============================================================================================
// Gram: G = Σ_rows x xᵀ  (Spark ALS.computeYtY: NormalEquation.add(y, 0.0) per src row, fp64)
// =============================================================================================
template <int KP, int W>
__device__ __forceinline__ void gram_body(const float* __restrict__ X, int64_t rb, int64_t re,
                                          double* __restrict__ out) {
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2, NTW = (NT + 3) / 4, NH = KP / 64;
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  f32x4 acc[NTW];
  double acc64[NTW][4];
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    acc[s] = zero4();
    for (int r = 0; r < 4; ++r) acc64[s][r] = 0.0;
  }
  int cnt = 0;
  for (int64_t r0 = rb; r0 < re; r0 += 4) {
    const int64_t row = r0 + g;
    f32x4 v[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) v[h] = row < re ? ld4(X + row * KP + 64 * h + 4 * i16) : zero4();
    static_for<0, NTW>([&](auto s) {
      constexpr int t = W + 4 * decltype(s)::value;
      if constexpr (t < NT) {
        constexpr TilePair p = upper_tile(t, NQ);
        acc[s] = mfma4(v[p.a >> 2][p.a & 3], v[p.b >> 2][p.b & 3], acc[s]);
      }
    });
    if (++cnt == 16) {  // 64 rows per fp32 partial, then fp64 (Spark accumulates in fp64)
      cnt = 0;
#pragma unroll
      for (int s = 0; s < NTW; ++s) {
        for (int r = 0; r < 4; ++r) acc64[s][r] += (double)acc[s][r];
        acc[s] = zero4();
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NTW; ++s) {
    const int t = W + 4 * s;
    if (t < NT)
      for (int r = 0; r < 4; ++r) out[((size_t)t * 64 + lane) * 4 + r] = acc64[s][r] + (double)acc[s][r];
  }
}

template <int KP>
__global__ __launch_bounds__(256) void gram_partial_kernel(const float* __restrict__ X, int64_t n,
                                                           int64_t per_blk, double* __restrict__ slab) {
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2;
  const int64_t rb = (int64_t)blockIdx.x * per_blk;
  const int64_t re = rb + per_blk < n ? rb + per_blk : n;
  double* out = slab + (size_t)blockIdx.x * NT * 256;
  const int wave = threadIdx.x >> 6;
  if (wave == 0) gram_body<KP, 0>(X, rb, re, out);
  else if (wave == 1) gram_body<KP, 1>(X, rb, re, out);
  else if (wave == 2) gram_body<KP, 2>(X, rb, re, out);
  else gram_body<KP, 3>(X, rb, re, out);
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
    gram_partial_kernel<128><<<nblk, 256, 0, s>>>(X, n, per, slab);
    gram_reduce_kernel<128><<<(nt * 256 + 255) / 256, 256, 0, s>>>(slab, nblk, G);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// =============================================================================================
// Rotation: Z = X · M   ([n][KP] x [KP][KP]); M staged in LDS, 64 rows per block iteration.
// =============================================================================================
template <int KP>
__global__ __launch_bounds__(256) void rotate_kernel(const float* __restrict__ X, const float* __restrict__ M,
                                                     float* __restrict__ Z, int64_t n) {
  constexpr int LDM = KP + 4, NJ = KP / 16;
  extern __shared__ __attribute__((aligned(16))) float sM[];
  for (int e = threadIdx.x; e < KP * KP / 4; e += 256) {
    const int r = (4 * e) / KP, c = (4 * e) % KP;
    *reinterpret_cast<f32x4*>(sM + r * LDM + c) = ld4(M + r * KP + c);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  for (int64_t b = blockIdx.x; b * 64 < n; b += gridDim.x) {
    const int64_t row = b * 64 + wave * 16 + i16;
    f32x4 acc[NJ];
#pragma unroll
    for (int J = 0; J < NJ; ++J) acc[J] = zero4();
    for (int c0 = 0; c0 < KP; c0 += 16) {
      const f32x4 a4 = row < n ? ld4(X + row * KP + c0 + 4 * g) : zero4();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float* mr = sM + (c0 + 4 * g + m) * LDM + i16;
#pragma unroll
        for (int J = 0; J < NJ; ++J) acc[J] = mfma4(a4[m], mr[16 * J], acc[J]);
      }
    }
#pragma unroll
    for (int J = 0; J < NJ; ++J)
      for (int r = 0; r < 4; ++r) {
        const int64_t rr = b * 64 + wave * 16 + 4 * g + r;
        if (rr < n) Z[rr * KP + 16 * J + i16] = acc[J][r];
      }
  }
}

hipError_t launch_rotate(int KP, const float* X, const float* M, float* Z, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 63) / 64;
  if (blocks > 2048) blocks = 2048;
  const size_t lds = (size_t)KP * (KP + 4) * sizeof(float);
  if (KP == 64) rotate_kernel<64><<<(int)blocks, 256, lds, s>>>(X, M, Z, n);
  else if (KP == 128) rotate_kernel<128><<<(int)blocks, 256, lds, s>>>(X, M, Z, n);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// =============================================================================================
// Light rows: push-through solve, one wave per dst row, degree d <= D.
//   S = (Z_j D^-1/2)(Z_j D^-1/2)ᵀ (d x d, MFMA over the KP columns), K = S + C⁻¹,
//   K v = C⁻¹ w (register Cholesky, lane i = row i), x' = D⁻¹ Z_jᵀ v.
// Entries with c = 0 (implicit zero ratings) contribute nothing to A or b and are masked out.
// =============================================================================================
__device__ __forceinline__ void rating_weights(float r, int implicit, float alpha, float& c, float& w) {
  if (implicit) {
    c = alpha * fabsf(r);
    w = r > 0.f ? 1.f + c : 0.f;
  } else {
    c = 1.f;
    w = r;
  }
}

template <int KP, int D>
__global__ __launch_bounds__(256) void solve_light_kernel(SolveArgs a) {
  constexpr int NB = D / 16, NT = NB * (NB + 1) / 2, LDK = D + 1, NHC = KP / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  float* Ks = smem + wave * D * LDK;
  const int64_t ridx = (int64_t)blockIdx.x * 4 + wave;
  if (ridx >= a.n_rows) return;  // wave-uniform; this kernel has no workgroup barrier
  const int j = a.rows[ridx];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);

  float r = 0.f, ce = 0.f, we = 0.f;
  int colE = 0;
  if (lane < d) {
    r = a.val[p0 + lane];
    colE = a.col[p0 + lane];
    rating_weights(r, a.implicit, a.alpha, ce, we);
  }
  const bool valid = lane < d && ce > 0.f;
  const int npos = a.implicit ? __popcll(__ballot(lane < d && r > 0.f)) : d;
  const float lamn = a.reg * (float)npos;

  int colB[NB];
  bool vB[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    colB[I] = __shfl(colE, 16 * I + i16);
    vB[I] = __shfl((int)valid, 16 * I + i16) != 0;
  }
  constexpr int NC = KP / 16;
  constexpr bool KEEPZ = D <= 32;  // keep the gathered rows in registers for the x' epilogue
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
  bool bad = false;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int c0 = 16 * c;
    const f32x4 dl = ld4(a.lam + c0 + 4 * g);
    float sd[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int cc = c0 + 4 * g + m;
      const float dd = dl[m] + lamn;
      if (cc < a.kreal && !(dd > 0.f)) bad = true;
      sd[m] = (cc < a.kreal && dd > 0.f) ? frsq(dd) : 0.f;
    }
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
  if (__any(bad) && lane == 0) atomicOr(a.err, 1);
  // S -> LDS (symmetric operands make S bitwise symmetric, so mirrored writes agree)
  static_for<0, NT>([&](auto t) {
    constexpr TilePair p = upper_tile(decltype(t)::value, NB);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * p.a + 4 * g + rr, cl = 16 * p.b + i16;
      Ks[row * LDK + cl] = acc[t][rr];
      Ks[cl * LDK + row] = acc[t][rr];
    }
  });
  WAVE_LDS_SYNC();
  const int me = lane < D ? lane : 0;
  const float cinv = valid ? frcp(ce) : 0.f;
  float kr[D];
#pragma unroll
  for (int m = 0; m < D; ++m) {
    const float v = Ks[me * LDK + m];
    kr[m] = (m == me) ? (valid ? v + cinv : 1.0f) : (valid ? v : 0.0f);
  }
  // Cholesky K = L Lᵀ, lane i holds row i (entries m <= i are L[i][m] when done)
  bool notpd = false;
  float dg = 1.f;  // 1 / L[me][me]
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const float piv = rdlane(kr[c], c);
    if (!(piv > 0.f)) notpd = true;
    const float inv = frsq(piv), s = piv * inv;
    kr[c] = (me == c) ? s : kr[c] * inv;
    dg = (me == c) ? inv : dg;
#pragma unroll
    for (int m = c + 1; m < D; ++m) kr[m] = fmaf(-kr[c], rdlane(kr[c], m), kr[m]);
  }
  if (notpd && lane == 0) atomicOr(a.err, 2);
  // forward: L y = C⁻¹ w
  float y = valid ? we * cinv : 0.f;
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const float yc = rdlane(y * dg, c);
    y = (me > c) ? fmaf(-kr[c], yc, y) : ((me == c) ? yc : y);
  }
  // transpose L through LDS: lane i gets column i (lt[m] = L[m][i])
  WAVE_LDS_SYNC();
  if (lane < D) {
#pragma unroll
    for (int m = 0; m < D; ++m) Ks[lane * LDK + m] = kr[m];
  }
  WAVE_LDS_SYNC();
  float lt[D];
#pragma unroll
  for (int m = 0; m < D; ++m) lt[m] = Ks[m * LDK + me];
  // backward: Lᵀ v = y
#pragma unroll
  for (int c = D - 1; c >= 0; --c) {
    const float vc = rdlane(y * dg, c);
    y = (me < c) ? fmaf(-lt[c], vc, y) : ((me == c) ? vc : y);
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
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) pr[m] += __shfl_xor(pr[m], o);
      if (i16 == 0) {
        const f32x4 dl = ld4(a.lam + 16 * c + 4 * g);
        f32x4 o4;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int cc = 16 * c + 4 * g + m;
          const float dd = dl[m] + lamn;
          o4[m] = (cc < a.kreal && dd > 0.f) ? pr[m] * frcp(dd) : 0.f;
        }
        *reinterpret_cast<f32x4*>(a.X + (int64_t)j * KP + 16 * c + 4 * g) = o4;
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
        const int e = e0 + u < d ? e0 + u : d - 1;
        ve[u] = e0 + u < d ? rdlane(y, e) : 0.f;
        const float* zr = a.Z + (int64_t)rdlane_i(colE, e) * KP + lane;
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
      const float dd = a.lam[c] + lamn;
      a.X[(int64_t)j * KP + c] = (c < a.kreal && dd > 0.f) ? xacc[h] * frcp(dd) : 0.f;
    }
  }
}

hipError_t launch_solve_light(int KP, int D, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  const int blocks = (int)((a.n_rows + 3) / 4);
  const size_t lds = (size_t)4 * D * (D + 1) * sizeof(float);
#define LIGHT(kp, dd) \
  if (KP == kp && D == dd) { solve_light_kernel<kp, dd><<<blocks, 256, lds, s>>>(a); return hipGetLastError(); }
  LIGHT(64, 16) LIGHT(64, 32) LIGHT(64, 64) LIGHT(128, 16) LIGHT(128, 32) LIGHT(128, 64)
#undef LIGHT
  return hipErrorInvalidValue;
}

// =============================================================================================
// Heavy rows: explicit A' = diag(Λ + λn) + Σ c z zᵀ, b' = Σ w z, then Cholesky + substitutions.
// One 256-thread workgroup per dst row, sized for 4 workgroups per CU (LDS <= 40 KiB):
//  build   the row's Z rows are gathered 32 at a time into a double-buffered LDS stage shared by
//          the 4 waves (one barrier per 32 ratings); each wave owns a fixed set of upper 16x16
//          tiles (permuted column blocks: one ds_read_b128 per lane per 64 columns) and
//          accumulates them with v_mfma_f32_16x16x4_f32 on √c-scaled rows (bitwise symmetric).
//  store   the tiles go to LDS as packed lower-triangular 16x17 tiles (the stage is dead by then).
//  factor  right-looking, 16-wide panels, two barriers per panel: the waves that own panel rows
//          factor the 16x16 diagonal tile redundantly in registers and solve their rows against
//          it with wave-uniform (SGPR) broadcasts of L11; the trailing update runs on MFMA.  b' is
//          carried as an extra row, so the forward substitution comes for free.
//  back    Lᵀx = y by one wave, no barriers.
// =============================================================================================
constexpr int HT_LD = 17, HT_SZ = 16 * HT_LD;
__device__ __forceinline__ int htile(int I, int J) { return (I * (I + 1) / 2 + J) * HT_SZ; }
__device__ __forceinline__ int hel(int r, int c) { return htile(r >> 4, c >> 4) + (r & 15) * HT_LD + (c & 15); }

template <int KP>
struct HeavyLds {
  static constexpr int NB = KP / 16, NTL = NB * (NB + 1) / 2;
  static constexpr int TILES = NTL * HT_SZ, STAGE = 2 * 32 * KP;
  static constexpr int BIG = TILES > STAGE ? TILES : STAGE;
  static constexpr int OFF_B = BIG, OFF_DIAG = OFF_B + KP, OFF_W = OFF_DIAG + KP, OFF_FLAG = OFF_W + 128;
  static constexpr int FLOATS = OFF_FLAG + 4;
};

template <int KP, int W>
__device__ __forceinline__ void heavy_build(const SolveArgs& a, int64_t p0, int d, float* smem) {
  using Lay = HeavyLds<KP>;
  constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2, NTW = (NT + 3) / 4, NH = KP / 64;
  constexpr int F4ROW = KP / 4, RPP = 256 / F4ROW, NPASS = 32 / RPP;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i16 = lane & 15;
  float* stage = smem;
  float* sw = smem + Lay::OFF_W;  // [buf][0..31] = sqrt(c), [buf][32..63] = w
  const int prow = tid / F4ROW, pch = (tid % F4ROW) * 4;
  f32x4 acc[NTW];
#pragma unroll
  for (int s = 0; s < NTW; ++s) acc[s] = zero4();
  f32x4 bacc[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) bacc[h] = zero4();
  int npos = 0;
  f32x4 stg[NPASS];
  float wsc = 0.f, ww = 0.f;
  auto gload = [&](int e0) {
    int cix[NPASS];
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int e = e0 + p * RPP + prow;
      cix[p] = e < d ? a.col[p0 + e] : -1;
    }
#pragma unroll
    for (int p = 0; p < NPASS; ++p) stg[p] = cix[p] >= 0 ? ld4(a.Z + (int64_t)cix[p] * KP + pch) : zero4();
    if (tid < 32) {
      const int e = e0 + tid;
      float r = 0.f, c = 0.f, w = 0.f;
      if (e < d) {
        r = a.val[p0 + e];
        rating_weights(r, a.implicit, a.alpha, c, w);
        npos += r > 0.f ? 1 : 0;
      }
      wsc = sqrtf(c);
      ww = w;
    }
  };
  auto lds_put = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NPASS; ++p)
      *reinterpret_cast<f32x4*>(stage + (buf * 32 + p * RPP + prow) * KP + pch) = stg[p];
    if (tid < 32) {
      sw[buf * 64 + tid] = wsc;
      sw[buf * 64 + 32 + tid] = ww;
    }
  };
  gload(0);
  lds_put(0);
  __syncthreads();
  const int nst = (d + 31) / 32;
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload((st + 1) * 32);
    const float* sb = stage + buf * 32 * KP;
#pragma unroll 2
    for (int q = 0; q < 8; ++q) {
      const int row = 4 * q + g;
      const float sc = sw[buf * 64 + row];
      f32x4 zs[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const f32x4 zv = *reinterpret_cast<const f32x4*>(sb + row * KP + 64 * h + 4 * i16);
        zs[h] = zv * sc;
        if (W == 0) bacc[h] += zv * sw[buf * 64 + 32 + row];
      }
      static_for<0, NTW>([&](auto s) {
        constexpr int t = W + 4 * decltype(s)::value;
        if constexpr (t < NT) {
          constexpr TilePair p = upper_tile(t, NQ);
          acc[s] = mfma4(zs[p.a >> 2][p.a & 3], zs[p.b >> 2][p.b & 3], acc[s]);
        }
      });
    }
    if (st + 1 < nst) lds_put(buf ^ 1);
    __syncthreads();
  }
  // stage is dead: store the lower triangle into packed tiles, b' into its vector
  static_for<0, NTW>([&](auto s) {
    constexpr int t = W + 4 * decltype(s)::value;
    if constexpr (t < NT) {
      constexpr TilePair p = upper_tile(t, NQ);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * g + r, jj = i16;
        if (p.a != p.b || i >= jj) {
          const int c1 = pcol(p.a, i), c2 = pcol(p.b, jj);
          smem[c1 > c2 ? hel(c1, c2) : hel(c2, c1)] = acc[s][r];
        }
      }
    }
  });
  if (W == 0) {
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        bacc[h][m] += __shfl_xor(bacc[h][m], 16);
        bacc[h][m] += __shfl_xor(bacc[h][m], 32);
      }
    if (lane < 16) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int m = 0; m < 4; ++m) smem[Lay::OFF_B + 64 * h + 4 * lane + m] = bacc[h][m];
    }
    // npos lives in lanes 0..31 of wave 0
    for (int o = 16; o > 0; o >>= 1) npos += __shfl_xor(npos, o);
    if (lane == 0) reinterpret_cast<int*>(smem + Lay::OFF_FLAG)[0] = a.implicit ? npos : d;
  }
}

// 16x16 Cholesky of the diagonal tile in registers (lane i16 = row i16).  dg = 1/L[i16][i16].
// A pivot that collapses below 2^-21 of its panel-start value is numerically singular in fp32
// (Spark's fp64 dppsv reports info > 0 on such systems); it is reported as not positive definite.
__device__ __forceinline__ bool chol16(float (&rr)[16], float& dg, int i) {
  bool notpd = false;
  float dstart[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) dstart[c] = rdlane(rr[c], c);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const float piv = rdlane(rr[c], c);
    if (!(piv > dstart[c] * 4.76837158e-07f)) notpd = true;
    const float inv = frsq(piv), s = piv * inv;
    rr[c] = (i == c) ? s : rr[c] * inv;
    dg = (i == c) ? inv : dg;
#pragma unroll
    for (int m = c + 1; m < 16; ++m) rr[m] = fmaf(-rr[c], rdlane(rr[c], m), rr[m]);
  }
  return notpd;
}

template <int KP>
__global__ __launch_bounds__(256, 4) void solve_heavy_kernel(SolveArgs a) {
  using Lay = HeavyLds<KP>;
  constexpr int NB = KP / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* bvec = smem + Lay::OFF_B;
  float* sdiag = smem + Lay::OFF_DIAG;
  int* s_flag = reinterpret_cast<int*>(smem + Lay::OFF_FLAG);  // [0] npos, [1] error bits
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, i16 = lane & 15;
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  if (tid == 0) s_flag[1] = 0;
  if (wave == 0) heavy_build<KP, 0>(a, p0, d, smem);
  else if (wave == 1) heavy_build<KP, 1>(a, p0, d, smem);
  else if (wave == 2) heavy_build<KP, 2>(a, p0, d, smem);
  else heavy_build<KP, 3>(a, p0, d, smem);
  __syncthreads();
  const float lamn = a.reg * (float)s_flag[0];
  for (int c = tid; c < KP; c += 256) smem[hel(c, c)] += c < a.kreal ? a.lam[c] + lamn : 1.0f;
  __syncthreads();
  for (int jb = 0; jb < NB; ++jb) {
    const int j0 = 16 * jb;
    const int nrow = KP - j0 - 16 + 1;  // rows below the panel + the b' row
    float rr[16];
    float dg = 1.f;
    bool notpd = false;
    if (wave * 64 < nrow) {
#pragma unroll
      for (int m = 0; m < 16; ++m) rr[m] = smem[htile(jb, jb) + i16 * HT_LD + m];
      notpd = chol16(rr, dg, i16);
      const int ridx = wave * 64 + lane;
      if (ridx < nrow) {  // L21 row = A21 row · L11⁻ᵀ with L11 broadcast from the registers
        const int i = j0 + 16 + ridx;
        float* src = i < KP ? smem + htile(i >> 4, jb) + (i & 15) * HT_LD : bvec + j0;
        float x[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = src[m];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          x[c] *= rdlane(dg, c);
#pragma unroll
          for (int m = c + 1; m < 16; ++m) x[m] = fmaf(-x[c], rdlane(rr[c], m), x[m]);
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) src[m] = x[m];
      }
    }
    __syncthreads();
    if (wave == 0 && lane < 16) {  // L11 back into its tile (read again only by the back substitution)
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m <= i16) smem[htile(jb, jb) + i16 * HT_LD + m] = rr[m];
      sdiag[j0 + i16] = dg;
      if (notpd) s_flag[1] = 2;
    }
    const int nrem = NB - jb - 1;
    const int ntr = nrem * (nrem + 1) / 2;
    for (int t = wave; t < ntr; t += 4) {
      int ti = 0, tt = t;  // lower tiles (I >= M), row-major
      while (tt > ti) { tt -= ti + 1; ++ti; }
      const int I = jb + 1 + ti, M = jb + 1 + tt;
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
    }
    for (int m = j0 + 16 + tid; m < KP; m += 256) {
      float s = bvec[m];
      const float* lr = smem + htile(m >> 4, jb) + (m & 15) * HT_LD;
#pragma unroll
      for (int c = 0; c < 16; ++c) s = fmaf(-bvec[j0 + c], lr[c], s);
      bvec[m] = s;
    }
    __syncthreads();
  }
  if (wave == 0) {  // back substitution Lᵀ x = y, single wave
    for (int jb = NB - 1; jb >= 0; --jb) {
      const int j0 = 16 * jb;
      float yv = bvec[j0 + i16];
      const float sdq = sdiag[j0 + i16];
      float lcol[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) lcol[m] = smem[htile(jb, jb) + m * HT_LD + i16];
#pragma unroll
      for (int i = 15; i >= 0; --i) {
        const float xi = rdlane(yv * sdq, i);
        yv = (i16 < i) ? fmaf(-lcol[i], xi, yv) : ((i16 == i) ? xi : yv);
      }
      if (lane < 16) bvec[j0 + i16] = yv;
      WAVE_LDS_SYNC();
      for (int m = lane; m < j0; m += 64) {
        float s = bvec[m];
        const float* lt = smem + htile(jb, m >> 4) + (m & 15);
#pragma unroll
        for (int c = 0; c < 16; ++c) s = fmaf(-lt[c * HT_LD], bvec[j0 + c], s);
        bvec[m] = s;
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
  }
}

// =============================================================================================
// NNLS rows (nonnegative = true; Spark NNLSSolver -> mllib/optimization/NNLS.scala).  Original basis
// (no rotation: the constraints are coordinate-wise): A = G + λn I + Σ c y yᵀ built exactly like
// the heavy rows (same LDS stage + MFMA + packed tiles) plus the G tiles, then Spark's projected
// gradient with CG acceleration, thread i = coordinate i, fp64 vectors and block reductions.
// =============================================================================================
template <int N>
__device__ __forceinline__ void block_sum(double (&v)[N], double* scr, int& phase) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < N; ++n)
    for (int o = 32; o > 0; o >>= 1) v[n] += __shfl_xor(v[n], o);
  double* sp = scr + phase * 32;
  if (lane == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n) sp[wave * 8 + n] = v[n];
  }
  __syncthreads();
#pragma unroll
  for (int n = 0; n < N; ++n) v[n] = ((sp[n] + sp[8 + n]) + sp[16 + n]) + sp[24 + n];
  phase ^= 1;
}

__device__ __forceinline__ double block_min(double v, double* scr, int& phase) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  double* sp = scr + phase * 32;
  if (lane == 0) sp[wave * 8] = v;
  __syncthreads();
  v = fmin(fmin(sp[0], sp[8]), fmin(sp[16], sp[24]));
  phase ^= 1;
  return v;
}

// (A v)_i for the symmetric matrix held as packed lower tiles; vec in LDS (fp64)
template <int KP>
__device__ __forceinline__ double sym_gemv_row(const float* smem, const double* vec, int i) {
  const int I = i >> 4, ii = i & 15;
  double acc = 0.0;
  for (int J = 0; J < I; ++J) {  // row i, tiles left of the diagonal
    const float* r = smem + htile(I, J) + ii * HT_LD;
#pragma unroll
    for (int c = 0; c < 16; ++c) acc += (double)r[c] * vec[16 * J + c];
  }
  {
    const float* t = smem + htile(I, I);
#pragma unroll
    for (int c = 0; c < 16; ++c) acc += (double)(c <= ii ? t[ii * HT_LD + c] : t[c * HT_LD + ii]) * vec[16 * I + c];
  }
  for (int J = I + 1; J < KP / 16; ++J) {  // column i of the tiles below the diagonal
    const float* t = smem + htile(J, I) + ii;
#pragma unroll
    for (int c = 0; c < 16; ++c) acc += (double)t[c * HT_LD] * vec[16 * J + c];
  }
  return acc;
}

template <int KP>
struct NnlsLds {
  static constexpr int BASE = HeavyLds<KP>::FLOATS;       // heavy layout first (tiles, b', flags)
  static constexpr int OFF_V = (BASE + 1) & ~1;            // fp64 vectors: x, grad, dir (KP each)
  static constexpr int OFF_SCR = OFF_V + 2 * 3 * KP;       // fp64 reduction scratch [2][4][8]
  static constexpr int FLOATS = OFF_SCR + 2 * 64;
};

__device__ __forceinline__ bool nnls_stop(double step, double ndir, double nx) {
  return isnan(step) || step < 1e-7 || step > 1e40 || ndir < 1e-12 * nx || ndir < 1e-32;
}

template <int KP>
__global__ __launch_bounds__(256) void solve_nnls_kernel(SolveArgs a, const float* __restrict__ Gt) {
  using Lay = HeavyLds<KP>;
  using NL = NnlsLds<KP>;
  constexpr int NTL = Lay::NTL;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* bvec = smem + Lay::OFF_B;
  int* s_flag = reinterpret_cast<int*>(smem + Lay::OFF_FLAG);
  double* vx = reinterpret_cast<double*>(smem + NL::OFF_V);
  double* vg = vx + KP;
  double* vd = vg + KP;
  double* scr = reinterpret_cast<double*>(smem + NL::OFF_SCR);
  const int tid = threadIdx.x, wave = tid >> 6;
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  if (tid == 0) s_flag[1] = 0;
  if (wave == 0) heavy_build<KP, 0>(a, p0, d, smem);
  else if (wave == 1) heavy_build<KP, 1>(a, p0, d, smem);
  else if (wave == 2) heavy_build<KP, 2>(a, p0, d, smem);
  else heavy_build<KP, 3>(a, p0, d, smem);
  __syncthreads();
  const float lamn = a.reg * (float)s_flag[0];
  for (int e = tid; e < NTL * HT_SZ; e += 256) smem[e] += Gt[e];   // A = G + Σ c y yᵀ
  __syncthreads();
  for (int c = tid; c < KP; c += 256) smem[hel(c, c)] += c < a.kreal ? lamn : 1.0f;
  const bool own = tid < KP;
  const int i = own ? tid : 0;
  const double bi = own ? (double)bvec[i] : 0.0;
  double xi = 0.0, last_dir = 0.0, last_norm = 0.0;
  if (own) vx[i] = 0.0;
  __syncthreads();
  int phase = 0, last_wall = 0;
  const int iter_max = 400 > 20 * a.kreal ? 400 : 20 * a.kreal;
  for (int iterno = 0; iterno < iter_max; ++iterno) {
    // residual = A x - b ; projected gradient
    const double res = own ? sym_gemv_row<KP>(smem, vx, i) - bi : 0.0;
    double gi = res;
    if (gi > 0.0 && xi == 0.0) gi = 0.0;
    if (own) vg[i] = gi;
    __syncthreads();
    const double agi = own ? sym_gemv_row<KP>(smem, vg, i) : 0.0;
    double r1[4] = {gi * gi, gi * res, gi * agi, xi * xi};
    block_sum<4>(r1, scr, phase);
    const double ngrad = r1[0], nx = r1[3];
    double step = r1[1] / (r1[2] + 1e-20);
    double di = gi, ndir;
    if (iterno > last_wall + 1) {
      const double alpha = ngrad / last_norm;
      di = gi + alpha * last_dir;
      if (own) vd[i] = di;
      __syncthreads();
      const double adi = own ? sym_gemv_row<KP>(smem, vd, i) : 0.0;
      double r2[3] = {di * res, di * adi, di * di};
      block_sum<3>(r2, scr, phase);
      const double dstep = r2[0] / (r2[1] + 1e-20);
      ndir = r2[2];
      if (nnls_stop(dstep, ndir, nx)) {
        di = gi;
        ndir = ngrad;
      } else {
        step = dstep;
      }
    } else {
      ndir = ngrad;
    }
    if (nnls_stop(step, ndir, nx)) break;
    // don't run through the walls: step = min(step, x_i / d_i over d_i > 0 with step d_i > x_i)
    const double cand = (own && step * di > xi) ? xi / di : INFINITY;
    step = fmin(step, block_min(cand, scr, phase));
    // take the step
    double hit = 0.0;
    if (own) {
      if (step * di > xi * (1 - 1e-14)) {
        xi = 0.0;
        hit = 1.0;
      } else {
        xi -= step * di;
      }
      vx[i] = xi;
    }
    double r3[1] = {hit};
    block_sum<1>(r3, scr, phase);
    if (r3[0] > 0.0) last_wall = iterno;
    last_dir = di;
    last_norm = ngrad;
  }
  if (own) a.X[(int64_t)j * KP + i] = i < a.kreal ? (float)xi : 0.f;
  if (tid == 0 && s_flag[1]) atomicOr(a.err, s_flag[1]);
}

hipError_t launch_solve_nnls(int KP, const SolveArgs& a, const float* Gt, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (KP == 64) solve_nnls_kernel<64><<<(int)a.n_rows, 256, NnlsLds<64>::FLOATS * 4, s>>>(a, Gt);
  else if (KP == 128) solve_nnls_kernel<128><<<(int)a.n_rows, 256, NnlsLds<128>::FLOATS * 4, s>>>(a, Gt);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
int nnls_gtile_floats(int KP) { const int nb = KP / 16; return nb * (nb + 1) / 2 * HT_SZ; }
int nnls_gtile_index(int r, int c) { return (r >> 4) * ((r >> 4) + 1) / 2 * HT_SZ + (c >> 4) * HT_SZ + (r & 15) * HT_LD + (c & 15); }

hipError_t launch_solve_heavy(int KP, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (KP == 64) solve_heavy_kernel<64><<<(int)a.n_rows, 256, HeavyLds<64>::FLOATS * 4, s>>>(a);
  else if (KP == 128) solve_heavy_kernel<128><<<(int)a.n_rows, 256, HeavyLds<128>::FLOATS * 4, s>>>(a);
  else return hipErrorInvalidValue;
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
__device__ __forceinline__ float f2j_dot(const float* __restrict__ x, const float* __restrict__ y, int k) {
#pragma clang fp contract(off)
  float acc = 0.f;
  for (int c = 0; c < k; ++c) {
    const float p = x[c] * y[c];
    acc = acc + p;
  }
  return acc;
}

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

// =============================================================================================
// Top-k (ALSRecommender.recommendForUsers / ALSModel.recommendForAll):
//  pass 1  MFMA fp32 scores of 16 src rows x a stripe of dst rows per wave, candidates above a
//          per-row threshold appended to LDS lists, lists compacted (bitonic) to the best KC;
//          the 4 waves' lists are merged and the best KC written out;
//  pass 2  exact F2J rescoring of the KC candidates, sort (score desc, id asc), certification:
//          any non-candidate has approx <= t (the KC-th approx score) so exact <= t + e; if the
//          k-th exact score is not > t + e the row is flagged for an exact full scan.
// =============================================================================================
constexpr int TK_CAP = 128;  // per (wave, src row) list capacity

// key order: higher score first, then lower index
__device__ __forceinline__ bool tk_before(float s1, int i1, float s2, int i2) {
  return s1 > s2 || (s1 == s2 && (unsigned)i1 < (unsigned)i2);
}

// Sort 64*NPL (score, idx) pairs held NPL per lane (element e = lane + 64*h) into tk order
// (best first).  Fully unrolled so every register index is a compile-time constant.
template <int NPL, int K, int JJ>
__device__ __forceinline__ void bitonic_step(float (&sc)[NPL], int (&ix)[NPL], int lane) {
  if constexpr (JJ >= 64) {
    constexpr int hj = JJ >> 6;
    static_for<0, NPL>([&](auto hc) {
      constexpr int h = decltype(hc)::value, hp = h ^ hj;
      if constexpr (hp > h) {
        const int e = lane + 64 * h;
        const bool up = (e & K) == 0;
        const bool sw = up ? tk_before(sc[hp], ix[hp], sc[h], ix[h]) : tk_before(sc[h], ix[h], sc[hp], ix[hp]);
        if (sw) { const float ts = sc[h]; sc[h] = sc[hp]; sc[hp] = ts; const int ti = ix[h]; ix[h] = ix[hp]; ix[hp] = ti; }
      }
    });
  } else {
    static_for<0, NPL>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      const float os = __shfl_xor(sc[h], JJ);
      const int oi = __shfl_xor(ix[h], JJ);
      const int e = lane + 64 * h;
      const bool lower = (lane & JJ) == 0;
      const bool up = (e & K) == 0;
      const bool other_first = tk_before(os, oi, sc[h], ix[h]);
      const bool take = (lower == up) ? other_first : !other_first;
      if (take) { sc[h] = os; ix[h] = oi; }
    });
  }
}
template <int NPL, int K, int JJ>
__device__ __forceinline__ void bitonic_merge(float (&sc)[NPL], int (&ix)[NPL], int lane) {
  if constexpr (JJ > 0) {
    bitonic_step<NPL, K, JJ>(sc, ix, lane);
    bitonic_merge<NPL, K, JJ / 2>(sc, ix, lane);
  }
}
template <int NPL, int K>
__device__ __forceinline__ void bitonic_stages(float (&sc)[NPL], int (&ix)[NPL], int lane) {
  if constexpr (K <= 64 * NPL) {
    bitonic_merge<NPL, K, K / 2>(sc, ix, lane);
    bitonic_stages<NPL, 2 * K>(sc, ix, lane);
  }
}
template <int NPL>
__device__ __forceinline__ void wave_bitonic(float (&sc)[NPL], int (&ix)[NPL]) {
  bitonic_stages<NPL, 2>(sc, ix, threadIdx.x & 63);
}

template <int KP>
__global__ __launch_bounds__(256) void topk_kernel(TopkArgs a) {
  constexpr int NC = KP / 16;  // 16-column chunks
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lsc = smem;                                           // [4][16][CAP]
  int* lix = reinterpret_cast<int*>(smem + 4 * 16 * TK_CAP);   // [4][16][CAP]
  int* lcnt = lix + 4 * 16 * TK_CAP;                           // [4][16]
  float* lthr = reinterpret_cast<float*>(lcnt + 64);           // [4][16]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int64_t sb = (int64_t)blockIdx.x * 16;
  if (threadIdx.x < 64) { lcnt[threadIdx.x] = 0; lthr[threadIdx.x] = -INFINITY; }
  // src fragments: lane holds row (sb + i16), columns c0 + 4g .. +3 for every chunk
  f32x4 su[NC];
  {
    const int64_t si = sb + i16;
    const int srow = si < a.n_src ? a.src_rows[si] : -1;
#pragma unroll
    for (int c = 0; c < NC; ++c) su[c] = srow >= 0 ? ld4(a.S + (int64_t)srow * KP + 16 * c + 4 * g) : zero4();
  }
  __syncthreads();
  float* wsc = lsc + wave * 16 * TK_CAP;
  int* wix = lix + wave * 16 * TK_CAP;
  int* wcnt = lcnt + wave * 16;
  float* wthr = lthr + wave * 16;
  for (int64_t j0 = (int64_t)wave * 64; j0 < a.n_dst; j0 += 256) {
    f32x4 acc[4];
#pragma unroll
    for (int J = 0; J < 4; ++J) acc[J] = zero4();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x4 tv[4];
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        const int64_t dj = j0 + 16 * J + i16;
        tv[J] = dj < a.n_dst ? ld4(a.T + dj * KP + 16 * c + 4 * g) : zero4();
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int J = 0; J < 4; ++J) acc[J] = mfma4(su[c][m], tv[J][m], acc[J]);
    }
    // append candidates: lane holds src rows 4g + r, dst j0 + 16J + i16
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = 4 * g + r;
      const float thr = wthr[sr];
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        const int64_t dj = j0 + 16 * J + i16;
        const float sc = acc[J][r];
        if (dj < a.n_dst && sc >= thr) {
          const int pos = atomicAdd(&wcnt[sr], 1);
          wsc[sr * TK_CAP + pos] = sc;
          wix[sr * TK_CAP + pos] = (int)dj;
        }
      }
    }
    WAVE_LDS_SYNC();
    // compact rows that could overflow on the next tile (each tile adds <= 64 per row)
    for (int sr = 0; sr < 16; ++sr) {
      const int cnt = wcnt[sr];
      if (cnt > TK_CAP - 64) {
        float s2[2];
        int i2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = lane + 64 * h;
          s2[h] = e < cnt ? wsc[sr * TK_CAP + e] : -INFINITY;
          i2[h] = e < cnt ? wix[sr * TK_CAP + e] : -1;
        }
        wave_bitonic<2>(s2, i2);
        WAVE_LDS_SYNC();
        wsc[sr * TK_CAP + lane] = s2[0];
        wix[sr * TK_CAP + lane] = i2[0];
        if (lane == 63) wthr[sr] = s2[0];
        if (lane == 0) wcnt[sr] = 64;
        WAVE_LDS_SYNC();
      }
    }
  }
  __syncthreads();
  // merge the 4 waves' lists per src row: wave w handles rows w, w+4, w+8, w+12
  for (int sr = wave; sr < 16; sr += 4) {
    const int64_t si = sb + sr;
    if (si >= a.n_src) break;
    float s8[8];
    int i8[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const int w = h >> 1, e = lane + 64 * (h & 1);
      const int cnt = lcnt[w * 16 + sr];
      s8[h] = e < cnt ? lsc[(w * 16 + sr) * TK_CAP + e] : -INFINITY;
      i8[h] = e < cnt ? lix[(w * 16 + sr) * TK_CAP + e] : -1;
    }
    wave_bitonic<8>(s8, i8);
    a.cand[si * TOPK_KC + lane] = i8[0];
    a.cand_score[si * TOPK_KC + lane] = s8[0];
  }
}

// One wave per src row: exact F2J rescoring of the KC candidates, sort, certify, write top-k.
template <int KP>
__global__ __launch_bounds__(256) void topk_rescore_kernel(TopkArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t si = (int64_t)blockIdx.x * 4 + wave;
  if (si >= a.n_src) return;
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  const int ci = a.cand[si * TOPK_KC + lane];
  const float approx = a.cand_score[si * TOPK_KC + lane];
  float ex = -INFINITY;
  if (ci >= 0) ex = f2j_dot(s, a.T + (int64_t)ci * KP, a.kreal);
  // t = smallest approx score kept (only meaningful when the list is full)
  float tmin = approx;
  for (int o = 32; o > 0; o >>= 1) tmin = fminf(tmin, __shfl_xor(tmin, o));
  const bool full = a.n_dst > TOPK_KC;
  // ||s||_2 in double for the error bound
  double nn = 0.0;
  for (int c = lane; c < a.kreal; c += 64) nn += (double)s[c] * (double)s[c];
  for (int o = 32; o > 0; o >>= 1) nn += __shfl_xor(nn, o);
  float sc1[1] = {ex};
  int ix1[1] = {ci};
  wave_bitonic<1>(sc1, ix1);
  const int k = a.k;
  const float kth = rdlane(sc1[0], k - 1);
  if (full) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double kk = (double)(a.kreal + 2);
    const double gam = kk * u / (1.0 - kk * u);
    const double e = 2.0 * gam * sqrt(nn) * (double)a.tmax_norm;
    if (!((double)kth > (double)tmin + e)) {
      if (lane == 0) a.need_exact[si] = 1;
    }
  }
  if (lane < k) {
    const int idx = ix1[0];
    a.out_ids[si * k + lane] = idx >= 0 ? a.dst_ids[idx] : -1;
    a.out_scores[si * k + lane] = idx >= 0 ? sc1[0] : __int_as_float(0x7fc00000);
  }
}

// Exact fallback: one workgroup (4 waves) per flagged src row; full F2J scan with a wave-level
// running top-64 per wave, merged at the end.
template <int KP>
__global__ __launch_bounds__(256) void topk_exact_kernel(TopkArgs a, const int32_t* rows) {
  __shared__ float msc[4][64];
  __shared__ int mix[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t si = rows[blockIdx.x];
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  float bs[2] = {-INFINITY, -INFINITY};
  int bi[2] = {-1, -1};
  for (int64_t j0 = (int64_t)wave * 64; j0 < a.n_dst; j0 += 256) {
    const int64_t dj = j0 + lane;
    bs[1] = dj < a.n_dst ? f2j_dot(s, a.T + dj * KP, a.kreal) : -INFINITY;
    bi[1] = dj < a.n_dst ? (int)dj : -1;
    wave_bitonic<2>(bs, bi);  // keeps the best 64 in bs[0]
  }
  msc[wave][lane] = bs[0];
  mix[wave][lane] = bi[0];
  __syncthreads();
  if (wave == 0) {
    float s4[4];
    int i4[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) { s4[h] = msc[h][lane]; i4[h] = mix[h][lane]; }
    wave_bitonic<4>(s4, i4);
    if (lane < a.k) {
      const int idx = i4[0];
      a.out_ids[si * a.k + lane] = idx >= 0 ? a.dst_ids[idx] : -1;
      a.out_scores[si * a.k + lane] = idx >= 0 ? s4[0] : __int_as_float(0x7fc00000);
    }
  }
}

hipError_t launch_topk(int KP, const TopkArgs& a, hipStream_t s) {
  if (a.n_src <= 0) return hipSuccess;
  const int blocks = (int)((a.n_src + 15) / 16);
  const size_t lds = (size_t)4 * 16 * TK_CAP * 8 + 128 * 4;
  if (KP == 64) {
    topk_kernel<64><<<blocks, 256, lds, s>>>(a);
    topk_rescore_kernel<64><<<(int)((a.n_src + 3) / 4), 256, 0, s>>>(a);
  } else if (KP == 128) {
    topk_kernel<128><<<blocks, 256, lds, s>>>(a);
    topk_rescore_kernel<128><<<(int)((a.n_src + 3) / 4), 256, 0, s>>>(a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_topk_exact(int KP, const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  if (KP == 64) topk_exact_kernel<64><<<(int)n_rows, 256, 0, s>>>(a, rows);
  else if (KP == 128) topk_exact_kernel<128><<<(int)n_rows, 256, 0, s>>>(a, rows);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace albedo
