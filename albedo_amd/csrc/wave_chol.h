// Blocked Cholesky solve of one SPD system held by ONE wave in MFMA accumulators (gfx950), shared by
// the heavy-row wave kernel (heavy_wave.hip: the k x k normal equation of Spark's CholeskySolver,
// reached from ALSRecommenderBuilder.scala:58) and the light rows' d x d push-through system
// (als_kernels.hip solve_light_kernel, d in (16, 64]).
//
//   A   NQ(NQ+1)/2 upper 16x16 tiles, tile (a, b) = acc[tix(a, b, NQ)] in the C/D layout of
//       v_mfma_f32_16x16x*: lane i + 16q holds rows 16a + 4q + r (r = 0..3), column 16b + i
//   b   bacc[A] in lane i + 16q = b[16A + i] (replicated over q)
//   x   xs[A], same layout as b
//
// Right-looking, 16-wide panels: the diagonal tile goes through LDS into the row layout of chol16
// (DPP broadcasts), its L⁻¹ comes from a 16-step v_fmac_f32_dpp substitution, the panel row is
// U = L⁻¹·T on f32 MFMA and the trailing tiles are updated with UᵀU on f32 MFMA -- the C/D layout of
// one MFMA is the A and B operand layout of the next, so no tile moves and no workgroup barrier is
// needed.  The right-hand side follows as a VALU column, then a block back substitution with the
// kept L⁻¹ tiles: each panel's L⁻¹ (A-operand layout) replaces its diagonal tile in the accumulators,
// which is dead once it has been factored.  scr: this wave's LDS scratch, 512 floats.
// Returns true when a pivot collapsed (not positive definite; wave-uniform).
#pragma once
#include "device_common.h"

namespace albedo {

// upper tile (a <= b) index, row-major over the upper triangle
__host__ __device__ constexpr int tix(int a, int b, int nq) { return a * nq - a * (a - 1) / 2 + (b - a); }

// fp16 hi (slots 0..3) and lo (slots 4..7) of four fp32 values: packed RNE conversion for hi, lo =
// fp16(x - hi) by v_fma_mix (x·1 - hi is exact in fp32, so one rounding)
__device__ __forceinline__ f16x8 split_hilo4(f32x4 v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  uint32_t w[4];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const f16x2 h = __builtin_convertvector((f32x2v{v[2 * p], v[2 * p + 1]}), f16x2);
    w[p] = __builtin_bit_cast(uint32_t, h);
    uint32_t l;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(l) : "v"(v[2 * p]), "v"(v[2 * p + 1]), "v"(w[p]));
    w[2 + p] = l;
  }
  return __builtin_bit_cast(f16x8, (u32x4{w[0], w[1], w[2], w[3]}));
}

// SPLIT: the trailing updates T -= UᵀU run on v_mfma_f32_16x16x32_f16 with U split into fp16 hi + lo
// (hi·hi + hi·lo + lo·hi in two MFMAs: k-slots 0..3 / 4..7 of a lane carry the same four rows as hi /
// lo, so the operands come straight from the C/D registers) instead of four f32 MFMAs: 32 instead of
// 128 matrix-core cycles per tile update.  The caller scales the system so that every U entry is
// below 2^14 (|U_ij| <= sqrt(A_jj): max diagonal < 2^28), keeping hi and lo in fp16's normal range.
// The diagonal block of a panel: rr (lane i: row i of a 16 x 16 SPD tile, in every 16-lane group) ->
// rr[m] = L[i][m] (m <= i) and x[r] = L⁻¹[r][i] (column i of the inverse Cholesky factor); returns
// whether a pivot collapsed (wave-uniform).  The Cholesky step c and the inverse's step c - 1 are
// independent (step c - 1 of the substitution needs column c - 1 of L and 1/L[c-1][c-1], final after
// Cholesky step c - 1), so they are issued interleaved: the two dependent chains overlap.  A pivot
// that collapses below 2^-21 of its start value is numerically singular in fp32 (Spark's fp64 dppsv
// reports info > 0 on such systems).
__device__ __forceinline__ bool diag_block(float (&rr)[16], float (&x)[16], int i16) {
  bool notpd = false;
  float d0 = 0.f, dg = 1.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) d0 = (i16 == c) ? rr[c] : d0;
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = (i16 == r) ? 1.f : 0.f;
  // step m of L x = e_i16 (right-looking: x_m, then every later row's update by x_m; each row still
  // accumulates its terms in increasing m, the same roundings as the dot-product order)
  auto inv_step = [&](auto MM) {
    constexpr int m = decltype(MM)::value;
    x[m] *= bc16_after_asm<m>(dg);
    static_for<m + 1, 16>([&](auto RR) {
      constexpr int r = decltype(RR)::value;
      fnmac_bc16<r, false>(x[r], rr[m], x[m]);  // L[r][m] from lane r
    });
  };
  static_for<0, 16>([&](auto CC) {
    constexpr int c = decltype(CC)::value;
    if (i16 == c && !(rr[c] > d0 * 4.76837158e-07f)) notpd = true;
    const float piv = bc16_after_asm<c>(rr[c]);
    const float inv = frsq(piv), sq = piv * inv;
    rr[c] = (i16 == c) ? sq : rr[c] * inv;
    dg = (i16 == c) ? inv : dg;
    static_for<c + 1, 16>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      fnmac_bc16<m, m == c + 1>(rr[m], rr[c], rr[c]);
    });
    if constexpr (c >= 1) inv_step(std::integral_constant<int, c - 1>{});
  });
  // the last step's results came from inline asm: two wait states before its DPP reads
  asm volatile("s_nop 1" : "+v"(rr[15]), "+v"(dg));
  inv_step(std::integral_constant<int, 15>{});
  return __any(notpd);
}

template <int NQ, bool SPLIT = false>
__device__ __forceinline__ bool wave_chol_solve(f32x4 (&acc)[NQ * (NQ + 1) / 2], float (&bacc)[NQ], float* scr,
                                                float (&xs)[NQ], const int lane = threadIdx.x & 63) {
  const int q = lane >> 4, i16 = lane & 15;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  bool notpd = false;
  static_for<0, NQ>([&](auto JB) {
    constexpr int jb = decltype(JB)::value, td = tix(jb, jb, NQ);
    // diagonal tile to the row layout of chol16 (lane i: row i, replicated over the 4 lane groups)
#pragma unroll
    for (int r = 0; r < 4; ++r) scr[(4 * q + r) * 16 + i16] = acc[td][r];
    if (q == 0) scr[256 + i16] = bacc[jb];  // b_jb alongside (the L⁻¹ image overwrites it later)
    WAVE_LDS_SYNC();
    const f32x4 bt = ld4(scr + 256 + 4 * q);  // lane i + 16q: b_jb[4q .. 4q+3] (the MFMA k layout)
    float rr[16], x[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 v = ld4(scr + 16 * i16 + 4 * u);
#pragma unroll
      for (int e = 0; e < 4; ++e) rr[4 * u + e] = v[e];
    }
    notpd |= __any(diag_block(rr, x, i16));
    if (q == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) scr[256 + 16 * r + i16] = x[r];
    }
    WAVE_LDS_SYNC();
    // L⁻¹ in the A-operand layout (lane i + 16q: L⁻¹[i][4q .. 4q+3]); it replaces the factored
    // diagonal tile in the accumulators (kept for the back substitution)
    const f32x4 lv = ld4(scr + 256 + 16 * i16 + 4 * q);
    acc[td] = lv;
    // panel row: U(jb, I) = L⁻¹ T(jb, I)  (A = L⁻¹ rows, B = the tile's C/D registers)
    static_for<jb + 1, NQ>([&](auto II) {
      constexpr int I = decltype(II)::value, t = tix(jb, I, NQ);
      f32x4 u = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) u = mfma4(lv[s], acc[t][s], u);
      acc[t] = u;
    });
    // RHS: y_jb = L⁻¹ b_jb, then b_M -= U(jb, M)ᵀ y_jb for the blocks below (VALU + shuffles: the
    // same products on the f32 MFMA -- 8 + 4 per block -- measured slower, they compete with the
    // other wave's build for the matrix core)
    float yp = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) yp = fmaf(lv[s], bt[s], yp);
    yp = rows4_sum(yp);
    bacc[jb] = yp;
    // y[4q .. 4q+3] to lane group q through the scratch (the L⁻¹ image's first row is already read)
    if (q == 0) scr[256 + i16] = yp;
    WAVE_LDS_SYNC();
    const f32x4 y4 = ld4(scr + 256 + 4 * q);
    static_for<jb + 1, NQ>([&](auto MM) {
      constexpr int M = decltype(MM)::value, t = tix(jb, M, NQ);
      float pv = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) pv = fmaf(acc[t][r], y4[r], pv);
      bacc[M] -= rows4_sum(pv);
    });
    // trailing tiles: T(M, I) -= U(jb, M)ᵀ U(jb, I), the next diagonal tile first
    if constexpr (SPLIT) {
      f16x8 ub[NQ];  // B operands [hi | lo] of the panel row's tiles
      static_for<jb + 1, NQ>([&](auto II) {
        constexpr int I = decltype(II)::value;
        ub[I] = split_hilo4(acc[tix(jb, I, NQ)]);
      });
      static_for<jb + 1, NQ>([&](auto MM) {
        constexpr int M = decltype(MM)::value;
        const u32x4 w = __builtin_bit_cast(u32x4, ub[M]) ^ 0x80008000u;  // -hi, -lo
        const f16x8 a1 = __builtin_bit_cast(f16x8, (u32x4{w[0], w[1], w[0], w[1]}));  // [-hi | -hi]
        const f16x8 a2 = __builtin_bit_cast(f16x8, (u32x4{w[2], w[3], 0u, 0u}));      // [-lo | 0]
        static_for<M, NQ>([&](auto II) {
          constexpr int I = decltype(II)::value, t = tix(M, I, NQ);
          acc[t] = mfma_h(a1, ub[I], acc[t]);  // -(hi_M·hi_I + hi_M·lo_I)
          acc[t] = mfma_h(a2, ub[I], acc[t]);  // -(lo_M·hi_I)
        });
      });
    } else {
      static_for<jb + 1, NQ>([&](auto MM) {
        constexpr int M = decltype(MM)::value, tm = tix(jb, M, NQ);
        static_for<M, NQ>([&](auto II) {
          constexpr int I = decltype(II)::value, t = tix(M, I, NQ), ti = tix(jb, I, NQ);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[t] = mfma4(-acc[tm][s], acc[ti][s], acc[t]);
        });
      });
    }
    WAVE_LDS_SYNC();  // scratch reads done before the next panel rewrites it
  });

  // ---- back substitution: x_jb = L_jb⁻ᵀ (y_jb - Σ_{M > jb} U(jb, M) x_M) ------------------------
  static_for<0, NQ>([&](auto KK) {
    constexpr int jb = NQ - 1 - decltype(KK)::value;
    float pr[4] = {0.f, 0.f, 0.f, 0.f};  // lane c + 16g: Σ_M U(jb, M)[4g + r][c] x_M[c]
    static_for<jb + 1, NQ>([&](auto MM) {
      constexpr int M = decltype(MM)::value, t = tix(jb, M, NQ);
#pragma unroll
      for (int r = 0; r < 4; ++r) pr[r] = fmaf(acc[t][r], xs[M], pr[r]);
    });
    float tq[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tq[r] = sum16_last(pr[r]);  // row 4g + r in lane 15 + 16g
    // lane i + 16q gets t_i = y_i - (row i's sum): row i lives in lane 15 + 16(i >> 2), slot i & 3,
    // gathered through the scratch (one store + one load instead of four shuffles)
    const f32x4 lv = acc[tix(jb, jb, NQ)];  // L⁻¹ of panel jb
    if (i16 == 15) *reinterpret_cast<f32x4*>(scr + 4 * q) = f32x4{tq[0], tq[1], tq[2], tq[3]};
    WAVE_LDS_SYNC();
    const float ti = bacc[jb] - scr[i16];
    // x = L⁻ᵀ t: lane k + 16q holds L⁻¹[k][4q + s]; x[4q + s] = Σ_k L⁻¹[k][4q + s] t_k
    float xq[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) xq[s] = sum16_last(lv[s] * ti);  // x[4g + s] in lane 15 + 16g
    if (i16 == 15) *reinterpret_cast<f32x4*>(scr + 16 + 4 * q) = f32x4{xq[0], xq[1], xq[2], xq[3]};
    WAVE_LDS_SYNC();
    xs[jb] = scr[16 + i16];
  });
  return notpd;
}

}  // namespace albedo
