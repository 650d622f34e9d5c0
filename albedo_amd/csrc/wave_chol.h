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
// kept L⁻¹ tiles.  scr: this wave's LDS scratch, WCHOL_SCR floats + NQ·64 f32x4 (L⁻¹ store).
// Returns true when a pivot collapsed (not positive definite; wave-uniform).
#pragma once
#include "device_common.h"

namespace albedo {

#ifdef WAVE_PROBE_CHOL_PHASES  // probes only (tools/probe/factortime.hip): shader-clock time per phase
__device__ unsigned long long* g_chol_ph;  // [row = blockIdx.x * 4 + wave][8]
#define WCHOL_T0() unsigned long long wc_t = __builtin_amdgcn_s_memtime(), wc_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define WCHOL_PH(k) { const unsigned long long wc_n = __builtin_amdgcn_s_memtime(); wc_acc[k] += wc_n - wc_t; wc_t = wc_n; }
#define WCHOL_OUT() \
  if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 8; ++k_) g_chol_ph[((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + k_] = wc_acc[k_]
#else
#define WCHOL_T0()
#define WCHOL_PH(k)
#define WCHOL_OUT()
#endif

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
// scratch layout: 16 x 16 images with a row stride of 20 floats (80 B), so the 16 rows a ds_read_b128
// lane group reads start on 16 disjoint 4-bank groups (a 64-B stride put rows i and i + 4 on the same
// banks); the diagonal tile at 0, b / L⁻¹ at WCHOL_IMG, the L⁻¹ store at WCHOL_SCR
constexpr int WCHOL_RS = 20, WCHOL_IMG = 16 * WCHOL_RS, WCHOL_SCR = 2 * 16 * WCHOL_RS;

template <int NQ, bool SPLIT = false>
__device__ __forceinline__ bool wave_chol_solve(f32x4 (&acc)[NQ * (NQ + 1) / 2], float (&bacc)[NQ], float* scr,
                                                float (&xs)[NQ]) {
  const int lane = threadIdx.x & 63, q = lane >> 4, i16 = lane & 15;
  // L⁻¹ of every panel in the A-operand layout (lane i + 16q: L⁻¹[i][4q .. 4q+3]), kept in the dead
  // stage for the back substitution: [NQ][64 lanes] f32x4 after the two scratch tiles
  f32x4* s_linv = reinterpret_cast<f32x4*>(scr + WCHOL_SCR);
  bool notpd = false;
  WCHOL_T0();
  static_for<0, NQ>([&](auto JB) {
    constexpr int jb = decltype(JB)::value, td = tix(jb, jb, NQ);
    // diagonal tile to the row layout of chol16 (lane i: row i, replicated over the 4 lane groups)
#pragma unroll
    for (int r = 0; r < 4; ++r) scr[(4 * q + r) * WCHOL_RS + i16] = acc[td][r];
    if (q == 0) scr[WCHOL_IMG + i16] = bacc[jb];  // b_jb alongside (the L⁻¹ image overwrites it later)
    WAVE_LDS_SYNC();
    float rr[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 v = ld4(scr + WCHOL_RS * i16 + 4 * u);
#pragma unroll
      for (int e = 0; e < 4; ++e) rr[4 * u + e] = v[e];
    }
    const f32x4 bt = ld4(scr + WCHOL_IMG + 4 * q);  // lane i + 16q: b_jb[4q .. 4q+3] (the MFMA k layout)
    float dg = 1.f;
    WCHOL_PH(0);
    notpd |= chol16(rr, dg, i16);
    WCHOL_PH(1);
    // chol16 ends in inline asm: two wait states before any DPP read of its results
    asm volatile("s_nop 1"
                 : "+v"(rr[0]), "+v"(rr[1]), "+v"(rr[2]), "+v"(rr[3]), "+v"(rr[4]), "+v"(rr[5]), "+v"(rr[6]),
                   "+v"(rr[7]), "+v"(rr[8]), "+v"(rr[9]), "+v"(rr[10]), "+v"(rr[11]), "+v"(rr[12]),
                   "+v"(rr[13]), "+v"(rr[14]), "+v"(rr[15]), "+v"(dg));
    // column i16 of L⁻¹: L x = e_i16 by forward substitution, L[r][m] broadcast from lane r.  Right-
    // looking (x_m, then every later row's update by x_m): the updates of one step are independent, so
    // the dependent chain is 16 steps long instead of 120 FMAs; each row still accumulates its terms
    // in increasing m (the same roundings as the dot-product order).
    float x[16];  // row r's running value until step r, then L⁻¹[r][i16]
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = (i16 == r) ? 1.f : 0.f;
    static_for<0, 16>([&](auto MM) {
      constexpr int m = decltype(MM)::value;
      x[m] *= bc16_after_asm<m>(dg);
      // one v_fmac_f32_dpp per term (asm keeps the broadcasts from being hoisted into registers)
      static_for<m + 1, 16>([&](auto RR) {
        constexpr int r = decltype(RR)::value;
        fnmac_bc16<r, false>(x[r], rr[m], x[m]);
      });
    });
    if (q == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) scr[WCHOL_IMG + WCHOL_RS * r + i16] = x[r];
    }
    WAVE_LDS_SYNC();
    const f32x4 lv = ld4(scr + WCHOL_IMG + WCHOL_RS * i16 + 4 * q);
    s_linv[jb * 64 + lane] = lv;
    WCHOL_PH(2);
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
    WCHOL_PH(3);
    float yp = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) yp = fmaf(lv[s], bt[s], yp);
    yp = rows4_sum(yp);
    bacc[jb] = yp;
    // y[4q .. 4q+3] to lane group q through the scratch (the L⁻¹ image's first row is already read)
    if (q == 0) scr[WCHOL_IMG + i16] = yp;
    WAVE_LDS_SYNC();
    const f32x4 y4 = ld4(scr + WCHOL_IMG + 4 * q);
    static_for<jb + 1, NQ>([&](auto MM) {
      constexpr int M = decltype(MM)::value, t = tix(jb, M, NQ);
      float pv = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) pv = fmaf(acc[t][r], y4[r], pv);
      bacc[M] -= rows4_sum(pv);
    });
    WCHOL_PH(4);
    // trailing tiles: T(M, I) -= U(jb, M)ᵀ U(jb, I), the next diagonal tile first
    if constexpr (SPLIT) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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
    WCHOL_PH(5);
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
    const f32x4 lv = s_linv[jb * 64 + lane];
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
  WCHOL_PH(6);
  WCHOL_OUT();
  return notpd;
}

}  // namespace albedo
