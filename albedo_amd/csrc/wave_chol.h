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
// Right-looking, 16-wide panels: the diagonal tile goes through LDS into a row layout, one 16-step
// Gaussian elimination with the inverse riding along gives its L⁻¹ (elim16_inverse), the panel row
// is U = L⁻¹·T on f32 MFMA and the trailing tiles are updated with UᵀU on MFMA -- the C/D layout of
// one MFMA is the A and B operand layout of the next, so no tile moves and no workgroup barrier is
// needed.  The right-hand side follows as a VALU column behind the trailing MFMAs, then a
// right-looking block back substitution with the L⁻¹ images.  scr: this wave's LDS scratch,
// wchol_scratch_floats(NQ) floats.
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

// row_c -> row_i update of the elimination below: x -= f · (x of lane C of the 16-lane row), one
// v_fmac_f32_dpp whose DPP source is the accumulator register itself (lane C's copy of the same
// entry).  Every VGPR a DPP instruction reads needs two wait states after its last write; the
// callers order the updates so that the previous write of x is at least two instructions back and
// f is written before the step's first update, which carries the s_nop (NOP = true).  The build
// re-checks the emitted code for exactly this rule (tools/isa_hazards.py).
template <int C, bool NOP>
__device__ __forceinline__ void elim_upd(float& x, float f) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, -%0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(x) : "v"(f), "n"(C));
  else
    asm volatile("v_fmac_f32_dpp %0, -%0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(x) : "v"(f), "n"(C));
}

// Lane group G's value of x in every lane (same lane within the 16-lane row): v_permlane16_swap
// leaves rows (0, 0, 2, 2) in its first result and (1, 1, 3, 3) in its second, v_permlane32_swap of
// that leaves (0, 1, 0, 1) / (2, 3, 2, 3); G picks the results at compile time, so the broadcast is
// two VALU instructions and no selects (tools/probe/permlane_probe.hip checks the semantics)
template <int G>
__device__ __forceinline__ float grp_bcast(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const uint32_t p = (G & 1) ? a[1] : a[0];
  const auto b = __builtin_amdgcn_permlane32_swap(p, p, false, false);
  return __uint_as_float((G & 2) ? b[1] : b[0]);
}

// Inverse Cholesky factor of a 16x16 SPD tile by Gaussian elimination with the inverse riding
// along, in one 16-step chain, the work spread over the four lane groups.  Row i of the
// concatenation [X | R] (X the tile, R starting as the identity) has 32 columns, and at step c
// exactly 16 of them change: X's c+1..15 and R's 0..c.  Lane i + 16q keeps, for each of the four
// columns m = 4q + s of its group, one register w[s]: X[i][m] until step m, then R[i][m] -- at step
// m column m of X has served as the pivot column and R's column m starts to change, so every lane
// updates exactly four live entries per step (the tile, replicated over the groups, took 15 - c
// updates plus the inverse's).  Step c: the pivot X[c][c] by readlane (uniform), the owner group
// G = c >> 2 forms the multipliers f_i = X[i][c] / X[c][c] (i > c) from its register, grp_bcast
// hands them to every group, the owner slot restarts as R's column c (e_c), and each
// w[s] -= f_i · (w[s] of lane c) -- one v_fmac_f32_dpp whose DPP source is the register itself (the
// owner slot becomes e_c - f, R's column c after step c).  The pivots are Cholesky's (d_i = L[i][i]²), R is the unit-lower inverse, so
// L⁻¹ = diag(d)^(-1/2) R, returned in the A-operand layout (lane i + 16q: L⁻¹[i][4q .. 4q+3]).
// The tile arrives in the MFMA C/D layout (lane i + 16q: D[4q + r][i] = D[i][4q + r] by symmetry),
// which is already this layout: no LDS round trip.  Step c + 1's pivot and multipliers are formed
// right after step c updates column c + 1 (its register goes first), so their latency hides behind
// step c's remaining updates.  notpd: a pivot collapsed below 2^-21 of its start value
// (numerically singular in fp32; wave-uniform).
__device__ __forceinline__ f32x4 elim16_inverse(f32x4 tile, int i16, int q, bool& notpd) {
  float w[4] = {tile[0], tile[1], tile[2], tile[3]};
  // start diagonal D[i][i] (lane i of group i >> 2, slot i & 3); the check runs in those lanes only
  const bool own = q == (i16 >> 2);
  float d0 = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) d0 = (own && (i16 & 3) == s) ? w[s] : d0;
  float dpiv = 1.f;
  uint64_t gmask[4];  // lanes of group g (the owner slot's switch to R)
#pragma unroll
  for (int g = 0; g < 4; ++g) gmask[g] = __ballot(q == g);
  float eye[4];  // R's start: lane i + 16q, slot s = (i == 4q + s)
#pragma unroll
  for (int s = 0; s < 4; ++s) eye[s] = (i16 == 4 * q + s) ? 1.f : 0.f;
  // multipliers of step c from the current register of column c (wave-uniform pivot by readlane)
  auto mult = [&](auto CC) {
    constexpr int c = decltype(CC)::value, G = c >> 2, S = c & 3;
    const float p = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w[S]), 16 * G + c));
    dpiv = (i16 == c) ? p : dpiv;
    const float fo = (i16 > c) ? w[S] * frcp(p) : 0.f;  // right in group G only
    return grp_bcast<G>(fo);
  };
  float f = mult(std::integral_constant<int, 0>{});
  static_for<0, 16>([&](auto CC) {
    constexpr int c = decltype(CC)::value, G = c >> 2, S = c & 3;
    // owner slot: X's column c is spent once its multipliers are formed; it restarts as R's column c
    // (e_c), and the step's own update below makes it e_c - f.  A volatile asm select: left to
    // itself the compiler sinks it next to the register's update, whose DPP read then follows the
    // write inside the two wait states (tools/isa_hazards.py); the owner slot's update goes last
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(w[S]) : "v"(eye[S]), "s"(gmask[G]));
    float fn = 0.f;
    if constexpr (c + 1 < 16) {
      constexpr int SN = (c + 1) & 3;
      elim_upd<c, true>(w[SN], f);  // column c + 1's register first: the next pivot
      fn = mult(std::integral_constant<int, c + 1>{});
      static_for<1, 4>([&](auto KK) {  // SN + 3 = S: the owner slot last
        constexpr int s = (SN + decltype(KK)::value) & 3;
        elim_upd<c, false>(w[s], f);
      });
    }
    f = fn;
  });
  notpd = __any(own && !(dpiv > d0 * 4.76837158e-07f));
  const float sc = frsq(dpiv);
  return f32x4{w[0] * sc, w[1] * sc, w[2] * sc, w[3] * sc};
}

// Sum over each 16-lane row with the result in every lane of the row: DPP quad permutes, then the
// half-row and row mirrors (each step adds the same two partial sums in every lane: all 16 lanes end
// bit-identical)
__device__ __forceinline__ float sum16_all(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true));  // row_half_mirror
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, true));  // row_mirror
  return x;
}

// SPLIT: the trailing updates T -= UᵀU run on v_mfma_f32_16x16x32_f16 with U split into fp16 hi + lo
// (hi·hi + hi·lo + lo·hi in two MFMAs: k-slots 0..3 / 4..7 of a lane carry the same four rows as hi /
// lo, so the operands come straight from the C/D registers) instead of four f32 MFMAs: 32 instead of
// 128 matrix-core cycles per tile update.  The caller scales the system so that every U entry is
// below 2^14 (|U_ij| <= sqrt(A_jj): max diagonal < 2^28), keeping hi and lo in fp16's normal range.
// Scratch (floats): one L⁻¹ image per panel (row-major), then y (16 per panel).  Images have a row
// stride of 20 floats (80 B): the four rows 4g + r the C/D reads of lane group g touch sit 16 banks
// apart.
constexpr int WCHOL_RS = 20, WCHOL_IMG = 16 * WCHOL_RS;
__host__ __device__ constexpr int wchol_scratch_floats(int nq) { return WCHOL_IMG * nq + 16 * nq; }

template <int NQ, bool SPLIT = false>
__device__ __forceinline__ bool wave_chol_solve(f32x4 (&acc)[NQ * (NQ + 1) / 2], float (&bacc)[NQ], float* scr,
                                                float (&xs)[NQ]) {
  const int lane = threadIdx.x & 63, q = lane >> 4, i16 = lane & 15;
  float* s_y = scr + WCHOL_IMG * NQ;  // y of every panel in the lane-group layout
  bool notpd = false;
  WCHOL_T0();
  static_for<0, NQ>([&](auto JB) {
    constexpr int jb = decltype(JB)::value, td = tix(jb, jb, NQ);
    float* img = scr + WCHOL_IMG * jb;  // this panel's L⁻¹, row-major
    WCHOL_PH(0);
    bool np;
    const f32x4 lv = elim16_inverse(acc[td], i16, q, np);  // lane i + 16q: L⁻¹[i][4q .. 4q+3]
    notpd |= np;
    WCHOL_PH(1);
    // L⁻¹ image: the RHS and the back substitution read it in the C/D layout
    *reinterpret_cast<f32x4*>(img + WCHOL_RS * i16 + 4 * q) = lv;
    // panel row: U(jb, I) = L⁻¹ T(jb, I)  (A = L⁻¹ rows, B = the tile's C/D registers)
    static_for<jb + 1, NQ>([&](auto II) {
      constexpr int I = decltype(II)::value, t = tix(jb, I, NQ);
      f32x4 u = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) u = mfma4(lv[s], acc[t][s], u);
      acc[t] = u;
    });
    // lane c + 16g: L⁻¹[4g + r][c] (the LDS pipe is in order: the image stores above come first)
    WAVE_LDS_FENCE();
    float lc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lc[r] = img[WCHOL_RS * (4 * q + r) + i16];
    WCHOL_PH(2);
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
    WCHOL_PH(3);
    // RHS, behind the trailing MFMAs: y_jb = L⁻¹ b_jb straight into the lane-group layout (lane c + 16g:
    // Σ_c L⁻¹[4g + r][c] b[c] summed over the row, y[4g + r] in every lane of group g), then
    // b_M -= U(jb, M)ᵀ y_jb for the blocks below (lane c + 16g: Σ_r U[4g + r][c] y[4g + r], summed
    // over the four groups) -- no LDS round trip on this chain
    float y4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) y4[r] = sum16_all(lc[r] * bacc[jb]);
    if (i16 == 0) *reinterpret_cast<f32x4*>(s_y + 16 * jb + 4 * q) = f32x4{y4[0], y4[1], y4[2], y4[3]};
    static_for<jb + 1, NQ>([&](auto MM) {
      constexpr int M = decltype(MM)::value, t = tix(jb, M, NQ);
      float pv = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) pv = fmaf(acc[t][r], y4[r], pv);
      bacc[M] -= rows4_sum(pv);
    });
    WCHOL_PH(4);
    WAVE_LDS_FENCE();  // the y store before any later read of it
  });

  // ---- back substitution: x_jb = L_jb⁻ᵀ (y_jb - Σ_{M > jb} U(jb, M) x_M), right-looking: as soon as
  // x_M is known every block above takes its products (lane c + 16g: U(jb, M)[4g + r][c] x_M[c]), so
  // the chain per block is one row sum, L⁻ᵀ on the lane-group layout and one cross-group sum
  float pr[NQ][4];
#pragma unroll
  for (int b = 0; b < NQ; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) pr[b][r] = 0.f;
  static_for<0, NQ>([&](auto KK) {
    constexpr int jb = NQ - 1 - decltype(KK)::value;
    const float* img = scr + WCHOL_IMG * jb;
    const f32x4 yb = ld4(s_y + 16 * jb + 4 * q);  // y[4g .. 4g+3]
    float xp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float t = yb[r] - sum16_all(pr[jb][r]);       // t[4g + r] in every lane of group g
      xp = fmaf(img[WCHOL_RS * (4 * q + r) + i16], t, xp);  // L⁻¹[4g + r][c] t[4g + r]
    }
    xs[jb] = rows4_sum(xp);  // x[c] in lane c of every group
    static_for<0, jb>([&](auto BB) {
      constexpr int b = decltype(BB)::value, t = tix(b, jb, NQ);
#pragma unroll
      for (int r = 0; r < 4; ++r) pr[b][r] = fmaf(acc[t][r], xs[jb], pr[b][r]);
    });
  });
  WCHOL_PH(6);
  WCHOL_OUT();
  return notpd;
}

}  // namespace albedo
