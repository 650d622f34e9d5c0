// Heavy rows, one WAVE per dst row (padded rank KP <= 128): the row's whole normal equation lives in
// that wave's MFMA accumulators from the first gathered rating to the last pivot.
//
// Same equation as solve_heavy_kernel (als_kernels.hip), in the eigenbasis of the src Gram
// (Spark ALS.computeFactors: NormalEquation.add per rating + CholeskySolver, reached from
// ALSRecommenderBuilder.scala:58):  A' = diag(Λ + λn) + Σ c z zᵀ,  b' = Σ w z,  A' x = b'.
//
//  gather   the row's factor rows arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
//           wave-instruction = 2 rows at KP = 128), 32 ratings per stage, into a per-wave raw fp32
//           stage.  No registers hold data in flight, so 8 waves per CU keep 8 stages in flight.
//  build    each lane reads its MFMA fragments (8 ratings of one column per 16-column block) out of
//           the stage, scales them by √c and the column's power of two, splits them into fp16
//           hi + lo and accumulates the NQ(NQ+1)/2 upper 16x16 tiles with hi·hi + hi·lo + lo·hi
//           on v_mfma_f32_16x16x32_f16 (fp32 accumulation; the numerics of heavy_build).  b' is an
//           fp32 VALU sum of w·z.  The stage is refilled as soon as the fragments are in registers.
//  factor   right-looking blocked Cholesky A' = UᵀU on the accumulator tiles themselves: per panel,
//           the diagonal tile goes through LDS into the row layout of chol16, L⁻¹ of the tile comes
//           from a 16-step DPP substitution, the panel row is U = L⁻¹·T on f32 MFMA and the trailing
//           tiles are updated with Uᵀ U on f32 MFMA -- the C/D layout of one MFMA is the A and B
//           operand layout of the next, so no tile moves.  The right-hand side follows as an extra
//           VALU column, then a block back substitution with the kept L⁻¹ tiles.
// Against the 4-wave workgroup kernel this trades 4 waves x 39 KB of LDS per row for one wave and
// 16.5 KB: twice the rows in flight per CU, and no workgroup barriers in the factorisation.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include "device_common.h"
#include "kernels.h"
#include "wave_chol.h"
#include "split_rec.h"

namespace albedo {
namespace {

#ifdef WAVE_PROBE_STAMPS  // probes only (tools/probe/wavetime.hip): per-row shader-clock stamps
__device__ unsigned long long* g_wave_stamps;  // [rows][4]: start, build done, factor done, stored
#define WAVE_STAMP(row, i) \
  if ((threadIdx.x & 63) == 0) g_wave_stamps[(row) * 4 + (i)] = __builtin_amdgcn_s_memtime()
#else
#define WAVE_STAMP(row, i) (void)0
#endif

typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) const void* glb_vp;

template <int KP>
struct WaveRow {
  static constexpr int NQ = KP / 16, NT = NQ * (NQ + 1) / 2;
  static constexpr int SPS = 32;                         // ratings per stage = one 16x16x32 k-step
  static constexpr int RB = 4 * KP;                      // bytes per factor row
  static constexpr int RPI = 1024 / RB;                  // rows per LDS-DMA wave-instruction
  static constexpr int LPR = 64 / RPI;                   // lanes per row in one instruction
  static constexpr int NI = SPS / RPI;                   // DMA instructions per stage
  static constexpr int STAGE = SPS * RB + 64 * (SPS / 8 - 1);  // + 64 B per 8-rating group (banks)
  static constexpr int WAVES = 4;                        // rows per workgroup (independent waves)
  static constexpr int LDS_WAVE = (STAGE + 255) & ~255;
  static constexpr int LDS = WAVES * LDS_WAVE + 2 * KP * 4;  // + column scales and inverses
  static_assert(RPI * RB == 1024 && 8 % RPI == 0, "DMA pieces never cross an 8-rating group");
  static_assert(LDS_WAVE >= 4 * wchol_scratch_floats(NQ), "the stage doubles as the factor's scratch");
};

// LDS byte offset of (rating r of the stage, column c).  Lane i + 16q reads ratings 8q..8q+7 of
// column 16A + i: the 64-B shift per 8-rating group puts the four q groups on different banks.
template <int KP>
__device__ __forceinline__ int soff(int r, int c) { return r * 4 * KP + 64 * (r >> 3) + 4 * c; }

// Pre-split stage layout (PRE): rating row r of the stage holds RB/16 chunks of 16 B (fp16 hi of the
// row's KP columns, then lo); chunk c sits at chunk position c ^ f(r), f(r) = 2·((r & 3) | ((r & 8) >> 1)).
// A transposed read (ds_read_b64_tr_b16) of one 16-column block takes, per 32-lane half, 8 rows whose
// f differ, i.e. 8 distinct 32-B bank windows: conflict-free.
__device__ __forceinline__ int pre_f(int r) { return 2 * ((r & 3) | ((r & 8) >> 1)); }
typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_vs __attribute__((__vector_size__(8)));
__device__ __forceinline__ f16x4v tr_read(const char* p) {
  const fp16x4_vs v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_vs*)(p));
  return __builtin_bit_cast(f16x4v, v);
}

// The build of one row's (or split-K chunk's) normal equation by one wave: ratings p0 .. p0+d-1 of
// the CSR, gathered 32 per stage into this wave's LDS stage st.  On return acc holds the NT upper
// tiles of Σ c·(cs z)(cs z)ᵀ (still column-scaled), bacc[A] (lane i + 16q) b'[16A + i] unscaled;
// returns the number of positive ratings.
template <int KP, bool IMPLICIT, bool PRE>
__device__ __forceinline__ int wave_build(const SolveArgs& a, int64_t p0, int d, char* st, const float* s_cs,
                                          f32x4 (&acc)[WaveRow<KP>::NT], float (&bacc)[WaveRow<KP>::NQ]) {
  using W = WaveRow<KP>;
  constexpr int NQ = W::NQ, NT = W::NT;
  const int lane = threadIdx.x & 63, q = lane >> 4, i16 = lane & 15;
  const int nst = (d + W::SPS - 1) / W::SPS;

#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  constexpr int CPL = KP / 64;  // b' columns per lane during the build: lane l sums CPL·l .. CPL·l+CPL-1
  float bpart[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) bpart[e] = 0.f;
  int npos = 0;

  // (col, val) of stage s: lane l holds rating 32 s + (l & 31), clamped to the row (zero weight)
  auto iload = [&](int s, int& c_out, float& r_out) {
    const int e = W::SPS * s + (lane & 31);
    const int64_t pe = p0 + (e < d ? e : d - 1);
    c_out = a.col[pe];
    r_out = a.val[pe];
    if constexpr (PRE) {  // past the row end: the zero row (its products vanish in A' and b')
      c_out = e < d ? c_out : (int)a.zero_row;
      r_out = e < d ? r_out : 0.f;
    }
  };
  // gather of one stage: piece u holds ratings RPI·u .. RPI·u + RPI-1, lane l the 16 B at
  // 4·(l % LPR) of rating RPI·u + l / LPR; the rating's src row is wave-uniform (readlane)
  auto dma = [&](int cidx) {
    static_for<0, W::NI>([&](auto U) {
      constexpr int u = decltype(U)::value;
      int row;
      if constexpr (W::RPI == 2) {
        const int r0 = rdlane_i(cidx, 2 * u), r1 = rdlane_i(cidx, 2 * u + 1);
        row = lane < 32 ? r0 : r1;
      } else {
        const int r0 = rdlane_i(cidx, 4 * u), r1 = rdlane_i(cidx, 4 * u + 1);
        const int r2 = rdlane_i(cidx, 4 * u + 2), r3 = rdlane_i(cidx, 4 * u + 3);
        row = q == 0 ? r0 : (q == 1 ? r1 : (q == 2 ? r2 : r3));
      }
      if constexpr (PRE) {
        const int rr = W::RPI * u + lane / W::LPR;  // row of the stage; chunk position lane % LPR
        const char* src = reinterpret_cast<const char*>(a.Zhl) + (int64_t)row * W::RB + 16 * ((lane % W::LPR) ^ pre_f(rr));
        __builtin_amdgcn_global_load_lds((glb_vp)src, (lds_vp)(st + 1024 * u), 16, 0, 0);
      } else {
        const float* src = a.Z + (int64_t)row * KP + 4 * (lane % W::LPR);
        __builtin_amdgcn_global_load_lds((glb_vp)src, (lds_vp)(st + soff<KP>(W::RPI * u, 0)), 16, 0, 0);
      }
    });
  };

  int c_cur = 0, c_nxt = 0;
  float r_cur = 0.f, r_nxt = 0.f;
  // the stage's fragments are in registers: refill the stage with s + 1, fetch the indices of s + 2
  auto next_stage = [&](int s) {
    dma(c_nxt);
    c_cur = c_nxt;
    r_cur = r_nxt;
    if (s + 2 < nst) iload(s + 2, c_nxt, r_nxt);
  };
  if (nst > 0) {
    iload(0, c_cur, r_cur);
    dma(c_cur);
    if (nst > 1) iload(1, c_nxt, r_nxt);
  }
  f32x4 bt = zero4();  // PRE: b' of every block in one tile (column 2A: w hi, 2A + 1: w lo)
  for (int s = 0; s < nst; ++s) {
    const bool in = W::SPS * s + (lane & 31) < d;
    npos += __popcll(__ballot(lane < 32 && in && r_cur > 0.f));
    float cw = 0.f, ww = 0.f;
    rating_weights(r_cur, IMPLICIT, a.alpha, cw, ww);
    auto tile = [&](auto AA, auto BB, const f16x8& ha, const f16x8& la, const f16x8& hb, const f16x8& lb) {
      constexpr int t = tix(decltype(AA)::value, decltype(BB)::value, NQ);
      acc[t] = mfma_h(ha, hb, acc[t]);
      acc[t] = mfma_h(ha, lb, acc[t]);
      acc[t] = mfma_h(la, hb, acc[t]);
    };
    if constexpr (PRE) {
      // W operand of the b' MFMAs: lane j + 16q holds w of ratings 8q .. 8q+7 (fp16 hi for even j,
      // lo for odd j), scaled by wsc
      const float wv = in ? ww * a.wsc : 0.f;
      f16x8 wop;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        float w = __shfl(wv, 8 * q + m);
        asm("" : "+v"(w));
        const _Float16 wh = (_Float16)w;
        wop[m] = (i16 & 1) ? (_Float16)(w - (float)wh) : wh;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this stage's DMA (and stage s+1's indices)
      // fragments by transposed reads: lane i + 16q gets column 16A + i of ratings 8q .. 8q+7; lane
      // 4qq + p of the group addresses row 8q + 4h + qq, columns 4p .. 4p+3 of the block
      f16x8 fh[NQ], fl[NQ];
      {
        const int qq = i16 >> 2, p = i16 & 3;
        static_for<0, NQ>([&](auto AA) {
          constexpr int A = decltype(AA)::value;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r = 8 * q + 4 * h + qq;
            const char* row = st + r * W::RB + 8 * (p & 1);
            const int ch = 2 * A + (p >> 1);
            const f16x4v vh = tr_read(row + 16 * (ch ^ pre_f(r)));
            const f16x4v vl = tr_read(row + 16 * ((ch + W::RB / 32) ^ pre_f(r)));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              fh[A][4 * h + e] = vh[e];
              fl[A][4 * h + e] = vl[e];
            }
          }
        });
      }
      WAVE_LDS_SYNC();
      if (s + 1 < nst) next_stage(s);
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, NQ>([&](auto AA) {
        constexpr int A = decltype(AA)::value;
        static_for<A, NQ>([&](auto BB) {
          tile(AA, BB, fh[A], fl[A], fh[decltype(BB)::value], fl[decltype(BB)::value]);
        });
        const f16x8 wa = ((i16 >> 1) == A) ? wop : f16x8{};
        bt = mfma_h(fh[A], wa, bt);
        bt = mfma_h(fl[A], wa, bt);
      });
    } else {
      const float sw = in ? sqrtf(cw) : 0.f;  // √c (0 past the row end)
      const float wv = in ? ww : 0.f;
      float sw8[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) sw8[m] = __shfl(sw, 8 * q + m);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this stage's DMA (and stage s+1's indices)
      // fragment of block A (lane i + 16q: ratings 8q .. 8q+7 of column 16A + i) -> fp16 hi / lo
      auto conv = [&](auto AA, f16x8& hv, f16x8& lv) {
        constexpr int A = decltype(AA)::value;
        float z[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) z[m] = *reinterpret_cast<const float*>(st + soff<KP>(8 * q + m, 16 * A + i16));
        const float csa = s_cs[16 * A + i16];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          float v = z[m] * (sw8[m] * csa);
          asm("" : "+v"(v));  // one fp32 rounding; hi and lo both from that value (see heavy_build)
          const _Float16 h = (_Float16)v;
          hv[m] = h;
          lv[m] = (_Float16)(v - (float)h);
        }
        __builtin_amdgcn_sched_barrier(0);  // one block's raw values live at a time (register cap)
      };
      // every block's fragments in registers (64 VGPRs at KP = 128, beside the tiles' 144)
      f16x8 fh[NQ], fl[NQ];
      static_for<0, NQ>([&](auto AA) { conv(AA, fh[decltype(AA)::value], fl[decltype(AA)::value]); });
      // b' += Σ_r w_r z_r: rows read whole (CPL consecutive columns per lane), w_r wave-uniform
#pragma unroll 4
      for (int r = 0; r < W::SPS; ++r) {
        const float wr = rdlane(wv, r);
        if constexpr (CPL == 2) {
          const float2 z2 = *reinterpret_cast<const float2*>(st + soff<KP>(r, 2 * lane));
          bpart[0] = fmaf(wr, z2.x, bpart[0]);
          bpart[1] = fmaf(wr, z2.y, bpart[1]);
        } else {
          bpart[0] = fmaf(wr, *reinterpret_cast<const float*>(st + soff<KP>(r, lane)), bpart[0]);
        }
      }
      WAVE_LDS_SYNC();
      if (s + 1 < nst) next_stage(s);
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, NQ>([&](auto AA) {
        static_for<decltype(AA)::value, NQ>([&](auto BB) {
          tile(AA, BB, fh[decltype(AA)::value], fl[decltype(AA)::value], fh[decltype(BB)::value],
               fl[decltype(BB)::value]);
        });
      });
    }
  }

  __builtin_amdgcn_sched_barrier(0);  // keep the factor's loads out of the build loop
  // ---- b' complete (sum over the four rating groups), tiles unscaled, diagonal Λ + λn ----------
  // b' to the factor's layout (lane i + 16q holds b'[16A + i] for every block A) through LDS
  float* bsc = reinterpret_cast<float*>(st);
  if constexpr (PRE) {  // bt: lane j + 16q holds column j (block j >> 1, w hi / lo), rows 4q .. 4q+3
#pragma unroll
    for (int r = 0; r < 4; ++r) bsc[16 * i16 + 4 * q + r] = bt[r];
    WAVE_LDS_SYNC();
    const float ib = a.inv_sw / a.wsc;  // Σ w·(√c·cs·z) / (√c·cs) = b'
#pragma unroll
    for (int A = 0; A < NQ; ++A)
      bacc[A] = (bsc[16 * (2 * A) + i16] + bsc[16 * (2 * A + 1) + i16]) * (s_cs[KP + 16 * A + i16] * ib);
    WAVE_LDS_SYNC();
  } else {
#pragma unroll
    for (int e = 0; e < CPL; ++e) bsc[CPL * lane + e] = bpart[e];
    WAVE_LDS_SYNC();
#pragma unroll
    for (int A = 0; A < NQ; ++A) bacc[A] = bsc[16 * A + i16];
    WAVE_LDS_SYNC();
  }
  return npos;
}

template <int KP, bool IMPLICIT, bool PRE>
__global__ __launch_bounds__(256, 2) void solve_wave_kernel(SolveArgs a) {
  using W = WaveRow<KP>;
  constexpr int NQ = W::NQ, NT = W::NT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: LDS-DMA bases in SGPRs
  float* s_cs = reinterpret_cast<float*>(lds + W::WAVES * W::LDS_WAVE);  // [KP] scales, [KP] inverses
  for (int e = threadIdx.x; e < 2 * KP; e += 256) s_cs[e] = a.colscale[e];
  __syncthreads();  // the only workgroup barrier: every wave below is on its own row
  const int64_t ridx = (int64_t)blockIdx.x * W::WAVES + wave;
  if (ridx >= a.n_rows) return;
  char* st = lds + wave * W::LDS_WAVE;
  const int j = a.rows[ridx];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  f32x4 acc[NT];
  float bacc[NQ];
  WAVE_STAMP(ridx, 0);
#ifdef WAVE_PROBE_FACTOR_ONLY  // probes only (tools/probe/factortime.hip): a synthetic SPD system
  static_for<0, NT>([&](auto T_) { acc[decltype(T_)::value] = f32x4{1e-3f, -2e-3f, 3e-3f, 1e-3f}; });
  static_for<0, NQ>([&](auto A_) {
    constexpr int A = decltype(A_)::value;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[tix(A, A, NQ)][r] = (4 * q + r == i16) ? 100.f + i16 : 1e-3f;
    bacc[A] = 1.f;
  });
  const int npos = d;
#else
  const int npos = wave_build<KP, IMPLICIT, PRE>(a, p0, d, st, s_cs, acc, bacc);
#endif
  WAVE_STAMP(ridx, 1);
  const float lamn = a.reg * (float)(IMPLICIT ? npos : d);
  const float* isc = s_cs + KP;
  // The system is scaled by s2 = 4^e (exact) so that its largest diagonal entry stays below 2^28:
  // every Cholesky entry |U_ij| <= sqrt(A_jj) is then below 2^14, the range the split-fp16 trailing
  // updates of wave_chol_solve<NQ, true> need.  x is unchanged ((s2·A') x = s2·b').
  float dmax = 0.f;
  static_for<0, NQ>([&](auto AA) {
    constexpr int A = decltype(AA)::value, t = tix(A, A, NQ);
    const int c = 16 * A + i16;
    const float ic = isc[c];
    float dv = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) dv = (4 * q + r == i16) ? acc[t][r] : dv;
    const float dadd = c < a.kreal ? a.lam[c] + lamn : 1.0f;
    dmax = fmaxf(dmax, fabsf(dv * (ic * ic) + dadd));
  });
  for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o));
  int ex = 0;
  frexpf(dmax, &ex);  // dmax < 2^ex
  int e2 = (28 - ex) >> 1;
  e2 = e2 > 60 ? 60 : (e2 < -60 ? -60 : e2);
  const float s2 = ldexpf(1.f, 2 * e2);
  static_for<0, NQ>([&](auto AA) {
    constexpr int A = decltype(AA)::value;
    const f32x4 ir = ld4(isc + 16 * A + 4 * q) * s2;
    bacc[A] *= s2;
    static_for<A, NQ>([&](auto BB) {
      constexpr int B = decltype(BB)::value, t = tix(A, B, NQ);
      const float ic = isc[16 * B + i16];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] *= ir[r] * ic;
      if constexpr (A == B) {
        const int c = 16 * A + i16;
        const float dadd = (c < a.kreal ? a.lam[c] + lamn : 1.0f) * s2;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r == i16) acc[t][r] += dadd;
      }
    });
  });

#ifdef WAVE_PROBE_BUILD_ONLY
  if (q == 0) for (int A = 0; A < NQ; ++A) a.X[(int64_t)j * KP + 16 * A + i16] = bacc[A] + acc[tix(A, A, NQ)][0];
  return;
#endif
  // ---- blocked Cholesky A' = UᵀU on the tiles, RHS alongside (wave_chol.h) -----------------------
  float xs[NQ];
  const bool notpd = wave_chol_solve<NQ, true>(acc, bacc, reinterpret_cast<float*>(st), xs);
  WAVE_STAMP(ridx, 2);
  bool nonfinite = false;
#pragma unroll
  for (int A = 0; A < NQ; ++A) {
    const int c = 16 * A + i16;
    const float v = c < a.kreal ? xs[A] : 0.f;
    nonfinite |= !isfinite(v);
    if (q == 0) a.X[(int64_t)j * KP + c] = v;
  }
  WAVE_STAMP(ridx, 3);
  const bool bad = notpd || __any(nonfinite);  // wave-uniform
  if (lane == 0 && bad) atomicOr(a.err, 2 | ALBEDO_EF_WAVE);
}

template <int KP>
hipError_t launch_wave_kp(const SolveArgs& a, hipStream_t s) {
  using W = WaveRow<KP>;
  static const hipError_t attr = allow_lds(solve_wave_kernel<KP, true, false>, W::LDS);
  static const hipError_t attr2 = allow_lds(solve_wave_kernel<KP, false, false>, W::LDS);
  static const hipError_t attr3 = allow_lds(solve_wave_kernel<KP, true, true>, W::LDS);
  static const hipError_t attr4 = allow_lds(solve_wave_kernel<KP, false, true>, W::LDS);
  for (hipError_t e : {attr, attr2, attr3, attr4})
    if (e != hipSuccess) return e;
  const int blocks = (int)((a.n_rows + W::WAVES - 1) / W::WAVES);
  if (a.Zhl) {
    if (a.implicit) solve_wave_kernel<KP, true, true><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a);
    else solve_wave_kernel<KP, false, true><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a);
  } else {
    if (a.implicit) solve_wave_kernel<KP, true, false><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a);
    else solve_wave_kernel<KP, false, false><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a);
  }
  return hipGetLastError();
}

// Split-K partial of one chunk per WAVE (kernels.h SplitArgs): the wave build of the chunk's
// chunk_len ratings, unscaled, into the fp32 record the fp64 chunk-order reduction sums.  Upper tile
// (A, B) in the C/D layout is stored as lower tile (B, A): lane i + 16q, slot r holds element
// (16B + i, 16A + 4q + r); diagonal-tile entries above the diagonal and the pad column are zeros.
template <int KP, bool IMPLICIT, bool PRE>
__global__ __launch_bounds__(256, 2) void wave_partial_kernel(SolveArgs a, SplitArgs sp) {
  using W = WaveRow<KP>;
  using R = SplitRec<KP>;
  constexpr int NQ = W::NQ, NT = W::NT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* s_cs = reinterpret_cast<float*>(lds + W::WAVES * W::LDS_WAVE);
  for (int e = threadIdx.x; e < 2 * KP; e += 256) s_cs[e] = a.colscale[e];
  __syncthreads();
  const int64_t slot = (int64_t)blockIdx.x * W::WAVES + wave;
  if (slot >= sp.n_chunks) return;
  char* st = lds + wave * W::LDS_WAVE;
  const int j = sp.chunk_row[slot];
  const int64_t rp0 = a.ptr[j], off = (int64_t)sp.chunk_idx[slot] * sp.chunk_len;
  const int64_t rest = a.ptr[j + 1] - rp0 - off;
  const int d = (int)(rest < sp.chunk_len ? rest : sp.chunk_len);
  f32x4 acc[NT];
  float bacc[NQ];
  const int npos = wave_build<KP, IMPLICIT, PRE>(a, rp0 + off, d, st, s_cs, acc, bacc);
  float* out = sp.partial + slot * R::FLOATS;
  const float* isc = s_cs + KP;
  static_for<0, NQ>([&](auto AA) {
    constexpr int A = decltype(AA)::value;
    const f32x4 ir = ld4(isc + 16 * A + 4 * q);
    static_for<A, NQ>([&](auto BB) {
      constexpr int B = decltype(BB)::value, t = tix(A, B, NQ);
      const float ic = isc[16 * B + i16];
      float* tl = out + htile(B, A) + i16 * HT_LD;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = A < B || 4 * q + r <= i16;
        tl[4 * q + r] = valid ? acc[t][r] * ir[r] * ic : 0.f;
      }
      if (q == 0) tl[16] = 0.f;
    });
  });
  if (q == 0) {
#pragma unroll
    for (int A = 0; A < NQ; ++A) out[R::OFF_B + 16 * A + i16] = bacc[A];
  }
  if (lane == 0) reinterpret_cast<int*>(out)[R::OFF_N] = npos;
}

template <int KP>
hipError_t launch_wave_partial_kp(const SolveArgs& a, const SplitArgs& sp, hipStream_t s) {
  using W = WaveRow<KP>;
  static const hipError_t e1 = allow_lds(wave_partial_kernel<KP, true, false>, W::LDS);
  static const hipError_t e2 = allow_lds(wave_partial_kernel<KP, false, false>, W::LDS);
  static const hipError_t e3 = allow_lds(wave_partial_kernel<KP, true, true>, W::LDS);
  static const hipError_t e4 = allow_lds(wave_partial_kernel<KP, false, true>, W::LDS);
  for (hipError_t e : {e1, e2, e3, e4})
    if (e != hipSuccess) return e;
  const int blocks = (int)((sp.n_chunks + W::WAVES - 1) / W::WAVES);
  if (a.Zhl) {
    if (a.implicit) wave_partial_kernel<KP, true, true><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a, sp);
    else wave_partial_kernel<KP, false, true><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a, sp);
  } else {
    if (a.implicit) wave_partial_kernel<KP, true, false><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a, sp);
    else wave_partial_kernel<KP, false, false><<<blocks, 64 * W::WAVES, W::LDS, s>>>(a, sp);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_wave_partial(int KP, const SolveArgs& a, const SplitArgs& s, hipStream_t st) {
  if (s.n_chunks <= 0) return hipSuccess;
  if (KP == 64) return launch_wave_partial_kp<64>(a, s, st);
  if (KP == 128) return launch_wave_partial_kp<128>(a, s, st);
  return hipErrorInvalidValue;
}

hipError_t launch_solve_wave(int KP, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  constexpr int64_t MAXR = (int64_t(1) << 31) / 64;  // 64 work-items per row; AQL grid sizes are 32-bit
  if (a.n_rows > MAXR) {
    for (int64_t r0 = 0; r0 < a.n_rows; r0 += MAXR) {
      SolveArgs b = a;
      b.rows = a.rows + r0;
      b.n_rows = a.n_rows - r0 < MAXR ? a.n_rows - r0 : MAXR;
      const hipError_t e = launch_solve_wave(KP, b, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (KP == 64) return launch_wave_kp<64>(a, s);
  if (KP == 128) return launch_wave_kp<128>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace albedo
