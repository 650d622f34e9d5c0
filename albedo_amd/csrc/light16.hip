// Light rows of degree d <= 16: the push-through solve of Spark's per-row normal equation
// (ALS.computeFactors -> NormalEquation + CholeskySolver, reached from ALSRecommenderBuilder.scala:58),
// one wave per row.  94 % of the users at c4 take this path.
//
//   x' = D⁻¹ Zᵀ v,  (C⁻¹ + Z D⁻¹ Zᵀ) v = C⁻¹ w,   D = Λ + λ·n (diagonal in the Gram's eigenbasis)
//
// The per-row work is small (d·KP gathered floats, a d x d system), so the kernel is bound by the
// wave's VALU instruction count rather than by HBM (r02 kernel: ~900 VALU instructions per row,
// SQ_ACTIVE_INST_VALU ≈ 100 % of the SIMD cycles).  This version is written for instruction count:
//   * every lane group loads entry i16 of the row itself (no cross-lane shuffles of the indices, the
//     diagonal of K added in the MFMA C layout where lane (i16, g) already owns entry i16's weight);
//   * S = (Z D^-1/2)(Z D^-1/2)ᵀ on split-fp16 MFMA, the hi / lo split with packed conversions
//     (v_cvt_pk_f16_f32: two elements per instruction);
//   * the d x d Cholesky runs only over the row's d columns (the forward substitution fused into it);
//   * L is transposed and x' = D⁻¹ Zᵀ v is formed through a small LDS stage (64 columns at a time,
//     lane = 2 columns, packed FMAs over the row's entries) instead of 16-lane DPP reductions.
// The arithmetic is the one of solve_light_kernel<KP, 16> (same S, same Cholesky and substitution
// order); only the final x' sum changes its addition order.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <type_traits>
#include "kernels.h"
#include "device_common.h"

namespace albedo {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int L16_LDK = 20;       // row stride of the K / L transposition scratch (floats)
constexpr int L16_COLS = 64;      // x' columns per LDS stage pass
constexpr int L16_SLD = L16_COLS + 4;  // stage row stride (floats)
__host__ __device__ constexpr int l16_wave_floats(int KP) { return 16 * L16_SLD + 2 * KP + 16; }  // stage, D^-1/2 of A, v, of B

// fp16 hi + lo of 8 fp32 values (already rounded to fp32: the caller pins them).  hi: packed RNE
// conversion; lo = fp16(x - hi) by v_fma_mix{lo,hi}_f16 (x·1 - hi is exact in fp32, so its single
// rounding to fp16 equals the convert-back / subtract / convert sequence, in 2 instead of 4
// instructions per pair)
__device__ __forceinline__ void split8(f32x4 a, f32x4 b, f16x8& hi, f16x8& lo) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x0 = p < 2 ? a[2 * p] : b[2 * p - 4], x1 = p < 2 ? a[2 * p + 1] : b[2 * p - 3];
    const f16x2 h = __builtin_convertvector((f32x2{x0, x1}), f16x2);
    hw[p] = __builtin_bit_cast(uint32_t, h);
    uint32_t l;  // both halves written (early clobber: the inputs are read after the first write)
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(l) : "v"(x0), "v"(x1), "v"(hw[p]));
    lw[p] = l;
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  hi = __builtin_bit_cast(f16x8, (u32x4{hw[0], hw[1], hw[2], hw[3]}));
  lo = __builtin_bit_cast(f16x8, (u32x4{lw[0], lw[1], lw[2], lw[3]}));
}

// entry i16 of a light row counts (Spark masks c = 0 ratings out of A and b)
__device__ __forceinline__ bool entry_valid(const SolveArgs& a, float r, int i16, int d) {
  float ce, we;
  rating_weights(r, a.implicit, a.alpha, ce, we);
  return i16 < d && ce > 0.f;
}

// One unit: a row of degree dA <= 16 (PAIR = false), or two rows of degree <= 8 solved side by side
// (PAIR: entries 0..7 of the 16-entry tile are row A's, 8..15 row B's; dB = 0 when B is absent).
// Each lane group holds entry i16's rating r and src row colE and the gathered rows zf (lane (i16, g):
// Z[entry i16][16c + 4g .. +3], zero for masked entries).  The two rows of a pair share the S tile,
// the Cholesky steps and the x' stage: K is block diagonal (the cross block is zeroed), so the
// factorisation of one block never touches the other (L's cross entries stay exactly 0), and each
// row's arithmetic is the one it would get alone.
// The live columns of a unit are tested at run time (wave-uniform degrees in SGPRs).  r04's
// degree-specialised units and the NaN-fill debug build (r05's light16 determinism probes) are not
// part of this kernel: tools/probe/history_builds.sh rebuilds them from the commits that had them.
template <int KP, bool PAIR>
__device__ __forceinline__ void light16_unit(const SolveArgs& a, int dA, int dB, float r, int colE,
                                             const f32x4 (&zf)[KP / 16], float* st, float* sdlA, float* sdlB,
                                             float* vsh, const float* s_lam, const float* s_csi,
                                             f32x2 (&xo)[KP / 64]) {
  constexpr int NQ = KP / 32, NHC = KP / 64;
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const int blk = PAIR ? (i16 >> 3) : 0, el = PAIR ? (i16 & 7) : i16;  // this lane's row and entry
  const int dme = (PAIR && blk) ? dB : dA;
  float ce = 0.f, we = 0.f;
  if (el < dme) rating_weights(r, a.implicit, a.alpha, ce, we);
  const bool valid = el < dme && ce > 0.f;
  const uint64_t pos = __ballot(el < dme && r > 0.f);
  const int nposA = a.implicit ? __popcll(pos & (PAIR ? 0xFFull : 0xFFFFull)) : dA;
  const int nposB = a.implicit ? __popcll(pos & 0xFF00ull) : dB;
  const float lamnA = a.reg * (float)nposA, lamnB = a.reg * (float)nposB;

  // D^-1/2 per row (lane: columns lane + 64h) and one power-of-two scale for the unit's fp16 operands
  float sdA[NHC], sdB[NHC];
  bool bad = false;
  float bnd = 0.f;
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    const int cc = lane + 64 * h;
    const float lm = s_lam[cc], cs = s_csi[cc];
    const float ddA = lm + lamnA;
    if (cc < a.kreal && !(ddA > 0.f)) bad = true;
    sdA[h] = (cc < a.kreal && ddA > 0.f) ? frsq(ddA) : 0.f;
    bnd = fmaxf(bnd, sdA[h] * cs);
    if constexpr (PAIR) {
      const float ddB = lm + lamnB;
      if (dB > 0 && cc < a.kreal && !(ddB > 0.f)) bad = true;
      sdB[h] = (cc < a.kreal && ddB > 0.f) ? frsq(ddB) : 0.f;
      if (dB > 0) bnd = fmaxf(bnd, sdB[h] * cs);
    }
  }
  bnd = wave_max_dpp(bnd);
  int ex = 0;
  frexpf(bnd * 8192.f, &ex);  // max |z_c · sd_c| < 2^13 · bnd < 2^ex
  const float sc = ldexpf(1.f, 13 - ex), usc = ldexpf(1.f, 2 * (ex - 13));
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    sdlA[lane + 64 * h] = sdA[h] * sc;
    if constexpr (PAIR) sdlB[lane + 64 * h] = sdB[h] * sc;
  }
  WAVE_LDS_SYNC();
  const float* sdl = (PAIR && blk) ? sdlB : sdlA;  // this lane's row

  // S = Zs Zsᵀ on split-fp16 MFMA (hi·hi + hi·lo + lo·hi); both operands are Zs, so the 32 k-slots
  // of step q may take columns 32q + 4g .. +3 and 32q + 16 + 4g .. +3
  f32x4 acc = zero4();
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    f32x4 v0 = zf[2 * q] * ld4(sdl + 32 * q + 4 * g);
    f32x4 v1 = zf[2 * q + 1] * ld4(sdl + 32 * q + 16 + 4 * g);
    asm("" : "+v"(v0), "+v"(v1));  // one fp32 rounding; hi and lo from that value (no fma_mix)
    f16x8 zh, zl;
    split8(v0, v1, zh, zl);
    acc = mfma_h(zh, zh, acc);
    acc = mfma_h(zh, zl, acc);
    acc = mfma_h(zl, zh, acc);
  }
  acc *= usc;
  // K = S + C⁻¹ (identity rows for masked / absent entries): lane (i16, g) holds K[4g + r][i16],
  // the diagonal is entry i16's own; PAIR: the cross block between the two rows is dropped
  const float cinv = valid ? frcp(ce) : 0.f;
  const float dadd = valid ? cinv : 1.0f;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    acc[rr] += (4 * g + rr == i16) ? dadd : 0.f;
    if constexpr (PAIR) acc[rr] = ((4 * g + rr) >> 3) == blk ? acc[rr] : 0.f;
  }
  if (__any(bad) && lane == 0) atomicOr(a.err, 1);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) st[(4 * g + rr) * L16_LDK + i16] = acc[rr];
  WAVE_LDS_SYNC();
  float kr[16];  // lane i16 (every group): row i16 of K
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 v = ld4(st + i16 * L16_LDK + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) kr[4 * u + e] = v[e];
  }
  // live column c: an entry of its row (c < dA, or PAIR: block B's c - 8 < dB)
  auto live = [&](int c) { return PAIR ? (c < 8 ? c < dA : c - 8 < dB) : c < dA; };

  // Cholesky K = L Lᵀ over the live columns (lane i holds row i: kr[m] = L[i][m], m <= i), with the
  // forward substitution L y = C⁻¹ w in the same steps; broadcasts of lane c by DPP row_newbcast
  float y = valid ? we * cinv : 0.f, dg = 1.f;
  bool notpd = false;
  static_for<0, 16>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    constexpr int cend = (PAIR && c < 8) ? 8 : 16;  // PAIR: the other block's rows are untouched
    if (!live(c)) return;
    // compiler-scheduled DPP broadcasts (bc16), not the asm helpers of device_common.h: with the asm
    // row_newbcast FMAs this kernel gave wrong results for a few paired rows from one run to the
    // next (tools/determinism.py: ~150 of 600K degree <= 8 rows at c2, always the second row of a
    // unit, 5-55 % off, each time a different set; the ISA scan finds no VALU-to-DPP read inside
    // two wait states), while the compiler-scheduled form is bit-identical across 20 half-sweeps
    const float piv = bc16<c>(kr[c]);
    if (!(piv > 0.f)) notpd = true;
    const float inv = frsq(piv), s = piv * inv;
    kr[c] = (i16 == c) ? s : kr[c] * inv;
    dg = (i16 == c) ? inv : dg;
    static_for<c + 1, cend>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      if (!live(m)) return;
      kr[m] = fmaf(-bc16<m>(kr[c]), kr[c], kr[m]);
    });
    const float yc = bc16<c>(y * dg);
    y = (i16 > c) ? fmaf(-kr[c], yc, y) : ((i16 == c) ? yc : y);
  });
  if (notpd && lane == 0) atomicOr(a.err, 2 | ALBEDO_EF_LIGHT16);
  // Lᵀ v = y: lane i needs column i of L (transposed through the scratch)
  if (g == 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<f32x4*>(st + i16 * L16_LDK + 4 * u) = f32x4{kr[4 * u], kr[4 * u + 1], kr[4 * u + 2], kr[4 * u + 3]};
  }
  WAVE_LDS_SYNC();
  float lt[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) lt[m] = st[m * L16_LDK + i16];  // L[m][i16] (m >= i16 used)
  static_for<0, 16>([&](auto cc) {
    constexpr int c = 15 - decltype(cc)::value;
    if (!live(c)) return;
    const float vc = bc16<c>(y * dg);
    y = (i16 < c) ? fmaf(-lt[c], vc, y) : ((i16 == c) ? vc : y);
  });
  if (g == 0) vsh[i16] = y;  // v (zero for masked / absent entries)

  // x' = D⁻¹ Zᵀ v through the stage: 64 columns per pass; lane l sums columns 2(l & 31), +1 over the
  // entries 8(l >> 5) + u.  Single row: u < min(8, d), the two halves meet by one cross-half shuffle;
  // PAIR: half 0 is row A, half 1 row B (u < max(dA, dB): absent entries are zero rows with v = 0).
  const int eh = lane >> 5, cl = 2 * (lane & 31);
  const int nu = PAIR ? (dA > dB ? dA : dB) : (dA < 8 ? dA : 8);
  const float* sdo = (PAIR && eh) ? sdlB : sdlA;
#pragma unroll
  for (int h = 0; h < KP / L16_COLS; ++h) {
    WAVE_LDS_SYNC();  // previous reads of the scratch / stage done
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      *reinterpret_cast<f32x4*>(st + i16 * L16_SLD + 16 * c4 + 4 * g) = zf[4 * h + c4];
    WAVE_LDS_SYNC();
    f32x2 xa = {0.f, 0.f};
    for (int u = 0; u < nu; ++u) {
      const int e = 8 * eh + u;
      const f32x2 z2 = *reinterpret_cast<const f32x2*>(st + e * L16_SLD + cl);
      xa += z2 * vsh[e];
    }
    if constexpr (!PAIR) {
      xa[0] += __shfl_xor(xa[0], 32);
      xa[1] += __shfl_xor(xa[1], 32);
    }
    // D⁻¹ = (sd·sc)² / sc² (exact power-of-two rescaling); the caller stores them once the next
    // unit's loads are issued
    const f32x2 s2 = *reinterpret_cast<const f32x2*>(sdo + L16_COLS * h + cl);
    xo[h] = xa * (s2 * s2 * usc);
  }
}

// Persistent waves over the unit list (unit i of the wave: wave id + i·waves), software-pipelined so
// that one dependent memory latency per unit remains exposed instead of four (rows -> ptr -> col/val
// -> Z).  Row descriptors {row, p0, degree} (a.desc) come by scalar loads two units ahead; the next
// unit's (col, val) entries are in flight while the current one computes; the Z gather of the next
// unit is issued as soon as the current unit's registers are free.  No vector load in the pipeline is
// conditional (masked entries read index 0 / gather the zero row a.zero_row), so the waits count only
// what they need; Λ and the column scales are staged in LDS once per workgroup.
// PAIR: unit u = rows 2u and 2u + 1 of the list (degree <= 8 each).
template <int KP, bool PAIR>
__global__ __launch_bounds__(256, KP <= 128 ? 5 : 4) void solve_light16_kernel(SolveArgs a) {
  constexpr int NC = KP / 16, WF = l16_wave_floats(KP);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int blk = PAIR ? (i16 >> 3) : 0, el = PAIR ? (i16 & 7) : i16;
  float* s_lam = smem + 4 * WF;  // [KP] Λ, then [KP] inverse column scales
  float* s_csi = s_lam + KP;
  for (int e = threadIdx.x; e < KP; e += 256) {
    s_lam[e] = a.lam[e];
    s_csi[e] = a.colscale[KP + e];
  }
  __syncthreads();  // the only workgroup barrier
  float* st = smem + wave * WF;     // K / L scratch, then the x' stage
  float* sdlA = st + 16 * L16_SLD;  // D^-1/2 · sc per column, row A
  float* vsh = sdlA + KP;           // v
  float* sdlB = vsh + 16;           // row B (PAIR)
  const int64_t n = a.n_rows, nu_ = PAIR ? (n + 1) / 2 : n, nw = (int64_t)gridDim.x * 4;
  int64_t uidx = (int64_t)blockIdx.x * 4 + wave;
  if (uidx >= nu_) return;
  auto desc = [&](int64_t i) {  // constant address space: a wave-uniform index becomes s_load_dwordx4
    if (i >= n) return int4{0, 0, 0, 0};
    typedef __attribute__((address_space(4))) const int cint;
    cint* q = (cint*)(a.desc) + 4 * i;
    return int4{q[0], q[1], q[2], q[3]};
  };
  struct Unit { int4 a, b; };  // row descriptors; b is zero without a second row
  auto unit = [&](int64_t u) {
    if (u >= nu_) return Unit{int4{0, 0, 0, 0}, int4{0, 0, 0, 0}};
    if constexpr (PAIR) return Unit{desc(2 * u), desc(2 * u + 1)};
    else return Unit{desc(u), int4{0, 0, 0, 0}};
  };
  auto entries = [&](const Unit& U, float& rr, int& cc) {
    const int4& dd = (PAIR && blk) ? U.b : U.a;
    const int64_t p0 = (int64_t)(uint32_t)dd.y | ((int64_t)dd.z << 32);
    const int64_t e = el < dd.w ? p0 + el : 0;  // unconditional load (index 0 always exists)
    rr = a.val[e];
    cc = a.col[e];
  };
  f32x4 zf[NC];
  auto gather = [&](const Unit& U, float rr, int cc) {
    const int dd = (PAIR && blk) ? U.b.w : U.a.w;
    const int64_t src = entry_valid(a, rr, el, dd) ? cc : a.zero_row;
#pragma unroll
    for (int c = 0; c < NC; ++c) zf[c] = ld4(a.Z + src * KP + 16 * c + 4 * g);
  };
  const int eh = lane >> 5, cl = 2 * (lane & 31);
  auto store = [&](const Unit& U, const f32x2 (&xo)[KP / L16_COLS]) {
    // single row: half 0 holds the columns; PAIR: half 0 row A, half 1 row B (if present)
    const int j = (PAIR && eh) ? U.b.x : U.a.x;
    const bool on = PAIR ? (eh == 0 || U.b.w > 0) : lane < 32;
    if (on) {
#pragma unroll
      for (int h = 0; h < KP / L16_COLS; ++h) *reinterpret_cast<f32x2*>(a.X + (int64_t)j * KP + L16_COLS * h + cl) = xo[h];
    }
  };
  Unit uA = unit(uidx);
  float r, rN = 0.f;
  int colE, cN = 0;
  entries(uA, r, colE);
  gather(uA, r, colE);
  Unit uB = unit(uidx + nw);
  entries(uB, rN, cN);
  Unit uC = unit(uidx + 2 * nw);
  for (;;) {
    f32x2 xo[KP / L16_COLS];
    light16_unit<KP, PAIR>(a, uA.a.w, uA.b.w, r, colE, zf, st, sdlA, sdlB, vsh, s_lam, s_csi, xo);
    const Unit done = uA;
    uidx += nw;
    if (uidx >= nu_) {
      store(done, xo);
      break;
    }
    uA = uB;
    uB = uC;
    r = rN;
    colE = cN;
    gather(uA, r, colE);
    entries(uB, rN, cN);  // unit uidx + nw (zero descriptors past the end: harmless loads of index 0)
    store(done, xo);      // after the loads: the next waits do not cover these stores
    uC = unit(uidx + 2 * nw);
  }
}

__global__ void row_desc_kernel(const int32_t* __restrict__ rows, int64_t n, const int64_t* __restrict__ ptr,
                                int4* __restrict__ desc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int j = rows[i];
  const int64_t p0 = ptr[j];
  desc[i] = int4{j, (int)(uint32_t)p0, (int)(p0 >> 32), (int)(ptr[j + 1] - p0)};
}

}  // namespace

// pair = true: the rows (all of degree <= 8) are solved two per unit
hipError_t launch_solve_light16(int KP, const SolveArgs& a, hipStream_t s, bool pair) {
  if (a.n_rows <= 0) return hipSuccess;
  if (!a.desc || a.n_cu <= 0) return hipErrorInvalidValue;
  const int per_cu = KP <= 128 ? 5 : 4;  // resident workgroups per CU (launch bounds)
  const int64_t units = pair ? (a.n_rows + 1) / 2 : a.n_rows;
  const int64_t need = (units + 3) / 4;
  const int blocks = (int)std::min<int64_t>(need, (int64_t)a.n_cu * per_cu);
  const size_t lds = ((size_t)4 * l16_wave_floats(KP) + 2 * KP) * sizeof(float);
#define L16(kp)                                                                  \
  if (KP == kp) {                                                                \
    if (pair) solve_light16_kernel<kp, true><<<blocks, 256, lds, s>>>(a);        \
    else solve_light16_kernel<kp, false><<<blocks, 256, lds, s>>>(a);            \
    return hipGetLastError();                                                    \
  }
  L16(64) L16(128) L16(256)
#undef L16
  return hipErrorInvalidValue;
}

hipError_t launch_row_desc(const int32_t* rows, int64_t n, const int64_t* ptr, int32_t* desc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  row_desc_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(rows, n, ptr, reinterpret_cast<int4*>(desc));
  return hipGetLastError();
}

}  // namespace albedo
