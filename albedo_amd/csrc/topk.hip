// Top-k recommendation (ALSModel.recommendForAll* / albedo's ALSRecommender.recommendForUsers,
// recommenders/ALSRecommender.scala:28-65: F2J sdot scores, BoundedPriorityQueue top-k,
// BoundedPriorityQueue.scala:30-53).  The score matrix is never materialised.
//
//  bound    s·t = s_P·t_P + s_⊥·t_⊥ in the eigenbasis of the dst Gram, P = its TOPK_M leading
//           directions, so s·t <= Σ_d max(s_d·lo_d, s_d·hi_d) + ‖s_⊥‖·R over any set of dst rows whose
//           t_P lie in the box [lo, hi] and whose ‖t_⊥‖ <= R.  Converged implicit-ALS item factors put
//           most of their energy in one or two directions (c4: 84 % / 92 %), so the bound is tight:
//           at c4 it keeps < 1 % of the dst chunks of a user against the 64th best score.
//  prepare  dst rows by descending ‖t_⊥‖ (device radix sort), packed as fp16 rows scaled by a power of
//           two, CH-row chunks with their box + R (and 16-chunk super-chunks), a probe image of the 256
//           largest-norm rows;
//  order    one wave per 16 src rows: scores against the probe rows on MFMA, the kt-th best v* -> the
//           starting threshold thr0 = v* minus the rounding difference to the scan; the src features
//           (s_P, ‖s_⊥‖, the pruning margin); a sort key that groups rows of similar depth and
//           direction;
//  mask     per scan workgroup, the chunks any of its rows can still need against thr0 (super-chunks
//           first): a bitmask;
//  scan     one workgroup per 64·G src rows over the masked chunks: the src rows' fp16 fragments stay in
//           registers, the dst rows stream through an LDS ring filled by LDS-DMA; a wave skips a chunk
//           none of its rows can use at the running thresholds; scores on v_mfma_f32_16x16x32_f16
//           started from minus the thresholds, hits appended to per-row lists in global memory, a
//           full list compacted to its best 64 by a wave bitonic sort, the kt-th best the new threshold;
//  select   one wave per src row: best 64 of the list, exact F2J rescoring, sort (score desc, id asc),
//           certification: every dst row outside the list had approx < its threshold <= t (a pruned
//           chunk only when bound + e < threshold), so its F2J score is <= t + e with e the fp16 + fp32
//           error bound; if the k-th exact score is not > t + e the row is re-scored by the exact scan
//           (topk_exact_kernel, which skips the chunks the bound excludes against its own k-th best).
// Output is bit-identical to BoundedPriorityQueue over ascending ids + TopByKeyAggregator.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>
#include "device_common.h"
#include "kernels.h"

namespace albedo {

typedef __attribute__((address_space(3))) void* tk_lds_vp;
inline int tk_grid(int64_t n, int per) {
  int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 8192));
}
size_t topk_sort_temp_bytes(int64_t n);
__global__ void topk_gather_rows_kernel(const int32_t* __restrict__ rows, const float* __restrict__ thr,
                                        const float* __restrict__ sf, const uint32_t* __restrict__ order, int64_t n,
                                        int32_t* __restrict__ out, float* __restrict__ thr_out, float* __restrict__ sf_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t o = order[i];
    out[i] = rows[o];
    thr_out[i] = thr[o];
#pragma unroll
    for (int f = 0; f < TOPK_SF; f += 4)
      *reinterpret_cast<f32x4*>(sf_out + i * TOPK_SF + f) = *reinterpret_cast<const f32x4*>(sf + (int64_t)o * TOPK_SF + f);
  }
}
typedef __attribute__((address_space(1))) const void* tk_glb_vp;

// ---------------------------------------------------------------------------------------------
// wave bitonic sort of 64·NPL (score, idx) pairs, NPL per lane (element e = lane + 64·h), into
// (score desc, idx asc) order.  Fully unrolled: every register index is a compile-time constant.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool tk_before(float s1, int i1, float s2, int i2) {
  return s1 > s2 || (s1 == s2 && (unsigned)i1 < (unsigned)i2);
}
// The value of lane l ^ JJ (JJ < 64) without the LDS crossbar (a __shfl_xor is a ds_bpermute, ~100+
// cycles of latency, and a compaction's bitonic sort is 27 dependent exchange steps): DPP quad
// permutes for 1 and 2, row_ror:8 for 8, two row shifts for 4, v_permlane16/32_swap for 16 / 32.
template <int JJ>
__device__ __forceinline__ int xor_lane(int v, int lane) {
  if constexpr (JJ == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  else if constexpr (JJ == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  else if constexpr (JJ == 4) {
    const int up = __builtin_amdgcn_mov_dpp(v, 0x104, 0xF, 0xF, false);  // row_shl:4: lane i + 4
    const int dn = __builtin_amdgcn_mov_dpp(v, 0x114, 0xF, 0xF, false);  // row_shr:4: lane i - 4
    return (lane & 4) ? dn : up;
  } else if constexpr (JJ == 8) return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
  else if constexpr (JJ == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane & 16) ? p[0] : p[1]);
  } else {
    static_assert(JJ == 32, "xor distance");
    const auto p = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane & 32) ? p[0] : p[1]);
  }
}

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
      const float os = __int_as_float(xor_lane<JJ>(__float_as_int(sc[h]), lane));
      const int oi = xor_lane<JJ>(ix[h], lane);
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


// ---------------------------------------------------------------------------------------------
// scan geometry.  A chunk is 16 KiB of fp16 dst rows (128 / 64 / 32 rows at KP = 64 / 128 / 256);
// NSTG chunks form the LDS ring.
// ---------------------------------------------------------------------------------------------
template <int KP, int G>
struct TkScan {
  static constexpr int RB = 2 * KP;              // bytes per fp16 dst row
  static constexpr int CB = 16384;               // dst bytes per chunk
  static constexpr int CH = CB / RB;             // dst rows per chunk
  static constexpr int NJ = CH / 16;             // 16-row tiles per chunk
  static constexpr int NQ = KP / 32;             // 32-deep MFMA steps per tile
  // G <= 4: two workgroups per CU (r05; at one per CU every wave is alone on its SIMD and the scan's
  // DMA, LDS, barrier and list latencies are all exposed): a 4-chunk ring, the first 2048 mask words in
  // LDS (the rest read from global memory by the mask window) -- 75 KB per workgroup.  G = 8 needs
  // more than 256 registers per lane (the AGPRs of a wave alone on its SIMD): one per CU, 6 chunks.
  // The src features live in registers (r04: LDS).
  static constexpr int OCC = G <= 4 ? 2 : 1;     // workgroups per CU
  static constexpr int NSTG = OCC == 2 ? 4 : 6;  // ring depth (chunks)
  static constexpr int SLOT = CB + 4 * 64;       // + each wave's copy of the chunk's bound box
  static constexpr int RING = NSTG * SLOT;
  static constexpr int RWG = 64 * G;             // src rows per workgroup (16·G per wave)
  static constexpr int DPW = CB / 1024 / 4;      // 1-KiB row DMAs per wave per chunk
  static constexpr int NVM = DPW + 1;            // DMA instructions per wave per chunk (rows + box)
  static constexpr int MASKW = OCC == 2 ? 2048 : 8192;  // mask words kept in LDS
  static constexpr int LDS = RING + RWG * 4 + MASKW * 4;
  static_assert(OCC * LDS <= 160 * 1024, "LDS budget");
};
template <int KP>
__host__ __device__ constexpr int topk_chunk_rows_dev() { return TkScan<KP, 2>::CH; }
// 16-B unit u of dst row `row` is stored at unit u ^ tk_sw(row): every ds_read_b128 lane group of a
// fragment read (16 rows x one unit, cdna ds_read_b128 groups) hits 16 distinct 16-B bank slots.
template <int KP>
__device__ __forceinline__ int tk_sw(int row) {
  if constexpr (KP == 64) return (row >> 1) & 7;
  else return row & 15;
}

__device__ __forceinline__ float agent_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int agent_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t agent_load64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Upper bound of s·t over the dst rows of a chunk (or super-chunk) feature record cf = {lo[M], hi[M],
// R}, for a src row with features sf = {s_P[M], ‖s_⊥‖}; fp32 arithmetic, its rounding is part of the
// margin stored with the src features (sf[TOPK_M + 1]).
__device__ __forceinline__ float tk_bound(const float* sf, const float* cf) {
  float b = sf[TOPK_M] * cf[2 * TOPK_M];
#pragma unroll
  for (int d = 0; d < TOPK_M; ++d) b += sf[d] * (sf[d] >= 0.f ? cf[TOPK_M + d] : cf[d]);
  return b;
}

// |F2J(s,t) - approx| for the fp16 pre-selection (select's certification bound, see there)
template <int KP>
__device__ __forceinline__ double tk_err(double ns, const TopkArgs& a) {
  const double u = 5.9604644775390625e-08;  // 2^-24
  const double kk = (double)(KP + 2);
  const double gam = kk * u / (1.0 - kk * u);
  const double rel = (9.765625e-04 + 2.384185791015625e-07 + 6.0 * gam) * (1.0 + 1.0 / 512.0);
  const double tm = (double)a.tmax_norm;
  const double absu = 2.98023223876953125e-08 * 1.001 * sqrt((double)KP) * (ns / (double)a.tsc + tm / (double)a.ssc) +
                      (double)KP * 8.9e-16 * (double)a.unscale;
  return rel * ns * tm + absu;
}

#ifdef ALBEDO_TOPK_PHASES  // probe builds only (tools/topk_phases.py): shader-clock time per scan phase
__device__ unsigned long long g_tk_ph[16];  // [0..7] cycles per phase summed over waves, [8..15] event counts
#define TKPH_T0() unsigned long long tk_t = __builtin_amdgcn_s_memtime(), tk_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tk_n[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define TKPH(k) { const unsigned long long tk_x = __builtin_amdgcn_s_memtime(); tk_acc[k] += tk_x - tk_t; tk_t = tk_x; }
#define TKPH_N(k, v) tk_n[k] += (v)
#define TKPH_OUT() if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 8; ++k_) { atomicAdd(&g_tk_ph[k_], tk_acc[k_]); atomicAdd(&g_tk_ph[8 + k_], tk_n[k_]); }
#else
#define TKPH_T0()
#define TKPH(k)
#define TKPH_N(k, v)
#define TKPH_OUT()
#endif

template <int KP, int G>
__global__ __launch_bounds__(256, (TkScan<KP, G>::OCC)) void topk_scan_kernel(TopkArgs a) {
  using C = TkScan<KP, G>;
  constexpr int NQ = C::NQ, NJ = C::NJ, RB = C::RB, CAP = TOPK_CAP, SF = TOPK_SF;
  // a list is compacted to its best 64 once it holds more than TRIG (<= TRIG + 16 <= 64·NSC entries):
  // frequent enough that the threshold follows the running kt-th best
  constexpr int TRIG = TOPK_TRIG, NSC = TOPK_CAP / 64;
  static_assert(TRIG + 16 <= 64 * NSC && TRIG + 16 <= CAP && TRIG + 16 <= 255, "compaction width, byte counters");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // one LDS object (glds pipelining)
  float* s_thr = reinterpret_cast<float*>(lds + C::RING);  // [RWG] thresholds (unscaled)
  uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_thr + C::RWG);  // [MASKW] this workgroup's mask
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rb0 = (int64_t)blockIdx.x * C::RWG;  // first src-list position of the workgroup
  const int wr0 = wave * 16 * G;                     // the wave's first row within the workgroup
  const char* Th = reinterpret_cast<const char*>(a.Th);
  const int64_t nch = a.n_chunks;
  char* const ring = lds;

  // src fragments: lane (i16, g) holds row 16gi + i16, columns 32q + 8g .. +7 (fp16, ·ssc)
  f16x8 sf[G][NQ];
  // minus the thresholds of rows 16gi + 4g + r in scaled units, in the MFMA C/D layout: every tile's
  // accumulation starts from them, so acc = score - threshold and a hit is acc >= 0 (one max over the
  // tile's accumulators instead of a compare per element).  No row: -inf.  Before a row's first
  // compaction: minus a lower bound of every score (-1.01·‖ŝ‖·max‖t̂‖ - 1), so every dst row passes.
  f32x4 nthr[G];
  uint32_t cntp[G];  // list lengths, one byte per row (see check_tile)
#pragma unroll
  for (int gi = 0; gi < G; ++gi) {
    const int64_t si = rb0 + wr0 + 16 * gi + i16;
    const int srow = si < a.n_src ? a.src_rows[si] : -1;
    const float* sp = a.S + (int64_t)(srow >= 0 ? srow : 0) * KP + 8 * g;  // loads unconditional (no
    const float keep = srow >= 0 ? 1.f : 0.f;                              // per-element waits)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4 v0 = ld4(sp + 32 * q), v1 = ld4(sp + 32 * q + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) sf[gi][q][e] = (_Float16)((e < 4 ? v0[e] : v1[e - 4]) * keep * a.ssc);
    }
    if (g == 0) s_thr[wr0 + 16 * gi + i16] = srow < 0 ? INFINITY : (a.thr0 ? a.thr0[si] : -INFINITY);
  }
  // src feature f of workgroup row w (global memory: read at setup only)
  auto sfeat = [&](int w, int f) -> float {
    const int64_t si = rb0 + w;
    return si < a.n_src && a.sfeat ? a.sfeat[si * SF + f] : 0.f;
  };
  const uint32_t* mw = a.mask ? a.mask + (int64_t)blockIdx.x * a.mask_words : nullptr;
  const int64_t mlds = mw ? (a.mask_words < C::MASKW ? a.mask_words : C::MASKW) : 0;
  for (int64_t w = tid; w < mlds; w += 256) s_mask[w] = mw[w];
  __syncthreads();  // no DMA in flight yet: a plain barrier
  const float tmax_sc = a.tmax_norm * a.tsc;
#pragma unroll
  for (int gi = 0; gi < G; ++gi) cntp[gi] = 0u;
#pragma unroll
  for (int gi = 0; gi < G; ++gi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int wrow = wr0 + 16 * gi + 4 * g + r;
      const float t0 = s_thr[wrow];
      nthr[gi][r] = t0 == INFINITY ? -INFINITY
                  : t0 == -INFINITY ? 1.01f * sfeat(wrow, TOPK_M + 2) * a.ssc * tmax_sc + 1.f : -(t0 * a.scaled);
    }

  // the chunk sequence: the set bits of this workgroup's mask (every chunk without one), ascending.
  // A window of 64 mask words (2048 chunks) is held in one VGPR (lane l: word base + l, from LDS;
  // beyond MASKW words from global memory): the next set bit is a ballot + ctz, and a new window is
  // read only when the walk leaves the current one (r04 read one LDS word per call and per empty
  // word: 8.5 % of the scan's wave-cycles).  Two cursors (DMA issue, consume) keep a window each.
  struct MaskWin { int64_t base; uint32_t word; };
  auto next_chunk = [&](int64_t x, MaskWin& mwin) -> int64_t {  // smallest chunk > x in the sequence (nch: none)
    int64_t c = x + 1;
    if (!mw) return c < nch ? c : nch;
    while (c < nch) {
      const int64_t w0 = c >> 5;
      if (w0 < mwin.base || w0 >= mwin.base + 64) {
        mwin.base = w0;
        const int64_t w = w0 + lane;
        mwin.word = w < mlds ? s_mask[w] : (w < a.mask_words ? mw[w] : 0u);
      }
      const int rel = (int)(w0 - mwin.base);
      const uint32_t word = lane < rel ? 0u : (lane == rel ? mwin.word & (~0u << (c & 31)) : mwin.word);
      const uint64_t nz = __ballot(word != 0u);
      if (nz) {
        const int L = __builtin_ctzll(nz);
        const uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)word, L);
        c = ((mwin.base + L) << 5) + __builtin_ctz(bits);
        return c < nch ? c : nch;
      }
      c = (mwin.base + 64) << 5;
    }
    return nch;
  };
  MaskWin win_iss{-((int64_t)1 << 40), 0u}, win_use{-((int64_t)1 << 40), 0u};

  // DMA of chunk c into ring slot `slot`: the wave's DPW KiB of rows (source addresses carry the
  // unit swizzle, the LDS image is lane-linear), then the wave's own copy of the chunk's bound box
  // (48 B, lanes 0-2)
  auto dma = [&](int64_t c, int slot) __attribute__((always_inline)) {
    char* base = ring + slot * C::SLOT;
    const int64_t j0 = c * C::CH;
#pragma unroll
    for (int m = 0; m < C::DPW; ++m) {
      const int ins = wave * C::DPW + m;
      const int off = ins * 1024 + 16 * lane;
      const int row = off / RB, up = (off % RB) / 16;
      const char* src = Th + (j0 + row) * RB + 16 * (up ^ tk_sw<KP>(row));
      __builtin_amdgcn_global_load_lds((tk_glb_vp)src, (tk_lds_vp)(base + ins * 1024), 16, 0, 0);
    }
    const float* cf = a.cfeat ? a.cfeat + c * TOPK_CF : a.S;  // any valid address when unpruned
    if (lane < TOPK_CF / 4)
      __builtin_amdgcn_global_load_lds((tk_glb_vp)(cf + 4 * lane), (tk_lds_vp)(base + C::CB + wave * 64), 16, 0, 0);
  };
  int64_t c_iss = -1;
  for (int u = 0; u < C::NSTG - 1; ++u) {
    c_iss = next_chunk(c_iss, win_iss);
    if (c_iss < nch) dma(c_iss, u);
  }

  // the bound test's src features (s_P, ‖s_⊥‖, margin) and thresholds of this lane's rows
  // lane + 64h in registers (r04 read them from LDS for every chunk); the thresholds are re-read after
  // a compaction raised some
  constexpr int BH = (16 * G + 63) / 64;
  float bsf[BH][TOPK_M + 2], bthr[BH];
#pragma unroll
  for (int h = 0; h < BH; ++h) {
    const int rr = lane + 64 * h < 16 * G ? lane + 64 * h : 0;
#pragma unroll
    for (int f = 0; f < TOPK_M + 2; ++f) bsf[h][f] = sfeat(wr0 + rr, f);
    bthr[h] = lane + 64 * h < 16 * G ? s_thr[wr0 + rr] : INFINITY;
  }
  TKPH_T0();
  // candidates of one 16-row tile (dst positions jt .. jt+15).  Slots come from a ballot prefix count
  // over the 16 lanes of a row's group; list lengths live in registers, one byte per row (cntp[gi]
  // byte r: row 16gi + 4g + r, the same in the 16 lanes of group g), so the append path touches no
  // LDS.  Lists above TRIG are compacted to their best 64.
  auto check_tile = [&](const f32x4 (&acc)[G], int64_t jt) __attribute__((always_inline)) {
    float mx = acc[0][0];
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[gi][r]);
    if (!__any(mx >= 0.f)) return;
    TKPH(2);
    TKPH_N(2, 1);
    const int64_t dj = jt + i16;
    const bool dv = dj < a.n_dst;
    const uint32_t below = (1u << i16) - 1u;
    bool over = false;
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool p = dv && acc[gi][r] >= 0.f;
        const uint64_t m = __ballot(p);
        if (m) {
          const uint32_t mg = (uint32_t)(m >> (16 * g)) & 0xffffu;
          const int wrow = wr0 + 16 * gi + 4 * g + r;
          const int cnt = (int)((cntp[gi] >> (8 * r)) & 0xffu);
          if (p) {
            const int64_t li = (rb0 + wrow) * CAP + cnt + __popc(mg & below);
            // score = acc + threshold; (score, position) in one 8-byte store
            a.lent[li] = uint2{__float_as_uint((acc[gi][r] - nthr[gi][r]) * a.unscale), (uint32_t)dj};
          }
          const int ncnt = cnt + __popc(mg);
          cntp[gi] += (uint32_t)__popc(mg) << (8 * r);
          over |= ncnt > TRIG;
        }
      }
    TKPH(3);  // appends
    if (!__any(over)) return;
    // wave-local rows to compact (bit 16gi + 4g + r)
    uint64_t f0 = 0, f1 = 0;
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint64_t m = __ballot(((cntp[gi] >> (8 * r)) & 0xffu) > (uint32_t)TRIG);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          if ((m >> (16 * gg)) & 1) {
            const int row = 16 * gi + 4 * gg + r;
            if (row < 64) f0 |= 1ull << row; else f1 |= 1ull << (row - 64);
          }
      }
    const uint64_t d0 = f0, d1 = f1;
    TKPH_N(3, 1);
    TKPH_N(4, __popcll(f0) + __popcll(f1));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's list stores are in L2
    TKPH(6);  // the drain of every outstanding VMEM op (ring DMAs included) before a compaction
    // two rows per batch: the list loads of both are in flight together (a compaction event flags
    // ~1.8 rows at c4); no drain after the batch (appends go to positions >= 64, and the next
    // compaction drains before it reads)
    while (f0 | f1) {
      int wl[2];
      bool on[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        on[k] = (f0 | f1) != 0;
        wl[k] = 0;
        if (f0) { wl[k] = __builtin_ctzll(f0); f0 &= f0 - 1; }
        else if (f1) { wl[k] = 64 + __builtin_ctzll(f1); f1 &= f1 - 1; }
      }
      float s2[2][NSC];
      int i2[2][NSC];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        uint32_t cw = 0;  // the row's length: byte (wl & 3) of cntp[wl >> 4] in lane 16·((wl >> 2) & 3)
#pragma unroll
        for (int gi = 0; gi < G; ++gi)
          if ((wl[k] >> 4) == gi) cw = (uint32_t)rdlane_i((int)cntp[gi], 16 * ((wl[k] >> 2) & 3));
        const int cnt = on[k] ? (int)((cw >> (8 * (wl[k] & 3))) & 0xffu) : 0;
        const int64_t lb = (rb0 + wr0 + wl[k]) * CAP;
#pragma unroll
        for (int h = 0; h < NSC; ++h) {
          const int e = lane + 64 * h;
          const uint64_t v = e < cnt ? agent_load64(reinterpret_cast<const uint64_t*>(a.lent + lb + e))
                                     : ((uint64_t)0xFFFFFFFFu << 32) | __float_as_uint(-INFINITY);
          s2[k][h] = __uint_as_float((uint32_t)v);
          i2[k][h] = (int)(uint32_t)(v >> 32);
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (!on[k]) continue;  // wave-uniform
        wave_bitonic<NSC>(s2[k], i2[k]);
        const int64_t lb = (rb0 + wr0 + wl[k]) * CAP;
        a.lent[lb + lane] = uint2{__float_as_uint(s2[k][0]), (uint32_t)i2[k][0]};
        const float tkt = rdlane(s2[k][0], a.kt - 1);  // the running kt-th best becomes the threshold
        if (lane == 0) s_thr[wr0 + wl[k]] = tkt;
      }
    }
    WAVE_LDS_SYNC();
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * gi + 4 * g + r;
        const bool done = row < 64 ? ((d0 >> row) & 1) : ((d1 >> (row - 64)) & 1);
        if (done) {
          nthr[gi][r] = -(s_thr[wr0 + row] * a.scaled);
          cntp[gi] = (cntp[gi] & ~(0xffu << (8 * r))) | (64u << (8 * r));
        }
      }
#pragma unroll
    for (int h = 0; h < BH; ++h)
      if (lane + 64 * h < 16 * G) bthr[h] = s_thr[wr0 + lane + 64 * h];
    TKPH(4);  // compaction loads + sorts + stores
  };

  int64_t it = 0, n_scored = 0;  // chunk iterations; chunks this wave scored (its `need` held)
  for (int64_t c = next_chunk(-1, win_use); c < nch; c = next_chunk(c, win_use), ++it) {
    TKPH(5);  // next_chunk (mask walk)
    // this wave's DMAs of chunk c have landed, then one barrier publishes every wave's part and retires
    // the previous slot.  vmcnt(0): r05 waited with a hand-counted vmcnt(NVM·(NSTG−2)), which assumed the
    // VM counter retires the LDS-DMA loads and the later list stores in issue order; the plain drain
    // measured no slower (c4 all users, scan 186.9 vs 192.1 ms, profiles/r06_bench_c4_topk_vmcnt0.json)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c_iss < nch) {
      c_iss = next_chunk(c_iss, win_iss);
      if (c_iss < nch) dma(c_iss, (int)((it + C::NSTG - 1) % C::NSTG));
    }
    TKPH(0);  // DMA wait + barrier + next DMA issue
    TKPH_N(0, 1);
    // can any row of this wave still take a dst row of chunk c (bound + margin >= its threshold)?
    const char* base = ring + (int)(it % C::NSTG) * C::SLOT;
    bool need = !a.cfeat;
    if (a.cfeat) {
      const float* cf = reinterpret_cast<const float*>(base + C::CB + wave * 64);
      float cfr[TOPK_CF];
#pragma unroll
      for (int f = 0; f < TOPK_CF; f += 4) {
        const f32x4 v = ld4(cf + f);
#pragma unroll
        for (int e = 0; e < 4; ++e) cfr[f + e] = v[e];
      }
#pragma unroll
      for (int h = 0; h < BH; ++h) need |= tk_bound(bsf[h], cfr) + bsf[h][TOPK_M + 1] >= bthr[h];
    }
    TKPH(1);  // chunk bound test
    if (!__any(need)) continue;
    ++n_scored;
    TKPH_N(1, 1);
    const int64_t j0 = c * C::CH;
    f16x8 df[2][NQ];
    auto rd = [&](int J, f16x8 (&d)[NQ]) __attribute__((always_inline)) {
      const int row = 16 * J + i16;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        d[q] = *reinterpret_cast<const f16x8*>(base + row * RB + 16 * ((4 * q + g) ^ tk_sw<KP>(row)));
    };
    rd(0, df[0]);
    f32x4 acc[2][G];
    static_for<0, NJ>([&](auto JJ) {
      constexpr int J = decltype(JJ)::value;
      if constexpr (J + 1 < NJ) rd(J + 1, df[(J + 1) & 1]);
#pragma unroll
      for (int gi = 0; gi < G; ++gi) acc[J & 1][gi] = mfma_h(sf[gi][0], df[J & 1][0], nthr[gi]);
#pragma unroll
      for (int q = 1; q < NQ; ++q)
#pragma unroll
        for (int gi = 0; gi < G; ++gi) acc[J & 1][gi] = mfma_h(sf[gi][q], df[J & 1][q], acc[J & 1][gi]);
      if constexpr (J > 0) check_tile(acc[(J - 1) & 1], j0 + 16 * (J - 1));
    });
    check_tile(acc[(NJ - 1) & 1], j0 + 16 * (NJ - 1));
    TKPH(2);  // MFMA scoring + tile checks (appends / compactions below are subtracted out)
  }
  TKPH_OUT();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup ends
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (i16 == 0) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t si = rb0 + wr0 + 16 * gi + 4 * g + r;
        if (si < a.n_src) a.lcnt[si] = (int)((cntp[gi] >> (8 * r)) & 0xffu);
      }
  }
  // dst rows this wave scored against its rows (topk_stats[2]: the MFMA work is 16·G src rows x these)
  if (a.scanned && lane == 0) atomicAdd(a.scanned, (unsigned long long)(n_scored * C::CH));
}

// F2J dots of a wave's candidate rows: lane L gets F2J(s, T[row_L]) (row_L < 0: -inf).  The rows
// arrive in 32-column blocks, eight lanes per row (128 coalesced bytes per row instead of one 16-B
// piece per lane and instruction), through the wave's LDS stage [64 rows][36 floats] (row stride 36:
// the b128 reads of 16 consecutive rows hit 16 distinct bank groups); each lane then walks its own row
// in F2J order (product, then add, left to right: f2j_dot_v4's value).
constexpr int TK_SEL_LD = 36;
template <int KP>
__device__ __forceinline__ float f2j_dot_rows(const float* __restrict__ s, const float* __restrict__ T, int row, int kreal,
                                              float* stg) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63, u = lane & 7;
  float* sv = stg + 64 * TK_SEL_LD;  // the src row
  for (int c = lane; c < KP; c += 64) sv[c] = s[c];
  int rowm[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) rowm[m] = __shfl(row, (lane >> 3) + 8 * m);
  float acc = 0.f;
  const float* tr = stg + lane * TK_SEL_LD;
  for (int cb = 0; cb < kreal; cb += 32) {
    f32x4 v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = rowm[m] >= 0 ? ld4(T + (int64_t)rowm[m] * KP + cb + 4 * u) : zero4();
    WAVE_LDS_SYNC();  // the previous block's reads are done
#pragma unroll
    for (int m = 0; m < 8; ++m) *reinterpret_cast<f32x4*>(stg + ((lane >> 3) + 8 * m) * TK_SEL_LD + 4 * u) = v[m];
    WAVE_LDS_SYNC();
    const int ce = kreal - cb < 32 ? kreal - cb : 32;
    if (ce == 32) {
#pragma unroll
      for (int c = 0; c < 32; c += 4) {
        const f32x4 t4 = ld4(tr + c), s4 = ld4(sv + cb + c);
        const float p0 = s4[0] * t4[0], p1 = s4[1] * t4[1], p2 = s4[2] * t4[2], p3 = s4[3] * t4[3];
        acc = acc + p0;
        acc = acc + p1;
        acc = acc + p2;
        acc = acc + p3;
      }
    } else {
      for (int c = 0; c < ce; ++c) {
        const float p = sv[cb + c] * tr[c];
        acc = acc + p;
      }
    }
  }
  return row >= 0 ? acc : -INFINITY;
}

template <int KP>
__device__ __forceinline__ void topk_select_row(const TopkArgs& a, int64_t si, int64_t so, float* stage, int* lid,
                                                float* lsc);

// One wave per src row: best 64 of the list, exact F2J rescoring, sort, certify, write top-k.
template <int KP>
__global__ __launch_bounds__(256) void topk_select_kernel(TopkArgs a) {
  __shared__ __attribute__((aligned(16))) float s_stage[4][64 * TK_SEL_LD + KP];
  // a range of output slots (in_pos): the workgroup's four consecutive lists leave as one contiguous
  // block of 16-B stores per array (written through PCIe into the caller's arrays, r06: whole 16-B
  // units instead of each wave's 4-B stores over its own 4k bytes)
  __shared__ __attribute__((aligned(16))) int s_oid[4 * TOPK_KC];
  __shared__ __attribute__((aligned(16))) float s_osc[4 * TOPK_KC];
  const int wave = threadIdx.x >> 6;
  const bool grouped = a.in_pos != nullptr;
  int64_t si = 0, so = 0;  // scan position, output slot
  if (grouped) {
    const int64_t l = (int64_t)blockIdx.x * 4 + wave;
    if (l < a.n_slots) {
      so = a.slot0 + l;
      si = a.in_pos[so];
      topk_select_row<KP>(a, si, so, s_stage[wave], s_oid + wave * a.k, s_osc + wave * a.k);
    }
    __syncthreads();
    const int64_t nu = min((int64_t)4, a.n_slots - (int64_t)blockIdx.x * 4);
    const int64_t so0 = a.slot0 + (int64_t)blockIdx.x * 4;  // a multiple of 4: so0·k·4 B is 16-B aligned
    const int tot = (int)nu * a.k;
    int* oi = a.out_ids + so0 * a.k;
    float* os = a.out_scores + so0 * a.k;
    for (int t = threadIdx.x; 4 * t < tot; t += 256) {
      if (4 * t + 4 <= tot) {
        *reinterpret_cast<int4*>(oi + 4 * t) = *reinterpret_cast<const int4*>(s_oid + 4 * t);
        *reinterpret_cast<float4*>(os + 4 * t) = *reinterpret_cast<const float4*>(s_osc + 4 * t);
      } else {
        for (int e = 4 * t; e < tot; ++e) {
          oi[e] = s_oid[e];
          os[e] = s_osc[e];
        }
      }
    }
    return;
  }
  si = (int64_t)blockIdx.x * 4 + wave;
  if (si >= a.n_src) return;
  so = a.out_pos ? (int64_t)a.out_pos[si] : si;
  topk_select_row<KP>(a, si, so, s_stage[wave], nullptr, nullptr);
}

// One src row of topk_select_kernel (a wave): best 64 of the list, exact F2J rescoring, sort, certify,
// top-k into the output slot (or into the workgroup's LDS lists when lid / lsc are given).
template <int KP>
__device__ __forceinline__ void topk_select_row(const TopkArgs& a, int64_t si, int64_t so, float* stage, int* lid,
                                                float* lsc) {
  constexpr int CAP = TOPK_CAP, NS = CAP / 64;
  const int lane = threadIdx.x & 63;
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  const int cnt = min(a.lcnt[si], CAP);
  float s2[NS];
  int i2[NS];
#pragma unroll
  for (int h = 0; h < NS; ++h) {
    const int e = lane + 64 * h;
    const uint2 v = e < cnt ? a.lent[si * CAP + e] : uint2{__float_as_uint(-INFINITY), 0xFFFFFFFFu};
    s2[h] = __uint_as_float(v.x);
    i2[h] = (int)v.y;
  }
  // a list of at most 64 entries sorts in one register (the same order: the padding sorts last)
  if (cnt <= 64) {
    float s1[1] = {s2[0]};
    int i1[1] = {i2[0]};
    wave_bitonic<1>(s1, i1);
    s2[0] = s1[0];
    i2[0] = i1[0];
  } else {
    wave_bitonic<NS>(s2, i2);
  }
  const float t = rdlane(s2[0], a.kt - 1);  // the kt-th approximate score (-inf when fewer)
  // Only the best kt candidates are rescored when the list can be certified (n_dst > TOPK_KC): a
  // candidate ranked below kt has approx <= t, so its F2J score is <= t + e, and a certified row has
  // its k-th exact score above t + e -- it cannot be in the top-k (nor tie).  A row that fails
  // certification is re-scored by the exact scan from the k-th exact score of these kt (still a
  // lower bound of the true k-th).  (Each rescored candidate reads a 512-B fp32 row from HBM.)
  const bool rescore = a.n_dst <= TOPK_KC || lane < a.kt;
  const int row = (i2[0] >= 0 && rescore) ? a.perm[i2[0]] : -1;
  const float ex = f2j_dot_rows<KP>(s, a.T, row, a.kreal, stage);
  // ‖s‖ for the certification bound: the order kernel's value rounded up (a larger ‖s‖ only widens
  // the bound), else computed here
  double nsr = 0.0;
  if (a.sfeat) {
    nsr = (double)a.sfeat[si * TOPK_SF + TOPK_M + 2];
  } else {
    double nn = 0.0;
    for (int c = lane; c < a.kreal; c += 64) nn += (double)s[c] * (double)s[c];
    for (int o = 32; o > 0; o >>= 1) nn += __shfl_xor(nn, o);
    nsr = sqrt(nn);
  }
  float sc1[1] = {ex};
  int ix1[1] = {row};
  wave_bitonic<1>(sc1, ix1);
  const int k = a.k;
  const float kth = rdlane(sc1[0], k - 1);
  if (a.n_dst > TOPK_KC) {
    // |F2J(s,t) - approx| <= fp16 rounding of both operands (2^-11 relative, 2^-25 absolute in the
    // scaled units) + fp32 accumulation of the MFMA started from -threshold (|threshold| <= 1.01·‖s‖·max‖t‖
    // + 1 scaled unit) and the add-back (4γ_{KP+2}) + F2J's own rounding (γ_{KP+2}), relative to ‖s‖·max‖t‖
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double kk = (double)(KP + 2);
    const double gam = kk * u / (1.0 - kk * u);
    const double rel = (9.765625e-04 + 2.384185791015625e-07 + 6.0 * gam) * (1.0 + 1.0 / 512.0);
    const double ns = nsr, tm = (double)a.tmax_norm;
    const double absu = 2.98023223876953125e-08 * 1.001 * sqrt((double)KP) *
                        (ns / (double)a.tsc + tm / (double)a.ssc) + (double)KP * 8.9e-16 * (double)a.unscale;
    const double e = rel * ns * tm + absu;
    // fewer than kt listed: the bound below needs t >= every threshold the scan used, which only a
    // list of kt entries guarantees
    if (cnt < a.kt || !((double)kth > (double)t + e)) {
      if (lane == 0) {
        a.need_exact[so] = 1;
        if (a.kth0) a.kth0[so] = kth;  // a lower bound of the true k-th F2J score: the rescan's start
      }
    }
  }
  if (lane < k) {
    const int idx = ix1[0];
    const int oid = idx >= 0 ? a.dst_ids[idx] : -1;
    const float osc = idx >= 0 ? sc1[0] : __int_as_float(0x7fc00000);
    if (lid) {
      lid[lane] = oid;
      lsc[lane] = osc;
    } else {
      a.out_ids[so * k + lane] = oid;
      a.out_scores[so * k + lane] = osc;
    }
  }
}


// Scan order, starting thresholds and features of the src rows.  One wave per 16 src rows scores them
// against the probe rows (the 256 largest-norm dst rows, fp16 like the scan) on MFMA and finds each
// row's exact kt-th best v* of those 256 by bisection on order-preserving keys.  thr0 = v* minus the
// accumulation difference between this pass and the scan (8γ_{KP+2}·‖s‖·max‖t‖) is a valid starting
// threshold: the probe rows above v* reach the list (their chunks' bound is >= their score), so the
// final kt-th approximate score is >= thr0.  Features (TOPK_SF floats): s_P (fp64 dots with the
// dst Gram's leading eigenvectors, rounded), ‖s_⊥‖ (rounded up, with a floor for the fp64 cancellation),
// the pruning margin e + 1.2e-5·‖s‖·max‖t‖ (e: select's approx error; 1.2e-5 covers the fp32 bound
// arithmetic and F2J's own rounding), ‖s‖ rounded up.  Sort key: thr0 / ‖s‖ (rows that stop at
// similar depths share a workgroup), its low a.order_dir_bits bits replaced by the direction of s_P.
template <int KP>
__global__ __launch_bounds__(256, 2) void topk_order_key_kernel(TopkArgs a, uint32_t* __restrict__ key,
                                                             uint32_t* __restrict__ val, float* __restrict__ thr0,
                                                             float* __restrict__ sfo) {
  constexpr int NQ = KP / 32, RB = 2 * KP;
  // the dst Gram's leading directions in LDS: every lane reads 32 columns x TOPK_M of them (as global
  // loads those were half of the kernel's vector memory instructions)
  __shared__ double sVP[TOPK_M * KP];
  for (int i = threadIdx.x; i < TOPK_M * KP; i += 256) sVP[i] = a.VP[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const int64_t sb = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 6) * 16;  // the wave's first position
  const int64_t si = sb + i16;
  const int srow = si < a.n_src ? a.src_rows[si] : -1;
  const float* sp = a.S + (int64_t)(srow >= 0 ? srow : 0) * KP + 8 * g;
  const float keep = srow >= 0 ? 1.f : 0.f;
  f16x8 sf[NQ];
  double ss = 0.0, spd[TOPK_M] = {};
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const f32x4 v0 = ld4(sp + 32 * q), v1 = ld4(sp + 32 * q + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (e < 4 ? v0[e] : v1[e - 4]) * keep;
      const int col = 32 * q + 8 * g + e;
      ss += (double)v * (double)v;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) spd[d] += (double)v * sVP[d * KP + col];
      sf[q][e] = (_Float16)(v * a.ssc);
    }
  }
  ss += __shfl_xor(ss, 16);
  ss += __shfl_xor(ss, 32);  // every lane: ‖s‖² of row i16
#pragma unroll
  for (int d = 0; d < TOPK_M; ++d) {
    spd[d] += __shfl_xor(spd[d], 16);
    spd[d] += __shfl_xor(spd[d], 32);
  }
  const char* Pr = reinterpret_cast<const char*>(a.probe);
  constexpr int NPJ = TOPK_NPROBE / 16;
  const int64_t n_probe = a.n_dst < TOPK_NPROBE ? a.n_dst : TOPK_NPROBE;
  // exact kt-th largest per row: bisection on order-preserving uint keys (count of keys >= mid over
  // the row's 16 lanes).  Lane (i16, g) holds probe column 16J + i16 of rows 4g + r.  Each 16-lane
  // count is a DPP butterfly (row_mirror, row_half_mirror, quad reversal, quad swap: every lane ends
  // with the row's total) -- a __shfl_xor step is an LDS permute, and 4 x 32 x 4 of them in dependent
  // chains made this kernel ~19 ms at 20M rows.
  auto row_count = [](int c) {
    c += __builtin_amdgcn_mov_dpp(c, 0x140, 0xF, 0xF, false);  // row_mirror: lane i^15
    c += __builtin_amdgcn_mov_dpp(c, 0x141, 0xF, 0xF, false);  // row_half_mirror: lane i^7
    c += __builtin_amdgcn_mov_dpp(c, 0x1B, 0xF, 0xF, false);   // quad_perm [3,2,1,0]: lane i^3
    c += __builtin_amdgcn_mov_dpp(c, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]: lane i^1
    return c;
  };
  // rows per pass: all four while their keys fit 128 VGPRs, else passes of two rows that recompute the
  // probe scores on MFMA (1024 probes in one pass hold 256 key VGPRs: one wave per SIMD, r06 +76 ms)
  constexpr int RP = NPJ * 4 <= 128 ? 4 : 2;
  uint32_t lo[4] = {0u, 0u, 0u, 0u};  // count(>= lo) >= kt always holds (TOPK_NPROBE keys >= 0)
  static_for<0, 4 / RP>([&](auto pc) {
    constexpr int P0 = decltype(pc)::value * RP;
    uint32_t u[NPJ][RP];
#pragma unroll
    for (int J = 0; J < NPJ; ++J) {
      const int64_t p = 16 * J + i16;
      f32x4 acc = zero4();
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const f16x8 d = *reinterpret_cast<const f16x8*>(Pr + p * RB + 16 * (4 * q + g));  // zero rows past n
        acc = mfma_h(sf[q], d, acc);
      }
#pragma unroll
      for (int rr = 0; rr < RP; ++rr) {
        const uint32_t bb = __float_as_uint(p < n_probe ? acc[P0 + rr] : -INFINITY);
        u[J][rr] = (bb & 0x80000000u) ? ~bb : (bb | 0x80000000u);
      }
      if constexpr (RP < 4) __builtin_amdgcn_sched_barrier(0);  // probe loads a few columns ahead only
    }
    uint32_t hi[RP];
#pragma unroll
    for (int rr = 0; rr < RP; ++rr) hi[rr] = 0xffffffffu;
    for (int it = 0; it < TOPK_BISECT; ++it) {
#pragma unroll
      for (int rr = 0; rr < RP; ++rr) {
        const uint32_t mid = lo[P0 + rr] + (uint32_t)(((uint64_t)hi[rr] - lo[P0 + rr] + 1) >> 1);
        int cnt = 0;
#pragma unroll
        for (int J = 0; J < NPJ; ++J) cnt += u[J][rr] >= mid ? 1 : 0;
        cnt = row_count(cnt);
        if (cnt >= a.kt) lo[P0 + rr] = mid;
        else hi[rr] = mid - 1u;
      }
    }
  });
  float vs[4];
#pragma unroll
  // key -> the smallest score of its bucket (the undecided low bits: zero); keys at or below -inf's
  // (0x007fffff; truncated, they would decode to NaN) are -inf
  for (int r = 0; r < 4; ++r)
    vs[r] = lo[r] < 0x00800000u ? -INFINITY : __uint_as_float((lo[r] & 0x80000000u) ? (lo[r] & 0x7fffffffu) : ~lo[r]);
  const int rsel = 4 * g + (i16 & 3);  // the row this lane reports in the group (lanes i16 < 4)
  const double nrm2 = __shfl(ss, rsel);
  const double nrm = sqrt(nrm2);
  double sq[TOPK_M];
  double pp = 0.0;
#pragma unroll
  for (int d = 0; d < TOPK_M; ++d) {
    sq[d] = __shfl(spd[d], rsel);
    pp += sq[d] * sq[d];
  }
  if (i16 < 4) {
    const int r = i16;
    const int64_t pr = sb + 4 * g + r;
    float v = vs[0];
#pragma unroll
    for (int rr = 1; rr < 4; ++rr) v = r == rr ? vs[rr] : v;
    if (pr < a.n_src) {
      const double kk = (double)(KP + 2) * 5.9604644775390625e-08;
      const double margin = (8.0 * kk / (1.0 - kk) + 9.5367431640625e-07) * nrm * (double)a.tmax_norm + 1e-30;
      const float t0 = v == -INFINITY ? -INFINITY : (float)((double)v * (double)a.unscale - margin);
      thr0[pr] = t0;
      const float k = nrm > 0.0 ? (float)((double)t0 / nrm) : INFINITY;
      const uint32_t bb = __float_as_uint(k);
      uint32_t kk32 = (bb & 0x80000000u) ? ~bb : (bb | 0x80000000u);
      if (a.order_dir_bits != 0 && nrm > 0.0) {
        // coarser depth, then the direction of s_P (lexicographic in u1, u2, u3 = s_P[1..3] / ‖s‖):
        // the rows of one workgroup then need similar chunks, so its mask union stays tight and its
        // waves skip fewer of the chunks it streams
        const int b1 = a.order_dir_bits & 255, b2 = (a.order_dir_bits >> 8) & 255, b3 = (a.order_dir_bits >> 16) & 255;
        const int db = b1 + b2 + b3;
        auto qz = [](double u, int bits) {
          const int m = (1 << bits) - 1;
          const int v = (int)((u + 1.0) * 0.5 * (double)(m + 1));
          return (uint32_t)(v < 0 ? 0 : (v > m ? m : v));
        };
        const uint32_t code = (qz(sq[1] / nrm, b1) << (b2 + b3)) | (qz(sq[2] / nrm, b2) << b3) | qz(sq[3] / nrm, b3);
        kk32 = (kk32 & ~((1u << db) - 1u)) | code;
      }
      key[pr] = kk32;
      val[pr] = (uint32_t)pr;
      float* o = sfo + pr * TOPK_SF;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) o[d] = (float)sq[d];
      o[TOPK_M] = __double2float_ru(sqrt(fmax(nrm2 - pp, 0.0) + 1e-13 * nrm2));
      o[TOPK_M + 1] = (float)(tk_err<KP>(nrm, a) + 1.2e-5 * nrm * (double)a.tmax_norm) * 1.0001f;
      o[TOPK_M + 2] = __double2float_ru(nrm);
      o[TOPK_M + 3] = 0.f;
    }
  }
}

size_t topk_order_temp_bytes(int64_t n_src) { return topk_sort_temp_bytes(n_src); }

// src_sorted[i] = src_rows[order[i]] (and thr0, features); order[i] = the position whose results
// slot i fills
hipError_t topk_order(int KP, const TopkArgs& a, void* temp, size_t temp_bytes, uint32_t* keys, uint32_t* order,
                      int32_t* src_sorted, float* thr_tmp, float* thr_sorted, float* sf_tmp, float* sf_sorted,
                      hipStream_t s) {
  const int64_t n = a.n_src;
  if (n <= 0) return hipSuccess;
  uint32_t* k0 = keys;
  uint32_t* k1 = keys + n;
  uint32_t* v0 = order + n;
  const int blocks = (int)((n + 63) / 64);
  if (KP == 64) topk_order_key_kernel<64><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp, sf_tmp);
  else if (KP == 128) topk_order_key_kernel<128><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp, sf_tmp);
  else topk_order_key_kernel<256><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp, sf_tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  // ascending thr0 / ‖s‖: rows with the lowest relative thresholds (the most chunks to scan, the most
  // candidates) fill the first workgroups, which the dispatcher starts first; the light ones then fill
  // in behind them instead of the heavy ones forming the launch's tail
  e = rocprim::radix_sort_pairs(temp, tb, k0, k1, v0, order, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  topk_gather_rows_kernel<<<tk_grid(n, 256), 256, 0, s>>>(a.src_rows, thr_tmp, sf_tmp, order, n, src_sorted,
                                                          thr_sorted, sf_sorted);
  return hipGetLastError();
}

// The chunks each scan workgroup can need: chunk c is needed when some row i of the workgroup has
// bound(s_i, c) + margin_i >= thr0_i; rows of a chunk that is not needed have approx < thr0 <= every
// threshold the scan will use, so the scan would not append any of them.  Super-chunks (16 chunks,
// the union box) are tested first.  One bit per chunk: word w holds chunks 32w .. 32w+31 (super-chunks
// 2w and 2w + 1).
__global__ __launch_bounds__(256) void topk_mask_kernel(TopkArgs a, int rwg, const float* __restrict__ supf,
                                                        int64_t n_super, uint32_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float rf[];  // [rwg][8]: s_P, ‖s_⊥‖, thr0 - margin
  __shared__ uint16_t ms[4096];                              // one batch of super-chunk masks
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * rwg;
  int nrow = 0;
  for (int i = tid; i < rwg; i += 256) {
    const int64_t p = p0 + i;
    float* o = rf + 8 * i;
    if (p < a.n_src) {
      const float* f = a.sfeat + p * TOPK_SF;
#pragma unroll
      for (int d = 0; d <= TOPK_M; ++d) o[d] = f[d];
      const float t0 = a.thr0 ? a.thr0[p] : -INFINITY;
      o[TOPK_M + 1] = t0 == -INFINITY ? -INFINITY : t0 - f[TOPK_M + 1];
    } else {
#pragma unroll
      for (int d = 0; d <= TOPK_M; ++d) o[d] = 0.f;
      o[TOPK_M + 1] = INFINITY;
    }
  }
  nrow = (int)std::min<int64_t>(rwg, a.n_src - p0);
  __syncthreads();
  // envelope of each group of MG rows: per direction the min / max of s_d, the max ‖s_⊥‖ and the
  // smallest threshold.  tk_bound is convex in each s_d (max(s_d·lo_d, s_d·hi_d)), so its maximum
  // over the group is at an end of [min s_d, max s_d]; fp32 rounding is monotonic, so evaluated in
  // tk_bound's order the envelope is >= every row's bound: a group whose envelope is below its
  // smallest threshold has no row that needs the chunk, and a chunk most groups reject costs
  // rwg / MG envelope tests instead of rwg row tests
  constexpr int MG = 32;
  __shared__ float genv[512 / MG][2 * TOPK_M + 2];  // smin[M], smax[M], max ‖s_⊥‖, min threshold
  const int ngrp = (nrow + MG - 1) / MG;
  if (tid < ngrp) {
    float mn[TOPK_M], mx[TOPK_M], sp = 0.f, th = INFINITY;
#pragma unroll
    for (int d = 0; d < TOPK_M; ++d) { mn[d] = INFINITY; mx[d] = -INFINITY; }
    for (int i = tid * MG; i < min(nrow, tid * MG + MG); ++i) {
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) { mn[d] = fminf(mn[d], rf[8 * i + d]); mx[d] = fmaxf(mx[d], rf[8 * i + d]); }
      sp = fmaxf(sp, rf[8 * i + TOPK_M]);
      th = fminf(th, rf[8 * i + TOPK_M + 1]);
    }
#pragma unroll
    for (int d = 0; d < TOPK_M; ++d) { genv[tid][d] = mn[d]; genv[tid][TOPK_M + d] = mx[d]; }
    genv[tid][2 * TOPK_M] = sp;
    genv[tid][2 * TOPK_M + 1] = th;
  }
  __syncthreads();
  auto needed = [&](const float* cf) {
    float c[TOPK_CF];
#pragma unroll
    for (int f = 0; f < TOPK_CF; f += 4) {
      const f32x4 v = ld4(cf + f);
#pragma unroll
      for (int e = 0; e < 4; ++e) c[f + e] = v[e];
    }
    for (int gq = 0; gq < ngrp; ++gq) {
      const float* e = genv[gq];
      float b = e[2 * TOPK_M] * c[2 * TOPK_M];  // tk_bound's order
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d)
        b += fmaxf(fmaxf(e[d] * c[d], e[d] * c[TOPK_M + d]), fmaxf(e[TOPK_M + d] * c[d], e[TOPK_M + d] * c[TOPK_M + d]));
      if (!(b >= e[2 * TOPK_M + 1])) continue;
      for (int i = gq * MG; i < min(nrow, gq * MG + MG); ++i)
        if (tk_bound(rf + 8 * i, c) >= rf[8 * i + TOPK_M + 1]) return true;
    }
    return false;
  };
  uint32_t* mrow = mask + (int64_t)blockIdx.x * a.mask_words;
  for (int64_t s0 = 0; s0 < n_super; s0 += 4096) {
    const int nb = (int)std::min<int64_t>(4096, n_super - s0);
    for (int j = tid; j < nb; j += 256) {
      const int64_t sup = s0 + j;
      uint32_t bits = 0u;
      if (needed(supf + sup * TOPK_CF)) {
        for (int c = 0; c < TOPK_SUPER; ++c) {
          const int64_t ch = sup * TOPK_SUPER + c;
          if (ch < a.n_chunks && needed(a.cfeat + ch * TOPK_CF)) bits |= 1u << c;
        }
      }
      ms[j] = (uint16_t)bits;
    }
    __syncthreads();
    for (int w = tid; w < (nb + 1) / 2; w += 256) {
      const uint32_t lo = ms[2 * w], hi = 2 * w + 1 < nb ? ms[2 * w + 1] : 0u;
      mrow[s0 / 2 + w] = lo | (hi << 16);
    }
    __syncthreads();
  }
}

// Exact path: one workgroup (4 waves) per src row, full F2J scan.  Each wave keeps its best 64·P
// (score desc, id asc) in registers, slots [0, P) sorted, and buffers up to 64·P newcomers in slots
// [P, 2P); a batch of 64 scores is only buffered when one of them reaches the current 64·P-th best,
// and a full buffer is merged by one bitonic sort of the 128·P slots.  The four waves' lists are
// merged at the end.  P = 1 serves the rows the MFMA pre-selection could not certify; P up to 8
// serves k up to 512 (recommendForAll* with k > 64, no pre-selection).  The dst rows are visited in
// the prepared chunk order and a chunk whose bound (+ F2J rounding) is below the wave's own 64·P-th
// best is skipped: none of its rows can enter the merged top-k (<= 64·P), ties included.  The bounds
// are evaluated 64 chunks at a time (a lane per chunk), so a pruned chunk costs a fraction of one
// feature-load latency instead of a dependent load per 64 rows.
// dcount != null (the certification rescans, r05): a persistent grid takes the rows rows[0 ..
// *dcount) from the counter *dnext, so the host never waits for the flagged count.
template <int KP, int P>
__global__ __launch_bounds__(256) void topk_exact_kernel(TopkArgs a, const int32_t* rows, int64_t row0,
                                                         const int* dcount, int* dnext) {
  __shared__ float msc[4][64 * P];
  __shared__ int mix[4][64 * P];
  __shared__ __attribute__((aligned(16))) float s_stage[4][64 * TK_SEL_LD + KP];  // f2j_dot_rows
  __shared__ int s_idx;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t it = 0;; ++it) {
  int64_t si;
  if (dcount) {
    if (threadIdx.x == 0) s_idx = atomicAdd(dnext, 1);
    __syncthreads();
    const int idx = s_idx;
    __syncthreads();  // s_idx read by every thread before the next claim rewrites it
    if (idx >= *dcount) return;  // workgroup-uniform
    si = rows[idx];
  } else {
    if (it > 0) return;
    si = rows ? rows[row0 + blockIdx.x] : row0 + (int64_t)blockIdx.x;
  }
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  float bs[2 * P];
  int bi[2 * P];
#pragma unroll
  for (int h = 0; h < 2 * P; ++h) { bs[h] = -INFINITY; bi[h] = -1; }
  int nin = 0;                // newcomer batches buffered (wave-uniform)
  // the kept list's last score once full; a rescan starts from the certification pass's k-th exact
  // score (a lower bound of the true k-th: rows strictly below it cannot enter the top-k)
  const float thr_init = a.kth0 ? a.kth0[si] : -INFINITY;
  float thr = thr_init;
  // this row's bound features (fp64, like the order kernel's)
  float sfe[TOPK_M + 1];
  float marg = 0.f;
  if (a.cfeat) {
    double nn = 0.0, sp[TOPK_M] = {};
    for (int c = lane; c < a.kreal; c += 64) {
      const double v = (double)s[c];
      nn += v * v;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) sp[d] += v * a.VP[d * KP + c];
    }
    for (int o = 32; o > 0; o >>= 1) {
      nn += __shfl_xor(nn, o);
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) sp[d] += __shfl_xor(sp[d], o);
    }
    double pp = 0.0;
#pragma unroll
    for (int d = 0; d < TOPK_M; ++d) {
      sfe[d] = (float)sp[d];
      pp += sp[d] * sp[d];
    }
    sfe[TOPK_M] = __double2float_ru(sqrt(fmax(nn - pp, 0.0) + 1e-13 * nn));
    marg = (float)(1.2e-5 * sqrt(nn) * (double)a.tmax_norm) * 1.0001f + 1e-30f;
  }
  // 64 dst rows (one per lane) -> F2J scores, buffered when one of them reaches the threshold
  auto score64 = [&](int64_t pj, bool in) {
    const int64_t dj = (a.perm && in) ? (int64_t)a.perm[pj] : pj;
    const float sc = f2j_dot_rows<KP>(s, a.T, in ? (int)dj : -1, a.kreal, s_stage[wave]);
    if (!__any(sc >= thr)) return;
    static_for<0, P>([&](auto hh) {
      constexpr int h = decltype(hh)::value;
      if (nin == h) { bs[P + h] = sc; bi[P + h] = in ? (int)dj : -1; }
    });
    if (++nin == P) {
      wave_bitonic<2 * P>(bs, bi);
#pragma unroll
      for (int h = P; h < 2 * P; ++h) { bs[h] = -INFINITY; bi[h] = -1; }
      nin = 0;
      thr = fmaxf(thr_init, rdlane(bs[P - 1], 63));
    }
  };
  if (a.cfeat) {
    // chunk-major: each lane tests the bound of one of the wave's next 64 chunks (one feature load
    // latency per 64 chunks, not per chunk), then the wave scores the rows of the chunks that pass,
    // re-testing each against the threshold as it rises
    const int ch = topk_chunk_rows_dev<KP>();
    for (int64_t c0 = (int64_t)wave * 64; c0 < a.n_chunks; c0 += 256) {
      const int64_t c = c0 + lane;
      float b = INFINITY;
      if (c < a.n_chunks) b = tk_bound(sfe, a.cfeat + c * TOPK_CF) + marg;
      uint64_t m = __ballot(c < a.n_chunks && !(b < thr));
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        if (rdlane(b, l) < thr) continue;  // the threshold rose past this chunk's bound
        const int64_t cc = c0 + l;
        for (int r0 = 0; r0 < ch; r0 += 64) {
          const int64_t pj = cc * ch + r0 + lane;
          score64(pj, r0 + lane < ch && pj < a.n_dst);
        }
      }
    }
  } else {
    for (int64_t j0 = (int64_t)wave * 64; j0 < a.n_dst; j0 += 256) score64(j0 + lane, j0 + lane < a.n_dst);
  }
  wave_bitonic<2 * P>(bs, bi);
#pragma unroll
  for (int h = 0; h < P; ++h) {
    msc[wave][64 * h + lane] = bs[h];
    mix[wave][64 * h + lane] = bi[h];
  }
  __syncthreads();
  if (wave == 0) {  // fold the other waves' lists in, one bitonic sort of 128·P slots each
    for (int w = 1; w < 4; ++w) {
#pragma unroll
      for (int h = 0; h < P; ++h) { bs[P + h] = msc[w][64 * h + lane]; bi[P + h] = mix[w][64 * h + lane]; }
      wave_bitonic<2 * P>(bs, bi);
    }
#pragma unroll
    for (int h = 0; h < P; ++h) {
      const int e = 64 * h + lane;
      if (e < a.k) {
        const int idx = bi[h];
        a.out_ids[si * a.k + e] = idx >= 0 ? a.dst_ids[idx] : -1;
        a.out_scores[si * a.k + e] = idx >= 0 ? bs[h] : __int_as_float(0x7fc00000);
      }
    }
  }
  __syncthreads();  // msc / mix read by wave 0 before the next row's waves rewrite them
  }
}

// ---------------------------------------------------------------------------------------------
// preparation of the dst side
// ---------------------------------------------------------------------------------------------
// per dst row r (one wave): t_P (fp64) = VP·t, pkey = bits of ‖t_⊥‖ rounded up (with a floor for the
// fp64 cancellation), nkey = bits of ‖t‖ rounded up; vals = r for both sorts
__global__ void topk_feat_kernel(const float* __restrict__ T, int64_t n, int KP, int kreal, const double* __restrict__ VP,
                                 double* __restrict__ tp, uint32_t* __restrict__ pkey, uint32_t* __restrict__ pval,
                                 uint32_t* __restrict__ nkey, uint32_t* __restrict__ nval) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    double s2 = 0.0, sp[TOPK_M] = {};
    for (int c = lane; c < kreal; c += 64) {
      const double v = (double)T[r * KP + c];
      s2 += v * v;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) sp[d] += v * VP[d * KP + c];
    }
    for (int o = 32; o > 0; o >>= 1) {
      s2 += __shfl_xor(s2, o);
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) sp[d] += __shfl_xor(sp[d], o);
    }
    if (lane == 0) {
      double pp = 0.0;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) {
        tp[r * TOPK_M + d] = sp[d];
        pp += sp[d] * sp[d];
      }
      pkey[r] = __float_as_uint(__double2float_ru(sqrt(fmax(s2 - pp, 0.0) + 1e-13 * s2)));
      pval[r] = (uint32_t)r;
      nkey[r] = __float_as_uint(__double2float_ru(sqrt(s2)));
      nval[r] = (uint32_t)r;
    }
  }
}
// Th[p] = fp16(T[perm[p]]·tsc) (zero rows past n)
__global__ void topk_pack_kernel(const float* __restrict__ T, int64_t n, int64_t n_pad, int KP, float tsc,
                                 const uint32_t* __restrict__ perm, _Float16* __restrict__ Th) {
  const int64_t tot = n_pad * KP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / KP;
    const int c = (int)(e % KP);
    Th[e] = p < n ? (_Float16)(T[(int64_t)perm[p] * KP + c] * tsc) : (_Float16)0.f;
  }
}
// chunk c (one wave): box of t_P over its rows (fp64, rounded outward) and R = max ‖t_⊥‖ (sorted keys)
__global__ void topk_chunk_feat_kernel(const double* __restrict__ tp, const uint32_t* __restrict__ perm,
                                       const uint32_t* __restrict__ pkey_sorted, int64_t n, int CH, int64_t n_chunks,
                                       float* __restrict__ cfeat) {
  const int lane = threadIdx.x & 63;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < n_chunks; c += (int64_t)gridDim.x * 4) {
    double lo[TOPK_M], hi[TOPK_M];
#pragma unroll
    for (int d = 0; d < TOPK_M; ++d) { lo[d] = INFINITY; hi[d] = -INFINITY; }
    float R = 0.f;
    for (int j = lane; j < CH; j += 64) {
      const int64_t p = c * CH + j;
      if (p < n) {
        const uint32_t r = perm[p];
#pragma unroll
        for (int d = 0; d < TOPK_M; ++d) {
          const double v = tp[(int64_t)r * TOPK_M + d];
          lo[d] = fmin(lo[d], v);
          hi[d] = fmax(hi[d], v);
        }
        R = fmaxf(R, __uint_as_float(pkey_sorted[p]));
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) {
        lo[d] = fmin(lo[d], __shfl_xor(lo[d], o));
        hi[d] = fmax(hi[d], __shfl_xor(hi[d], o));
      }
      R = fmaxf(R, __shfl_xor(R, o));
    }
    if (lane == 0) {
      float* o = cfeat + c * TOPK_CF;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) {
        o[d] = lo[d] == INFINITY ? 0.f : __double2float_rd(lo[d]);
        o[TOPK_M + d] = hi[d] == -INFINITY ? 0.f : __double2float_ru(hi[d]);
      }
      o[2 * TOPK_M] = R;
      for (int f = 2 * TOPK_M + 1; f < TOPK_CF; ++f) o[f] = 0.f;
    }
  }
}
// super-chunk s: the union of its TOPK_SUPER chunk boxes
__global__ void topk_super_feat_kernel(const float* __restrict__ cfeat, int64_t n_chunks, int64_t n_super,
                                       float* __restrict__ supf) {
  for (int64_t sidx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sidx < n_super; sidx += (int64_t)gridDim.x * blockDim.x) {
    float o[TOPK_CF];
#pragma unroll
    for (int d = 0; d < TOPK_M; ++d) { o[d] = INFINITY; o[TOPK_M + d] = -INFINITY; }
    o[2 * TOPK_M] = 0.f;
    for (int c = 0; c < TOPK_SUPER; ++c) {
      const int64_t ch = sidx * TOPK_SUPER + c;
      if (ch >= n_chunks) break;
      const float* f = cfeat + ch * TOPK_CF;
#pragma unroll
      for (int d = 0; d < TOPK_M; ++d) {
        o[d] = fminf(o[d], f[d]);
        o[TOPK_M + d] = fmaxf(o[TOPK_M + d], f[TOPK_M + d]);
      }
      o[2 * TOPK_M] = fmaxf(o[2 * TOPK_M], f[2 * TOPK_M]);
    }
    for (int f = 2 * TOPK_M + 1; f < TOPK_CF; ++f) o[f] = 0.f;
    for (int f = 0; f < TOPK_CF; ++f) supf[sidx * TOPK_CF + f] = o[f];
  }
}

namespace {
template <int KP>
constexpr int tk_chunk_rows() { return TkScan<KP, 2>::CH; }
}  // namespace

int topk_chunk_rows(int KP) {
  return KP == 64 ? tk_chunk_rows<64>() : KP == 128 ? tk_chunk_rows<128>() : tk_chunk_rows<256>();
}

size_t topk_sort_temp_bytes(int64_t n) {
  size_t tb = 0, ta = 0;
  (void)rocprim::radix_sort_pairs_desc(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (size_t)n, 0, 32, (hipStream_t)0);
  (void)rocprim::radix_sort_pairs(nullptr, ta, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0, 32, (hipStream_t)0);
  return std::max(tb, ta);
}

hipError_t topk_prepare(int KP, int kreal, const float* T, int64_t n, float tsc, const double* VP, void* temp,
                        size_t temp_bytes, uint32_t* keys, uint32_t* perm, uint32_t* nperm, double* tp, void* Th,
                        float* cfeat, float* supf, void* probe, hipStream_t s) {
  const int CH = topk_chunk_rows(KP);
  const int64_t n_pad = (n + CH - 1) / CH * CH, n_chunks = n_pad / CH;
  const int64_t n_super = (n_chunks + TOPK_SUPER - 1) / TOPK_SUPER;
  uint32_t* pk0 = keys;          // ‖t_⊥‖ keys, unsorted / sorted
  uint32_t* pk1 = keys + n;
  uint32_t* nk0 = keys + 2 * n;  // ‖t‖ keys
  uint32_t* nk1 = keys + 3 * n;
  topk_feat_kernel<<<tk_grid(n, 4), 256, 0, s>>>(T, n, KP, kreal, VP, tp, pk0, perm + n, nk0, nperm + n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  e = rocprim::radix_sort_pairs_desc(temp, tb, pk0, pk1, perm + n, perm, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  e = rocprim::radix_sort_pairs_desc(temp, tb, nk0, nk1, nperm + n, nperm, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  topk_pack_kernel<<<tk_grid(n_pad * KP, 256), 256, 0, s>>>(T, n, n_pad, KP, tsc, perm, reinterpret_cast<_Float16*>(Th));
  topk_pack_kernel<<<tk_grid(TOPK_NPROBE * KP, 256), 256, 0, s>>>(T, std::min<int64_t>(n, TOPK_NPROBE), TOPK_NPROBE, KP, tsc, nperm,
                                                          reinterpret_cast<_Float16*>(probe));
  topk_chunk_feat_kernel<<<tk_grid(n_chunks, 4), 256, 0, s>>>(tp, perm, pk1, n, CH, n_chunks, cfeat);
  topk_super_feat_kernel<<<tk_grid(n_super, 256), 256, 0, s>>>(cfeat, n_chunks, n_super, supf);
  return hipGetLastError();
}

hipError_t launch_topk_mask(const TopkArgs& a, int rows_per_wg, const float* supf, int64_t n_super, uint32_t* mask,
                            hipStream_t s) {
  const int64_t n_wg = (a.n_src + rows_per_wg - 1) / rows_per_wg;
  if (n_wg <= 0) return hipSuccess;
  topk_mask_kernel<<<(int)n_wg, 256, (size_t)rows_per_wg * 8 * 4, s>>>(a, rows_per_wg, supf, n_super, mask);
  return hipGetLastError();
}

template <int KP, int G>
hipError_t launch_scan(const TopkArgs& a, hipStream_t s) {
  using C = TkScan<KP, G>;
  static const hipError_t attr = allow_lds(topk_scan_kernel<KP, G>, C::LDS);
  if (attr != hipSuccess) return attr;
  topk_scan_kernel<KP, G><<<(int)((a.n_src + C::RWG - 1) / C::RWG), 256, C::LDS, s>>>(a);
  return hipGetLastError();
}

// src rows per scan workgroup: register blocking G = 4 (two workgroups per CU: r05, c4 all users
// scan 649 -> 438 ms against G = 8 at one per CU), smaller while it leaves CUs without two workgroups
int topk_rows_per_workgroup(int KP, int64_t n_src, int n_cu) {
  int gmax = KP <= 128 ? 8 : 4;
  // ALBEDO_TOPK_GMAX: A/B knob, read per call like the other knobs; only 2, 4 or 8 are accepted
  const char* e = std::getenv("ALBEDO_TOPK_GMAX");
  const int ge = e && *e ? std::atoi(e) : 4;
  const int gcap = (ge == 2 || ge == 4 || ge == 8) ? ge : 4;
  gmax = std::min(gmax, std::max(2, gcap));
  for (int G = gmax; G > 2; G /= 2)
    if (n_src >= (int64_t)2 * n_cu * 64 * G) return 64 * G;
  return 128;
}

template <int KP>
hipError_t launch_topk_kp(const TopkArgs& a, int n_cu, hipStream_t s) {
  hipError_t e;
  const int rows = topk_rows_per_workgroup(KP, a.n_src, n_cu);
  if (rows == 512) e = launch_scan<KP, (KP <= 128 ? 8 : 4)>(a, s);
  else if (rows == 256) e = launch_scan<KP, 4>(a, s);
  else e = launch_scan<KP, 2>(a, s);
  return e;
}

hipError_t launch_topk(int KP, const TopkArgs& a, int n_cu, hipStream_t s) {
  if (a.n_src <= 0) return hipSuccess;
  if (KP == 64) return launch_topk_kp<64>(a, n_cu, s);
  if (KP == 128) return launch_topk_kp<128>(a, n_cu, s);
  if (KP == 256) return launch_topk_kp<256>(a, n_cu, s);
  return hipErrorInvalidValue;
}

#ifdef ALBEDO_TOPK_PHASES
extern "C" int als_debug_topk_phases(unsigned long long* out16, int reset) {
  if (out16 && hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_tk_ph), 16 * 8) != hipSuccess) return 4;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tk_ph), z, sizeof z) != hipSuccess) return 4;
  }
  return 0;
}
#endif

hipError_t launch_topk_select(int KP, const TopkArgs& a, hipStream_t s) {
  const int64_t n = a.in_pos ? a.n_slots : a.n_src;
  if (n <= 0) return hipSuccess;
  const int blocks = (int)((n + 3) / 4);
  if (KP == 64) topk_select_kernel<64><<<blocks, 256, 0, s>>>(a);
  else if (KP == 128) topk_select_kernel<128><<<blocks, 256, 0, s>>>(a);
  else if (KP == 256) topk_select_kernel<256><<<blocks, 256, 0, s>>>(a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// max_r ||T[r][0..kreal)||_2 (fp64), stored as the bits of a non-negative double
__global__ void rownorm_max_kernel(const float* __restrict__ T, int64_t n, int KP, int kreal,
                                   unsigned long long* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  double best = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    double s2 = 0.0;
    for (int c = lane; c < kreal; c += 64) s2 += (double)T[r * KP + c] * (double)T[r * KP + c];
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    best = fmax(best, s2);
  }
  if (lane == 0) atomicMax(out, (unsigned long long)__double_as_longlong(sqrt(best)));
}

hipError_t launch_rownorm_max(const float* T, int64_t n, int KP, int kreal, unsigned long long* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, 8, s);
  if (e != hipSuccess || n <= 0) return e;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  rownorm_max_kernel<<<(int)blocks, 256, 0, s>>>(T, n, KP, kreal, out);
  return hipGetLastError();
}

template <int KP, int P>
hipError_t topk_exact_p(const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  for (int64_t r0 = 0; r0 < n_rows; r0 += max_rows_per_launch(256)) {
    const int64_t n = std::min<int64_t>(n_rows - r0, max_rows_per_launch(256));
    topk_exact_kernel<KP, P><<<(int)n, 256, 0, s>>>(a, rows, r0, nullptr, nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
template <int KP, int P>
hipError_t topk_exact_dev_p(const TopkArgs& a, const int32_t* rows, const int* dcount, int* dnext, int grid, hipStream_t s) {
  topk_exact_kernel<KP, P><<<grid, 256, 0, s>>>(a, rows, 0, dcount, dnext);
  return hipGetLastError();
}
template <int KP>
hipError_t topk_exact_kp(const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  if (a.k <= 64) return topk_exact_p<KP, 1>(a, rows, n_rows, s);
  if (a.k <= 128) return topk_exact_p<KP, 2>(a, rows, n_rows, s);
  if (a.k <= 256) return topk_exact_p<KP, 4>(a, rows, n_rows, s);
  if (a.k <= TOPK_MAX) return topk_exact_p<KP, 8>(a, rows, n_rows, s);
  return hipErrorInvalidValue;
}
// need[i] != 0 -> flags[atomicAdd(cnt, 1)] = i (order irrelevant: the rescan writes each row's own
// slot); cnt[2] accumulates the call's total
__global__ void topk_flag_compact_kernel(const int32_t* __restrict__ need, int64_t n, int32_t* __restrict__ flags,
                                         int* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (need[i]) {
      flags[atomicAdd(cnt, 1)] = (int32_t)i;
      atomicAdd(cnt + 2, 1);
    }
}
hipError_t launch_topk_exact_flagged(int KP, const TopkArgs& a, const int32_t* need, int64_t n, int32_t* flags, int* cnt,
                                     int n_cu, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  topk_flag_compact_kernel<<<tk_grid(n, 256), 256, 0, s>>>(need, n, flags, cnt);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int grid = (int)std::min<int64_t>(n, (int64_t)4 * n_cu);
  const int* dcount = cnt;
  int* dnext = cnt + 1;
  if (a.k > 64) return hipErrorInvalidValue;  // the certification path is k <= TOPK_KC
  if (KP == 64) return topk_exact_dev_p<64, 1>(a, flags, dcount, dnext, grid, s);
  if (KP == 128) return topk_exact_dev_p<128, 1>(a, flags, dcount, dnext, grid, s);
  if (KP == 256) return topk_exact_dev_p<256, 1>(a, flags, dcount, dnext, grid, s);
  return hipErrorInvalidValue;
}

__global__ void invert_perm_kernel(const uint32_t* __restrict__ perm, int64_t n, uint32_t* __restrict__ inv) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    inv[perm[i]] = (uint32_t)i;
}
hipError_t launch_invert_perm(const uint32_t* perm, int64_t n, uint32_t* inv, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  invert_perm_kernel<<<tk_grid(n, 256), 256, 0, s>>>(perm, n, inv);
  return hipGetLastError();
}

__global__ void iota_i32_kernel(int32_t* __restrict__ out, int64_t n, int64_t start) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)(start + i);
}
hipError_t launch_iota_i32(int32_t* out, int64_t n, int64_t start, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  iota_i32_kernel<<<tk_grid(n, 256), 256, 0, s>>>(out, n, start);
  return hipGetLastError();
}

hipError_t launch_topk_exact(int KP, const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  if (KP == 64) return topk_exact_kp<64>(a, rows, n_rows, s);
  if (KP == 128) return topk_exact_kp<128>(a, rows, n_rows, s);
  if (KP == 256) return topk_exact_kp<256>(a, rows, n_rows, s);
  return hipErrorInvalidValue;
}

}  // namespace albedo
