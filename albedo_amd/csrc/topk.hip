// Top-k recommendation (ALSModel.recommendForAll* / albedo's ALSRecommender.recommendForUsers,
// recommenders/ALSRecommender.scala:28-65: F2J sdot scores, BoundedPriorityQueue top-k,
// BoundedPriorityQueue.scala:30-53).  The score matrix is never materialised.
//
//  prepare  dst rows ordered by descending L2 norm (device radix sort), packed as fp16 rows scaled by
//           a power of two, plus the norm of every chunk's first row (the largest of that chunk and of
//           everything after it);
//  scan     one workgroup per 64·G src rows: the src rows' fp16 fragments stay in registers, the dst
//           rows stream through an LDS ring filled by LDS-DMA; scores on v_mfma_f32_16x16x32_f16, each
//           compared with its row's threshold (the 64th best so far) and appended to a per-row list in
//           global memory; a full list is compacted to its best 64 by a wave bitonic sort.  Because the
//           dst rows arrive by descending norm, Cauchy-Schwarz ends the scan early: once
//           ‖s‖·‖t_j‖ <= threshold for every row of the workgroup, no later dst row can enter;
//  select   one wave per src row: best 64 of the list by approximate score, exact F2J rescoring of
//           those 64, sort (score desc, id asc), certification: every dst row outside the 64 has
//           approx <= t (the 64th approx score) or was pruned with ‖s‖‖t_j‖ <= t, so its F2J score is
//           <= t + e with e the fp16 + fp32 error bound; if the k-th exact score is not > t + e the row
//           is re-scored by the exact full scan (topk_exact_kernel).
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
                                        const uint32_t* __restrict__ order, int64_t n, int32_t* __restrict__ out,
                                        float* __restrict__ thr_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = rows[order[i]];
    thr_out[i] = thr[order[i]];
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

// ---------------------------------------------------------------------------------------------
// scan geometry.  A chunk is 16 KiB of fp16 dst rows (128 / 64 / 32 rows at KP = 64 / 128 / 256) plus
// one 256-B DMA per wave carrying the chunk's head norm; NSTG chunks form the LDS ring.
// ---------------------------------------------------------------------------------------------
template <int KP, int G>
struct TkScan {
  static constexpr int RB = 2 * KP;              // bytes per fp16 dst row
  static constexpr int CB = 16384;               // dst bytes per chunk
  static constexpr int CH = CB / RB;             // dst rows per chunk
  static constexpr int NJ = CH / 16;             // 16-row tiles per chunk
  static constexpr int NQ = KP / 32;             // 32-deep MFMA steps per tile
  static constexpr int NSTG = G >= 4 ? 6 : 4;    // ring depth (chunks)
  static constexpr int SLOT = CB + 4 * 256;      // + one norm DMA per wave
  static constexpr int RWG = 64 * G;             // src rows per workgroup (16·G per wave)
  static constexpr int DPW = CB / 1024 / 4;      // 1-KiB row DMAs per wave per chunk
  static constexpr int NVM = DPW + 1;            // DMA instructions per wave per chunk
  static constexpr int LDS = NSTG * SLOT + 2 * RWG * 4 + 8 * 4;
  static_assert(LDS <= 160 * 1024, "LDS budget");
};
// Per-wave rings (WV): every wave streams the dst rows through its own 4-deep ring of 8 KiB chunks and
// runs without workgroup barriers: a wave's list compactions stall only that wave, and each wave
// stops on its own rows' vote.  Four times the L2 -> LDS traffic of the shared ring.
template <int KP, int G, bool WV>
struct TkGeo {
  static constexpr int RB = 2 * KP;
  static constexpr int CHP = TkScan<KP, G>::CH;            // rows per prepared chunk (head[] entries)
  static constexpr int CB = WV ? 8192 : 16384;             // dst bytes per ring chunk
  static constexpr int CH = CB / RB;
  static constexpr int NJ = CH / 16;
  static constexpr int NQ = KP / 32;
  static constexpr int NSTG = WV ? 4 : TkScan<KP, G>::NSTG;
  static constexpr int SLOT = CB + (WV ? 256 : 4 * 256);
  static constexpr int RING = (WV ? 4 : 1) * NSTG * SLOT;  // ring bytes of the workgroup
  static constexpr int RWG = 64 * G;
  static constexpr int DPW = WV ? CB / 1024 : CB / 1024 / 4;
  static constexpr int NVM = DPW + 1;
  static constexpr int LDS = RING + 2 * RWG * 4 + 8 * 4;
  static_assert(LDS <= 160 * 1024 && CH % 16 == 0 && CHP % CH == 0, "LDS budget, chunk geometry");
};
// 16-B unit u of dst row `row` is stored at unit u ^ tk_sw(row): every ds_read_b128 lane group of a
// fragment read (16 rows x one unit, cdna ds_read_b128 groups) hits 16 distinct 16-B bank slots.
template <int KP>
__host__ __device__ constexpr int topk_chunk_rows_dev() { return TkScan<KP, 2>::CH; }
template <int KP>
__device__ __forceinline__ int tk_sw(int row) {
  if constexpr (KP == 64) return (row >> 1) & 7;
  else return row & 15;
}

// LDS store the compiler's wait insertion does not see (it would drain the LDS-DMA queue before a
// plain LDS write); ordered by the explicit lgkmcnt wait ahead of the next barrier
__device__ __forceinline__ void lds_store_asm(int* p, int v) {
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)p;
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ float agent_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int agent_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int KP, int G, bool WV>
__global__ __launch_bounds__(256, 1) void topk_scan_kernel(TopkArgs a) {
  using C = TkGeo<KP, G, WV>;
  constexpr int NQ = C::NQ, NJ = C::NJ, RB = C::RB, CAP = TOPK_CAP;
  // a list is compacted to its best 64 once it holds more than TRIG (<= TRIG + 16 <= 64·NSC entries):
  // frequent enough that the threshold follows the running 64th best
  constexpr int TRIG = TOPK_TRIG, NSC = TOPK_CAP / 64;
  static_assert(TRIG + 16 <= 64 * NSC && TRIG + 16 <= CAP && TRIG + 16 <= 255, "compaction width, byte counters");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // one LDS object (glds pipelining)
  float* s_thr = reinterpret_cast<float*>(lds + C::RING);            // [RWG] thresholds (unscaled)
  float* s_nrm = s_thr + C::RWG;                                      // [RWG] ‖s‖ rounded up
  int* s_flag = reinterpret_cast<int*>(s_nrm + C::RWG);           // [2][4] per-wave "done" votes
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rb0 = (int64_t)blockIdx.x * C::RWG;  // first src-list position of the workgroup
  const int wr0 = wave * 16 * G;                     // the wave's first row within the workgroup
  const char* Th = reinterpret_cast<const char*>(a.Th);
  const int64_t nch = a.n_chunks * (C::CHP / C::CH);
  char* const ring = lds + (WV ? wave * C::NSTG * C::SLOT : 0);

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
    double ss = 0.0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4 v0 = ld4(sp + 32 * q), v1 = ld4(sp + 32 * q + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (e < 4 ? v0[e] : v1[e - 4]) * keep;
        ss += (double)v * (double)v;
        sf[gi][q][e] = (_Float16)(v * a.ssc);
      }
    }
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    if (g == 0) {
      const int wrow = wr0 + 16 * gi + i16;
      s_nrm[wrow] = __double2float_ru(sqrt(ss));
      s_thr[wrow] = srow < 0 ? INFINITY : (a.thr0 ? a.thr0[si] : -INFINITY);
    }
  }
  if (tid < 8) s_flag[tid] = 0;
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
                  : t0 == -INFINITY ? 1.01f * s_nrm[wrow] * a.ssc * tmax_sc + 1.f : -(t0 * a.scaled);
    }

  // DMA of chunk c into ring slot `slot`: the wave's DPW KiB of rows (source addresses carry the
  // unit swizzle, the LDS image is lane-linear), then the chunk's head norm (every lane the same word)
  auto dma = [&](int64_t c, int slot) __attribute__((always_inline)) {
    char* base = ring + slot * C::SLOT;
    const int64_t j0 = c * C::CH;
#pragma unroll
    for (int m = 0; m < C::DPW; ++m) {
      const int ins = WV ? m : wave * C::DPW + m;
      const int off = ins * 1024 + 16 * lane;
      const int row = off / RB, up = (off % RB) / 16;
      const char* src = Th + (j0 + row) * RB + 16 * (up ^ tk_sw<KP>(row));
      __builtin_amdgcn_global_load_lds((tk_glb_vp)src, (tk_lds_vp)(base + ins * 1024), 16, 0, 0);
    }
    __builtin_amdgcn_global_load_lds((tk_glb_vp)(a.head + j0 / C::CHP), (tk_lds_vp)(base + C::CB + (WV ? 0 : wave * 256)),
                                     4, 0, 0);
  };
  for (int c = 0; c < C::NSTG - 1; ++c)
    if (c < nch) dma(c, c);

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
            a.lscore[li] = (acc[gi][r] - nthr[gi][r]) * a.unscale;  // score = acc + threshold
            a.lidx[li] = (int)dj;
          }
          const int ncnt = cnt + __popc(mg);
          cntp[gi] += (uint32_t)__popc(mg) << (8 * r);
          over |= ncnt > TRIG;
        }
      }
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's list stores are in L2
    while (f0 | f1) {
      int wl;
      if (f0) { wl = __builtin_ctzll(f0); f0 &= f0 - 1; }
      else { wl = 64 + __builtin_ctzll(f1); f1 &= f1 - 1; }
      uint32_t cw = 0;  // the row's length: byte (wl & 3) of cntp[wl >> 4] in lane 16·((wl >> 2) & 3)
#pragma unroll
      for (int gi = 0; gi < G; ++gi)
        if ((wl >> 4) == gi) cw = (uint32_t)rdlane_i((int)cntp[gi], 16 * ((wl >> 2) & 3));
      const int cnt = (int)((cw >> (8 * (wl & 3))) & 0xffu);
      const int64_t lb = (rb0 + wr0 + wl) * CAP;
      float s2[NSC];
      int i2[NSC];
#pragma unroll
      for (int h = 0; h < NSC; ++h) {
        const int e = lane + 64 * h;
        s2[h] = e < cnt ? agent_load(a.lscore + lb + e) : -INFINITY;
        i2[h] = e < cnt ? agent_load(a.lidx + lb + e) : -1;
      }
      wave_bitonic<NSC>(s2, i2);
      a.lscore[lb + lane] = s2[0];
      a.lidx[lb + lane] = i2[0];
      const float tkt = rdlane(s2[0], a.kt - 1);  // the running kt-th best becomes the threshold
      if (lane == 0) s_thr[wr0 + wl] = tkt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
  };

  int64_t c = 0;
  for (; c < nch; ++c) {
    // this wave's DMAs of chunk c have landed (in-order VM counter; later list stores only make the
    // wait stricter), then one barrier publishes every wave's part and retires slot (c-1) % NSTG
    if (c + C::NSTG - 2 < nch && !a.drain) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::NVM * (C::NSTG - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!WV) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (c > 0) {
        const int* fl = s_flag + ((c - 1) & 1) * 4;
        if (fl[0] & fl[1] & fl[2] & fl[3]) break;  // every row of the workgroup is complete
      }
    }
    if (c + C::NSTG - 1 < nch) dma(c + C::NSTG - 1, (int)((c + C::NSTG - 1) % C::NSTG));
    const char* base = ring + (int)(c % C::NSTG) * C::SLOT;
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
    // vote: every row's threshold already bounds ‖s‖·‖t_j‖ for all j from this chunk on
    {
      const float hn = *reinterpret_cast<const float*>(base + C::CB + (WV ? 0 : wave * 256)) * 1.00000095367431640625f;
      bool ok = true;
      if (lane < 16 * G) ok = s_nrm[wr0 + lane] * hn <= s_thr[wr0 + lane];
      if (16 * G > 64) ok = ok && s_nrm[wr0 + 64 + lane] * hn <= s_thr[wr0 + 64 + lane];
      // no vote before the 256 dst rows behind the starting thresholds are scanned (their 64 best
      // must reach the lists)
      const bool done = !__any(!ok) && (c + 1) * C::CH >= 256;
      if constexpr (WV) {
        if (done) {
          ++c;
          break;
        }
      } else {
        if (lane == 0) lds_store_asm(s_flag + (c & 1) * 4 + wave, done ? 1 : 0);
      }
    }
  }
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
  // dst rows scanned, summed over waves
  if (a.scanned && (WV ? lane == 0 : tid == 0)) atomicAdd(a.scanned, (unsigned long long)(c * C::CH * (WV ? 1 : 4)));
}

// One wave per src row: best 64 of the list, exact F2J rescoring, sort, certify, write top-k.
template <int KP>
__global__ __launch_bounds__(256) void topk_select_kernel(TopkArgs a) {
  constexpr int CAP = TOPK_CAP, NS = CAP / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t si = (int64_t)blockIdx.x * 4 + wave;
  if (si >= a.n_src) return;
  const int64_t so = a.out_pos ? (int64_t)a.out_pos[si] : si;  // output slot of scan position si
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  const int cnt = min(a.lcnt[si], CAP);
  float s2[NS];
  int i2[NS];
#pragma unroll
  for (int h = 0; h < NS; ++h) {
    const int e = lane + 64 * h;
    s2[h] = e < cnt ? a.lscore[si * CAP + e] : -INFINITY;
    i2[h] = e < cnt ? a.lidx[si * CAP + e] : -1;
  }
  wave_bitonic<NS>(s2, i2);
  const float t = rdlane(s2[0], a.kt - 1);  // the kt-th approximate score (-inf when fewer)
  const int row = i2[0] >= 0 ? a.perm[i2[0]] : -1;
  float ex = -INFINITY;
  if (row >= 0) ex = f2j_dot_v4(s, a.T + (int64_t)row * KP, a.kreal);
  double nn = 0.0;
  for (int c = lane; c < a.kreal; c += 64) nn += (double)s[c] * (double)s[c];
  for (int o = 32; o > 0; o >>= 1) nn += __shfl_xor(nn, o);
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
    const double ns = sqrt(nn), tm = (double)a.tmax_norm;
    const double absu = 2.98023223876953125e-08 * 1.001 * sqrt((double)KP) *
                        (ns / (double)a.tsc + tm / (double)a.ssc) + (double)KP * 8.9e-16 * (double)a.unscale;
    const double e = rel * ns * tm + absu;
    // fewer than 64 listed (a scan that stopped before 64 rows reached a starting threshold): the
    // bound below needs t >= the last threshold, which only a full list guarantees
    if (cnt < a.kt || !((double)kth > (double)t + e)) {
      if (lane == 0) a.need_exact[so] = 1;
    }
  }
  if (lane < k) {
    const int idx = ix1[0];
    a.out_ids[so * k + lane] = idx >= 0 ? a.dst_ids[idx] : -1;
    a.out_scores[so * k + lane] = idx >= 0 ? sc1[0] : __int_as_float(0x7fc00000);
  }
}

// Scan order and starting thresholds of the src rows.  A workgroup's scan ends when its slowest row
// can stop, so rows that stop at similar depths go together.  One wave per 16 src rows scores them
// against the 256 largest-norm dst rows with the scan's own fp16 operands on MFMA, and v* = the
// 64th best of those 256 (bisection on order-preserving keys): a lower bound of the row's final
// 64th best.  thr0 = v* minus the
// rounding difference between this accumulation and the scan's (8γ_{KP+2}·‖s‖·max‖t‖) is a valid
// starting threshold: the 64 dst rows above v* reach the list, so the final 64th approximate score
// is >= thr0.  key = thr0 / ‖s‖: the row can stop once ‖t_j‖ <= threshold / ‖s‖, so a larger key
// stops earlier (order-preserving uint of the float, sorted descending with the positions as values).
template <int KP>
__global__ __launch_bounds__(256) void topk_order_key_kernel(TopkArgs a, uint32_t* __restrict__ key,
                                                             uint32_t* __restrict__ val, float* __restrict__ thr0) {
  constexpr int NQ = KP / 32, RB = 2 * KP;
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const int64_t sb = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 6) * 16;  // the wave's first position
  const int64_t si = sb + i16;
  const int srow = si < a.n_src ? a.src_rows[si] : -1;
  const float* sp = a.S + (int64_t)(srow >= 0 ? srow : 0) * KP + 8 * g;
  const float keep = srow >= 0 ? 1.f : 0.f;
  f16x8 sf[NQ];
  double ss = 0.0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const f32x4 v0 = ld4(sp + 32 * q), v1 = ld4(sp + 32 * q + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (e < 4 ? v0[e] : v1[e - 4]) * keep;
      ss += (double)v * (double)v;
      sf[q][e] = (_Float16)(v * a.ssc);
    }
  }
  ss += __shfl_xor(ss, 16);
  ss += __shfl_xor(ss, 32);  // every lane: ‖s‖² of row i16
  const char* Th = reinterpret_cast<const char*>(a.Th);
  const int64_t n_pad = a.n_chunks * (int64_t)topk_chunk_rows_dev<KP>();
  // order-preserving uint keys of the 256 scores: lane (i16, g) holds column 16J + i16 of rows 4g + r
  uint32_t u[16][4];
#pragma unroll
  for (int J = 0; J < 16; ++J) {
    const int64_t p = 16 * J + i16;
    f32x4 acc = zero4();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      f16x8 d = {};
      if (p < n_pad) d = *reinterpret_cast<const f16x8*>(Th + p * RB + 16 * (4 * q + g));
      acc = mfma_h(sf[q], d, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t bb = __float_as_uint(p < a.n_dst ? acc[r] : -INFINITY);
      u[J][r] = (bb & 0x80000000u) ? ~bb : (bb | 0x80000000u);
    }
  }
  // exact 64th largest per row: bisection on the key (count of keys >= mid over the row's 16 lanes)
  float vs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t lo = 0u, hi = 0xffffffffu;  // count(>= lo) >= kt always holds (256 keys >= 0)
    for (int it = 0; it < 32; ++it) {
      const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) >> 1);
      int cnt = 0;
#pragma unroll
      for (int J = 0; J < 16; ++J) cnt += u[J][r] >= mid ? 1 : 0;
      for (int o = 1; o < 16; o <<= 1) cnt += __shfl_xor(cnt, o);
      if (cnt >= a.kt) lo = mid;
      else hi = mid - 1u;
    }
    vs[r] = __uint_as_float((lo & 0x80000000u) ? (lo & 0x7fffffffu) : ~lo);
  }
  const double nrm = sqrt(__shfl(ss, 4 * g + (i16 & 3)));  // ‖s‖ of row 4g + r (all lanes take part)
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
      key[pr] = (bb & 0x80000000u) ? ~bb : (bb | 0x80000000u);
      val[pr] = (uint32_t)pr;
    }
  }
}

size_t topk_order_temp_bytes(int64_t n_src) { return topk_sort_temp_bytes(n_src); }

// src_sorted[i] = src_rows[order[i]], thr_sorted[i] = thr0[order[i]]; order[i] = the position whose
// results slot i fills
hipError_t topk_order(int KP, const TopkArgs& a, void* temp, size_t temp_bytes, uint32_t* keys, uint32_t* order,
                      int32_t* src_sorted, float* thr_tmp, float* thr_sorted, hipStream_t s) {
  const int64_t n = a.n_src;
  if (n <= 0) return hipSuccess;
  uint32_t* k0 = keys;
  uint32_t* k1 = keys + n;
  uint32_t* v0 = order + n;
  const int blocks = (int)((n + 63) / 64);
  if (KP == 64) topk_order_key_kernel<64><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp);
  else if (KP == 128) topk_order_key_kernel<128><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp);
  else topk_order_key_kernel<256><<<blocks, 256, 0, s>>>(a, k0, v0, thr_tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  e = rocprim::radix_sort_pairs_desc(temp, tb, k0, k1, v0, order, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  topk_gather_rows_kernel<<<tk_grid(n, 256), 256, 0, s>>>(a.src_rows, thr_tmp, order, n, src_sorted, thr_sorted);
  return hipGetLastError();
}

// Exact path: one workgroup (4 waves) per src row, full F2J scan.  Each wave keeps its best 64·P
// (score desc, id asc) in registers, slots [0, P) sorted, and buffers up to 64·P newcomers in slots
// [P, 2P); a batch of 64 scores is only buffered when one of them reaches the current 64·P-th best,
// and a full buffer is merged by one bitonic sort of the 128·P slots.  The four waves' lists are
// merged at the end.  P = 1 serves the rows the MFMA pre-selection could not certify; P up to 8
// serves k up to 512 (recommendForAll* with k > 64, no pre-selection).
template <int KP, int P>
__global__ __launch_bounds__(256) void topk_exact_kernel(TopkArgs a, const int32_t* rows, int64_t row0) {
  __shared__ float msc[4][64 * P];
  __shared__ int mix[4][64 * P];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t si = rows ? rows[row0 + blockIdx.x] : row0 + (int64_t)blockIdx.x;
  const int srow = a.src_rows[si];
  const float* s = a.S + (int64_t)srow * KP;
  float bs[2 * P];
  int bi[2 * P];
#pragma unroll
  for (int h = 0; h < 2 * P; ++h) { bs[h] = -INFINITY; bi[h] = -1; }
  int nin = 0;                // newcomer batches buffered (wave-uniform)
  float thr = -INFINITY;      // the kept list's last score once full
  // with the prepared norm order (a.perm / a.head) dst rows are visited by descending norm and a wave
  // stops once ‖s‖·‖t_j‖ bounds every later F2J score below its own 64·P-th best (which is <= the
  // merged k-th): F2J(s, t) <= ‖s‖‖t‖(1 + (KP+2)·2^-24), covered by the 2^-14 factor
  float snrm = 0.f;
  if (a.perm) {
    double nn = 0.0;
    for (int c = lane; c < a.kreal; c += 64) nn += (double)s[c] * (double)s[c];
    for (int o = 32; o > 0; o >>= 1) nn += __shfl_xor(nn, o);
    snrm = __double2float_ru(sqrt(nn)) * 1.00006103515625f;
  }
  const int ch = topk_chunk_rows_dev<KP>();
  for (int64_t j0 = (int64_t)wave * 64; j0 < a.n_dst; j0 += 256) {
    if (a.perm && thr > -INFINITY && snrm * a.head[j0 / ch] < thr) break;
    const int64_t pj = j0 + lane;
    const int64_t dj = (a.perm && pj < a.n_dst) ? (int64_t)a.perm[pj] : pj;
    const float sc = pj < a.n_dst ? f2j_dot_v4(s, a.T + dj * KP, a.kreal) : -INFINITY;
    if (!__any(sc >= thr)) continue;
    static_for<0, P>([&](auto hh) {
      constexpr int h = decltype(hh)::value;
      if (nin == h) { bs[P + h] = sc; bi[P + h] = pj < a.n_dst ? (int)dj : -1; }
    });
    if (++nin == P) {
      wave_bitonic<2 * P>(bs, bi);
#pragma unroll
      for (int h = P; h < 2 * P; ++h) { bs[h] = -INFINITY; bi[h] = -1; }
      nin = 0;
      thr = rdlane(bs[P - 1], 63);
    }
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
}

// ---------------------------------------------------------------------------------------------
// preparation of the dst side
// ---------------------------------------------------------------------------------------------
// key[j] = bits of ‖T_j‖ rounded up to fp32 (non-negative floats order as unsigned), val[j] = j
__global__ void topk_norm_keys_kernel(const float* __restrict__ T, int64_t n, int KP, int kreal,
                                      uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    double s2 = 0.0;
    for (int c = lane; c < kreal; c += 64) s2 += (double)T[r * KP + c] * (double)T[r * KP + c];
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    if (lane == 0) {
      key[r] = __float_as_uint(__double2float_ru(sqrt(s2)));
      val[r] = (uint32_t)r;
    }
  }
}
// Th[p] = fp16(T[perm[p]]·tsc) (zero rows past n), head[c] = ‖T_{perm[c·CH]}‖ (0 past n)
__global__ void topk_pack_kernel(const float* __restrict__ T, int64_t n, int64_t n_pad, int KP, float tsc,
                                 const uint32_t* __restrict__ perm, const uint32_t* __restrict__ skey, int CH,
                                 _Float16* __restrict__ Th, float* __restrict__ head) {
  const int64_t tot = n_pad * KP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / KP;
    const int c = (int)(e % KP);
    Th[e] = p < n ? (_Float16)(T[(int64_t)perm[p] * KP + c] * tsc) : (_Float16)0.f;
    if (c == 0 && p % CH == 0) head[p / CH] = p < n ? __uint_as_float(skey[p]) : 0.f;
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
  size_t tb = 0;
  (void)rocprim::radix_sort_pairs_desc(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (size_t)n, 0, 32, (hipStream_t)0);
  return tb;
}

hipError_t topk_prepare(int KP, int kreal, const float* T, int64_t n, float tsc, void* temp, size_t temp_bytes,
                        uint32_t* keys, uint32_t* perm, void* Th, float* head, hipStream_t s) {
  const int CH = topk_chunk_rows(KP);
  const int64_t n_pad = (n + CH - 1) / CH * CH;
  uint32_t* k0 = keys;
  uint32_t* k1 = keys + n;
  uint32_t* v0 = perm + n;  // perm has 2n slots: [n, 2n) holds the unsorted values
  topk_norm_keys_kernel<<<tk_grid(n, 4), 256, 0, s>>>(T, n, KP, kreal, k0, v0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  e = rocprim::radix_sort_pairs_desc(temp, tb, k0, k1, v0, perm, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  topk_pack_kernel<<<tk_grid(n_pad * KP, 256), 256, 0, s>>>(T, n, n_pad, KP, tsc, perm, k1, CH,
                                                            reinterpret_cast<_Float16*>(Th), head);
  return hipGetLastError();
}

template <int KP, int G>
hipError_t launch_scan(const TopkArgs& a, hipStream_t s) {
  // default: one ring per workgroup; "wave": per-wave rings (measured 2.69 s vs 2.60 s at c4: the
  // waves of a workgroup stop together, so the barriers cost little and the 4x ring traffic shows)
  static const char* ev = std::getenv("ALBEDO_TOPK_SCAN");
  const bool wv = ev && std::string(ev) == "wave";
  if (wv) {
    using C = TkGeo<KP, G, true>;
    static const hipError_t attr = allow_lds(topk_scan_kernel<KP, G, true>, C::LDS);
    if (attr != hipSuccess) return attr;
    topk_scan_kernel<KP, G, true><<<(int)((a.n_src + C::RWG - 1) / C::RWG), 256, C::LDS, s>>>(a);
  } else {
    using C = TkGeo<KP, G, false>;
    static const hipError_t attr = allow_lds(topk_scan_kernel<KP, G, false>, C::LDS);
    if (attr != hipSuccess) return attr;
    topk_scan_kernel<KP, G, false><<<(int)((a.n_src + C::RWG - 1) / C::RWG), 256, C::LDS, s>>>(a);
  }
  return hipGetLastError();
}

// src rows per scan workgroup: the largest register blocking (G = 8 at KP <= 128, 4 at KP = 256)
// that still gives every CU two workgroups, down to G = 2
int topk_rows_per_workgroup(int KP, int64_t n_src, int n_cu) {
  int gmax = KP <= 128 ? 8 : 4;
  if (const char* e = std::getenv("ALBEDO_TOPK_GMAX")) {  // experiments: cap the register blocking
    const int v = std::atoi(e);
    if (v == 2 || v == 4 || v == 8) gmax = std::min(gmax, v);
  }
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
  if (e != hipSuccess) return e;
  topk_select_kernel<KP><<<(int)((a.n_src + 3) / 4), 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_topk(int KP, const TopkArgs& a, int n_cu, hipStream_t s) {
  if (a.n_src <= 0) return hipSuccess;
  if (KP == 64) return launch_topk_kp<64>(a, n_cu, s);
  if (KP == 128) return launch_topk_kp<128>(a, n_cu, s);
  if (KP == 256) return launch_topk_kp<256>(a, n_cu, s);
  return hipErrorInvalidValue;
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
    topk_exact_kernel<KP, P><<<(int)n, 256, 0, s>>>(a, rows, r0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
template <int KP>
hipError_t topk_exact_kp(const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  if (a.k <= 64) return topk_exact_p<KP, 1>(a, rows, n_rows, s);
  if (a.k <= 128) return topk_exact_p<KP, 2>(a, rows, n_rows, s);
  if (a.k <= 256) return topk_exact_p<KP, 4>(a, rows, n_rows, s);
  if (a.k <= TOPK_MAX) return topk_exact_p<KP, 8>(a, rows, n_rows, s);
  return hipErrorInvalidValue;
}
hipError_t launch_topk_exact(int KP, const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  if (KP == 64) return topk_exact_kp<64>(a, rows, n_rows, s);
  if (KP == 128) return topk_exact_kp<128>(a, rows, n_rows, s);
  if (KP == 256) return topk_exact_kp<256>(a, rows, n_rows, s);
  return hipErrorInvalidValue;
}

}  // namespace albedo
