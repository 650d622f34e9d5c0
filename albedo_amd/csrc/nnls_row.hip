// NNLS rows at KP = 256 (nonnegative = true; Spark NNLSSolver -> mllib/optimization/NNLS.scala,
// reached from ALS.computeFactors): the per-row kernel of the rows the lockstep kernel (nnls_batch.hip)
// does not take.  Same problem and iteration as solve_nnls_kernel / nnls_reg_iterate (als_kernels.hip):
//   A = G + λn I + Σ c y yᵀ  (original basis),  b = Σ w y,
// Spark's projected gradient with CG acceleration, its stopping rules, wall clamp and restarts, one
// product A·g per iteration (A·dir = A·g + alpha·A·lastDir), the residual following the steps with an
// exact refresh every 64 iterations.
//
// What changes is where A lives.  The 1024-thread kernel keeps all of A (256 KiB) in the registers of
// one workgroup and needs the whole LDS for its build, so a CU iterates ONE row: every iteration is a
// chain of reductions, barriers and fp64 scalar steps (~4K cycles, profiles/r05_nnlstime_*) with the
// CU idle in between.  Here a row takes 8 waves and keeps only the upper 16x16 tiles (136 of 256) in
// registers, in the MFMA C layout its build leaves them in, so TWO rows iterate on each CU and their
// latency chains overlap:
//   waves 0-5   one off-diagonal 64x64 group pair (GI < GJ) each: 4 x 4 tiles, 64 VGPRs
//   waves 6-7   two diagonal groups each: 2 x 10 upper tiles, 80 VGPRs
// (group G = row blocks 4G .. 4G+3).  A·v from upper tiles: a tile (I, J) gives the row partial
// A_IJ v_J (a sum over its columns: 16-lane DPP transpose-reduce) and, off the diagonal, the column
// partial A_IJᵀ v_I (a sum over its rows: in-lane, then across the four lane rows by permlane swaps).
// Every coordinate then has exactly five partials in LDS (three from the off-diagonal pairs of its
// group, the row and column parts of its diagonal group), summed in a fixed order by its owner.
// Owners: waves 0-3, lane l of wave w owns coordinate 64w + l (x, residual, directions in fp64).
// Build: the heavy rows' stage scheme (als_kernels.hip heavy_build) at 32 ratings per stage, √c-scaled
// rows split into fp16 hi + lo, three MFMAs per tile, double-buffered images (64 KiB); split-K rows
// arrive as reduced records (SplitRec) and are read straight into the registers.
// Measured (r06, profiles/r06_nnlsrow_*): c5 sweep 3437 -> 2854 ms (per-row NNLS 2245 -> 1659 ms);
// probe rows of degree 60 / 200 at 1.55 / 1.76 us per row-iteration per CU against 1.97 / 2.11 for the
// 1024-thread kernel.  Per iteration (~4.6K cycles per workgroup) the owners spend 0.8K before B1,
// 1.3K on their product, 0.9K after it and 1.0K on the step; the diagonal-group waves' product
// (2.5K) is what B2 waits for.  Degree-2000 rows build slower than in the 1024-thread kernel (its
// pipelined 64-rating stages); those are a small share of c5's per-row stars.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <algorithm>
#include "kernels.h"
#include "device_common.h"
#include "split_rec.h"
#include "nnls_common.h"

namespace albedo {

#ifdef ALBEDO_NNLS_TIMING  // probes only (tools/probe/nnlstime.hip): loop phase cycles of waves 0 and 6
__device__ unsigned long long albedo_nrow_ph[64][2][8];
#define NR_T0() unsigned long long nr_t = clock64(), nr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define NR_PH(k) { const unsigned long long nr_n = clock64(); nr_acc[k] += nr_n - nr_t; nr_t = nr_n; }
#define NR_OUT() \
  if ((threadIdx.x == 0 || threadIdx.x == 384) && blockIdx.x < 64) \
    for (int q = 0; q < 8; ++q) albedo_nrow_ph[blockIdx.x][threadIdx.x ? 1 : 0][q] = nr_acc[q]
#else
#define NR_T0()
#define NR_PH(k)
#define NR_OUT()
#endif

namespace {

struct NRow {
  static constexpr int KP = 256, NTH = 512, NW = 8;
  static constexpr int SPS = 32, CS = 2 * SPS, IMG = KP * CS;  // bytes per fp16 image (hi or lo)
  static constexpr int NST = 4;                                // ratings per thread per stage
  // LDS (floats): 2 buffers x (hi, lo) images, then the iteration's vectors
  static constexpr int OFF_B = 4 * IMG / 4;                    // b' [KP]
  static constexpr int OFF_G = OFF_B + KP;                     // fp32 product input [KP]
  static constexpr int OFF_P = OFF_G + KP;                     // product partials [5][KP]
  static constexpr int OFF_R1 = OFF_P + 5 * KP;                // fp64 [8][16] sums / minima (B1)
  static constexpr int OFF_R2 = OFF_R1 + 256;                  // fp64 [8][16] (B2)
  static constexpr int OFF_FLAG = OFF_R2 + 256;                // npos, error bits, stop
  static constexpr int FLOATS = OFF_FLAG + 4;
};
static_assert(NRow::OFF_R1 % 2 == 0, "fp64 alignment");
static_assert(NRow::NW * NRow::KP <= NRow::OFF_B, "b' partials fit the dead images");
static_assert(2 * NRow::FLOATS * 4 <= 160 * 1024, "two workgroups per CU");

// byte offset of (column, byte within its 32 ratings) in one image: 16-B units xor-swizzled per column
// (the layout of heavy_build's images at 32 ratings per stage: conflict-free fragment reads)
__device__ __forceinline__ int nr_img_off(int col, int byteoff) {
  const int sw = (col ^ (3 * (col >> 3))) & 3;
  return col * NRow::CS + ((((byteoff >> 4) ^ sw) & 3) << 4) + (byteoff & 15);
}
__device__ __forceinline__ uint32_t nr_pack_h2(float a, float b) {
  f16x2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, h);
}

// upper tile u of a 4 x 4 block group, row-major: (0,0) (0,1) (0,2) (0,3) (1,1) (1,2) (1,3) (2,2) (2,3) (3,3)
struct TAB { int a, b; };
__host__ __device__ constexpr TAB ut4(int u) { return u < 4 ? TAB{0, u} : u < 7 ? TAB{1, u - 3} : u < 9 ? TAB{2, u - 5} : TAB{3, 3}; }

// 16 values per lane -> lane i of each 16-lane row holds the row-sum of value i: four halving steps
// with the partners i^15, i^7, i^3, i^1 (row_mirror, row_half_mirror, quad perms); a lane keeps the
// half whose index bit matches its own lane bit and receives the partner's copy of it
__device__ __forceinline__ float nr_rowsum16(float (&h)[16], int i16) {
  const bool b3 = i16 & 8, b2 = i16 & 4, b1 = i16 & 2, b0 = i16 & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b3 ? h[k + 8] : h[k], send = b3 ? h[k] : h[k + 8];
    h[k] = keep + dppf<0x140>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b2 ? h[k + 4] : h[k], send = b2 ? h[k] : h[k + 4];
    h[k] = keep + dppf<0x141>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b1 ? h[k + 2] : h[k], send = b1 ? h[k] : h[k + 2];
    h[k] = keep + dppf<0x1B>(send);
  }
  const float keep = b0 ? h[1] : h[0], send = b0 ? h[0] : h[1];
  return keep + dppf<0xB1>(send);
}
// (u, w): lanes 0-31 get u's sum over the two halves, lanes 32-63 w's (v_permlane32_swap);
// rows 0, 2 get u's sum over the row pairs (0,1) / (2,3), rows 1, 3 w's (v_permlane16_swap)
__device__ __forceinline__ float nr_halve32(float u, float w) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(u), __float_as_int(w), false, false);
  return __int_as_float((int)r[0]) + __int_as_float((int)r[1]);
}
__device__ __forceinline__ float nr_halve16(float u, float w) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(u), __float_as_int(w), false, false);
  return __int_as_float((int)r[0]) + __int_as_float((int)r[1]);
}
// 4 values per lane -> lane row q holds the sum of value q over the four rows (same lane i16)
__device__ __forceinline__ float nr_colsum4(const float (&p)[4]) {
  return nr_halve16(nr_halve32(p[0], p[2]), nr_halve32(p[1], p[3]));
}

// the lane index through an empty asm: address arithmetic derived from it is redone where it is used
// instead of being hoisted out of the NNLS loop (dozens of loop-invariant LDS addresses spill at the
// 128 VGPRs of four waves per SIMD)
__device__ __forceinline__ int nr_lane() {
  int l = (int)threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}

// a / b through v_rcp_f64 and two Newton corrections (the quotients of the NNLS step, the CG weight and
// the wall ratios: b > 0, or a NaN that the stopping rule catches either way)
__device__ __forceinline__ double nr_div(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}

// Tile sets.  Four 16-block groups G (row blocks 4G .. 4G+3); the upper tiles are the 6 off-diagonal
// group pairs (16 tiles each) and the 4 diagonal groups (10 each).
//   MODE 0, waves 0-5:  pair (0,1) (0,2) (0,3) (1,2) (1,3) (2,3); waves 0-3 are also the owners
//   MODE 1, waves 6-7:  diagonal groups 2(w - 6), 2(w - 6) + 1
// (r06 measured the alternative with the owners on 16 tiles and 18-tile diagonal + half-pair waves
// beside them: its owner loop spilled and every row-iteration was ~30 % slower.)  Segment s of a wave:
// 4 row blocks from BI, 4 column blocks from BJ, upper tiles only when UP (BI == BJ).  Every coordinate
// of group X gets its partials in the LDS slots 0-2 (the three pairs (X, Y) or (Y, X): slot Y if Y < X,
// else Y - 1) and 3 / 4 (the row / column parts of its diagonal group).
template <int MODE> struct NSeg;
template <> struct NSeg<0> {
  static constexpr int N = 1, NT = 16;
  static constexpr bool up(int) { return false; }
  static constexpr int to(int) { return 0; }
};
template <> struct NSeg<1> {
  static constexpr int N = 2, NT = 20;
  static constexpr bool up(int) { return true; }
  static constexpr int to(int s) { return 10 * s; }
};
// tile index of (row block i, column block jb) within a segment
__host__ __device__ constexpr int seg_tile(bool up, int i, int jb) {
  return up ? (i == 0 ? jb : i == 1 ? 3 + jb : i == 2 ? 5 + jb : 9) : 4 * i + jb;
}
// segment / row block / column block of tile t (inverse of to + seg_tile)
template <int MODE>
__host__ __device__ constexpr int tile_seg(int t) { return MODE == 0 ? 0 : t / 10; }
template <int MODE>
__host__ __device__ constexpr int tile_i(int t) { return MODE == 0 ? t >> 2 : ut4(t % 10).a; }
template <int MODE>
__host__ __device__ constexpr int tile_j(int t) { return MODE == 0 ? t & 3 : ut4(t % 10).b; }

// One row; both modes run the same sequence of workgroup barriers.
template <int MODE, bool PRE>
__device__ __forceinline__ void nnls_row_body(const SolveArgs& a, const float* __restrict__ Gt, float* smem, int j,
                                              int64_t p0, int d, const float* __restrict__ rec) {
  using R = NRow;
  using S = NSeg<MODE>;
  constexpr int KP = R::KP, NT = S::NT;
  const int tid = threadIdx.x, lane = tid & 63, g4 = lane >> 4, i16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int* s_flag = reinterpret_cast<int*>(smem + R::OFF_FLAG);
  // segment bases and LDS slots (wave-uniform)
  const int GI = wave < 3 ? 0 : wave < 5 ? 1 : 2, GJ = wave < 3 ? wave + 1 : wave < 5 ? wave - 1 : 3;  // MODE 0
  const int G0 = 2 * (wave - 6);                                                                    // MODE 1
  auto segBI = [&](int s) { return MODE == 0 ? 4 * GI : 4 * (G0 + s); };
  auto segBJ = [&](int s) { return MODE == 0 ? 4 * GJ : 4 * (G0 + s); };
  auto slot_row = [&](int) { return MODE == 0 ? GJ - 1 : 3; };
  auto slot_col = [&](int) { return MODE == 0 ? GI : 4; };
  auto rb = [&](int t) { return segBI(tile_seg<MODE>(t)) + tile_i<MODE>(t); };
  auto cb = [&](int t) { return segBJ(tile_seg<MODE>(t)) + tile_j<MODE>(t); };

  NR_T0();
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  if constexpr (!PRE) {
    // ---- build: stage st holds ratings 32 st .. 32 st + 31; thread (wave, lane) stages ratings
    // 32 st + 4 wave + m (m < 4), columns 4 lane .. 4 lane + 3
    const int xr = lane & 3;
    f32x4 bp = zero4();
    int npos = 0;
    int ci[R::NST];
    float rv[R::NST];
    auto iload = [&](int st) {
#pragma unroll
      for (int m = 0; m < R::NST; ++m) {
        const int e = R::SPS * st + R::NST * wave + m;
        const int64_t pe = p0 + (e < d ? e : d - 1);
        ci[m] = a.col[pe];
        rv[m] = a.val[pe];
      }
    };
    auto put = [&](int buf, int st) {
      const f32x4 csc = ld4(a.colscale + 4 * lane);  // re-read per stage (L1): 4 VGPRs fewer across the MFMAs
      f32x4 zr[R::NST];
#pragma unroll
      for (int m = 0; m < R::NST; ++m) zr[m] = ld4(a.Z + (int64_t)ci[m] * KP + 4 * lane);
      float sq[R::NST], wv[R::NST];
#pragma unroll
      for (int m = 0; m < R::NST; ++m) {
        float c = 0.f, w = 0.f;
        rating_weights(rv[m], a.implicit, a.alpha, c, w);
        const bool in = R::SPS * st + R::NST * wave + m < d;
        sq[m] = in ? sqrtf(c) : 0.f;
        wv[m] = in ? w : 0.f;
        npos += (lane == 0 && in && rv[m] > 0.f) ? 1 : 0;
        bp += zr[m] * wv[m];
      }
      u32x2 hp[4], lp[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2) {
          float v0 = zr[2 * m2][q] * (sq[2 * m2] * csc[q]);
          float v1 = zr[2 * m2 + 1][q] * (sq[2 * m2 + 1] * csc[q]);
          asm("" : "+v"(v0), "+v"(v1));  // one fp32 rounding; hi and lo from that value (heavy_build)
          const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
          hp[q][m2] = nr_pack_h2(h0, h1);
          lp[q][m2] = nr_pack_h2(v0 - (float)h0, v1 - (float)h1);
        }
      // write slot i = column 4 lane + (i ^ xr): spreads one instruction's stores over the banks; the
      // data hp[i ^ xr] picked by two selects per slot and stored at once (no permuted copies live)
      const bool s0 = xr & 1, s1 = xr & 2;
      char* himg = reinterpret_cast<char*>(smem) + (2 * buf) * R::IMG;
      char* limg = himg + R::IMG;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x2 ha = s0 ? hp[i ^ 1] : hp[i], hb = s0 ? hp[i ^ 3] : hp[i ^ 2];
        const u32x2 la = s0 ? lp[i ^ 1] : lp[i], lb = s0 ? lp[i ^ 3] : lp[i ^ 2];
        const int off = nr_img_off(4 * lane + (i ^ xr), 8 * wave);
        *reinterpret_cast<u32x2*>(himg + off) = s1 ? hb : ha;
        *reinterpret_cast<u32x2*>(limg + off) = s1 ? lb : la;
      }
    };
    const int nst = (d + R::SPS - 1) / R::SPS;
    if (nst > 0) {
      iload(0);
      put(0, 0);
      if (nst > 1) iload(1);
    }
    for (int st = 0; st < nst; ++st) {
      __syncthreads();  // stage st's images are complete; every wave is done with stage st - 1's
      const char* himg = reinterpret_cast<const char*>(smem) + (2 * (st & 1)) * R::IMG;
      const char* limg = himg + R::IMG;
      // row fragments one block at a time, column fragments re-read per row block (registers:
      // the accumulators + 16 fragment VGPRs at four waves per SIMD)
      static_for<0, S::N>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        constexpr bool UP = S::up(s);
        const int BI = segBI(s), BJ = segBJ(s);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ro = nr_img_off(16 * (BI + i) + i16, 16 * g4);
          const f16x8 rh = *reinterpret_cast<const f16x8*>(himg + ro);
          const f16x8 rl = *reinterpret_cast<const f16x8*>(limg + ro);
#pragma unroll
          for (int jb = UP ? i : 0; jb < 4; ++jb) {
            f16x8 ch = rh, cl = rl;
            if (!UP || jb != i) {
              const int off = nr_img_off(16 * (BJ + jb) + i16, 16 * g4);
              ch = *reinterpret_cast<const f16x8*>(himg + off);
              cl = *reinterpret_cast<const f16x8*>(limg + off);
            }
            const int t = S::to(s) + seg_tile(UP, i, jb);
            acc[t] = mfma_h(rh, ch, acc[t]);
            acc[t] = mfma_h(rh, cl, acc[t]);
            acc[t] = mfma_h(rl, ch, acc[t]);
          }
          __builtin_amdgcn_sched_barrier(0);  // one row block's fragments live at a time (VGPRs)
        }
      });
      if (st + 1 < nst) {  // next stage into the other buffer (its last readers passed this barrier)
        put((st + 1) & 1, st + 1);
        if (st + 2 < nst) iload(st + 2);
      }
    }
    __syncthreads();  // every MFMA has read its fragments: the images are dead
    *reinterpret_cast<f32x4*>(smem + wave * KP + 4 * lane) = bp;
    if (npos) atomicAdd(&s_flag[0], npos);
    __syncthreads();
    if (tid < KP) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < R::NW; ++q) s += smem[q * KP + tid];
      smem[R::OFF_B + tid] = s;
    }
  } else {
    if (tid == 0) s_flag[0] = reinterpret_cast<const int*>(rec)[SplitRec<KP>::OFF_N];
    if (tid < KP) smem[R::OFF_B + tid] = rec[SplitRec<KP>::OFF_B + tid];
  }
  __syncthreads();
  // ---- A = (unscaled build | record) + G + λn I, upper tiles in the MFMA C layout:
  // acc[t][r] = A[16 rb(t) + 4 g4 + r][16 cb(t) + i16]
  const float lamn = a.reg * (float)(a.implicit ? s_flag[0] : d);
  const float* isc = a.colscale + KP;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c2 = 16 * cb(t) + i16;
    const f32x4 ir = PRE ? zero4() : ld4(isc + 16 * rb(t) + 4 * g4);
    const float ic = PRE ? 0.f : isc[c2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c1 = 16 * rb(t) + 4 * g4 + r;
      const int hi = c1 > c2 ? c1 : c2, lo = c1 > c2 ? c2 : c1;
      float v = PRE ? rec[hel(hi, lo)] : acc[t][r] * ir[r] * ic;
      v += Gt[nel(hi, lo)];
      if (c1 == c2) v += c1 < a.kreal ? lamn : 1.0f;
      acc[t][r] = v;
    }
    __builtin_amdgcn_sched_barrier(0);  // one tile's G loads in flight at a time (no spills)
  }

  // ---- the iteration (nnls_reg_iterate's, with four owner waves and eight product waves)
  float* sG = smem + R::OFF_G;
  float* sP = smem + R::OFF_P;
  double* sR1 = reinterpret_cast<double*>(smem + R::OFF_R1);
  double* sR2 = reinterpret_cast<double*>(smem + R::OFF_R2);
  int* sStop = s_flag + 2;
  const bool own = MODE == 0 && wave < 4;  // wave-uniform
  const int c_own = 64 * wave + lane;
  const float bi = own ? smem[R::OFF_B + c_own] : 0.f;
  // A·v (v in sG): partials to sP, returns this lane's share of vᵀAv
  auto product = [&]() -> float {
    const int L = nr_lane(), g4 = L >> 4, i16 = L & 15;
    float tv = 0.f;
    static_for<0, S::N>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr bool UP = S::up(s);
      const int BI = segBI(s), BJ = segBJ(s);
      float gJ[4], h[16], pc[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        gJ[jb] = sG[16 * (BJ + jb) + i16];
        pc[jb] = 0.f;
      }
      // row block i at a time: its v_I fragment (4 values) lives only for its tiles
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 gI = ld4(sG + 16 * (BI + i) + 4 * g4);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[4 * i + r] = 0.f;
#pragma unroll
        for (int jb = UP ? i : 0; jb < 4; ++jb) {
          const f32x4 T = acc[S::to(s) + seg_tile(UP, i, jb)];
#pragma unroll
          for (int r = 0; r < 4; ++r) h[4 * i + r] = fmaf(T[r], gJ[jb], h[4 * i + r]);
          if (!UP || jb != i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) pc[jb] = fmaf(T[r], gI[r], pc[jb]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) tv = fmaf(h[4 * i + r], gI[r], tv);
      }
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) tv = fmaf(pc[jb], gJ[jb], tv);  // the transposed tiles' share of vᵀAv
      const float rsum = nr_rowsum16(h, i16);  // row 16 (BI + (i16 >> 2)) + 4 g4 + (i16 & 3)
      const float csum = nr_colsum4(pc);       // column 16 (BJ + g4) + i16
      sP[slot_row(s) * KP + 16 * (BI + (i16 >> 2)) + 4 * g4 + (i16 & 3)] = rsum;
      sP[slot_col(s) * KP + 16 * (BJ + g4) + i16] = csum;
    });
    return tv;
  };
  auto ysum = [&]() -> float {  // the owner's coordinate of the last product, fixed order
    const int co = 64 * wave + nr_lane();
    float y = sP[co];
#pragma unroll
    for (int s = 1; s < 5; ++s) y += sP[s * KP + co];
    return y;
  };
  double xi = 0.0, axi = 0.0, last_dir = 0.0, a_last = 0.0;
  float hit = 0.f;
  double last_norm = 0.0, last_dad = 0.0;
  double ngrad = 0.0, gres = 0.0, nx = 0.0, gal = 0.0, alpha = 0.0, dc = 0.0;
  bool cg = false;
  int last_wall = 0, iterno = 0;
  bool stopped = false;  // owner waves only (the others learn it at the next barrier)
  const int iter_max = 400 > 20 * a.kreal ? 400 : 20 * a.kreal;
  // the owners' fp64 chains first on their SIMDs (r06 probe: deg 60 rows 6.55 -> 6.37 ms, deg 200 even)
  if (own) __builtin_amdgcn_s_setprio(1);
  NR_PH(7);  // build + assembly
  for (; iterno < iter_max; ++iterno) {
    const int lane = nr_lane(), g4 = lane >> 4, c_own = 64 * wave + lane;
    if (iterno > 0 && (iterno & 63) == 0) {  // exact residual refresh: A·x
      if (own && !stopped) sG[c_own] = (float)xi;
      if (tid == 0) sStop[0] = stopped;
      __syncthreads();
      if (sStop[0]) break;
      (void)product();
      __syncthreads();
      if (own) axi = (double)ysum();
      NR_PH(6);
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
      if ((lane & 15) == 0) {  // row q holds sum q and minimum q
        sR1[g4 * 16 + wave] = s;
        sR1[64 + g4 * 16 + wave] = m;
      }
      sG[c_own] = (float)gi;
    }
    if (tid == 0) sStop[0] = stopped;
    NR_PH(0);
    __syncthreads();  // B1
    NR_PH(1);
    if (sStop[0]) break;
    double t_gag = (double)product();
    NR_PH(2);
    if (own) {
      {  // lane l: sum / minimum l >> 4 of owner wave l & 15
        const bool wv = (lane & 15) < 4;
        const double t0 = row16_all<false>(wv ? sR1[lane] : 0.0);
        const double t1 = row16_all<true>(wv ? sR1[64 + lane] : INFINITY);
        ngrad = rdlane_d(t0, 0);
        gres = rdlane_d(t0, 16);
        nx = rdlane_d(t0, 32);
        gal = rdlane_d(t0, 48);
        if (-rdlane_d(t1, 0) > 0.0) last_wall = iterno - 1;  // the previous step's wall hits
      }
      cg = iterno > last_wall + 1;
      alpha = cg ? uni(nr_div(ngrad, last_norm)) : 0.0;
      dc = cg ? gi + alpha * last_dir : 0.0;
      // sums: g·A·g partials, ‖dir‖², dir·res; minima: wall ratios of g and of dir
      const double t[8] = {t_gag, dc * dc, dc * res, 0.0, gi > 0.0 ? nr_div(xi, gi) : INFINITY,
                           (cg && dc > 0.0) ? nr_div(xi, dc) : INFINITY, INFINITY, INFINITY};
      double s, m;
      wave_reduce8(t, s, m);
      if ((lane & 15) == 0) {
        sR2[g4 * 16 + wave] = s;
        sR2[64 + g4 * 16 + wave] = m;
      }
    } else {
      t_gag = row16_sum(t_gag);
      t_gag += dpp64z<0x142>(t_gag);  // row_bcast:15
      t_gag += dpp64z<0x143>(t_gag);  // row_bcast:31 -> lane 63
      if (lane == 63) sR2[wave] = t_gag;
    }
    NR_PH(3);
    __syncthreads();  // B2
    NR_PH(4);
    if (own) {
      double s0, s1;
      {  // lane l: sum / minimum l >> 4 of wave l & 15 (sum 0 from every wave, the rest from the owners)
        const bool ownv = (lane & 15) < 4;
        s0 = row16_all<false>(((g4 == 0 ? (lane & 15) < R::NW : ownv)) ? sR2[lane] : 0.0);
        s1 = row16_all<true>(ownv ? sR2[64 + lane] : INFINITY);
      }
      const double gag = rdlane_d(s0, 0), ndc = rdlane_d(s0, 16), dres = rdlane_d(s0, 32);
      const double mg = rdlane_d(s1, 0), md = rdlane_d(s1, 16);
      const double agi = (double)ysum();
      double step = nr_div(gres, gag + 1e-20);
      double di = gi, adi = agi, ndir = ngrad, dad_used = gag;
      bool use_dc = false;
      if (cg) {
        const double dad = gag + 2.0 * alpha * gal + alpha * alpha * last_dad;
        const double dstep = nr_div(dres, dad + 1e-20);
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
    NR_PH(5);
    if (stopped) continue;  // owner waves: on to the next pass's first barrier, which ends the loop
  }
  NR_OUT();
  // iterations in Spark's count: the pass whose stopping rule fired (the loop ran one pass further)
  if (stopped) --iterno;
  if (own) a.X[(int64_t)j * KP + c_own] = c_own < a.kreal ? (float)xi : 0.f;
  if (tid == 0 && s_flag[1]) atomicOr(a.err, s_flag[1]);
  if (tid == 0 && a.iters) {
    atomicAdd(&a.iters[0], (unsigned long long)iterno);
    atomicMax(&a.iters[1], (unsigned long long)iterno);
  }
}

template <bool PRE>
__global__ __launch_bounds__(NRow::NTH, 4) void solve_nnls_row_kernel(SolveArgs a, const float* __restrict__ Gt) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  const float* rec = PRE ? a.prebuilt + (size_t)blockIdx.x * SplitRec<NRow::KP>::FLOATS : nullptr;
  int* s_flag = reinterpret_cast<int*>(smem + NRow::OFF_FLAG);
  if (threadIdx.x == 0) {
    s_flag[0] = 0;
    s_flag[1] = 0;
    s_flag[2] = 0;
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < 6) nnls_row_body<0, PRE>(a, Gt, smem, j, p0, d, rec);
  else nnls_row_body<1, PRE>(a, Gt, smem, j, p0, d, rec);
}

}  // namespace

hipError_t launch_solve_nnls_row256(const SolveArgs& a, const float* Gt, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  const size_t lds = (size_t)NRow::FLOATS * 4;
  static const hipError_t attr = allow_lds(solve_nnls_row_kernel<false>, lds);
  static const hipError_t attr2 = allow_lds(solve_nnls_row_kernel<true>, lds);
  if (attr != hipSuccess) return attr;
  if (attr2 != hipSuccess) return attr2;
  const int64_t cap = max_rows_per_launch(NRow::NTH);  // 32-bit AQL grid size in work-items
  for (int64_t r0 = 0; r0 < a.n_rows; r0 += cap) {
    SolveArgs b = a;
    b.rows = a.rows + r0;
    b.n_rows = std::min<int64_t>(a.n_rows - r0, cap);
    if (a.prebuilt) {
      b.prebuilt = a.prebuilt + (size_t)r0 * SplitRec<NRow::KP>::FLOATS;
      solve_nnls_row_kernel<true><<<(int)b.n_rows, NRow::NTH, lds, s>>>(b, Gt);
    } else {
      solve_nnls_row_kernel<false><<<(int)b.n_rows, NRow::NTH, lds, s>>>(b, Gt);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace albedo
