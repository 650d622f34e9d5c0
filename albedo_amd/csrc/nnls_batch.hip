// NNLS rows of low degree (d <= DL), sixteen rows per workgroup in lockstep.
//
// Same problem and iteration as solve_nnls_kernel (als_kernels.hip; Spark NNLSSolver ->
// mllib/optimization/NNLS.scala, reached from ALS.computeFactors with nonnegative = true):
//   A = G + λn I + Ỹᵀ Ỹ   (Ỹ = the row's d src factor rows scaled by √c),   b = Σ w y,
// projected gradient with CG acceleration, Spark's stopping rules, wall clamp and restarts; the
// residual follows the steps (A·x_new = A·x - step·A·dir) with an exact refresh every 64 iterations.
//
// What changes is how A·v is formed.  A light row's A is the common Gram G plus a rank-d term, so a
// workgroup iterates up to 16 rows ("slots") at once and never forms A:
//   G·[v_0 .. v_15]   one 16-column GEMM on v_mfma_f32_16x16x32_f16 with G and every v split into
//                     fp16 hi + lo (hi·hi + hi·lo + lo·hi, fp32 accumulation: 22-bit operands, as the
//                     heavy build), G by a power of two, each slot's v by a power of two from a bound
//                     on max|v| the reductions already carry; G streams from L2 (it is shared by every
//                     workgroup), v goes through LDS;
//   Ỹᵀ(Ỹ v)           per slot, fp32, from the slot's Ỹ rows in LDS (d x KP);
//   λn v              per slot.
// The Ỹ budget is 96 KiB, so the slot count trades against the degree limit: SV slots of degree
// <= 24576 / (SV·KP) (KP = 256: 16 x 6, 8 x 12, 4 x 24, 2 x 48, 1 x 96); the G·V cost is the same
// for any SV (16 MFMA columns), the per-row cost falls as 1/SV.
// Lane layout = the MFMA C/D layout: wave w owns row blocks I = w·RBW .. w·RBW + RBW-1; lane l holds
// slot j = l & 15 and coordinates 16 I + 4 (l >> 4) + t, t = 0..3.  Every per-slot vector lives in
// that layout in registers (fp64, as in the explicit kernel); per-slot sums reduce over the four lane
// groups (shuffles) and the waves (LDS, one barrier), and every lane of a slot ends with the same
// value, so each slot runs its own state machine under uniform control flow.
//
// Slots are refilled from a global row counter when RT of them are idle: the workgroup is
// persistent (one per CU) and drains when the counter passes the row list.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <utility>
#include "device_common.h"
#include "kernels.h"

namespace albedo {
namespace {

constexpr int YBUDGET = 24576;  // floats of Ỹ per workgroup (96 KiB)

#ifdef ALBEDO_BATCH_TIMING  // probes only: loop phase cycles summed over iterations (thread 0)
__device__ unsigned long long albedo_batch_ph[64][9];
#define BT_T0() unsigned long long bt_t = clock64(), bt_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}
#define BT_PH(k) { const unsigned long long bt_n = clock64(); bt_acc[k] += bt_n - bt_t; bt_t = bt_n; }
#define BT_OUT() \
  if (threadIdx.x == 0 && blockIdx.x < 64) for (int q = 0; q < 9; ++q) albedo_batch_ph[blockIdx.x][q] = bt_acc[q]
#else
#define BT_T0()
#define BT_PH(k)
#define BT_OUT()
#endif

template <int KP, int SV>
struct NBatch {
  static constexpr int NQ = KP / 16;                 // 16-row blocks of G
  static constexpr int NS = KP / 32;                 // 32-deep k-steps of the f16 MFMA
  static constexpr int NW = KP >= 128 ? 8 : 4;       // waves
  static constexpr int RBW = NQ / NW;                // row blocks per wave (1 or 2)
  static constexpr int NTH = 64 * NW;
  static constexpr int S = 16;                       // MFMA columns; slots SV <= 16 of them
  static constexpr int DL = YBUDGET / (SV * KP);     // degree limit of a slot
  static constexpr int DLP = (DL + 3) & ~3;
  static constexpr int YS = DL * KP + 4;             // floats per slot; +4: slot j starts on bank 4j
  static constexpr int RT = SV >= 4 ? SV / 4 : 1;    // refill when this many slots are idle
  // LDS, in floats
  static constexpr int OFF_Y = 0;                            // [SV][YS]
  static constexpr int OFF_V = SV * YS;                      // [hi|lo][NS][4][16][8] halves
  static constexpr int OFF_P = OFF_V + KP * S;               // [NW][SV][DLP]: Ỹv partials
  static constexpr int OFF_U = OFF_P + NW * SV * DLP;        // [SV][DLP]: Ỹv per slot
  static constexpr int AS = KP + 4;                          // A·lastDir row stride (banks)
  static constexpr int OFF_A = OFF_U + SV * DLP;             // [SV][AS]: A·lastDir per slot (fp32)
  static constexpr int OFF_R = (OFF_A + SV * AS + 3) & ~3;   // doubles [2][NW][16][RS]
  // R: doubles [2][NW][16][RS]; RS = 9 (8 values + 1 pad): the slot stride of 18 dwords puts the 16
  // slots' b64 accesses on 16 distinct bank pairs (at 8 they shared 4: the SQ counters of r06 showed
  // 2.7 bank-conflict cycles per LDS instruction in this kernel)
  static constexpr int RS = 9;
  static constexpr int OFF_C = OFF_R + 2 * 2 * NW * S * RS;     // ints: [0] refill base, [4 + j] slot j's row
  static constexpr int FLOATS = OFF_C + 4 + S;
  static_assert(NW * RBW == NQ && NQ % 2 == 0 && RBW <= 2, "row blocks split evenly over the waves");
  static_assert(DL >= 1 && FLOATS * 4 <= 160 * 1024, "LDS");
};

__device__ __forceinline__ bool stop_rule(double step, double ndir, double nx) {
  return isnan(step) || step < 1e-7 || step > 1e40 || ndir < 1e-12 * nx || ndir < 1e-32;
}

// 2^(14 - E) for bound < 2^E: |v| <= bound maps below 2^14, in fp16's range with room for lo
__device__ __forceinline__ float pow2_scale(double bound) {
  if (!(bound > 0.0) || !isfinite(bound)) return 1.0f;
  int e;
  (void)frexp(bound, &e);
  e = 14 - e;
  e = e > 100 ? 100 : (e < -100 ? -100 : e);
  return ldexpf(1.0f, e);
}

// Sum / max over the four 16-lane rows of the wave (lanes l, l^16, l^32, l^48), every lane getting
// the same result: v_permlane16_swap pairs rows (0,1) and (2,3), v_permlane32_swap the two halves --
// VALU only, no LDS round trip (a shuffle is two).  Both partners add in the same order, so the
// result is bit-identical in all four lanes (the slot state machine relies on that).
template <bool MAX>
__device__ __forceinline__ float rows4(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float p = __uint_as_float(a[0]), q = __uint_as_float(a[1]);
  const float s = MAX ? fmaxf(p, q) : p + q;
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  const float u = __uint_as_float(b[0]), v = __uint_as_float(b[1]);
  return MAX ? fmaxf(u, v) : u + v;
}
template <bool MAX>
__device__ __forceinline__ double rows4(double x) {
  auto swap16 = [](double d) {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(d), (unsigned)__double2loint(d), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(d), (unsigned)__double2hiint(d), false, false);
    return std::make_pair(__hiloint2double((int)hi[0], (int)lo[0]), __hiloint2double((int)hi[1], (int)lo[1]));
  };
  auto swap32 = [](double d) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(d), (unsigned)__double2loint(d), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(d), (unsigned)__double2hiint(d), false, false);
    return std::make_pair(__hiloint2double((int)hi[0], (int)lo[0]), __hiloint2double((int)hi[1], (int)lo[1]));
  };
  const auto a = swap16(x);
  const double s = MAX ? fmax(a.first, a.second) : a.first + a.second;
  const auto b = swap32(s);
  return MAX ? fmax(b.first, b.second) : b.first + b.second;
}

// G·gs in MFMA A-operand order, fp16 hi then lo: element ((I·NS + s)·64 + l)·8 + h holds
// G[16 I + (l & 15)][32 s + 8 (l >> 4) + h] (one 1-KiB b128 load per wave per 32-deep k-step)
__global__ void nnls_gfrag_kernel(const float* __restrict__ Gt, _Float16* __restrict__ Gh, int KP, float gs) {
  const int NS = KP / 32;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= KP * KP) return;
  const int h = e & 7, l = (e >> 3) & 63, s = (e >> 9) % NS, I = (e >> 9) / NS;
  const int r = 16 * I + (l & 15), c = 32 * s + 8 * (l >> 4) + h;
  float v = ((r >> 4) >= (c >> 4) ? Gt[nel(r, c)] : Gt[nel(c, r)]) * gs;
  asm("" : "+v"(v));  // hi and lo from the one fp32 value
  const _Float16 hi = (_Float16)v;
  Gh[e] = hi;
  Gh[KP * KP + e] = (_Float16)(v - (float)hi);
}

template <int KP, int SV>
__global__ __launch_bounds__((NBatch<KP, SV>::NTH), 1) void nnls_batch_kernel(SolveArgs a, const _Float16* __restrict__ Gh,
                                                                            float ginv, unsigned int* __restrict__ counter) {
  using NB = NBatch<KP, SV>;
  constexpr int RBW = NB::RBW, NW = NB::NW, DL = NB::DL, DLP = NB::DLP, YS = NB::YS, S = NB::S, NS = NB::NS;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Lane coordinates, re-derived every iteration from an opaque copy of threadIdx.x (see the loop
  // head): otherwise the compiler hoists dozens of LDS addresses out of the loop and spills them.
  int j = lane & 15, g = lane >> 4;
  bool slot_lane = j < SV;                          // columns past SV stay empty
  float* Yj = smem + NB::OFF_Y + (slot_lane ? j : 0) * YS;  // this lane's slot
  float* Aj = smem + NB::OFF_A + (slot_lane ? j : 0) * NB::AS;  // its A·lastDir (fp32)
  double* R = reinterpret_cast<double*>(smem + NB::OFF_R);
  int* ctl = reinterpret_cast<int*>(smem + NB::OFF_C);
  _Float16* Vh = reinterpret_cast<_Float16*>(smem + NB::OFF_V);

  // this wave's G fragments (hi; lo follows at + KP·KP halves), streamed from L2 by every product
  const _Float16* gwave = Gh + ((int64_t)(w * RBW) * NS * 64 + lane) * 8;

  auto coord = [&](int rb, int t) { return 16 * (w * RBW + rb) + 4 * g + t; };
  BT_T0();

  // Per-slot reductions over the slot's KP coordinates: the four lane groups by shuffles, the waves
  // through LDS (buffer `buf`, values at `off`..): the first NSUM values are summed, the next NMAX
  // take the maximum.  Every lane of a slot ends with the same values.
  auto slot_reduce = [&](auto NSUMC, auto NMAXC, double* v, int buf, int off) {
    constexpr int NSUM = decltype(NSUMC)::value, N = NSUM + decltype(NMAXC)::value;
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] = n < NSUM ? rows4<false>(v[n]) : rows4<true>(v[n]);
    double* rp = R + buf * NW * S * NB::RS + off;
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < N; ++n) rp[(w * S + j) * NB::RS + n] = v[n];
    }
    __syncthreads();
    // readout split over the four lane groups: group g combines waves g·NW/4 .. of the slot's partials
    // and the lane-group sum finishes (2 LDS reads per value and lane at NW = 8 instead of 8), in the
    // fixed order ((w0 w1)(w2 w3))((w4 w5)(w6 w7)), bit-identical in every lane of the slot
    constexpr int WPG = NW / 4;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double t = rp[((WPG * g) * S + j) * NB::RS + n];
#pragma unroll
      for (int u = 1; u < WPG; ++u)
        t = n < NSUM ? t + rp[((WPG * g + u) * S + j) * NB::RS + n] : fmax(t, rp[((WPG * g + u) * S + j) * NB::RS + n]);
      v[n] = n < NSUM ? rows4<false>(t) : rows4<true>(t);
    }
  };

  // y_n = A·v_n for NV per-slot vectors (fp32 in, fp32 out); vs[n]: the slot's power-of-two scale
  // of v_n for the fp16 split; lamn = λn (1 on pad coordinates)
  auto product = [&](auto NVV, const float (*vin)[RBW][4], const float* vs, float (*yout)[RBW][4], float lamn) {
    constexpr int NV = decltype(NVV)::value;
    static_assert(NV == 1, "the V / P / U buffers hold one vector");
    // B fragments: coordinate 32 s + 8 gg + h of slot j at hi/lo [((s·4 + gg)·16 + j)·8 + h]
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      _Float16* vh = Vh + n * 2 * KP * S;
      _Float16* vl = vh + KP * S;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        const int I = w * RBW + rb;
        const int off = (((I >> 1) * 4 + 2 * (I & 1) + (g >> 1)) * 16 + j) * 8 + 4 * (g & 1);
        f16x4 hv, lv;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float v = vin[n][rb][t] * vs[n];
          asm("" : "+v"(v));
          const _Float16 h = (_Float16)v;
          hv[t] = h;
          lv[t] = (_Float16)(v - (float)h);
        }
        *reinterpret_cast<f16x4*>(vh + off) = hv;
        *reinterpret_cast<f16x4*>(vl + off) = lv;
      }
    }
    // Ỹ v partials over this lane's coordinates (each Ỹ fragment read once for every vector),
    // summed over the four lane groups, one partial per wave and slot
#pragma unroll 2
    for (int e = 0; e < DL; ++e) {
      float p[NV];
#pragma unroll
      for (int n = 0; n < NV; ++n) p[n] = 0.f;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        const f32x4 y4 = ld4(Yj + e * KP + 16 * (w * RBW + rb) + 4 * g);
#pragma unroll
        for (int n = 0; n < NV; ++n)
          p[n] = fmaf(y4[0], vin[n][rb][0], fmaf(y4[1], vin[n][rb][1], fmaf(y4[2], vin[n][rb][2],
                 fmaf(y4[3], vin[n][rb][3], p[n]))));
      }
#pragma unroll
      for (int n = 0; n < NV; ++n) {
        p[n] = rows4<false>(p[n]);
        if (g == 0 && slot_lane) smem[NB::OFF_P + ((n * NW + w) * SV + j) * DLP + e] = p[n];
      }
    }
    __syncthreads();
    BT_PH(3);
    // per-slot Ỹ v: sum of the partials in a fixed order
    for (int idx = tid; idx < NV * SV * DL; idx += NB::NTH) {
      const int n = idx / (SV * DL), jj = (idx / DL) % SV, e = idx % DL;
      const float* P = smem + NB::OFF_P + n * NW * SV * DLP + jj * DLP + e;
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) t += P[q * SV * DLP];
      smem[NB::OFF_U + (n * SV + jj) * DLP + e] = t;
    }
    // G·V on split-fp16 MFMA
    f32x4 acc[NV][RBW];
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) acc[n][rb] = zero4();
    // (k-step, row block) pairs in sequence, the next pair's G fragments in flight
    f16x8 gh = *reinterpret_cast<const f16x8*>(gwave), gl = *reinterpret_cast<const f16x8*>(gwave + KP * KP);
#pragma unroll 2
    for (int q = 0; q < NS * RBW; ++q) {
      const int ks = q / RBW, rb = q % RBW;
      f16x8 nh = gh, nl = gl;
      if (q + 1 < NS * RBW) {
        const int ks1 = (q + 1) / RBW, rb1 = (q + 1) % RBW;
        nh = *reinterpret_cast<const f16x8*>(gwave + rb1 * NS * 512 + ks1 * 512);
        nl = *reinterpret_cast<const f16x8*>(gwave + KP * KP + rb1 * NS * 512 + ks1 * 512);
      }
#pragma unroll
      for (int n = 0; n < NV; ++n) {
        const _Float16* vh = Vh + n * 2 * KP * S + ((ks * 4 + g) * 16 + j) * 8;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(vh);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(vh + KP * S);
        f32x4 c = acc[n][0];
        if (RBW > 1 && rb == 1) c = acc[n][RBW > 1 ? 1 : 0];
        c = mfma_h(gh, bh, c);
        c = mfma_h(gh, bl, c);
        c = mfma_h(gl, bh, c);
        if (RBW > 1 && rb == 1) acc[n][RBW > 1 ? 1 : 0] = c;
        else acc[n][0] = c;
      }
      gh = nh;
      gl = nl;
    }
    __syncthreads();
    BT_PH(4);
    // Ỹᵀ (Ỹ v) + λn v + G v
    float wv[NV][RBW][4];
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) wv[n][rb][t] = 0.f;
    // four ratings per step: the slot's Ỹv from one b128 read per vector
    const float* Uj = smem + NB::OFF_U + (slot_lane ? j : 0) * DLP;
#pragma unroll 1
    for (int e4 = 0; e4 < DLP; e4 += 4) {
      f32x4 u4[NV];
#pragma unroll
      for (int n = 0; n < NV; ++n) u4[n] = slot_lane ? ld4(Uj + n * SV * DLP + e4) : zero4();
#pragma unroll
      for (int ee = 0; ee < 4; ++ee) {
        if (DL % 4 != 0 && e4 + ee >= DL) break;
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) {
          const f32x4 y4 = ld4(Yj + (e4 + ee) * KP + 16 * (w * RBW + rb) + 4 * g);
#pragma unroll
          for (int n = 0; n < NV; ++n)
#pragma unroll
            for (int t = 0; t < 4; ++t) wv[n][rb][t] = fmaf(y4[t], u4[n][ee], wv[n][rb][t]);
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const float unscale = ginv / vs[n];  // powers of two: exact
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float lc = coord(rb, t) < a.kreal ? lamn : 1.0f;
          yout[n][rb][t] = acc[n][rb][t] * unscale + fmaf(lc, vin[n][rb][t], wv[n][rb][t]);
        }
    }
  };

  // slot state (every lane of a slot holds the slot's scalars)
  // ald = A·lastDir: A·dir = A·g + alpha·A·lastDir (linearity), so one product per iteration
  // (ald in fp32: it is an fp32 product's value carried forward, the registers go to the products)
  double x[RBW][4], ax[RBW][4], ld[RBW][4];
  float bb[RBW][4];
  bool act = false;
  // (the slot's row lives in LDS, ctl[4 + j], and its λn in one register: the loop is at the 256-VGPR
  // budget, and every register freed there is a spill less)
  int iterno = 0, last_wall = 0;
  float lamn = 0.f;
  double last_norm = 0.0, hit = 0.0, last_dad = 0.0;
  const int iter_max = 400 > 20 * a.kreal ? 400 : 20 * a.kreal;
  bool exhausted = false;
  int wg_iter = 0;

  for (;;) {
    {
      int ot = tid;
      asm volatile("" : "+v"(ot));
      j = ot & 15;
      g = (ot >> 4) & 3;
      slot_lane = j < SV;
      Yj = smem + NB::OFF_Y + (slot_lane ? j : 0) * YS;
      Aj = smem + NB::OFF_A + (slot_lane ? j : 0) * NB::AS;
    }
    // ---- refill idle slots (uniform: every wave sees the same slot flags) ----------------------
    const unsigned idle = (unsigned)__ballot(slot_lane && !act) & ((1u << SV) - 1u);
    const int nidle = __popc(idle);
    if (!exhausted && (nidle >= NB::RT || nidle == SV)) {
      __syncthreads();  // Ỹ of the idle slots is no longer read
      if (tid == 0) ctl[0] = (int)atomicAdd(counter, (unsigned)nidle);
      __syncthreads();
      const int64_t base = ctl[0];
      if (base + nidle >= a.n_rows) exhausted = true;
      if (slot_lane && !act) {
        const int64_t r = base + __popc(idle & ((1u << j) - 1u));
        if (r < a.n_rows) {
          act = true;
          const int row = a.rows[r];
          if (w == 0 && g == 0) ctl[4 + j] = row;
          const int64_t p0 = a.ptr[row];
          const int dd = (int)(a.ptr[row + 1] - p0);
          if (dd > DL) atomicOr(a.err, 4);  // host bucketing guarantees d <= DL
          int npos = 0;
#pragma unroll
          for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
            for (int t = 0; t < 4; ++t) bb[rb][t] = 0.f;
#pragma unroll 1
          for (int e = 0; e < DL; ++e) {
            const bool in = e < dd;
            const int col = in ? a.col[p0 + e] : 0;
            const float rv = in ? a.val[p0 + e] : 0.f;
            float cw = 0.f, ww = 0.f;
            rating_weights(rv, a.implicit, a.alpha, cw, ww);
            const float sc = in ? sqrtf(cw) : 0.f;
            if (!in) ww = 0.f;
            npos += (in && rv > 0.f) ? 1 : 0;
#pragma unroll
            for (int rb = 0; rb < RBW; ++rb) {
              const int c0 = 16 * (w * RBW + rb) + 4 * g;
              const f32x4 z = in ? ld4(a.Z + (int64_t)col * KP + c0) : zero4();
              *reinterpret_cast<f32x4*>(Yj + e * KP + c0) = f32x4{sc * z[0], sc * z[1], sc * z[2], sc * z[3]};
#pragma unroll
              for (int t = 0; t < 4; ++t) bb[rb][t] = fmaf(ww, z[t], bb[rb][t]);
            }
          }
#pragma unroll
          for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              x[rb][t] = ax[rb][t] = ld[rb][t] = 0.0;
            }
#pragma unroll
          for (int rb = 0; rb < RBW; ++rb) *reinterpret_cast<f32x4*>(Aj + 16 * (w * RBW + rb) + 4 * g) = zero4();
          lamn = a.reg * (float)(a.implicit ? npos : dd);
          iterno = 0;
          last_wall = 0;
          last_norm = 0.0;
          last_dad = 0.0;
          hit = 0.0;
        }
      }
      __syncthreads();  // the new Ỹ rows before any product reads them
    }
    BT_PH(0);
    if ((__ballot(slot_lane && act) & ((1u << SV) - 1u)) == 0) break;  // drained (implies exhausted)

    // ---- exact residual refresh (A·x) every 64 workgroup iterations -----------------------------
    if (wg_iter > 0 && (wg_iter & 63) == 0) {
      float xin[1][RBW][4], yo[1][RBW][4];
      double xm[1] = {0.0};
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          xin[0][rb][t] = (float)x[rb][t];
          xm[0] = fmax(xm[0], fabs(x[rb][t]));
        }
      slot_reduce(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, xm, 0, 6);
      const float vs[1] = {pow2_scale(xm[0])};
      product(std::integral_constant<int, 1>{}, xin, vs, yo, lamn);
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) ax[rb][t] = (double)yo[0][rb][t];
    }
    ++wg_iter;
    BT_PH(1);

    // ---- residual, projected gradient (recomputed where needed: registers go to the products) ------
    auto grad = [&](int rb, int t) {
      const double res = ax[rb][t] - (double)bb[rb][t];
      return (res > 0.0 && x[rb][t] == 0.0) ? 0.0 : res;
    };
    double r1[6] = {0.0, 0.0, 0.0, hit, 0.0, 0.0};  // Σg², Σg·res, Σx², wall hits, Σg·A·lastDir | max|g|
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double res = ax[rb][t] - (double)bb[rb][t];
        const double gv = grad(rb, t);
        r1[0] += gv * gv;
        r1[1] += gv * res;
        r1[2] += x[rb][t] * x[rb][t];
        r1[4] += gv * (double)Aj[16 * (w * RBW + rb) + 4 * g + t];
        r1[5] = fmax(r1[5], fabs(gv));
      }
    slot_reduce(std::integral_constant<int, 5>{}, std::integral_constant<int, 1>{}, r1, 0, 0);
    BT_PH(2);
    if (r1[3] > 0.0) last_wall = iterno - 1;
    const double ngrad = r1[0], nx = r1[2];
    const bool cg = iterno > last_wall + 1;
    const double alpha = cg ? ngrad / last_norm : 0.0;

    // ---- A·grad (A·dir = A·grad + alpha·A·lastDir) --------------------------------------------------
    float vin[1][RBW][4], yo[1][RBW][4];
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) vin[0][rb][t] = (float)grad(rb, t);
    const float vs[1] = {pow2_scale(r1[5])};
    product(std::integral_constant<int, 1>{}, vin, vs, yo, lamn);
    BT_PH(5);
    // Σg·Ag, Σd·res, Σd² | and the wall ratios of both candidate directions: -min x_i/g_i over
    // g_i > 0, -min x_i/d_i over d_i > 0 (Spark clamps the step to the smallest x_i/dir_i below it;
    // the minimum over every positive dir_i gives the same clamp, so the ratio rides in this
    // reduction instead of a third one after the direction is chosen).  d·Ad = g·Ag + 2 alpha
    // g·A·lastDir + alpha² lastDir·A·lastDir (the previous step's curvature).
    // (the lane's smallest ratios are selected by cross-multiplication, then divided once each)
    double r2[5] = {0.0, 0.0, 0.0, -INFINITY, -INFINITY};
    double ng = 0.0, dg = 0.0, nd = 0.0, ddn = 0.0;  // numerator / denominator of the lane's minima
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double res = ax[rb][t] - (double)bb[rb][t];
        const double gv = grad(rb, t);
        const double dc = cg ? gv + alpha * ld[rb][t] : 0.0;
        r2[0] += gv * (double)yo[0][rb][t];
        r2[1] += dc * res;
        r2[2] += dc * dc;
        if (gv > 0.0 && (dg == 0.0 || x[rb][t] * dg < ng * gv)) {
          ng = x[rb][t];
          dg = gv;
        }
        if (dc > 0.0 && (ddn == 0.0 || x[rb][t] * ddn < nd * dc)) {
          nd = x[rb][t];
          ddn = dc;
        }
      }
    if (dg > 0.0) r2[3] = -(ng / dg);
    if (ddn > 0.0) r2[4] = -(nd / ddn);
    slot_reduce(std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{}, r2, 1, 0);
    BT_PH(6);
    double step = r1[1] / (r2[0] + 1e-20), ndir = ngrad, dad_used = r2[0];
    bool use_dc = false;
    if (cg) {
      const double dad = r2[0] + 2.0 * alpha * r1[4] + alpha * alpha * last_dad;
      const double dstep = r2[1] / (dad + 1e-20);
      if (!stop_rule(dstep, r2[2], nx)) {  // else: reject the CG direction
        step = dstep;
        ndir = r2[2];
        dad_used = dad;
        use_dc = true;
      }
    }
    const bool stop = !act || stop_rule(step, ndir, nx);
    // don't run through the walls
    step = fmin(step, -(use_dc ? r2[4] : r2[3]));
    BT_PH(7);
    bool finish = act && stop;
    if (act && !stop) {
      hit = 0.0;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        float* ap = Aj + 16 * (w * RBW + rb) + 4 * g;
        const f32x4 a4 = ld4(ap);
        f32x4 an;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const double gv = grad(rb, t);
          const double di = use_dc ? gv + alpha * ld[rb][t] : gv;
          const double agi = (double)yo[0][rb][t];
          const double adi = use_dc ? agi + alpha * (double)a4[t] : agi;
          if (step * di > x[rb][t] * (1 - 1e-14)) {
            x[rb][t] = 0.0;
            hit = 1.0;
          } else {
            x[rb][t] -= step * di;
          }
          ax[rb][t] -= step * adi;
          ld[rb][t] = di;
          an[t] = (float)adi;
        }
        if (slot_lane) *reinterpret_cast<f32x4*>(ap) = an;
      }
      last_norm = ngrad;
      last_dad = dad_used;
      ++iterno;
      finish = iterno >= iter_max;
    }
    if (finish) {
      bool nonfinite = false;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        float o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          o[t] = coord(rb, t) < a.kreal ? (float)x[rb][t] : 0.f;
          nonfinite |= !isfinite(o[t]);
        }
        *reinterpret_cast<f32x4*>(a.X + (int64_t)ctl[4 + j] * KP + coord(rb, 0)) = f32x4{o[0], o[1], o[2], o[3]};
      }
      if (nonfinite) atomicOr(a.err, 2);
      if (a.iters && w == 0 && g == 0) {
        atomicAdd(&a.iters[0], (unsigned long long)iterno);
        atomicMax(&a.iters[1], (unsigned long long)iterno);
      }
      act = false;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          x[rb][t] = ax[rb][t] = ld[rb][t] = 0.0;
          bb[rb][t] = 0.f;
        }
      hit = 0.0;
      last_dad = 0.0;
    }
    BT_PH(8);
  }
  BT_OUT();
}

template <int KP, int SV>
hipError_t launch_batch_sv(const SolveArgs& a, const _Float16* Gh, float ginv, unsigned int* counter, int n_cu,
                           hipStream_t s) {
  using NB = NBatch<KP, SV>;
  static const hipError_t attr = allow_lds(nnls_batch_kernel<KP, SV>, NB::FLOATS * 4);
  if (attr != hipSuccess) return attr;
  hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  const int64_t want = (a.n_rows + SV - 1) / SV;
  const int blocks = (int)(want < n_cu ? want : n_cu);
  nnls_batch_kernel<KP, SV><<<blocks, NB::NTH, NB::FLOATS * 4, s>>>(a, Gh, ginv, counter);
  return hipGetLastError();
}

template <int KP>
hipError_t launch_batch_kp(int sv, const SolveArgs& a, const _Float16* Gh, float ginv, unsigned int* counter,
                           int n_cu, hipStream_t s) {
  switch (sv) {
    case 16: return launch_batch_sv<KP, 16>(a, Gh, ginv, counter, n_cu, s);
    case 8: return launch_batch_sv<KP, 8>(a, Gh, ginv, counter, n_cu, s);
    case 4: return launch_batch_sv<KP, 4>(a, Gh, ginv, counter, n_cu, s);
    case 2: return launch_batch_sv<KP, 2>(a, Gh, ginv, counter, n_cu, s);
    case 1: return launch_batch_sv<KP, 1>(a, Gh, ginv, counter, n_cu, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int nnls_batch_max_degree(int KP, int slots) { return (slots >= 1 && slots <= 16) ? YBUDGET / (slots * KP) : 0; }

hipError_t launch_nnls_gfrag(int KP, const float* Gt, float gscale, void* Gfrag, hipStream_t s) {
  nnls_gfrag_kernel<<<(KP * KP + 255) / 256, 256, 0, s>>>(Gt, reinterpret_cast<_Float16*>(Gfrag), KP, gscale);
  return hipGetLastError();
}

hipError_t launch_nnls_batch(int KP, int slots, const SolveArgs& a, const void* Gfrag, float gscale,
                             unsigned int* counter, int n_cu, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  const _Float16* Gh = reinterpret_cast<const _Float16*>(Gfrag);
  const float ginv = 1.0f / gscale;
  if (KP == 64) return launch_batch_kp<64>(slots, a, Gh, ginv, counter, n_cu, s);
  if (KP == 128) return launch_batch_kp<128>(slots, a, Gh, ginv, counter, n_cu, s);
  if (KP == 256) return launch_batch_kp<256>(slots, a, Gh, ginv, counter, n_cu, s);
  return hipErrorInvalidValue;
}

}  // namespace albedo
