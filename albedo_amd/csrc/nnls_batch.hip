// NNLS rows of low degree (d <= DL), sixteen rows per workgroup in lockstep.
//
// Same problem and iteration as solve_nnls_kernel (als_kernels.hip; Spark NNLSSolver ->
// mllib/optimization/NNLS.scala, reached from ALS.computeFactors with nonnegative = true):
//   A = G + λn I + Ỹᵀ Ỹ   (Ỹ = the row's d src factor rows scaled by √c),   b = Σ w y,
// projected gradient with CG acceleration, Spark's stopping rules, wall clamp and restarts; the
// residual follows the steps (A·x_new = A·x - step·A·dir) with an exact refresh every 64 iterations.
//
// What changes is how A·v is formed.  A light row's A is the common Gram G plus a rank-d term, so a
// workgroup keeps G in registers as MFMA A-operand fragments and iterates 16 rows ("slots") at once:
//   G·[v_0 .. v_15]   one 16-column GEMM on v_mfma_f32_16x16x4_f32 (exact fp32 products, like the
//                     explicit kernel's fp32 FMAs) -- G is read from registers, never from LDS;
//   Ỹᵀ(Ỹ v)           per slot, from the slot's Ỹ rows in LDS (d x KP fp32);
//   λn v              per slot.
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
#include "device_common.h"
#include "kernels.h"

namespace albedo {
namespace {

template <int KP>
struct NBatch {
  static constexpr int NQ = KP / 16;                 // 16-row blocks of G
  static constexpr int NW = KP >= 128 ? 8 : 4;       // waves
  static constexpr int RBW = NQ / NW;                // row blocks per wave
  static constexpr int NTH = 64 * NW;
  static constexpr int S = 16;                       // slots (the MFMA's 16 columns)
  static constexpr int DL = 1536 / KP;               // max degree: Ỹ of 16 slots = 96 KiB
  static constexpr int DLP = (DL + 3) & ~3;
  static constexpr int YS = DL * KP + 4;             // floats per slot; +4: slot j starts on bank 4j
  static constexpr int RT = 4;                       // refill when this many slots are idle
  // LDS, in floats
  static constexpr int OFF_Y = 0;                            // [S][YS]
  static constexpr int OFF_V = S * YS;                       // [2][NQ][4][16][4]: B fragments
  static constexpr int OFF_P = OFF_V + 2 * KP * S;           // [2][NW][16][DLP]: Ỹv partials
  static constexpr int OFF_U = OFF_P + 2 * NW * S * DLP;      // [2][16][DLP]: Ỹv per slot
  static constexpr int OFF_R = (OFF_U + 2 * S * DLP + 3) & ~3;  // doubles [3][NW][16][4]
  static constexpr int OFF_C = OFF_R + 2 * 3 * NW * S * 4;      // ints
  static constexpr int FLOATS = OFF_C + 4;
  static_assert(NW * RBW == NQ, "row blocks split evenly over the waves");
  static_assert(FLOATS * 4 <= 160 * 1024, "LDS");
};

__device__ __forceinline__ bool stop_rule(double step, double ndir, double nx) {
  return isnan(step) || step < 1e-7 || step > 1e40 || ndir < 1e-12 * nx || ndir < 1e-32;
}

// G in MFMA A-operand order, fp32: Gfrag[((I·NQ + m)·64 + l)·4 + u] = G[16 I + (l & 15)][16 m + 4 u + (l >> 4)]
// (one 1-KiB coalesced b128 load per wave serves four 16x16x4 steps of row block I)
__global__ void nnls_gfrag_kernel(const float* __restrict__ Gt, float* __restrict__ Gfrag, int KP) {
  const int NQ = KP / 16;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= KP * KP) return;
  const int u = e & 3, l = (e >> 2) & 63, m = (e >> 8) % NQ, I = (e >> 8) / NQ;
  const int r = 16 * I + (l & 15), c = 16 * m + 4 * u + (l >> 4);
  Gfrag[e] = (r >> 4) >= (c >> 4) ? Gt[nel(r, c)] : Gt[nel(c, r)];
}

template <int KP>
__global__ __launch_bounds__(NBatch<KP>::NTH, 1) void nnls_batch_kernel(SolveArgs a, const float* __restrict__ Gfrag,
                                                                        unsigned int* __restrict__ counter) {
  using NB = NBatch<KP>;
  constexpr int RBW = NB::RBW, NW = NB::NW, DL = NB::DL, DLP = NB::DLP, YS = NB::YS, S = NB::S, NQ = NB::NQ;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, j = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* Yj = smem + NB::OFF_Y + j * YS;  // this lane's slot
  double* R = reinterpret_cast<double*>(smem + NB::OFF_R);
  int* ctl = reinterpret_cast<int*>(smem + NB::OFF_C);

  // this wave's G fragments, streamed from L2 by every product (256 KiB at KP = 256: G is shared by
  // every workgroup and stays cached; holding it in registers would leave none for the slot state)
  const float* gwave = Gfrag + ((int64_t)(w * RBW) * NQ * 64 + lane) * 4;

  auto coord = [&](int rb, int t) { return 16 * (w * RBW + rb) + 4 * g + t; };

  // per-slot sums over the slot's KP coordinates: lane groups by shuffles, waves through LDS
  auto slot_sum = [&](auto NN, double* v, int red) {
    constexpr int N = decltype(NN)::value;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      v[n] += __shfl_xor(v[n], 16);
      v[n] += __shfl_xor(v[n], 32);
    }
    double* rp = R + red * NW * S * 4;
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < N; ++n) rp[(w * S + j) * 4 + n] = v[n];
    }
    __syncthreads();
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double t = rp[j * 4 + n];
#pragma unroll
      for (int u = 1; u < NW; ++u) t += rp[(u * S + j) * 4 + n];
      v[n] = t;
    }
  };
  auto slot_min = [&](double v) {
    v = fmin(v, __shfl_xor(v, 16));
    v = fmin(v, __shfl_xor(v, 32));
    double* rp = R + 2 * NW * S * 4;
    if (g == 0) rp[(w * S + j) * 4] = v;
    __syncthreads();
    double t = rp[j * 4];
#pragma unroll
    for (int u = 1; u < NW; ++u) t = fmin(t, rp[(u * S + j) * 4]);
    return t;
  };

  // y_n = A·v_n for NV per-slot vectors (fp32 in, fp32 out), lamc = λn (or 1 on pad coordinates)
  auto product = [&](auto NVV, const float (*vin)[RBW][4], float (*yout)[RBW][4], float lamn) {
    constexpr int NV = decltype(NVV)::value;
    // B fragments: coordinate 16 m + 4 u + gg of slot j at ((m·4 + gg)·16 + j)·4 + u
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      float* V = smem + NB::OFF_V + n * KP * S;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) V[(((w * RBW + rb) * 4 + t) * 16 + j) * 4 + g] = vin[n][rb][t];
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
        p[n] += __shfl_xor(p[n], 16);
        p[n] += __shfl_xor(p[n], 32);
        if (g == 0) smem[NB::OFF_P + ((n * NW + w) * S + j) * DLP + e] = p[n];
      }
    }
    __syncthreads();
    // per-slot Ỹ v: sum of the partials in a fixed order
    for (int idx = tid; idx < NV * S * DL; idx += NB::NTH) {
      const int n = idx / (S * DL), jj = (idx / DL) % S, e = idx % DL;
      const float* P = smem + NB::OFF_P + n * NW * S * DLP + jj * DLP + e;
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) t += P[q * S * DLP];
      smem[NB::OFF_U + (n * S + jj) * DLP + e] = t;
    }
    // G·V on MFMA
    f32x4 acc[NV][RBW];
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) acc[n][rb] = zero4();
    f32x4 gq[RBW], gn[RBW];
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb) gq[rb] = ld4(gwave + rb * NQ * 256);
#pragma unroll 2
    for (int m = 0; m < NQ; ++m) {
      if (m + 1 < NQ) {  // next row-block column group in flight while this one is on MFMA
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) gn[rb] = ld4(gwave + rb * NQ * 256 + (m + 1) * 256);
      }
      f32x4 vb[NV];
#pragma unroll
      for (int n = 0; n < NV; ++n) vb[n] = ld4(smem + NB::OFF_V + n * KP * S + ((m * 4 + g) * 16 + j) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int n = 0; n < NV; ++n)
#pragma unroll
          for (int rb = 0; rb < RBW; ++rb) acc[n][rb] = mfma4(gq[rb][u], vb[n][u], acc[n][rb]);
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) gq[rb] = gn[rb];
    }
    __syncthreads();
    // Ỹᵀ (Ỹ v) + λn v + G v
    float wv[NV][RBW][4];
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) wv[n][rb][t] = 0.f;
#pragma unroll 2
    for (int e = 0; e < DL; ++e) {
      float un[NV];
#pragma unroll
      for (int n = 0; n < NV; ++n) un[n] = smem[NB::OFF_U + (n * S + j) * DLP + e];
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        const f32x4 y4 = ld4(Yj + e * KP + 16 * (w * RBW + rb) + 4 * g);
#pragma unroll
        for (int n = 0; n < NV; ++n)
#pragma unroll
          for (int t = 0; t < 4; ++t) wv[n][rb][t] = fmaf(y4[t], un[n], wv[n][rb][t]);
      }
    }
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float lc = coord(rb, t) < a.kreal ? lamn : 1.0f;
          yout[n][rb][t] = acc[n][rb][t] + fmaf(lc, vin[n][rb][t], wv[n][rb][t]);
        }
  };

  // slot state (every lane of a slot holds the slot's scalars)
  double x[RBW][4], ax[RBW][4], ld[RBW][4];
  float bb[RBW][4];
  bool act = false;
  int row = 0, iterno = 0, last_wall = 0, npos = 0, dd = 0;
  double last_norm = 0.0, hit = 0.0;
  const int iter_max = 400 > 20 * a.kreal ? 400 : 20 * a.kreal;
  bool exhausted = false;
  int wg_iter = 0;

  for (;;) {
    // ---- refill idle slots (uniform: every wave sees the same slot flags) ----------------------
    const unsigned idle = (unsigned)__ballot(lane < 16 && !act) & 0xFFFFu;
    const int nidle = __popc(idle);
    if (!exhausted && (nidle >= NB::RT || nidle == S)) {
      __syncthreads();  // Ỹ of the idle slots is no longer read
      if (tid == 0) ctl[0] = (int)atomicAdd(counter, (unsigned)nidle);
      __syncthreads();
      const int64_t base = ctl[0];
      if (base + nidle >= a.n_rows) exhausted = true;
      if (!act) {
        const int64_t r = base + __popc(idle & ((1u << j) - 1u));
        if (r < a.n_rows) {
          act = true;
          row = a.rows[r];
          const int64_t p0 = a.ptr[row];
          dd = (int)(a.ptr[row + 1] - p0);
          if (dd > DL) atomicOr(a.err, 4);  // host bucketing guarantees d <= DL
          npos = 0;
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
            for (int t = 0; t < 4; ++t) x[rb][t] = ax[rb][t] = ld[rb][t] = 0.0;
          iterno = 0;
          last_wall = 0;
          last_norm = 0.0;
          hit = 0.0;
        }
      }
      __syncthreads();  // the new Ỹ rows before any product reads them
    }
    if (__ballot(lane < 16 && act) == 0) break;  // drained (implies exhausted)
    const float lamn = a.reg * (float)(a.implicit ? npos : dd);

    // ---- exact residual refresh (A·x) every 64 workgroup iterations -----------------------------
    if (wg_iter > 0 && (wg_iter & 63) == 0) {
      float xin[1][RBW][4], yo[1][RBW][4];
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) xin[0][rb][t] = (float)x[rb][t];
      product(std::integral_constant<int, 1>{}, xin, yo, lamn);
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) ax[rb][t] = (double)yo[0][rb][t];
    }
    ++wg_iter;

    // ---- residual, projected gradient ------------------------------------------------------------
    double gi[RBW][4];
    double r1[4] = {0.0, 0.0, 0.0, hit};
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double res = ax[rb][t] - (double)bb[rb][t];
        double gv = res;
        if (gv > 0.0 && x[rb][t] == 0.0) gv = 0.0;
        gi[rb][t] = gv;
        r1[0] += gv * gv;
        r1[1] += gv * res;
        r1[2] += x[rb][t] * x[rb][t];
      }
    slot_sum(std::integral_constant<int, 4>{}, r1, 0);
    if (r1[3] > 0.0) last_wall = iterno - 1;
    const double ngrad = r1[0], nx = r1[2];
    const bool cg = iterno > last_wall + 1;
    const double alpha = cg ? ngrad / last_norm : 0.0;

    // ---- A·grad and A·dir --------------------------------------------------------------------------
    float vin[2][RBW][4], yo[2][RBW][4];
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        vin[0][rb][t] = (float)gi[rb][t];
        vin[1][rb][t] = cg ? (float)(gi[rb][t] + alpha * ld[rb][t]) : 0.f;
      }
    product(std::integral_constant<int, 2>{}, vin, yo, lamn);
    double r2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double res = ax[rb][t] - (double)bb[rb][t];
        const double dc = cg ? gi[rb][t] + alpha * ld[rb][t] : 0.0;
        r2[0] += gi[rb][t] * (double)yo[0][rb][t];
        r2[1] += dc * res;
        r2[2] += dc * (double)yo[1][rb][t];
        r2[3] += dc * dc;
      }
    slot_sum(std::integral_constant<int, 4>{}, r2, 1);
    double step = r1[1] / (r2[0] + 1e-20), ndir = ngrad;
    bool use_dc = false;
    if (cg) {
      const double dstep = r2[1] / (r2[2] + 1e-20);
      if (!stop_rule(dstep, r2[3], nx)) {  // else: reject the CG direction
        step = dstep;
        ndir = r2[3];
        use_dc = true;
      }
    }
    const bool stop = !act || stop_rule(step, ndir, nx);
    // don't run through the walls: step = min(step, x_i / d_i over d_i > 0 with step d_i > x_i)
    double cand = INFINITY;
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double di = use_dc ? gi[rb][t] + alpha * ld[rb][t] : gi[rb][t];
        if (!stop && step * di > x[rb][t]) cand = fmin(cand, x[rb][t] / di);
      }
    step = fmin(step, slot_min(cand));
    bool finish = act && stop;
    if (act && !stop) {
      hit = 0.0;
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const double di = use_dc ? gi[rb][t] + alpha * ld[rb][t] : gi[rb][t];
          float y0v = yo[0][rb][t], y1v = yo[1][rb][t];
          asm("" : "+v"(y0v), "+v"(y1v));  // a select of values, not of array slots (scratch)
          const double adi = (double)(use_dc ? y1v : y0v);
          if (step * di > x[rb][t] * (1 - 1e-14)) {
            x[rb][t] = 0.0;
            hit = 1.0;
          } else {
            x[rb][t] -= step * di;
          }
          ax[rb][t] -= step * adi;
          ld[rb][t] = di;
        }
      last_norm = ngrad;
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
        *reinterpret_cast<f32x4*>(a.X + (int64_t)row * KP + coord(rb, 0)) = f32x4{o[0], o[1], o[2], o[3]};
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
    }
  }
}

template <int KP>
hipError_t launch_batch_kp(const SolveArgs& a, const float* Gfrag, unsigned int* counter, int n_cu, hipStream_t s) {
  using NB = NBatch<KP>;
  static const hipError_t attr = allow_lds(nnls_batch_kernel<KP>, NB::FLOATS * 4);
  if (attr != hipSuccess) return attr;
  hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  const int64_t want = (a.n_rows + NB::S - 1) / NB::S;
  const int blocks = (int)(want < n_cu ? want : n_cu);
  nnls_batch_kernel<KP><<<blocks, NB::NTH, NB::FLOATS * 4, s>>>(a, Gfrag, counter);
  return hipGetLastError();
}

}  // namespace

int nnls_batch_max_degree(int KP) { return KP == 64 ? NBatch<64>::DL : KP == 128 ? NBatch<128>::DL : NBatch<256>::DL; }

hipError_t launch_nnls_batch(int KP, const SolveArgs& a, const float* Gt, float* Gfrag, unsigned int* counter,
                             int n_cu, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  nnls_gfrag_kernel<<<(KP * KP + 255) / 256, 256, 0, s>>>(Gt, Gfrag, KP);
  if (KP == 64) return launch_batch_kp<64>(a, Gfrag, counter, n_cu, s);
  if (KP == 128) return launch_batch_kp<128>(a, Gfrag, counter, n_cu, s);
  if (KP == 256) return launch_batch_kp<256>(a, Gfrag, counter, n_cu, s);
  return hipErrorInvalidValue;
}

}  // namespace albedo
