// Eigenbasis of the src Gram on the device (the step between Spark's computeYtY and the per-row
// solves, ALS.computeFactors reached from ALSRecommenderBuilder.scala:58; the engine's restatement
// solves every row in the basis where YᵀY is diagonal, als_engine.cpp half_sweep).
//
// The src factors X live in an orthogonal basis B_s (original = X·B_sᵀ) and the dst side's current
// basis B_t = B_s(prev)·P(prev) holds the eigenvectors of this side's previous Gram in original
// coordinates, so  W = B_sᵀ·B_t  nearly diagonalises the new Gram G (the factors change little from
// one sweep to the next):  M = Wᵀ G W  is swept by a cyclic parallel Jacobi in fp64 (one workgroup,
// M in LDS, the 64 disjoint pairs of a round-robin round rotated at once, V = W·J accumulated in
// global memory) until the off-diagonal mass is below 1e-28 of the diagonal's (JAC_TOL).  Then P = V, Λ = diag,
// and the new dst basis B_t = B_s·P.  From a warm start the sweep count is small (2-4); from the
// identity (first half-sweep) it is the usual 6-10.  Deterministic: fixed pairing, fixed order.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include "device_common.h"
#include "kernels.h"

namespace albedo {
namespace {

// C = op(A)·op(B) for KP x KP fp64 row-major matrices (TA / TB: transpose), one thread per element
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void dgemm_kp_kernel(const double* __restrict__ A, const double* __restrict__ B,
                                                       double* __restrict__ C, int KP) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= KP * KP) return;
  const int i = e / KP, j = e % KP;
  double acc = 0.0;
  for (int m = 0; m < KP; ++m) {
    const double a = TA ? A[m * KP + i] : A[i * KP + m];
    const double b = TB ? B[j * KP + m] : B[m * KP + j];
    acc = fma(a, b, acc);
  }
  C[e] = acc;
}

constexpr int JAC_THREADS = 1024;
// Sweep budget.  A run that spends it without meeting the tolerance below reports a negative sweep
// count (-(sweeps + 1)), and the engine fails the half-sweep as the host eigensolver it replaced did
// (ALS_E_NOT_POSITIVE_DEFINITE, "did not converge"): the light push-through solves assume Λ is the
// diagonal of the Gram in the basis P.  ALBEDO_JAC_MAX_SWEEPS lowers the budget (test knob).
constexpr int JAC_MAX_SWEEPS = 30;
int jacobi_max_sweeps() {
  const char* e = std::getenv("ALBEDO_JAC_MAX_SWEEPS");
  if (e && *e) return std::max(0, std::min(JAC_MAX_SWEEPS, std::atoi(e)));
  return JAC_MAX_SWEEPS;
}
// Convergence: off-diagonal mass <= 1e-28 of the diagonal's (off-diagonal norm 1e-14 of the diagonal's,
// about fp64 rounding at k <= 256: a backward error of the order of a Householder + QL solve).  The
// small eigenpairs need it: at 1e-9 the directions of eigenvalues near 1e-9·‖G‖ keep components of the
// large ones, and the per-row systems built on them (D = Λ + λn, push-through S = Z D⁻¹ Zᵀ) lose
// positive definiteness in fp32.  Below 1e-20, a sweep that does not halve the mass (the rounding floor) also stops.
constexpr double JAC_TOL = 1e-28;

// round r of the round-robin over n (even) players: pair i = (a, b); player n-1 is fixed
__device__ __forceinline__ void rr_pair(int r, int i, int n, int& a, int& b) {
  const int m = n - 1;
  if (i == 0) {
    a = r % m;
    b = m;
  } else {
    a = (r + i) % m;
    b = (r - i + m) % m;
  }
  if (a > b) { const int t = a; a = b; b = t; }
}

// M (KP x KP, global, the leading k x k block meaningful) -> eigenvalues w[0..k), VT = Vᵀ (in: Wᵀ,
// out: (W·J)ᵀ = Jᵀ·Wᵀ: the rotations act on rows of VT, contiguous in memory).
// LDSM: M is swept in LDS (k <= 128: 129 x 128 doubles); else in place in global memory (the
// workgroup's own stores, ordered by its barriers).
template <bool LDSM>
__global__ __launch_bounds__(JAC_THREADS) void jacobi_kernel(double* __restrict__ Mg, double* __restrict__ VT,
                                                             double* __restrict__ w, int k, int KP, int max_sweeps,
                                                             int* __restrict__ sweeps_out) {
  extern __shared__ double sm[];
  __shared__ double cs[2 * 128];  // c, s of the round's pairs (k <= 256: at most 128 pairs)
  __shared__ int pq[2 * 128];     // p, q
  __shared__ double red[JAC_THREADS / 64][2];
  __shared__ int done;
  double prev_off = INFINITY;  // thread 0's
  const int ld = LDSM ? k + 1 : KP;  // LDS: padded row stride (column walks spread over the banks)
  double* M = LDSM ? sm : Mg;
  const int tid = threadIdx.x;
  if constexpr (LDSM)
    for (int e = tid; e < k * k; e += JAC_THREADS) M[(e / k) * ld + e % k] = Mg[(e / k) * KP + e % k];
  const int n = k + (k & 1);  // players; index k (odd k) is a dummy that never rotates
  const int np = n / 2;
  __syncthreads();
  int sweep = 0;
  for (;; ++sweep) {
    // convergence: off-diagonal mass against the diagonal's (fixed-order block reduction)
    double off = 0.0, dia = 0.0;
    for (int e = tid; e < k * k; e += JAC_THREADS) {
      const int i = e / k, j = e % k;
      const double v = M[i * ld + j];
      if (i == j) dia += v * v;
      else off += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) {
      off += __shfl_xor(off, o);
      dia += __shfl_xor(dia, o);
    }
    if ((tid & 63) == 0) {
      red[tid >> 6][0] = off;
      red[tid >> 6][1] = dia;
    }
    __syncthreads();
    if (tid == 0) {
      double so = 0.0, sd = 0.0;
      for (int i = 0; i < JAC_THREADS / 64; ++i) {
        so += red[i][0];
        sd += red[i][1];
      }
      done = !(so > JAC_TOL * sd) || (!(so > 1e-20 * sd) && !(so < 0.5 * prev_off));  // or at the rounding floor
      if (!done && sweep >= max_sweeps) done = 2;  // the sweep budget is spent: not converged
      prev_off = so;
    }
    __syncthreads();
    if (done) break;
    for (int r = 0; r < n - 1; ++r) {
      if (tid < np) {  // this round's rotation of pair tid
        int p, q;
        rr_pair(r, tid, n, p, q);
        double c = 1.0, s = 0.0;
        if (q < k) {
          const double apq = M[p * ld + q];
          if (apq != 0.0) {
            const double th = (M[q * ld + q] - M[p * ld + p]) / (2.0 * apq);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
            c = 1.0 / sqrt(fma(t, t, 1.0));
            s = t * c;
          }
        }
        cs[tid] = c;
        cs[128 + tid] = s;
        pq[tid] = p;
        pq[128 + tid] = q < k ? q : p;  // the dummy pair rotates nothing
      }
      __syncthreads();
      // rows p, q of M  (M <- Jᵀ M)
      for (int e = tid; e < np * k; e += JAC_THREADS) {
        const int i = e / k, j = e % k;
        const int p = pq[i], q = pq[128 + i];
        if (p == q) continue;
        const double c = cs[i], s = cs[128 + i];
        const double a = M[p * ld + j], b = M[q * ld + j];
        M[p * ld + j] = c * a - s * b;
        M[q * ld + j] = s * a + c * b;
      }
      __syncthreads();
      // columns p, q of M (M <- M J) and of V (V <- V J)
      for (int e = tid; e < np * k; e += JAC_THREADS) {
        const int i = e / k, j = e % k;
        const int p = pq[i], q = pq[128 + i];
        if (p == q) continue;
        const double c = cs[i], s = cs[128 + i];
        const double a = M[j * ld + p], b = M[j * ld + q];
        M[j * ld + p] = c * a - s * b;
        M[j * ld + q] = s * a + c * b;
      }
      for (int e = tid; e < np * KP; e += JAC_THREADS) {  // VT = Vᵀ: rows p, q (contiguous)
        const int i = e / KP, j = e % KP;
        const int p = pq[i], q = pq[128 + i];
        if (p == q) continue;
        const double c = cs[i], s = cs[128 + i];
        const double a = VT[p * KP + j], b = VT[q * KP + j];
        VT[p * KP + j] = c * a - s * b;
        VT[q * KP + j] = s * a + c * b;
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < KP; i += JAC_THREADS) w[i] = i < k ? M[i * ld + i] : 0.0;
  if (tid == 0 && sweeps_out) *sweeps_out = done == 2 ? -sweep - 1 : sweep;  // < 0: did not converge
}

// k <= 128: JAC_WG workgroups sweep identical copies of M in LDS (same code, same inputs, fixed
// order: bit-identical rotations) and each applies the rotations to its own JAC_WG-th of the columns of
// VT, also in LDS, so no global memory is touched inside the sweeps.  One round = the rotations of the
// round's disjoint pairs computed from M, a barrier, then M <- Jᵀ M J as 2 x 2 blocks (pair a's rows x
// pair b's columns: both sides of the similarity in one pass) and VT's rows, a barrier.
constexpr int JAC_WG = 8;
__global__ __launch_bounds__(JAC_THREADS) void jacobi_lds_kernel(const double* __restrict__ Mg, double* __restrict__ VTg,
                                                                 double* __restrict__ w, int k, int KP, int max_sweeps,
                                                                 int* __restrict__ sweeps_out) {
  extern __shared__ double sm[];
  __shared__ double cs[2 * 64];
  __shared__ int pq[2 * 64];
  __shared__ double red[JAC_THREADS / 64][2];
  __shared__ int done;
  double prev_off = INFINITY;  // thread 0's
  const int ld = k + 1;           // M row stride (column walks spread over the banks)
  const int nc = KP / JAC_WG;     // VT columns of this workgroup
  const int c0 = blockIdx.x * nc;
  double* M = sm;
  double* VT = sm + k * ld;       // [KP][nc]
  const int tid = threadIdx.x;
  for (int e = tid; e < k * k; e += JAC_THREADS) M[(e / k) * ld + e % k] = Mg[(e / k) * KP + e % k];
  for (int e = tid; e < KP * nc; e += JAC_THREADS) VT[e] = VTg[(e / nc) * KP + c0 + e % nc];
  const int n = k + (k & 1);  // players; index k (odd k) is a dummy that never rotates
  const int np = n / 2;
  __syncthreads();
  int sweep = 0;
  for (;; ++sweep) {
    double off = 0.0, dia = 0.0;
    for (int e = tid; e < k * k; e += JAC_THREADS) {
      const int i = e / k, j = e % k;
      const double v = M[i * ld + j];
      if (i == j) dia += v * v;
      else off += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) {
      off += __shfl_xor(off, o);
      dia += __shfl_xor(dia, o);
    }
    if ((tid & 63) == 0) {
      red[tid >> 6][0] = off;
      red[tid >> 6][1] = dia;
    }
    __syncthreads();
    if (tid == 0) {
      double so = 0.0, sd = 0.0;
      for (int i = 0; i < JAC_THREADS / 64; ++i) {
        so += red[i][0];
        sd += red[i][1];
      }
      done = !(so > JAC_TOL * sd) || (!(so > 1e-20 * sd) && !(so < 0.5 * prev_off));  // or at the rounding floor
      if (!done && sweep >= max_sweeps) done = 2;  // the sweep budget is spent: not converged
      prev_off = so;
    }
    __syncthreads();
    if (done) break;
    for (int r = 0; r < n - 1; ++r) {
      if (tid < np) {
        int p, q;
        rr_pair(r, tid, n, p, q);
        double c = 1.0, s = 0.0;
        if (q < k) {
          const double apq = M[p * ld + q];
          if (apq != 0.0) {
            const double th = (M[q * ld + q] - M[p * ld + p]) / (2.0 * apq);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
            c = 1.0 / sqrt(fma(t, t, 1.0));
            s = t * c;
          }
        }
        cs[tid] = c;
        cs[64 + tid] = s;
        pq[tid] = p;
        pq[64 + tid] = q;  // q = k: the dummy (odd k), its row / column do not exist
      }
      __syncthreads();
      // M <- Jᵀ M J on 2 x 2 blocks: rows {pa, qa} x columns {pb, qb}
      for (int e = tid; e < np * np; e += JAC_THREADS) {
        const int ia = e / np, ib = e % np;
        const int pa = pq[ia], qa = pq[64 + ia], pb = pq[ib], qb = pq[64 + ib];
        const double ca = cs[ia], sa = cs[64 + ia], cb = cs[ib], sb = cs[64 + ib];
        const bool ha = qa < k, hb = qb < k;
        const double m00 = M[pa * ld + pb];
        const double m01 = hb ? M[pa * ld + qb] : 0.0;
        const double m10 = ha ? M[qa * ld + pb] : 0.0;
        const double m11 = (ha && hb) ? M[qa * ld + qb] : 0.0;
        // rows: [r0; r1] = [ca -sa; sa ca] [m0x; m1x]
        const double r00 = ca * m00 - sa * m10, r01 = ca * m01 - sa * m11;
        const double r10 = sa * m00 + ca * m10, r11 = sa * m01 + ca * m11;
        // columns: [x0 x1] [cb sb; -sb cb]
        M[pa * ld + pb] = r00 * cb - r01 * sb;
        if (hb) M[pa * ld + qb] = r00 * sb + r01 * cb;
        if (ha) M[qa * ld + pb] = r10 * cb - r11 * sb;
        if (ha && hb) M[qa * ld + qb] = r10 * sb + r11 * cb;
      }
      // VT <- Jᵀ VT: rows pa, qa of this workgroup's columns
      for (int e = tid; e < np * nc; e += JAC_THREADS) {
        const int ia = e / nc, j = e % nc;
        const int pa = pq[ia], qa = pq[64 + ia];
        if (qa >= k) continue;
        const double ca = cs[ia], sa = cs[64 + ia];
        const double a = VT[pa * nc + j], b = VT[qa * nc + j];
        VT[pa * nc + j] = ca * a - sa * b;
        VT[qa * nc + j] = sa * a + ca * b;
      }
      __syncthreads();
    }
  }
  for (int e = tid; e < KP * nc; e += JAC_THREADS) VTg[(e / nc) * KP + c0 + e % nc] = VT[e];
  if (blockIdx.x == 0) {
    for (int i = tid; i < KP; i += JAC_THREADS) w[i] = i < k ? M[i * ld + i] : 0.0;
    if (tid == 0 && sweeps_out) *sweeps_out = done == 2 ? -sweep - 1 : sweep;  // < 0: did not converge
  }
}

// P32 = (float) V; lam32 = max(w, 0); ub (the rotation's column-scale bound, als_engine.cpp):
// sqrt(max(w_j, 0) + 1e-6 max(w_max, 0)) * 1.001 as float bits; wmm = {min w, max w}
__global__ __launch_bounds__(256) void eig_finish_kernel(const double* __restrict__ w, const double* __restrict__ VT, int k,
                                                         int KP, float* __restrict__ P32, float* __restrict__ lam32,
                                                         unsigned* __restrict__ ub, double* __restrict__ wmm) {
  __shared__ double smax;
  if (threadIdx.x == 0) {
    double mx = -INFINITY, mn = INFINITY;
    for (int i = 0; i < k; ++i) {
      mx = fmax(mx, w[i]);
      mn = fmin(mn, w[i]);
    }
    smax = mx;
    if (blockIdx.x == 0) {
      wmm[0] = mn;
      wmm[1] = mx;
    }
  }
  __syncthreads();
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < KP * KP; e += gridDim.x * blockDim.x)
    P32[e] = (float)VT[(e % KP) * KP + e / KP];  // P = V = VTᵀ
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < KP; j += blockDim.x) {
      lam32[j] = j < k ? (float)fmax(w[j], 0.0) : 0.f;
      const float u = j < k ? (float)(sqrt(fmax(w[j], 0.0) + 1e-6 * fmax(smax, 0.0)) * 1.001) : 0.f;
      ub[j] = __float_as_uint(u);
    }
}

__global__ void ns_combine_kernel(double* __restrict__ WT, const double* __restrict__ M, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) WT[e] = 1.5 * WT[e] - 0.5 * M[e];
}

__global__ void identity_kernel(double* __restrict__ B, int KP) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < KP * KP) B[e] = (e / KP == e % KP) ? 1.0 : 0.0;
}

// Bt32[i][j] = (float) B[j][i] (the rotation matrix of materialize: original = X · Bᵀ)
__global__ void basis_t32_kernel(const double* __restrict__ B, float* __restrict__ Bt, int KP) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < KP * KP) Bt[e] = (float)B[(e % KP) * KP + e / KP];
}

}  // namespace

size_t eig_scratch_doubles(int KP) { return (size_t)3 * KP * KP + KP + 2 + 2; }

hipError_t launch_device_eig(int KP, int k, const double* G, const double* Bs, const double* Bt_in, double* Bt_out,
                             double* scratch, float* P32, float* lam32, unsigned* ub, hipStream_t s) {
  if (k < 1 || k > KP || KP > 256) return hipErrorInvalidValue;
  double* WT = scratch;              // Wᵀ (warm start), then Vᵀ
  double* T = WT + KP * KP;          // G·W
  double* M = T + KP * KP;           // Wᵀ G W
  double* w = M + KP * KP;           // eigenvalues [KP]
  double* wmm = w + KP;              // {min, max}
  int* sweeps = reinterpret_cast<int*>(wmm + 2);
  const int g = (KP * KP + 255) / 256;
  dgemm_kp_kernel<true, false><<<g, 256, 0, s>>>(Bt_in, Bs, WT, KP);  // Wᵀ = B_tᵀ B_s
  // One Newton-Schulz step towards the orthogonal polar factor: Wᵀ <- (3 Wᵀ - Wᵀ W Wᵀ) / 2.  Without it
  // the warm start couples the two bases' orthogonality errors (P = W·J inherits both, B_t = B_s·P
  // adds them again): they grow ~2.5x per half-sweep, and after ~40 halves the rotated Gram is no
  // longer the Gram of the original factors (measured: tools/debug_c1.py).  One step squares the
  // error (W is orthogonal to rounding plus the previous half's drift).
  dgemm_kp_kernel<false, true><<<g, 256, 0, s>>>(WT, WT, T, KP);     // Wᵀ W
  dgemm_kp_kernel<false, false><<<g, 256, 0, s>>>(T, WT, M, KP);     // Wᵀ W Wᵀ
  ns_combine_kernel<<<g, 256, 0, s>>>(WT, M, KP * KP);
  dgemm_kp_kernel<false, true><<<g, 256, 0, s>>>(G, WT, T, KP);      // G W
  dgemm_kp_kernel<false, false><<<g, 256, 0, s>>>(WT, T, M, KP);     // Wᵀ G W
  if (k <= 128) {
    const size_t lds = ((size_t)k * (k + 1) + (size_t)KP * (KP / JAC_WG)) * sizeof(double);
    static const hipError_t attr = allow_lds(jacobi_lds_kernel, ((size_t)128 * 129 + 128 * 16) * 8);
    if (attr != hipSuccess) return attr;
    jacobi_lds_kernel<<<JAC_WG, JAC_THREADS, lds, s>>>(M, WT, w, k, KP, jacobi_max_sweeps(), sweeps);
  } else {
    jacobi_kernel<false><<<1, JAC_THREADS, 0, s>>>(M, WT, w, k, KP, jacobi_max_sweeps(), sweeps);
  }
  eig_finish_kernel<<<std::max(1, std::min(64, g)), 256, 0, s>>>(w, WT, k, KP, P32, lam32, ub, wmm);
  dgemm_kp_kernel<false, true><<<g, 256, 0, s>>>(Bs, WT, Bt_out, KP);  // B_t = B_s P = B_s (Vᵀ)ᵀ
  // and one Newton-Schulz step on B_t itself: the rotations' roundings (c² + s² = 1 + O(u), a few
  // hundred per row and half-sweep) would otherwise grow the columns' norms linearly over a fit
  // (1e-12 after 60 halves, measured); B_t <- B_t (3I - B_tᵀ B_t) / 2 keeps both bases orthogonal to
  // rounding for any fit length
  dgemm_kp_kernel<true, false><<<g, 256, 0, s>>>(Bt_out, Bt_out, T, KP);  // B_tᵀ B_t
  dgemm_kp_kernel<false, false><<<g, 256, 0, s>>>(Bt_out, T, M, KP);     // B_t B_tᵀ B_t
  ns_combine_kernel<<<g, 256, 0, s>>>(Bt_out, M, KP * KP);
  return hipGetLastError();
}

// {min w, max w} and the Jacobi sweep count of the last launch_device_eig (device pointers into scratch)
const double* eig_minmax(const double* scratch, int KP) { return scratch + (size_t)3 * KP * KP + KP; }
const int* eig_sweeps(const double* scratch, int KP) {
  return reinterpret_cast<const int*>(scratch + (size_t)3 * KP * KP + KP + 2);
}

__global__ void diag_scan_kernel(const void* __restrict__ p, int64_t n, bool f16, unsigned long long* __restrict__ out) {
  unsigned long long bad = 0, first = ~0ull;
  unsigned mx = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = f16 ? (float)reinterpret_cast<const _Float16*>(p)[i] : reinterpret_cast<const float*>(p)[i];
    if (!isfinite(v)) {
      ++bad;
      if ((unsigned long long)i < first) first = (unsigned long long)i;
    } else {
      mx = max(mx, __float_as_uint(fabsf(v)));
    }
  }
  if (bad) {
    atomicAdd(out, bad);
    atomicMin(out + 1, first);
  }
  if (mx) atomicMax(out + 2, (unsigned long long)mx);
}

hipError_t launch_diag_scan(const void* p, int64_t n, bool f16, unsigned long long* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  diag_scan_kernel<<<(int)blocks, 256, 0, s>>>(p, n, f16, out);
  return hipGetLastError();
}

hipError_t launch_identity(double* B, int KP, hipStream_t s) {
  identity_kernel<<<(KP * KP + 255) / 256, 256, 0, s>>>(B, KP);
  return hipGetLastError();
}

hipError_t launch_basis_t32(const double* B, float* Bt, int KP, hipStream_t s) {
  basis_t32_kernel<<<(KP * KP + 255) / 256, 256, 0, s>>>(B, Bt, KP);
  return hipGetLastError();
}

}  // namespace albedo
