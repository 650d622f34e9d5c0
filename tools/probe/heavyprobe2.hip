// Probe: solve_heavy_kernel on synthetic rows vs an fp64 host solve of the same normal equation.
//   (Λ + λn)I + Σ c z zᵀ) x = Σ w z   with the kernel's own inputs (no engine, no rotation).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include "../../albedo_amd/csrc/als_kernels.hip"
using namespace albedo;
template <int KP>
__global__ __launch_bounds__(Heavy<KP>::NTH) void dump_build_kernel(SolveArgs a, float* outA, float* outb) {
  using H = Heavy<KP>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* s_flag = reinterpret_cast<int*>(smem + H::OFF_FLAG);
  const int tid = threadIdx.x;
  const int j = a.rows[blockIdx.x];
  const int64_t p0 = a.ptr[j];
  const int d = (int)(a.ptr[j + 1] - p0);
  if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; }
  heavy_build_all<KP>(a, p0, d, smem);
  for (int e = tid; e < KP * KP; e += H::NTH) {
    const int r = e / KP, c = e % KP;
    outA[(size_t)blockIdx.x * KP * KP + e] = smem[r >= c ? hel(r, c) : hel(c, r)];
  }
  for (int c = tid; c < KP; c += H::NTH) outb[(size_t)blockIdx.x * KP + c] = smem[H::OFF_B + c];
}

static void solve64(int k, std::vector<double>& A, std::vector<double>& b) {  // Cholesky in place
  for (int j = 0; j < k; ++j) {
    double s = A[j * k + j];
    for (int m = 0; m < j; ++m) s -= A[j * k + m] * A[j * k + m];
    const double d = sqrt(s);
    A[j * k + j] = d;
    for (int i = j + 1; i < k; ++i) {
      double t = A[i * k + j];
      for (int m = 0; m < j; ++m) t -= A[i * k + m] * A[j * k + m];
      A[i * k + j] = t / d;
    }
  }
  for (int i = 0; i < k; ++i) { double s = b[i]; for (int m = 0; m < i; ++m) s -= A[i * k + m] * b[m]; b[i] = s / A[i * k + i]; }
  for (int i = k - 1; i >= 0; --i) { double s = b[i]; for (int m = i + 1; m < k; ++m) s -= A[m * k + i] * b[m]; b[i] = s / A[i * k + i]; }
}
int main(int argc, char** argv) {
  const int KP = argc > 1 ? atoi(argv[1]) : 64, k = argc > 2 ? atoi(argv[2]) : 50;
  const int nsrc = 600;
  const int nrows = argc > 3 ? atoi(argv[3]) : 8;
  std::vector<int> degs(nrows);
  for (int j = 0; j < nrows; ++j) degs[j] = 1 + (j * 7) % 64;
  std::mt19937 rng(3);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> Z((size_t)nsrc * KP, 0.f), lam(KP, 0.f);
  for (int c = 0; c < k; ++c) lam[c] = 50.f * expf(-0.1f * c) + 0.01f;
  for (int r = 0; r < nsrc; ++r) for (int c = 0; c < k; ++c) Z[(size_t)r * KP + c] = nd(rng) * sqrtf(lam[c] / nsrc);
  std::vector<int64_t> ptr(nrows + 1, 0);
  std::vector<int32_t> col, rows(nrows);
  std::vector<float> val;
  for (int j = 0; j < nrows; ++j) {
    rows[j] = j;
    for (int e = 0; e < degs[j]; ++e) { col.push_back((int32_t)(rng() % nsrc)); val.push_back(1.0f); }
    ptr[j + 1] = (int64_t)col.size();
  }
  float *dZ, *dlam, *dX, *dval, *dcs; int64_t* dptr; int32_t *dcol, *drows; int* derr; unsigned* dtmp;
  hipMalloc(&dZ, Z.size() * 4); hipMalloc(&dlam, KP * 4); hipMalloc(&dX, (size_t)nrows * KP * 4);
  hipMalloc(&dval, val.size() * 4); hipMalloc(&dptr, ptr.size() * 8); hipMalloc(&dcol, col.size() * 4);
  hipMalloc(&drows, nrows * 4); hipMalloc(&derr, 4); hipMalloc(&dcs, 2 * KP * 4); hipMalloc(&dtmp, KP * 4);
  hipMemcpy(dZ, Z.data(), Z.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dlam, lam.data(), KP * 4, hipMemcpyHostToDevice);
  hipMemcpy(dval, val.data(), val.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dptr, ptr.data(), ptr.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dcol, col.data(), col.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(drows, rows.data(), nrows * 4, hipMemcpyHostToDevice);
  hipMemset(derr, 0, 4);
  const float alpha = 40.f, reg = 0.5f;
  for (int scaled = 0; scaled < 2; ++scaled) {
    if (scaled) launch_colscale(KP, dZ, nsrc, alpha, dtmp, dcs, 0);
    else { std::vector<float> one(2 * KP, 1.f); hipMemcpy(dcs, one.data(), 2 * KP * 4, hipMemcpyHostToDevice); }
    SolveArgs a{};
    a.Z = dZ; a.ptr = dptr; a.col = dcol; a.val = dval; a.rows = drows; a.n_rows = nrows; a.lam = dlam; a.X = dX;
    a.kreal = k; a.implicit = 1; a.alpha = alpha; a.reg = reg; a.err = derr; a.colscale = dcs;
    hipError_t e;
    const char* big = getenv("BIGLDS");
    if (big && KP == 64) {
      const size_t lds = (size_t)atoi(big);
      hipFuncSetAttribute((const void*)solve_heavy_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      solve_heavy_kernel<64><<<nrows, 256, lds, 0>>>(a); e = hipGetLastError();
    } else e = launch_solve_heavy(KP, a, 0);
    hipDeviceSynchronize();
    std::vector<float> hA((size_t)nrows * KP * KP), hb((size_t)nrows * KP);
    if (KP == 64) {
      float *dA, *db; hipMalloc(&dA, hA.size() * 4); hipMalloc(&db, hb.size() * 4);
      dump_build_kernel<64><<<nrows, 256, Heavy<64>::FLOATS * 4, 0>>>(a, dA, db);
      hipMemcpy(hA.data(), dA, hA.size() * 4, hipMemcpyDeviceToHost);
      hipMemcpy(hb.data(), db, hb.size() * 4, hipMemcpyDeviceToHost);
    }
    std::vector<float> X((size_t)nrows * KP);
    hipMemcpy(X.data(), dX, X.size() * 4, hipMemcpyDeviceToHost);
    int err = 0; hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost);
    printf("KP %d k %d colscale %s: launch %d err %d\n", KP, k, scaled ? "on" : "off(1)", (int)e, err);
    for (int j = 0; j < nrows; ++j) {
      std::vector<double> A((size_t)k * k, 0.0), b(k, 0.0);
      const int d = degs[j];
      for (int c = 0; c < k; ++c) A[c * k + c] = lam[c] + (double)reg * d;
      for (int64_t p = ptr[j]; p < ptr[j + 1]; ++p) {
        const float* z = &Z[(size_t)col[p] * KP];
        const double cc = alpha * 1.0, w = 1.0 + cc;
        for (int r = 0; r < k; ++r) { b[r] += w * z[r]; for (int c = 0; c < k; ++c) A[r * k + c] += cc * z[r] * (double)z[c]; }
      }
      std::vector<double> As(A), bs(b);
      {  // emulated split-fp16 build: hi·hi + hi·lo + lo·hi of v = √c z · cs (host fp64 sums)
        std::vector<float> cs(2 * KP);
        hipMemcpy(cs.data(), dcs, 2 * KP * 4, hipMemcpyDeviceToHost);
        for (int r = 0; r < k; ++r) for (int c = 0; c < k; ++c) As[r * k + c] = (r == c) ? lam[c] + (double)reg * d : 0.0;
        for (int64_t p = ptr[j]; p < ptr[j + 1]; ++p) {
          const float* z = &Z[(size_t)col[p] * KP];
          std::vector<double> hi(k), lo(k);
          for (int r = 0; r < k; ++r) {
            const float v = z[r] * (sqrtf(alpha) * cs[r]);
            const _Float16 h = (_Float16)v; hi[r] = (double)(float)h; lo[r] = (double)(float)(_Float16)(v - (float)h);
            hi[r] /= cs[r]; lo[r] /= cs[r];
          }
          for (int r = 0; r < k; ++r) for (int c = 0; c < k; ++c) As[r * k + c] += hi[r] * hi[c] + hi[r] * lo[c] + lo[r] * hi[c];
        }
      }
      if (scaled && KP == 64 && j < 400) {  // compare the kernel's Σ c z zᵀ tiles with the emulated split sums
        double worst = 0; int wr = -1, wc = -1;
        for (int r = 0; r < k; ++r) for (int c = 0; c < k; ++c) {
          const double em = As[r * k + c] - ((r == c) ? lam[c] + (double)reg * d : 0.0);
          const double ex = A[r * k + c] - ((r == c) ? lam[c] + (double)reg * d : 0.0);
          const double dv = fabs(hA[(size_t)j * KP * KP + r * KP + c] - em) / (fabs(ex) + 1e-30);
          if (fabs(hA[(size_t)j * KP * KP + r * KP + c] - em) > 1e-5 * sqrt(fabs(A[r*k+r]*A[c*k+c])) && dv > worst) { worst = dv; wr = r; wc = c; }
        }
        if (wr >= 0) printf("  row %d: A entry (%d,%d) kernel %.9g emul %.9g exact %.9g\n", j, wr, wc, hA[(size_t)j*KP*KP+wr*KP+wc],
                            As[wr*k+wc] - ((wr==wc) ? lam[wc] + (double)reg * d : 0.0), A[wr*k+wc] - ((wr==wc) ? lam[wc] + (double)reg * d : 0.0));
      }
      solve64(k, A, b);
      solve64(k, As, bs);
      double mes = 0;
      for (int c = 0; c < k; ++c) mes = fmax(mes, fabs(bs[c] - b[c]));
      double me = 0, mx = 0;
      for (int c = 0; c < k; ++c) { me = fmax(me, fabs(X[(size_t)j * KP + c] - b[c])); mx = fmax(mx, fabs(b[c])); }
      if (me / mx > 1e-5 || j < 4) printf("  row %d deg %4d: rel err %.3e  emulated split %.3e\n", j, d, me / mx, mes / mx);
    }
  }
  return 0;
}
