// Probe: solve_heavy_kernel on synthetic rows vs an fp64 host solve of the same normal equation.
//   (Λ + λn)I + Σ c z zᵀ) x = Σ w z   with the kernel's own inputs (no engine, no rotation).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include "../../albedo_amd/csrc/kernels.h"
using namespace albedo;
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
  const int nsrc = 600, nrows = 8;
  const int degs[nrows] = {1, 4, 4, 9, 31, 32, 33, 200};
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
    hipError_t e = launch_solve_heavy(KP, a, 0);
    hipDeviceSynchronize();
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
      solve64(k, A, b);
      double me = 0, mx = 0;
      for (int c = 0; c < k; ++c) { me = fmax(me, fabs(X[(size_t)j * KP + c] - b[c])); mx = fmax(mx, fabs(b[c])); }
      printf("  row deg %4d: rel err %.3e\n", d, me / mx);
    }
  }
  return 0;
}
