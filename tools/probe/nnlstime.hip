// Timing probe (not a test): solve_nnls_kernel loop phases (cycles per iteration, wave 0's view)
//   ./nnlstime KP NSRC NROWS DEG
// Phases: 0 residual/grad, 1 r1 reduce, 2 v write + barrier, 3 products, 4 barrier after products,
// 5 r2 reduce, 6 wall min, 7 update.  G = the Gram of the random (nonnegative) src factors.
#define ALBEDO_NNLS_TIMING
#include "../../albedo_amd/csrc/als_kernels.hip"
#include "../../albedo_amd/csrc/nnls_row.hip"
#include "../../albedo_amd/csrc/heavy_wave.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace albedo;
__device__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void fillZ(float* Z, int64_t n, int KP, int kreal) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Z[i] = (i % KP) < kreal ? ((mix(i) >> 40) * (1.0f / 16777216.0f)) * 0.1f : 0.f;
}
__global__ void fillCSR(int32_t* col, float* val, int64_t nnz, int64_t nsrc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    col[i] = (int32_t)(mix(i * 7 + 3) % nsrc);
    val[i] = 1.0f;
  }
}
template <int KP>
void bench(int64_t nsrc, int nrows, int deg) {
  float *Z, *val, *X, *lam, *cs, *Gt; int64_t* ptr; int32_t *col, *rows; int* err; unsigned long long* it;
  const int64_t nnz = (int64_t)nrows * deg;
  hipMalloc(&Z, nsrc * KP * 4); hipMalloc(&val, nnz * 4); hipMalloc(&col, nnz * 4); hipMalloc(&X, (size_t)nrows * KP * 4);
  hipMalloc(&lam, KP * 4); hipMalloc(&cs, 2 * KP * 4); hipMalloc(&ptr, (nrows + 1) * 8); hipMalloc(&rows, nrows * 4);
  hipMalloc(&err, 4); hipMalloc(&it, 16);
  fillZ<<<4096, 256>>>(Z, nsrc * KP, KP, KP);
  fillCSR<<<4096, 256>>>(col, val, nnz, nsrc);
  std::vector<float> hz(nsrc * KP);
  hipMemcpy(hz.data(), Z, hz.size() * 4, hipMemcpyDeviceToHost);
  std::vector<double> G((size_t)KP * KP, 0.0);
  for (int64_t r = 0; r < nsrc; ++r)
    for (int i = 0; i < KP; ++i)
      for (int j = 0; j <= i; ++j) G[(size_t)i * KP + j] += (double)hz[r * KP + i] * hz[r * KP + j];
  const int ngt = nnls_gtile_floats(KP);
  std::vector<float> gt(ngt, 0.f);
  for (int i = 0; i < KP; ++i)
    for (int j = 0; j < 16 * ((i >> 4) + 1); ++j) gt[nnls_gtile_index(i, j)] = (float)(j <= i ? G[(size_t)i * KP + j] : G[(size_t)j * KP + i]);
  hipMalloc(&Gt, ngt * 4);
  hipMemcpy(Gt, gt.data(), ngt * 4, hipMemcpyHostToDevice);
  std::vector<int64_t> hp(nrows + 1); std::vector<int32_t> hr(nrows);
  for (int i = 0; i <= nrows; ++i) hp[i] = (int64_t)i * deg;
  for (int i = 0; i < nrows; ++i) hr[i] = i;
  hipMemcpy(ptr, hp.data(), hp.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> hl(KP, 0.f), hc(2 * KP, 1.f);
  for (int i = 0; i < KP; ++i) { hc[i] = 2048.f; hc[KP + i] = 1.f / 2048.f; }
  hipMemcpy(lam, hl.data(), KP * 4, hipMemcpyHostToDevice);
  hipMemcpy(cs, hc.data(), 2 * KP * 4, hipMemcpyHostToDevice);
  hipMemset(err, 0, 4); hipMemset(it, 0, 16);
  SolveArgs a{};
  a.Z = Z; a.ptr = ptr; a.col = col; a.val = val; a.rows = rows; a.n_rows = nrows; a.lam = lam; a.X = X;
  a.kreal = KP; a.implicit = 1; a.alpha = 40.f; a.reg = 0.5f; a.err = err; a.colscale = cs; a.iters = it;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  // the other per-row kernel's X first (ALBEDO_NNLS_ROW=1024 <-> the 512-thread one at KP = 256)
  std::vector<float> xo((size_t)nrows * KP), xn((size_t)nrows * KP);
  const char* sel = getenv("ALBEDO_NNLS_ROW");
  const bool is_old = sel && atoi(sel) == 1024;
  if (KP == 256) {
    setenv("ALBEDO_NNLS_ROW", is_old ? "512" : "1024", 1);
    launch_solve_nnls(KP, a, Gt, 0);
    hipMemcpy(xo.data(), X, xo.size() * 4, hipMemcpyDeviceToHost);
    setenv("ALBEDO_NNLS_ROW", is_old ? "1024" : "512", 1);
  }
  launch_solve_nnls(KP, a, Gt, 0);
  hipMemset(it, 0, 16);
  hipEventRecord(e0, 0);
  launch_solve_nnls(KP, a, Gt, 0);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  if (KP == 256) {
    hipMemcpy(xn.data(), X, xn.size() * 4, hipMemcpyDeviceToHost);
    double num = 0, den = 0, worst = 0; long zero_mismatch = 0;
    for (int r = 0; r < nrows; ++r) {
      double rn = 0, rd = 0;
      for (int c = 0; c < KP; ++c) {
        const double dlt = (double)xn[(size_t)r * KP + c] - xo[(size_t)r * KP + c];
        rn = fmax(rn, fabs(dlt)); rd = fmax(rd, fabs((double)xo[(size_t)r * KP + c]));
        zero_mismatch += (xn[(size_t)r * KP + c] == 0.f) != (xo[(size_t)r * KP + c] == 0.f);
      }
      num = fmax(num, rn); den = fmax(den, rd); worst = fmax(worst, rd > 0 ? rn / rd : rn);
    }
    int herr = 0; hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
    printf("%s vs the other kernel: max|dx|/max|x| %.3e, worst row %.3e, zero-pattern mismatches %ld, err %d\n",
           is_old ? "1024-thread" : "512-thread", den > 0 ? num / den : num, worst, zero_mismatch, herr);
  }
  unsigned long long hit[2]; hipMemcpy(hit, it, 16, hipMemcpyDeviceToHost);
  unsigned long long ph[64][8];
  hipMemcpyFromSymbol(ph, HIP_SYMBOL(albedo_nnls_ph), sizeof(ph));
  double tot[8] = {0}; unsigned long long iters = 0;
  for (int b = 0; b < 64 && b < nrows; ++b) for (int q = 0; q < 8; ++q) tot[q] += ph[b][q];
  const double mean_it = (double)hit[0] / nrows;
  printf("KP %d rows %d deg %d: %.2f ms, mean iterations %.1f (max %llu), %.2f us per row-iteration per CU\n", KP, nrows, deg, ms,
         mean_it, hit[1], ms * 1e3 / (hit[0] / 256.0));
  double s = 0; for (int q = 0; q < 8; ++q) s += tot[q];
  printf("phase share (64 blocks): ");
  for (int q = 0; q < 8; ++q) printf("%d:%.3f ", q, tot[q] / s);
  printf("\ncycles per iteration (block 0..63 avg): %.0f\n", s / (hit[0] * 64.0 / nrows));
  if (KP == 256 && !is_old) {  // the 512-thread kernel: waves 0 (owner) and 6 (diagonal groups)
    unsigned long long nph[64][2][8];
    hipMemcpyFromSymbol(nph, HIP_SYMBOL(albedo_nrow_ph), sizeof(nph));
    const double its = hit[0] * 64.0 / nrows;
    for (int w = 0; w < 2; ++w) {
      printf("512-thread wave %d cycles per iteration by phase (0 pre-B1, 1 B1, 2 product, 3 post-product, 4 B2, 5 step, 6 refresh, 7 build/iter):", w ? 6 : 0);
      for (int q = 0; q < 8; ++q) {
        double t = 0; for (int b = 0; b < 64 && b < nrows; ++b) t += nph[b][w][q];
        printf(" %.0f", t / its);
      }
      printf("\n");
    }
  }
  (void)iters;
}
int main(int argc, char** argv) {
  const int KP = atoi(argv[1]);
  const int64_t nsrc = atoll(argv[2]);
  const int nrows = atoi(argv[3]), deg = atoi(argv[4]);
  if (KP == 128) bench<128>(nsrc, nrows, deg);
  if (KP == 256) bench<256>(nsrc, nrows, deg);
  return 0;
}
