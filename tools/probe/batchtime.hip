// Timing probe (not a test): nnls_batch_kernel loop phases (cycles per workgroup iteration, wave 0)
//   ./batchtime KP SV NSRC NROWS DEG
// Phases: 0 refill, 1 refresh, 2 grad + r1 reduce, 3 V split/write + Ỹv partials + barrier,
// 4 partial sums + G·V MFMA + barrier, 5 Ỹᵀu + assemble, 6 r2 reduce, 7 wall min, 8 update.
#define ALBEDO_BATCH_TIMING
#include "../../albedo_amd/csrc/nnls_batch.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace albedo;
__device__ uint64_t mixb(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void fillZb(float* Z, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Z[i] = ((mixb(i) >> 40) * (1.0f / 16777216.0f)) * 0.1f;
}
__global__ void fillCSRb(int32_t* col, float* val, int64_t nnz, int64_t nsrc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    col[i] = (int32_t)(mixb(i * 7 + 3) % nsrc);
    val[i] = 1.0f;
  }
}
int main(int argc, char** argv) {
  const int KP = atoi(argv[1]), SV = atoi(argv[2]);
  const int64_t nsrc = atoll(argv[3]);
  const int nrows = atoi(argv[4]), deg = atoi(argv[5]);
  float *Z, *val, *X, *Gt; int64_t* ptr; int32_t *col, *rows; int* err; unsigned long long* it; unsigned* cnt; void* gf;
  const int64_t nnz = (int64_t)nrows * deg;
  hipMalloc(&Z, nsrc * KP * 4); hipMalloc(&val, nnz * 4); hipMalloc(&col, nnz * 4); hipMalloc(&X, (size_t)nrows * KP * 4);
  hipMalloc(&ptr, (nrows + 1) * 8); hipMalloc(&rows, nrows * 4); hipMalloc(&err, 4); hipMalloc(&it, 16); hipMalloc(&cnt, 64);
  hipMalloc(&gf, KP * KP * 4);
  fillZb<<<4096, 256>>>(Z, nsrc * KP);
  fillCSRb<<<4096, 256>>>(col, val, nnz, nsrc);
  std::vector<float> hz(nsrc * KP);
  hipMemcpy(hz.data(), Z, hz.size() * 4, hipMemcpyDeviceToHost);
  std::vector<double> G((size_t)KP * KP, 0.0);
  for (int64_t r = 0; r < nsrc; ++r)
    for (int i = 0; i < KP; ++i)
      for (int j = 0; j <= i; ++j) G[(size_t)i * KP + j] += (double)hz[r * KP + i] * hz[r * KP + j];
  const int ngt = (KP / 16) * (KP / 16 + 1) / 2 * 256;
  std::vector<float> gt(ngt, 0.f);
  double gmax = 0;
  for (int i = 0; i < KP; ++i)
    for (int j = 0; j < 16 * ((i >> 4) + 1); ++j) {
      const double v = j <= i ? G[(size_t)i * KP + j] : G[(size_t)j * KP + i];
      gt[nel(i, j)] = (float)v;
      gmax = std::max(gmax, std::fabs(v));
    }
  int ex; std::frexp(gmax, &ex);
  const float gs = (float)std::ldexp(1.0, 15 - ex);
  hipMalloc(&Gt, ngt * 4);
  hipMemcpy(Gt, gt.data(), ngt * 4, hipMemcpyHostToDevice);
  std::vector<int64_t> hp(nrows + 1); std::vector<int32_t> hr(nrows);
  for (int i = 0; i <= nrows; ++i) hp[i] = (int64_t)i * deg;
  for (int i = 0; i < nrows; ++i) hr[i] = i;
  hipMemcpy(ptr, hp.data(), hp.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice);
  hipMemset(err, 0, 4); hipMemset(it, 0, 16);
  SolveArgs a{};
  a.Z = Z; a.ptr = ptr; a.col = col; a.val = val; a.rows = rows; a.n_rows = nrows; a.X = X;
  a.kreal = KP; a.implicit = 1; a.alpha = 40.f; a.reg = 0.5f; a.err = err; a.iters = it;
  launch_nnls_gfrag(KP, Gt, gs, gf, 0);
  launch_nnls_batch(KP, SV, a, gf, gs, cnt, 256, 0);
  hipMemset(it, 0, 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  launch_nnls_batch(KP, SV, a, gf, gs, cnt, 256, 0);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long hit[2]; hipMemcpy(hit, it, 16, hipMemcpyDeviceToHost);
  unsigned long long ph[64][9];
  hipMemcpyFromSymbol(ph, HIP_SYMBOL(albedo_batch_ph), sizeof(ph));
  double tot[9] = {0}, s = 0;
  for (int b = 0; b < 64; ++b) for (int q = 0; q < 9; ++q) tot[q] += ph[b][q];
  for (int q = 0; q < 9; ++q) s += tot[q];
  const double wg_iters = (double)hit[0] / SV;  // approx (slots busy)
  printf("KP %d SV %d rows %d deg %d: %.2f ms, mean iterations %.1f (max %llu); %.3f us per row-iteration (chip)\n", KP, SV,
         nrows, deg, ms, (double)hit[0] / nrows, hit[1], ms * 1e3 / hit[0] * 256);
  printf("phase cycles per WG-iteration (64 WGs): ");
  const double per = s / (wg_iters * 64.0 / ((nrows + SV - 1) / SV < 256 ? (nrows + SV - 1) / SV : 256));
  for (int q = 0; q < 9; ++q) printf("%d:%.0f ", q, tot[q] / s * per);
  printf(" total %.0f\n", per);
  int herr; hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
  printf("err %d\n", herr);
  return 0;
}
