// Timing probe (not a test): solve_heavy_kernel phases on synthetic rows.
//   ./heavytime KP NSRC NROWS DEG   -> ms for build-only (PH=1), factor-only (PH=2), full (PH=3)
#define ALBEDO_HEAVY_TIMING
#include "../../albedo_amd/csrc/als_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace albedo;
__device__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void fillZ(float* Z, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Z[i] = ((mix(i) >> 40) * (1.0f / 16777216.0f) - 0.5f) * 0.2f;
}
__global__ void fillCSR(int32_t* col, float* val, int64_t nnz, int64_t nsrc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    col[i] = (int32_t)(mix(i * 7 + 3) % nsrc);
    val[i] = 1.0f;
  }
}
template <int KP, int PH>
float run(const SolveArgs& a, int reps) {
  size_t lds = Heavy<KP>::FLOATS * 4;
  if (getenv("OCC")) { const size_t want = 160 * 1024 / atoi(getenv("OCC")); if (want > lds) lds = want - 64; }
  hipFuncSetAttribute((const void*)solve_heavy_kernel<KP, PH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  solve_heavy_kernel<KP, PH><<<(int)a.n_rows, Heavy<KP>::NTH, lds, 0>>>(a);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) solve_heavy_kernel<KP, PH><<<(int)a.n_rows, Heavy<KP>::NTH, lds, 0>>>(a);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}
template <int KP>
void bench(int64_t nsrc, int nrows, int deg) {
  float *Z, *val, *X, *lam, *cs; int64_t* ptr; int32_t *col, *rows; int* err;
  const int64_t nnz = (int64_t)nrows * deg;
  hipMalloc(&Z, nsrc * KP * 4); hipMalloc(&val, nnz * 4); hipMalloc(&col, nnz * 4); hipMalloc(&X, (size_t)nrows * KP * 4);
  hipMalloc(&lam, KP * 4); hipMalloc(&cs, 2 * KP * 4); hipMalloc(&ptr, (nrows + 1) * 8); hipMalloc(&rows, nrows * 4); hipMalloc(&err, 4);
  fillZ<<<4096, 256>>>(Z, nsrc * KP);
  fillCSR<<<4096, 256>>>(col, val, nnz, nsrc);
  std::vector<int64_t> hp(nrows + 1); std::vector<int32_t> hr(nrows);
  for (int i = 0; i <= nrows; ++i) hp[i] = (int64_t)i * deg;
  for (int i = 0; i < nrows; ++i) hr[i] = i;
  hipMemcpy(ptr, hp.data(), hp.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> hl(KP, 10.f), hc(2 * KP, 1.f);
  for (int i = 0; i < KP; ++i) { hc[i] = 2048.f; hc[KP + i] = 1.f / 2048.f; }
  hipMemcpy(lam, hl.data(), KP * 4, hipMemcpyHostToDevice);
  hipMemcpy(cs, hc.data(), 2 * KP * 4, hipMemcpyHostToDevice);
  hipMemset(err, 0, 4);
  SolveArgs a{};
  a.Z = Z; a.ptr = ptr; a.col = col; a.val = val; a.rows = rows; a.n_rows = nrows; a.lam = lam; a.X = X;
  a.kreal = KP; a.implicit = 1; a.alpha = 40.f; a.reg = 0.5f; a.err = err; a.colscale = cs;
  const double bytes = (double)nnz * (8 + 4.0 * KP) + (nrows + 1) * 8.0 + (double)nrows * 4 * KP;
  const float t1 = run<KP, 1>(a, 3), t2 = run<KP, 2>(a, 3), t3 = run<KP, 3>(a, 3);
  {
    unsigned long long ts[64][48];
    hipMemcpyFromSymbol(ts, HIP_SYMBOL(albedo_heavy_ts), sizeof(ts));
    printf("stamps (cycles from start, block 5): ");
    for (int k = 1; k < 48; ++k) if (ts[5][k] > ts[5][0] && ts[5][k] - ts[5][0] < 100000000ull) printf("%d:%llu ", k, ts[5][k] - ts[5][0]);
    printf("\n");
  }
  printf("KP %d nsrc %lld rows %d deg %d: build-only %.2f ms (%.0f GB/s)  factor-only %.2f ms (%.2f us/row-slot)  full %.2f ms (%.0f GB/s)\n",
         KP, (long long)nsrc, nrows, deg, t1, bytes / t1 / 1e6, t2, t2 * 1e3 / (nrows / 1024.0), t3, bytes / t3 / 1e6);
  hipFree(Z); hipFree(val); hipFree(col); hipFree(X); hipFree(lam); hipFree(cs); hipFree(ptr); hipFree(rows); hipFree(err);
}
int main(int argc, char** argv) {
  const int KP = atoi(argv[1]);
  const int64_t nsrc = atoll(argv[2]);
  const int nrows = atoi(argv[3]), deg = atoi(argv[4]);
  if (KP == 64) bench<64>(nsrc, nrows, deg);
  if (KP == 128) bench<128>(nsrc, nrows, deg);
  if (KP == 256) bench<256>(nsrc, nrows, deg);
  return 0;
}
