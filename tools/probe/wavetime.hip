// Timing probe (not a test): solve_wave_kernel<128> (PRE path, the c4 default) on synthetic rows of a
// fixed degree gathered from a 20M-row pre-split table (HBM-resident like c4's Z_user).
//   ./wavetime NSRC "d1,d2,..." STARS_PER_TEST      (build with -DWAVE_PROBE_STAMPS)
//   ./wavetime_bo ...                                (+ -DWAVE_PROBE_BUILD_ONLY: the factor skipped)
// Prints per degree: ms per launch, algorithmic GB/s (SURVEY §8(d) bytes), and from the per-row
// shader-clock stamps the mean build / factor / store cycles of a row.
#include "../../albedo_amd/csrc/heavy_wave.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
using namespace albedo;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// pre-split rows: fp16 hi of values in [-1, 1), lo = 0 (timing does not depend on the values)
__global__ void fill_hl(_Float16* Zhl, int64_t nrow, int KP) {
  const int64_t n = nrow * 2 * KP;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % (2 * KP));
    Zhl[i] = c < KP ? (_Float16)(((mix64(i) >> 40) * (1.0f / 8388608.0f)) - 1.0f) : (_Float16)0.f;
  }
}
__global__ void fill_csr(int32_t* col, float* val, int64_t nnz, int64_t nsrc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    col[i] = (int32_t)(mix64(i * 7 + 3) % nsrc);
    val[i] = 1.0f;
  }
}

int main(int argc, char** argv) {
  constexpr int KP = 128;
  const int64_t nsrc = argc > 1 ? atoll(argv[1]) : 20000000;
  std::vector<int> degs;
  {
    std::string s = argc > 2 ? argv[2] : "80,160,320,640,1280,4096";
    size_t p = 0;
    while (p < s.size()) { degs.push_back(atoi(s.c_str() + p)); p = s.find(',', p); if (p == std::string::npos) break; ++p; }
  }
  const int64_t stars = argc > 3 ? atoll(argv[3]) : 200000000;
  void* Zhl; float *Z, *val, *X, *lam, *cs; int64_t* ptr; int32_t *col, *rows; int* err; unsigned long long* stamps;
  CK(hipMalloc(&Zhl, (nsrc + 1) * KP * 4));
  CK(hipMalloc(&Z, 16 * KP * 4));
  fill_hl<<<8192, 256>>>((_Float16*)Zhl, nsrc + 1, KP);
  CK(hipMemset((char*)Zhl + nsrc * KP * 4, 0, KP * 4));
  CK(hipMalloc(&val, stars * 4)); CK(hipMalloc(&col, stars * 4));
  fill_csr<<<8192, 256>>>(col, val, stars, nsrc);
  const int64_t maxrows = stars / 65 + 1;
  CK(hipMalloc(&X, maxrows * KP * 4)); CK(hipMalloc(&ptr, (maxrows + 1) * 8)); CK(hipMalloc(&rows, maxrows * 4));
  CK(hipMalloc(&lam, KP * 4)); CK(hipMalloc(&cs, 2 * KP * 4)); CK(hipMalloc(&err, 4));
  CK(hipMalloc(&stamps, maxrows * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_stamps), &stamps, sizeof(stamps)));
  std::vector<float> hl(KP, 10.f), hc(2 * KP, 1.f);
  CK(hipMemcpy(lam, hl.data(), KP * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(cs, hc.data(), 2 * KP * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int deg : degs) {
    const int64_t nrows = stars / deg;
    std::vector<int64_t> hp(nrows + 1); std::vector<int32_t> hr(nrows);
    for (int64_t i = 0; i <= nrows; ++i) hp[i] = i * deg;
    for (int64_t i = 0; i < nrows; ++i) hr[i] = (int32_t)i;
    CK(hipMemcpy(ptr, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(err, 0, 4));
    SolveArgs a{};
    a.Z = Z; a.Zhl = Zhl; a.zero_row = nsrc; a.wsc = 1.f; a.inv_sw = 1.f;
    a.ptr = ptr; a.col = col; a.val = val; a.rows = rows; a.n_rows = nrows; a.lam = lam; a.X = X;
    a.kreal = KP; a.implicit = 1; a.alpha = 40.f; a.reg = 0.5f; a.err = err; a.colscale = cs; a.n_cu = 256;
    CK(launch_solve_wave(KP, a, 0));
    CK(hipDeviceSynchronize());
    const int reps = 3;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) CK(launch_solve_wave(KP, a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::vector<unsigned long long> ts(nrows * 4);
    CK(hipMemcpy(ts.data(), stamps, ts.size() * 8, hipMemcpyDeviceToHost));
    double sb = 0, sf = 0, ss = 0; int64_t n = 0;
    for (int64_t i = 0; i < nrows; i += 7) {
      const unsigned long long* t = &ts[i * 4];
      if (t[1] < t[0]) continue;
#ifndef WAVE_PROBE_BUILD_ONLY
      if (t[3] < t[1]) continue;
#endif
      sb += (double)(t[1] - t[0]);
#ifndef WAVE_PROBE_BUILD_ONLY
      sf += (double)(t[2] - t[1]); ss += (double)(t[3] - t[2]);
#endif
      ++n;
    }
    const double bytes = (double)nrows * deg * (8 + 4.0 * KP) + (nrows + 1) * 8.0 + (double)nrows * 4 * KP;
    int herr = 0; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("deg %5d rows %8lld: %8.3f ms  %6.0f GB/s alg  cycles/row build %9.0f factor %8.0f store %6.0f  (%.1f ns/row-launch, err %d)\n",
           deg, (long long)nrows, ms, bytes / ms / 1e6, n ? sb / n : 0.0, n ? sf / n : 0.0, n ? ss / n : 0.0,
           ms * 1e6 / nrows, herr);
    fflush(stdout);
  }
  return 0;
}
