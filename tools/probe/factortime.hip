// Timing probe (not a test): the wave kernel's factorisation alone (WAVE_PROBE_FACTOR_ONLY: a
// synthetic SPD system instead of the build) at 2 waves per SIMD (the kernel's occupancy) and at 1
// (one workgroup per CU, forced by the LDS request): cycles per row from the shader-clock stamps.
//   ./factortime NROWS
#define WAVE_PROBE_STAMPS
#define WAVE_PROBE_FACTOR_ONLY
#define WAVE_PROBE_CHOL_PHASES
#include "../../albedo_amd/csrc/heavy_wave.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace albedo;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
int main(int argc, char** argv) {
  constexpr int KP = 128;
  using W = WaveRow<KP>;
  const int64_t nrows = argc > 1 ? atoll(argv[1]) : 1000000;
  float *X, *lam, *cs; int64_t* ptr; int32_t* rows; int* err; unsigned long long* stamps;
  CK(hipMalloc(&X, nrows * KP * 4)); CK(hipMalloc(&ptr, (nrows + 1) * 8)); CK(hipMalloc(&rows, nrows * 4));
  CK(hipMalloc(&lam, KP * 4)); CK(hipMalloc(&cs, 2 * KP * 4)); CK(hipMalloc(&err, 4));
  CK(hipMalloc(&stamps, nrows * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_stamps), &stamps, sizeof(stamps)));
  unsigned long long* ph;
  CK(hipMalloc(&ph, nrows * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chol_ph), &ph, sizeof(ph)));
  std::vector<int64_t> hp(nrows + 1); std::vector<int32_t> hr(nrows);
  for (int64_t i = 0; i <= nrows; ++i) hp[i] = i * 80;
  for (int64_t i = 0; i < nrows; ++i) hr[i] = (int32_t)i;
  CK(hipMemcpy(ptr, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> hl(KP, 10.f), hc(2 * KP, 1.f);
  CK(hipMemcpy(lam, hl.data(), KP * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(cs, hc.data(), 2 * KP * 4, hipMemcpyHostToDevice));
  CK(hipMemset(err, 0, 4));
  SolveArgs a{};
  a.ptr = ptr; a.rows = rows; a.n_rows = nrows; a.lam = lam; a.X = X; a.kreal = KP; a.implicit = 1; a.alpha = 40.f;
  a.reg = 0.5f; a.err = err; a.colscale = cs; a.n_cu = 256;
  auto k = solve_wave_kernel<KP, true, false>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int occ : {2, 1}) {
    const size_t lds = occ == 2 ? W::LDS : 100 * 1024;
    const int blocks = (int)((nrows + W::WAVES - 1) / W::WAVES);
    k<<<blocks, 64 * W::WAVES, lds, 0>>>(a);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    k<<<blocks, 64 * W::WAVES, lds, 0>>>(a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> ts(nrows * 4);
    CK(hipMemcpy(ts.data(), stamps, ts.size() * 8, hipMemcpyDeviceToHost));
    double sf = 0; int64_t n = 0;
    for (int64_t i = 0; i < nrows; i += 7) {
      const unsigned long long* t = &ts[i * 4];
      if (t[2] < t[1]) continue;
      sf += (double)(t[2] - t[1]);
      ++n;
    }
    std::vector<unsigned long long> hph(nrows * 8);
    CK(hipMemcpy(hph.data(), ph, hph.size() * 8, hipMemcpyDeviceToHost));
    double pa[8] = {0}; int64_t pn = 0;
    for (int64_t i = 0; i < nrows; i += 7, ++pn)
      for (int q = 0; q < 8; ++q) pa[q] += (double)hph[i * 8 + q];
    printf("  phases (cycles/row): diag-to-rows %.0f  elim16 %.0f  image+U %.0f  trailing %.0f  rhs %.0f  sync %.0f  back-sub %.0f\n",
           pa[0] / pn, pa[1] / pn, pa[2] / pn, pa[3] / pn, pa[4] / pn, pa[5] / pn, pa[6] / pn);
    int herr = 0; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("waves/SIMD %d: %8.3f ms for %lld rows (%.1f ns/row), factor cycles/row %.0f, err %d\n", occ, ms,
           (long long)nrows, ms * 1e6 / nrows, n ? sf / n : 0.0, herr);
  }
  return 0;
}
