/*
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): C/OpenMP restatement of albedo's top-k scorer,
 * the same definition as oracle/spark_als.py:recommend_for_all, for full-size parity checks.
 *   score(s, t)   F2J sdot (ALSRecommender.scala:51): fp32 products added left to right, no FMA
 *                 (this file is compiled with -ffp-contract=off; the 5-way unroll of sdot.f is
 *                 left-to-right too, so the order is plain sequential)
 *   top-k         BoundedPriorityQueue over dst rows in ascending id order (BoundedPriorityQueue.scala:
 *                 45-53: replace the lowest only when strictly greater, so ties keep the lower id) +
 *                 TopByKeyAggregator's sort = the best `num` by (score desc, id asc)
 * The dst rows are visited in blocks of 64, transposed, so the sequential sum over the rank runs
 * along SIMD lanes of 64 independent rows (the per-row order is unchanged).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* worse(a, b): a ranks below b under (score desc, id asc) */
static inline int worse(float sa, int32_t ia, float sb, int32_t ib) { return sa < sb || (sa == sb && ia > ib); }

static void heap_down(float* hs, int32_t* hi, int n, int i) {
  for (;;) {
    int l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && worse(hs[l], hi[l], hs[m], hi[m])) m = l;
    if (r < n && worse(hs[r], hi[r], hs[m], hi[m])) m = r;
    if (m == i) return;
    float ts = hs[i]; hs[i] = hs[m]; hs[m] = ts;
    int32_t ti = hi[i]; hi[i] = hi[m]; hi[m] = ti;
    i = m;
  }
}
static void heap_up(float* hs, int32_t* hi, int i) {
  while (i > 0) {
    int p = (i - 1) / 2;
    if (!worse(hs[i], hi[i], hs[p], hi[p])) return;
    float ts = hs[i]; hs[i] = hs[p]; hs[p] = ts;
    int32_t ti = hi[i]; hi[i] = hi[p]; hi[p] = ti;
    i = p;
  }
}

/* src_f [n_src][k], dst_f [n_dst][k] with dst_ids ascending; out [n_src][num] (-1 / NaN padded) */
int oracle_recommend(int64_t n_src, const float* src_f, int64_t n_dst, const int32_t* dst_ids, const float* dst_f,
                     int k, int num, int32_t* out_ids, float* out_sc, int nthreads) {
  for (int64_t j = 1; j < n_dst; ++j)
    if (dst_ids[j] <= dst_ids[j - 1]) return -2;
  const int64_t nb = (n_dst + 63) / 64;
  float* Tt = malloc(sizeof(float) * (size_t)nb * 64 * k); /* block b: [k][64] */
  if (!Tt) return -1;
#pragma omp parallel for num_threads(nthreads) schedule(static)
  for (int64_t b = 0; b < nb; ++b)
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < 64; ++j) {
        const int64_t r = b * 64 + j;
        Tt[((size_t)b * k + i) * 64 + j] = r < n_dst ? dst_f[r * k + i] : 0.f;
      }
  const int m = num < n_dst ? num : (int)n_dst;
#pragma omp parallel num_threads(nthreads)
  {
    float* hs = malloc(sizeof(float) * (m > 0 ? m : 1));
    int32_t* hi = malloc(sizeof(int32_t) * (m > 0 ? m : 1));
#pragma omp for schedule(dynamic, 4)
    for (int64_t q = 0; q < n_src; ++q) {
      const float* s = src_f + q * k;
      int n = 0;
      for (int64_t b = 0; b < nb; ++b) {
        float acc[64];
        for (int j = 0; j < 64; ++j) acc[j] = 0.f;
        const float* blk = Tt + (size_t)b * k * 64;
        for (int i = 0; i < k; ++i) {
          const float si = s[i];
          for (int j = 0; j < 64; ++j) acc[j] = acc[j] + si * blk[i * 64 + j];
        }
        const int jn = (b * 64 + 64 <= n_dst) ? 64 : (int)(n_dst - b * 64);
        for (int j = 0; j < jn; ++j) {
          const int64_t r = b * 64 + j;
          if (n < m) {
            hs[n] = acc[j];
            hi[n] = (int32_t)r;
            heap_up(hs, hi, n++);
          } else if (m > 0 && worse(hs[0], hi[0], acc[j], (int32_t)r)) {
            hs[0] = acc[j];
            hi[0] = (int32_t)r;
            heap_down(hs, hi, m, 0);
          }
        }
      }
      /* heap sort: repeatedly move the worst to the back -> best first */
      for (int e = n - 1; e > 0; --e) {
        float ts = hs[0]; hs[0] = hs[e]; hs[e] = ts;
        int32_t ti = hi[0]; hi[0] = hi[e]; hi[e] = ti;
        heap_down(hs, hi, e, 0);
      }
      for (int e = 0; e < num; ++e) {
        out_ids[q * num + e] = e < n ? dst_ids[hi[e]] : -1;
        out_sc[q * num + e] = e < n ? hs[e] : NAN;
      }
    }
    free(hs);
    free(hi);
  }
  free(Tt);
  return 0;
}
