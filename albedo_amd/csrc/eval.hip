// Ranking evaluation on the device (albedo evaluators/RankingEvaluator.scala:83-139 ->
// mllib RankingMetrics.ndcgAt):
//
//  actual    intoUserActualItems (:111-129): rank() over (user ORDER BY starred_at DESC) <= k, then
//            collect_list, then evaluate's slice(0, k) (:91-92).  rank() keeps every row with fewer
//            than k strictly later rows, so after the slice the list is exactly the first k rows in
//            (key desc, item asc) order (the deterministic collect_list order the host evaluator
//            imposes): one wave per user selects them with a wave bitonic sort.
//  predicted intoUserPredictedItems (:131-139) of the top-k lists (score desc, id asc): the lists
//            als_recommend produces, kept on the device.
//  ndcgAt    per user n = min(max(|pred|, |labSet|), k), dcg = Σ_{i<n} [pred_i ∈ lab] g_i,
//            maxDcg = Σ_{i<min(n,|labSet|)} g_i (|labSet| = distinct items of the actual list),
//            g_i = 1 / ln(i + 2) from the host's libm (the same
//            table the host evaluator uses), summed in index order: per-user values are bit-identical
//            to the host evaluator's.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>
#include <algorithm>
#include <cstdint>
#include "device_common.h"
#include "kernels.h"

namespace albedo {
namespace {

inline int ev_grid(int64_t n, int per) {
  const int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 16384));
}

// raw user id -> dense row (binary search over the ascending ids); unknown ids -> 0xFFFFFFFF, which
// sorts last and is dropped (the evaluator's inner join)
__global__ void ev_map_rows_kernel(const int32_t* __restrict__ user, int64_t n, const int32_t* __restrict__ ids,
                                   int64_t n_ids, uint32_t* __restrict__ row, uint32_t* __restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = user[i];
    int64_t lo = 0, hi = n_ids;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ids[mid] < u) lo = mid + 1;
      else hi = mid;
    }
    row[i] = (lo < n_ids && ids[lo] == u) ? (uint32_t)lo : 0xFFFFFFFFu;
    idx[i] = (uint32_t)i;
  }
}

// (key desc, item asc) order of the actual lists; "before" = ranks earlier
__device__ __forceinline__ bool ev_before(int64_t k1, int32_t i1, int64_t k2, int32_t i2) {
  return k1 > k2 || (k1 == k2 && i1 < i2);
}

// wave bitonic sort of 128 (key, item) pairs, 2 per lane (element e = lane + 64h), into ev_before order
__device__ __forceinline__ void ev_bitonic128(int64_t (&ky)[2], int32_t (&it)[2]) {
  const int lane = threadIdx.x & 63;
  for (int K = 2; K <= 128; K <<= 1) {
    for (int J = K >> 1; J > 0; J >>= 1) {
      if (J == 64) {  // across the two registers of a lane
        const bool up = (lane & K) == 0;  // K = 128: element e < 128 -> always "up"
        const bool sw = up ? ev_before(ky[1], it[1], ky[0], it[0]) : ev_before(ky[0], it[0], ky[1], it[1]);
        if (sw) {
          const int64_t tk = ky[0]; ky[0] = ky[1]; ky[1] = tk;
          const int32_t ti = it[0]; it[0] = it[1]; it[1] = ti;
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = lane + 64 * h;
          const int64_t ok = __shfl_xor(ky[h], J);
          const int32_t oi = __shfl_xor(it[h], J);
          const bool lower = (lane & J) == 0;
          const bool up = (e & K) == 0;
          const bool other_first = ev_before(ok, oi, ky[h], it[h]);
          if ((lower == up) ? other_first : !other_first) { ky[h] = ok; it[h] = oi; }
        }
      }
    }
  }
}

// one wave per user run: the first min(k, cnt) entries in (key desc, item asc) order
__global__ __launch_bounds__(256) void ev_actual_kernel(const uint32_t* __restrict__ sidx, const int64_t* __restrict__ off,
                                                       const int32_t* __restrict__ cnt, int64_t n_runs,
                                                       const int64_t* __restrict__ key, const int32_t* __restrict__ item,
                                                       int k, int32_t* __restrict__ act, int32_t* __restrict__ act_n) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_runs) return;
  const int64_t o = off[r];
  const int n = cnt[r];
  int64_t ky[2] = {INT64_MIN, INT64_MIN};
  int32_t it[2] = {INT32_MAX, INT32_MAX};  // empty slots rank last
  for (int b = 0; b < n; b += 64) {  // kept best 64 in slot 0, the next 64 entries in slot 1
    const int e = b + lane;
    if (e < n) {
      const uint32_t j = sidx[o + e];
      ky[1] = key[j];
      it[1] = item[j];
    } else {
      ky[1] = INT64_MIN;
      it[1] = INT32_MAX;
    }
    ev_bitonic128(ky, it);
  }
  const int m = min(n, k);
  if (lane < k) act[r * k + lane] = lane < m ? it[0] : -1;
  if (lane == 0) act_n[r] = m;
}

// one wave per evaluated user: ndcgAt(k) of the predicted list against the actual list
__global__ __launch_bounds__(256) void ev_ndcg_kernel(const int32_t* __restrict__ pred, const int32_t* __restrict__ act,
                                                     const int32_t* __restrict__ act_n, int64_t n_users, int k,
                                                     const double* __restrict__ gain, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n_users) return;
  const int32_t p = lane < k ? pred[u * k + lane] : -1;
  const int nl = act_n[u];
  const int32_t lab = lane < nl ? act[u * k + lane] : -1;
  bool hit = false, dup = false;
  for (int j = 0; j < nl; ++j) {
    const int32_t v = __shfl(lab, j);
    hit |= (p >= 0 && p == v);
    dup |= (j < lane && v == lab);  // an earlier entry holds the same item
  }
  // |labSet|: mllib takes the size of the label SET (a user's duplicated (user, item) rows count once)
  const int ns = __popcll(__ballot(lane < nl && !dup));
  const int np = __popcll(__ballot(lane < k && p >= 0));  // the lists are dense: -1 only at the tail
  const uint64_t hits = __ballot(hit);
  if (lane == 0) {
    double v = 0.0;
    if (ns > 0) {
      const int n = min(max(np, ns), k);
      double dcg = 0.0, mx = 0.0;
      for (int i = 0; i < n; ++i) {
        if (i < np && ((hits >> i) & 1)) dcg += gain[i];
        if (i < ns) mx += gain[i];
      }
      v = dcg / mx;
    }
    out[u] = v;
  }
}

}  // namespace

size_t eval_sort_temp_bytes(int64_t n) {
  size_t a = 0, b = 0, c = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0, 32, (hipStream_t)0);
  (void)rocprim::run_length_encode(nullptr, b, (uint32_t*)nullptr, (size_t)n, (uint32_t*)nullptr, (int32_t*)nullptr,
                                   (int64_t*)nullptr, (hipStream_t)0);
  (void)rocprim::exclusive_scan(nullptr, c, (int32_t*)nullptr, (int64_t*)nullptr, (int64_t)0, (size_t)n,
                                rocprim::plus<int64_t>(), (hipStream_t)0);
  return std::max(a, std::max(b, c));
}

hipError_t eval_group_users(const int32_t* user, int64_t n, const int32_t* ids, int64_t n_ids, void* temp,
                            size_t temp_bytes, uint32_t* row, uint32_t* row_sorted, uint32_t* idx, uint32_t* idx_sorted,
                            uint32_t* runs, int32_t* counts, int64_t* offsets, int64_t* n_runs, hipStream_t s) {
  ev_map_rows_kernel<<<ev_grid(n, 256), 256, 0, s>>>(user, n, ids, n_ids, row, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  e = rocprim::radix_sort_pairs(temp, tb, row, row_sorted, idx, idx_sorted, (size_t)n, 0, 32, s);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  e = rocprim::run_length_encode(temp, tb, row_sorted, (size_t)n, runs, counts, n_runs, s);
  if (e != hipSuccess) return e;
  int64_t nr = 0;
  e = hipMemcpyAsync(&nr, n_runs, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  return rocprim::exclusive_scan(temp, tb, counts, offsets, (int64_t)0, (size_t)nr, rocprim::plus<int64_t>(), s);
}

hipError_t eval_actual_lists(const uint32_t* idx_sorted, const int64_t* offsets, const int32_t* counts, int64_t n_runs,
                             const int64_t* key, const int32_t* item, int k, int32_t* act, int32_t* act_n,
                             hipStream_t s) {
  if (n_runs <= 0) return hipSuccess;
  if (k < 1 || k > 64) return hipErrorInvalidValue;
  for (int64_t r0 = 0; r0 < n_runs; r0 += max_rows_per_launch(64)) {
    const int64_t nr = std::min<int64_t>(n_runs - r0, max_rows_per_launch(64));
    ev_actual_kernel<<<(int)((nr + 3) / 4), 256, 0, s>>>(idx_sorted, offsets + r0, counts + r0, nr, key, item, k,
                                                        act + r0 * k, act_n + r0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t eval_ndcg(const int32_t* pred, const int32_t* act, const int32_t* act_n, int64_t n_users, int k,
                     const double* gain, double* out, hipStream_t s) {
  if (n_users <= 0) return hipSuccess;
  if (k < 1 || k > 64) return hipErrorInvalidValue;
  for (int64_t u0 = 0; u0 < n_users; u0 += max_rows_per_launch(64)) {
    const int64_t nu = std::min<int64_t>(n_users - u0, max_rows_per_launch(64));
    ev_ndcg_kernel<<<(int)((nu + 3) / 4), 256, 0, s>>>(pred + u0 * k, act + u0 * k, act_n + u0, nu, k, gain, out + u0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace albedo
