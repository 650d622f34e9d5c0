// Ingest on device: raw-id COO -> dense id remap + CSR in both orientations, and the seeded
// synthetic star-matrix generator.
//
// Reference semantics: Spark ALS.fit casts (user, item) with checkedCast to Int and the rating to
// Float, then partitionRatings/makeBlocks build per-block CSR InBlocks keyed by the sorted unique
// ids (ml/recommendation/ALS.scala, reached from ALSRecommenderBuilder.scala:58 with the input of
// DatasetUtils.scala:111-123).  Here one device-wide radix sort per key replaces the shuffle.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <cstdint>
#include <vector>
#include "kernels.h"

namespace albedo {

namespace {

struct Scratch {  // grow-only device scratch, freed at scope exit
  std::vector<void*> ptrs;
  ~Scratch() { for (void* p : ptrs) (void)hipFree(p); }
  template <class T>
  hipError_t alloc(T** p, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, n * sizeof(T) > 0 ? n * sizeof(T) : 16);
    if (e != hipSuccess) return e;
    ptrs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return hipSuccess;
  }
};

#define TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

__global__ void flip_keys_kernel(const int32_t* in, uint32_t* out, uint32_t* idx, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = (uint32_t)in[i] ^ 0x80000000u;  // order-preserving for signed ints
    idx[i] = (uint32_t)i;
  }
}
__global__ void head_flags_kernel(const uint32_t* ks, uint32_t* flags, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = (i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}
__global__ void scatter_dense_kernel(const uint32_t* ks, const uint32_t* perm, const uint32_t* rank,
                                     int32_t* dense, int32_t* uniq, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = rank[i] - 1;
    dense[perm[i]] = (int32_t)r;
    if (i == 0 || ks[i] != ks[i - 1]) uniq[r] = (int32_t)(ks[i] ^ 0x80000000u);
  }
}
__global__ void make_pair_keys_kernel(const int32_t* dst, const int32_t* src, uint64_t* keys,
                                      unsigned long long* counts, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = ((uint64_t)(uint32_t)dst[i] << 32) | (uint32_t)src[i];
    atomicAdd(&counts[dst[i]], 1ull);
  }
}
__global__ void split_keys_kernel(const uint64_t* keys, int32_t* col, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    col[i] = (int32_t)(keys[i] & 0xffffffffull);
}

inline int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}
inline unsigned bits_for(uint64_t v) {
  unsigned b = 0;
  while (b < 32 && (1ull << b) <= v) ++b;
  return b == 0 ? 1 : b;
}

}  // namespace

hipError_t remap_ids(const int32_t* d_ids, int64_t n, int32_t* d_dense, int32_t** d_unique,
                     int64_t* n_unique, hipStream_t s) {
  Scratch sc;
  uint32_t *k0, *k1, *v0, *v1, *fl;
  TRY(sc.alloc(&k0, n)); TRY(sc.alloc(&k1, n)); TRY(sc.alloc(&v0, n)); TRY(sc.alloc(&v1, n));
  TRY(sc.alloc(&fl, n));
  flip_keys_kernel<<<grid_for(n), 256, 0, s>>>(d_ids, k0, v0, n);
  size_t tb = 0;
  TRY(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, (size_t)n, 0, 32, s));
  void* tmp; TRY(sc.alloc((char**)&tmp, tb));
  TRY(rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, (size_t)n, 0, 32, s));
  head_flags_kernel<<<grid_for(n), 256, 0, s>>>(k1, fl, n);
  size_t tb2 = 0;
  TRY(rocprim::inclusive_scan(nullptr, tb2, fl, k0, (size_t)n, rocprim::plus<uint32_t>(), s));
  void* tmp2; TRY(sc.alloc((char**)&tmp2, tb2));
  TRY(rocprim::inclusive_scan(tmp2, tb2, fl, k0, (size_t)n, rocprim::plus<uint32_t>(), s));
  uint32_t last = 0;
  TRY(hipMemcpyAsync(&last, k0 + (n - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  *n_unique = last;
  TRY(hipMalloc(d_unique, (size_t)last * sizeof(int32_t)));
  scatter_dense_kernel<<<grid_for(n), 256, 0, s>>>(k1, v1, k0, d_dense, *d_unique, n);
  TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

namespace {
// dense src index -> position in the padded all-gathered layout (rank r's rows at r * maxrows)
__global__ void padded_remap_kernel(const int32_t* __restrict__ in, int64_t n, ShardStarts st, int64_t chpad,
                                    int32_t* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = in[e];
    int r = 0;
    while (r + 1 < st.world && st.s[r + 1] <= d) ++r;
    const int64_t l = d - st.s[r];  // local row of rank r; chunk-major gathered layout
    out[e] = (int32_t)((l / chpad) * st.world * chpad + r * chpad + l % chpad);
  }
}
}  // namespace

hipError_t padded_remap(const int32_t* d_in, int64_t n, const ShardStarts& st, int64_t chpad, int32_t* d_out,
                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  padded_remap_kernel<<<(int)blocks, 256, 0, s>>>(d_in, n, st, chpad, d_out);
  return hipGetLastError();
}

hipError_t build_csr(const int32_t* d_dst, const int32_t* d_src, const float* d_val, int64_t n,
                     int64_t n_dst, int64_t n_src, int64_t* d_ptr, int32_t* d_col, float* d_valout,
                     hipStream_t s) {
  Scratch sc;
  uint64_t *k0, *k1;
  float* vtmp;
  unsigned long long* cnt;
  TRY(sc.alloc(&k0, n)); TRY(sc.alloc(&k1, n)); TRY(sc.alloc(&vtmp, n));
  TRY(sc.alloc(&cnt, n_dst + 1));
  TRY(hipMemsetAsync(cnt, 0, (n_dst + 1) * sizeof(unsigned long long), s));
  make_pair_keys_kernel<<<grid_for(n), 256, 0, s>>>(d_dst, d_src, k0, cnt, n);
  TRY(hipMemcpyAsync(vtmp, d_val, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  const unsigned end_bit = 32 + bits_for((uint64_t)n_dst);
  (void)n_src;
  size_t tb = 0;
  TRY(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, vtmp, d_valout, (size_t)n, 0, end_bit, s));
  void* tmp; TRY(sc.alloc((char**)&tmp, tb));
  TRY(rocprim::radix_sort_pairs(tmp, tb, k0, k1, vtmp, d_valout, (size_t)n, 0, end_bit, s));
  split_keys_kernel<<<grid_for(n), 256, 0, s>>>(k1, d_col, n);
  size_t tb2 = 0;
  TRY(rocprim::exclusive_scan(nullptr, tb2, cnt, (unsigned long long*)d_ptr, 0ull, (size_t)(n_dst + 1),
                              rocprim::plus<unsigned long long>(), s));
  void* tmp2; TRY(sc.alloc((char**)&tmp2, tb2));
  TRY(rocprim::exclusive_scan(tmp2, tb2, cnt, (unsigned long long*)d_ptr, 0ull, (size_t)(n_dst + 1),
                              rocprim::plus<unsigned long long>(), s));
  TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

// ---------------------------------------------------------------------------------------------
// Synthetic generator: device twin of albedo_amd/synthetic.py `generate` (same splitmix64 draws,
// same inverse-CDF sampling, same first-slot-keeps de-duplication rounds).
// ---------------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint64_t smix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double unif(uint64_t key, uint64_t idx) {
  return (double)(smix(idx + key) >> 11) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ int32_t sample_pos(const double* cw, int64_t I, const int32_t* perm, double u) {
  const double x = u * cw[I - 1];
  int64_t lo = 0, hi = I;  // first j with cw[j] > x (numpy searchsorted side='right')
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cw[mid] > x) hi = mid; else lo = mid + 1;
  }
  if (lo > I - 1) lo = I - 1;
  return perm[lo];
}
__global__ void synth_init_kernel(uint64_t key0, const int64_t* prefix, int64_t U, const double* cw, int64_t I,
                                  const int32_t* perm, int32_t* row, int32_t* item, int64_t n) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = U;  // row = last r with prefix[r] <= s
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (prefix[mid] <= s) lo = mid; else hi = mid - 1;
    }
    row[s] = (int32_t)lo;
    item[s] = sample_pos(cw, I, perm, unif(key0, (uint64_t)s));
  }
}
__global__ void synth_keys_kernel(const int32_t* row, const int32_t* item, int64_t I, uint64_t* keys,
                                  uint32_t* slots, int64_t n) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
    keys[s] = (uint64_t)row[s] * (uint64_t)I + (uint64_t)item[s];
    slots[s] = (uint32_t)s;
  }
}
__global__ void synth_dups_kernel(const uint64_t* ks, const uint32_t* slots, uint8_t* dup,
                                  unsigned long long* ndup, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool d = i > 0 && ks[i] == ks[i - 1];
    dup[slots[i]] = d ? 1 : 0;
    if (d) atomicAdd(ndup, 1ull);
  }
}
__global__ void synth_resample_kernel(uint64_t key, const uint8_t* dup, const double* cw, int64_t I,
                                      const int32_t* perm, int32_t* item, int64_t n) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x)
    if (dup[s]) item[s] = sample_pos(cw, I, perm, unif(key, (uint64_t)s));
}
__global__ void synth_alive_kernel(const uint8_t* dup, uint32_t* alive, int64_t n) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x)
    alive[s] = dup[s] ? 0u : 1u;
}
__global__ void synth_emit_kernel(const int32_t* row, const int32_t* item, const uint32_t* alive,
                                  const uint32_t* pos, int32_t* u_out, int32_t* i_out, float* r_out, int64_t n) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
    if (!alive[s]) continue;
    const uint32_t p = pos[s];
    u_out[p] = (int32_t)(((int64_t)row[s] * 0x9E3779B1ll + 0x2545F491ll) & 0x7FFFFFFF);
    i_out[p] = (int32_t)(((int64_t)item[s] * 0x85EBCA77ll + 0x1B873593ll) & 0x7FFFFFFF);
    r_out[p] = 1.0f;
  }
}
uint64_t host_smix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t stream_key(uint64_t seed, uint64_t stream) { return host_smix(seed ^ (stream * 0xD1B54A32D192ED03ull)); }
}  // namespace

hipError_t synth_fill(uint64_t seed, int rounds, int64_t U, int64_t I, const int64_t* d_prefix,
                      const double* d_cw, const int32_t* d_perm, int32_t* d_user, int32_t* d_item,
                      float* d_rating, int64_t n, int64_t* n_out, hipStream_t s) {
  Scratch sc;
  int32_t *row, *item;
  uint64_t *k0, *k1;
  uint32_t *s0, *s1, *alive, *pos;
  uint8_t* dup;
  unsigned long long* ndup;
  TRY(sc.alloc(&row, n)); TRY(sc.alloc(&item, n)); TRY(sc.alloc(&k0, n)); TRY(sc.alloc(&k1, n));
  TRY(sc.alloc(&s0, n)); TRY(sc.alloc(&s1, n)); TRY(sc.alloc(&dup, n)); TRY(sc.alloc(&ndup, 1));
  synth_init_kernel<<<grid_for(n), 256, 0, s>>>(stream_key(seed, 2), d_prefix, U, d_cw, I, d_perm, row, item, n);
  size_t tb = 0;
  TRY(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, s0, s1, (size_t)n, 0, 64, s));
  void* tmp; TRY(sc.alloc((char**)&tmp, tb));
  auto find_dups = [&](unsigned long long* hcount) -> hipError_t {
    synth_keys_kernel<<<grid_for(n), 256, 0, s>>>(row, item, I, k0, s0, n);
    TRY(rocprim::radix_sort_pairs(tmp, tb, k0, k1, s0, s1, (size_t)n, 0, 64, s));  // stable
    TRY(hipMemsetAsync(ndup, 0, sizeof(unsigned long long), s));
    synth_dups_kernel<<<grid_for(n), 256, 0, s>>>(k1, s1, dup, ndup, n);
    TRY(hipMemcpyAsync(hcount, ndup, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    return hipStreamSynchronize(s);
  };
  bool clean = false;
  for (int attempt = 1; attempt <= rounds; ++attempt) {
    unsigned long long nd = 0;
    TRY(find_dups(&nd));
    if (nd == 0) { clean = true; break; }
    synth_resample_kernel<<<grid_for(n), 256, 0, s>>>(stream_key(seed, 2 + attempt), dup, d_cw, I, d_perm, item, n);
  }
  if (!clean) {
    unsigned long long nd = 0;
    TRY(find_dups(&nd));
  } else {
    TRY(hipMemsetAsync(dup, 0, n, s));
  }
  TRY(sc.alloc(&alive, n)); TRY(sc.alloc(&pos, n));
  synth_alive_kernel<<<grid_for(n), 256, 0, s>>>(dup, alive, n);
  size_t tb2 = 0;
  TRY(rocprim::exclusive_scan(nullptr, tb2, alive, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
  void* tmp2; TRY(sc.alloc((char**)&tmp2, tb2));
  TRY(rocprim::exclusive_scan(tmp2, tb2, alive, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
  synth_emit_kernel<<<grid_for(n), 256, 0, s>>>(row, item, alive, pos, d_user, d_item, d_rating, n);
  uint32_t lp = 0, la = 0;
  TRY(hipMemcpyAsync(&lp, pos + (n - 1), 4, hipMemcpyDeviceToHost, s));
  TRY(hipMemcpyAsync(&la, alive + (n - 1), 4, hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  *n_out = (int64_t)lp + la;
  return hipGetLastError();
}

}  // namespace albedo
