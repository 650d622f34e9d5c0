// Host-side numerics of the engine: the fp64 symmetric eigensolver used to diagonalise the Gram
// matrix each half-sweep, and the Spark-style (best effort) factor initialisation.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "host_math.h"

namespace albedo {

// ---------------------------------------------------------------------------------------------
// Symmetric eigendecomposition (Householder tridiagonalisation + implicit QL, EISPACK tred2/tql2
// as in the public-domain JAMA formulation).  a: n x n row-major symmetric.  On return w holds the
// eigenvalues ascending and v (row-major) the eigenvectors as columns: a = v diag(w) vᵀ.
// ---------------------------------------------------------------------------------------------
// (transposed storage: V[c * n + r] holds element (r, c), so the column sweeps of the JAMA code
// run along contiguous rows; the input is symmetric, the output is the transformation transposed)
static void tred2(int n, double* V, double* d, double* e) {
  for (int j = 0; j < n; j++) d[j] = V[j * n + (n - 1)];
  for (int i = n - 1; i > 0; i--) {
    double scale = 0.0, h = 0.0;
    for (int k = 0; k < i; k++) scale += std::fabs(d[k]);
    if (scale == 0.0) {
      e[i] = d[i - 1];
      for (int j = 0; j < i; j++) {
        d[j] = V[j * n + (i - 1)];
        V[j * n + i] = 0.0;
        V[i * n + j] = 0.0;
      }
    } else {
      for (int k = 0; k < i; k++) {
        d[k] /= scale;
        h += d[k] * d[k];
      }
      double f = d[i - 1];
      double g = std::sqrt(h);
      if (f > 0) g = -g;
      e[i] = scale * g;
      h = h - f * g;
      d[i - 1] = f - g;
      for (int j = 0; j < i; j++) e[j] = 0.0;
      for (int j = 0; j < i; j++) {
        f = d[j];
        V[i * n + j] = f;
        g = e[j] + V[j * n + j] * f;
        for (int k = j + 1; k <= i - 1; k++) {
          g += V[j * n + k] * d[k];
          e[k] += V[j * n + k] * f;
        }
        e[j] = g;
      }
      f = 0.0;
      for (int j = 0; j < i; j++) {
        e[j] /= h;
        f += e[j] * d[j];
      }
      const double hh = f / (h + h);
      for (int j = 0; j < i; j++) e[j] -= hh * d[j];
      for (int j = 0; j < i; j++) {
        f = d[j];
        g = e[j];
        for (int k = j; k <= i - 1; k++) V[j * n + k] -= (f * e[k] + g * d[k]);
        d[j] = V[j * n + (i - 1)];
        V[j * n + i] = 0.0;
      }
    }
    d[i] = h;
  }
  for (int i = 0; i < n - 1; i++) {
    V[i * n + (n - 1)] = V[i * n + i];
    V[i * n + i] = 1.0;
    const double h = d[i + 1];
    if (h != 0.0) {
      for (int k = 0; k <= i; k++) d[k] = V[(i + 1) * n + k] / h;
      for (int j = 0; j <= i; j++) {
        double g = 0.0;
        for (int k = 0; k <= i; k++) g += V[(i + 1) * n + k] * V[j * n + k];
        for (int k = 0; k <= i; k++) V[j * n + k] -= g * d[k];
      }
    }
    for (int k = 0; k <= i; k++) V[(i + 1) * n + k] = 0.0;
  }
  for (int j = 0; j < n; j++) {
    d[j] = V[j * n + (n - 1)];
    V[j * n + (n - 1)] = 0.0;
  }
  V[(n - 1) * n + (n - 1)] = 1.0;
  e[0] = 0.0;
}

static bool tql2(int n, double* V, double* d, double* e) {
  for (int i = 1; i < n; i++) e[i - 1] = e[i];
  e[n - 1] = 0.0;
  double f = 0.0, tst1 = 0.0;
  const double eps = std::ldexp(1.0, -52);
  for (int l = 0; l < n; l++) {
    tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
    int m = l;
    while (m < n) {
      if (std::fabs(e[m]) <= eps * tst1) break;
      m++;
    }
    if (m > l) {
      int iter = 0;
      do {
        if (++iter > 200) return false;
        double g = d[l];
        double p = (d[l + 1] - g) / (2.0 * e[l]);
        double r = std::hypot(p, 1.0);
        if (p < 0) r = -r;
        d[l] = e[l] / (p + r);
        d[l + 1] = e[l] * (p + r);
        const double dl1 = d[l + 1];
        double h = g - d[l];
        for (int i = l + 2; i < n; i++) d[i] -= h;
        f = f + h;
        p = d[m];
        double c = 1.0, c2 = c, c3 = c;
        const double el1 = e[l + 1];
        double s = 0.0, s2 = 0.0;
        for (int i = m - 1; i >= l; i--) {
          c3 = c2;
          c2 = c;
          s2 = s;
          g = c * e[i];
          h = c * p;
          r = std::hypot(p, e[i]);
          e[i + 1] = s * r;
          s = e[i] / r;
          c = p / r;
          p = c * d[i] - s * g;
          d[i + 1] = h + s * (c * g + s * d[i]);
          double* __restrict__ vi = V + (size_t)i * n;  // V holds the vectors as rows here
          double* __restrict__ vi1 = vi + n;
          for (int k = 0; k < n; k++) {
            h = vi1[k];
            vi1[k] = s * vi[k] + c * h;
            vi[k] = c * vi[k] - s * h;
          }
        }
        p = -s * s2 * c3 * el1 * e[l] / dl1;
        e[l] = s * p;
        d[l] = c * p;
      } while (std::fabs(e[l]) > eps * tst1);
    }
    d[l] = d[l] + f;
    e[l] = 0.0;
  }
  for (int i = 0; i < n - 1; i++) {
    int k = i;
    double p = d[i];
    for (int j = i + 1; j < n; j++)
      if (d[j] < p) {
        k = j;
        p = d[j];
      }
    if (k != i) {
      d[k] = d[i];
      d[i] = p;
      for (int j = 0; j < n; j++) std::swap(V[(size_t)i * n + j], V[(size_t)k * n + j]);
    }
  }
  return true;
}

static void transpose(int n, double* V) {
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++) std::swap(V[(size_t)i * n + j], V[(size_t)j * n + i]);
}

bool sym_eig(int n, const double* a, double* w, double* v) {
  std::memcpy(v, a, sizeof(double) * n * n);
  std::vector<double> e(n, 0.0);
  if (n == 1) {
    w[0] = a[0];
    v[0] = 1.0;
    return true;
  }
  tred2(n, v, w, e.data());  // leaves the transformation transposed: vectors as rows
  const bool ok = tql2(n, v, w, e.data());  // QL rotations on contiguous rows
  transpose(n, v);
  return ok;
}

// ---------------------------------------------------------------------------------------------
// Spark-style init (ml/recommendation/ALS.scala initialize; util/random/XORShiftRandom.scala;
// scala.util.hashing.MurmurHash3.bytesHash / byteswap64; java.util.Random.nextGaussian;
// netlib snrm2/sscal).  Best effort: SURVEY.md §7.1 item 6 (unverifiable offline).  The same
// restatement lives in oracle/spark_als.py and tests compare the two bit for bit.
// ---------------------------------------------------------------------------------------------
namespace {
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mix_last(uint32_t h, uint32_t k) {
  k *= 0xCC9E2D51u;
  k = rotl32(k, 15);
  k *= 0x1B873593u;
  return h ^ k;
}
inline uint32_t mix(uint32_t h, uint32_t k) {
  h = mix_last(h, k);
  h = rotl32(h, 13);
  return h * 5 + 0xE6546B64u;
}
inline uint32_t avalanche(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
uint32_t murmur3_bytes(const uint8_t* data, int n, uint32_t seed) {
  uint32_t h = seed;
  int i = 0;
  for (; n - i >= 4; i += 4) {
    const uint32_t k = (uint32_t)data[i] | ((uint32_t)data[i + 1] << 8) | ((uint32_t)data[i + 2] << 16) |
                       ((uint32_t)data[i + 3] << 24);
    h = mix(h, k);
  }
  const int rem = n - i;
  uint32_t k = 0;
  if (rem == 3) k ^= (uint32_t)data[i + 2] << 16;
  if (rem >= 2) k ^= (uint32_t)data[i + 1] << 8;
  if (rem >= 1) {
    k ^= data[i];
    h = mix_last(h, k);
  }
  return avalanche(h ^ (uint32_t)n);
}
uint64_t hash_seed(int64_t seed) {
  uint8_t bytes[64] = {0};
  const uint64_t u = (uint64_t)seed;
  for (int b = 0; b < 8; ++b) bytes[b] = (uint8_t)(u >> (56 - 8 * b));
  const uint32_t low = murmur3_bytes(bytes, 64, 0x3C074A61u);
  const uint32_t high = murmur3_bytes(bytes, 64, low);
  return ((uint64_t)high << 32) | (uint64_t)low;
}
uint64_t byteswap64(uint64_t v) {
  uint64_t hc = v * 0x9E3775CD9E3775CDull;
  hc = __builtin_bswap64(hc);
  return hc * 0x9E3775CD9E3775CDull;
}
struct XorShift {
  uint64_t s;
  bool have = false;
  double nextg = 0.0;
  explicit XorShift(int64_t init) : s(hash_seed(init)) {}
  int32_t next(int bits) {
    s ^= s << 21;
    s ^= s >> 35;
    s ^= s << 4;
    return (int32_t)(uint32_t)(s & ((1ull << bits) - 1));
  }
  int64_t next_long() {
    const int64_t hi = (int64_t)next(32);
    const int64_t lo = (int64_t)next(32);
    return (int64_t)((uint64_t)hi << 32) + lo;
  }
  double next_double() {
    return (double)(((int64_t)next(26) << 27) + next(27)) * (1.0 / 9007199254740992.0);
  }
  double next_gaussian() {
#pragma clang fp contract(off)
    if (have) {
      have = false;
      return nextg;
    }
    double v1, v2, sq;
    do {
      v1 = 2 * next_double() - 1;
      v2 = 2 * next_double() - 1;
      sq = v1 * v1 + v2 * v2;
    } while (sq >= 1 || sq == 0);
    const double mul = std::sqrt(-2 * std::log(sq) / sq);
    nextg = v2 * mul;
    have = true;
    return v1 * mul;
  }
};
float f2j_snrm2(const float* x, int n) {
#pragma clang fp contract(off)
  float scale = 0.f, ssq = 1.f;
  for (int i = 0; i < n; ++i) {
    if (x[i] != 0.f) {
      const float a = std::fabs(x[i]);
      if (scale < a) {
        const float q = scale / a;
        ssq = 1.f + ssq * (q * q);
        scale = a;
      } else {
        const float q = a / scale;
        ssq = ssq + q * q;
      }
    }
  }
  return scale * std::sqrt(ssq);
}
}  // namespace

void spark_side_seeds(int64_t seed, int64_t* user_seed, int64_t* item_seed) {
  XorShift g(seed);
  *user_seed = g.next_long();
  *item_seed = g.next_long();
}

void spark_initialize(const int32_t* ids_sorted, int64_t n, int rank, int64_t side_seed, int num_blocks,
                      float* out, int64_t ld) {
#pragma clang fp contract(off)
  std::vector<std::vector<int64_t>> rows(num_blocks);
  for (int64_t i = 0; i < n; ++i) {
    int b = (int)(((int64_t)ids_sorted[i] % num_blocks + num_blocks) % num_blocks);
    rows[b].push_back(i);
  }
  // one generator per block, as Spark's per-block XORShiftRandom: each block's stream is sequential
  // (the Gaussian draws are rejection-sampled), the blocks are independent -> one thread per block
  auto block = [&](int b) {
#pragma clang fp contract(off)
    std::vector<float> v(rank);
    XorShift rnd((int64_t)byteswap64((uint64_t)side_seed ^ (uint64_t)b));
    for (int64_t r : rows[b]) {
      for (int c = 0; c < rank; ++c) v[c] = (float)rnd.next_gaussian();
      const float nrm = f2j_snrm2(v.data(), rank);
      const float inv = 1.0f / nrm;
      for (int c = 0; c < rank; ++c) out[r * ld + c] = v[c] * inv;
    }
  };
  if (n < (int64_t)1 << 16) {  // small inputs: no thread start-up
    for (int b = 0; b < num_blocks; ++b) block(b);
    return;
  }
  // a fixed pool of min(hardware threads, blocks) workers taking block indices from a counter (each
  // block keeps its own generator, so the output does not depend on which worker draws it); a pool
  // that cannot start a thread runs the remaining blocks on the caller's
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nw = (int)std::min<int64_t>(hw, num_blocks);
  std::atomic<int> next{0};
  auto worker = [&]() {
    for (int b = next.fetch_add(1); b < num_blocks; b = next.fetch_add(1)) block(b);
  };
  std::vector<std::thread> th;
  th.reserve(nw);
  for (int w = 1; w < nw; ++w) {
    try {
      th.emplace_back(worker);
    } catch (const std::system_error&) {
      break;
    }
  }
  worker();
  for (auto& t : th) t.join();
}

// Contiguous shards of [0, n) balanced by nnz (ptr = CSR row pointer of the side, n + 1 entries).
void plan_shards(const int64_t* ptr, int64_t n, int world, int64_t* starts) {
  const int64_t total = ptr[n];
  starts[0] = 0;
  int64_t r = 0;
  for (int w = 1; w < world; ++w) {
    const int64_t target = (total * w + world - 1) / world;
    while (r < n && ptr[r] < target) ++r;
    starts[w] = std::max(starts[w - 1], r);
  }
  starts[world] = n;
}

}  // namespace albedo
