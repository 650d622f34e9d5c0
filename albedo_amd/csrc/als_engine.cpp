// libalbedo_als.so host engine: the C ABI of include/albedo_als.h.
//
// Mirrors Spark MLlib 2.2.0 ALS.train as reached from ALSRecommenderBuilder.scala:46-58:
//   userFactors = initialize(...); itemFactors = initialize(...)
//   for iter in 1..maxIter: itemFactors = computeFactors(userFactors -> items)
//                           userFactors = computeFactors(itemFactors -> users)
// Each computeFactors call is one half-sweep here (half_sweep()):
//   G = Σ y yᵀ over the src rows (MFMA, fp64 partials)    [+ all-reduce across ranks]
//   G = P Λ Pᵀ (host fp64 eigensolver);  Z = X_src · P    [+ all-gather of the Z shard]
//   every dst row solved in the eigenbasis (light: push-through, heavy: explicit Cholesky)
// Factors are stored in a per-side basis B (original = X · Bᵀ); solving from src basis B_s with
// rotation P puts the dst solution in basis B_s·P, so only one rotation GEMM runs per half-sweep.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "albedo_als.h"
#include "host_math.h"
#include "kernels.h"

using namespace albedo;

namespace {

thread_local std::string g_err;
std::mutex g_fork_mu;  // parent / fork lifetimes (als_fork: forks may be destroyed from any thread)

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess)                                                                          \
      return fail(e_ == hipErrorOutOfMemory ? ALS_E_OUT_OF_MEMORY : ALS_E_HIP,                     \
                  std::string("HIP error: ") + hipGetErrorString(e_) + " in " #x);                 \
  } while (0)
#define NCCLCHK(x)                                                                                 \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) return fail(ALS_E_RCCL, std::string("RCCL error: ") + ncclGetErrorString(r_) + " in " #x); \
  } while (0)
#define TRYC(x)                    \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != ALS_OK) return rc_; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  bool owned = true;  // false: a view of another context's buffer (als_fork), never freed here
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p && owned) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    owned = true;
  }
  void share(const DevBuf& o) {
    release();
    p = o.p;
    bytes = o.bytes;
    owned = false;
  }
  hipError_t ensure(size_t b) {
    if (!owned) return hipErrorNotSupported;  // a view (als_fork) is never resized or written through
    if (b <= bytes && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, b ? b : 16);
    if (e == hipSuccess) bytes = b;
    return e;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

enum { B_L16 = 0, B_L32 = 1, B_L64 = 2, B_L96 = 3, B_HEAVY = 4, NBUCKET = 5 };

struct Side {
  int64_t n = 0;                 // rows (unique raw ids)
  std::vector<int32_t> ids;      // ascending
  std::vector<int64_t> starts;   // shard starts over dense rows (world + 1)
  int64_t maxrows = 0;           // max own rows over ranks
  // Gathered (padded) layout, chunk-major so that one chunk of every rank is contiguous: rank r's
  // local row i sits at (i / chpad)·world·chpad + r·chpad + i % chpad.  world = 1: nch = 1 and
  // the position is i.  prows() = nch·world·chpad rows.
  int nch = 1, world = 1;
  int64_t chpad = 0;
  int64_t own0 = 0, own_n = 0;   // this rank's dense row range
  // dst CSR of this side restricted to own rows (local row index; col = padded src position)
  DevBuf d_ptr, d_col, d_val;
  int64_t own_nnz = 0;
  std::vector<int64_t> h_deg;    // degree per own row
  DevBuf d_rows;                 // own local rows grouped by bucket
  DevBuf d_desc;                 // int4 per d_rows entry: {row, p0 lo, p0 hi, degree} (light16 prefetch)
  int64_t boff[NBUCKET + 1] = {0};
  int64_t bnnz[NBUCKET] = {0};
  float vmax = 0.f;              // max |rating| over own dst rows (heavy-build fp16 scaling)
  float vmin = 0.f;              // min |rating| over own dst rows: vmin == vmax -> one confidence c
  DevBuf d_X;                    // [own_n][KP] factors in basis B
  DevBuf d_Z;                    // [prows][KP] rotated factors (src role), gathered layout
  DevBuf d_Xfull;                // world > 1: [prows][KP] every rank's X (basis B), gathered layout
  bool full_valid = false;       // d_Xfull holds the current X (gathered behind the solve on st2)
  int64_t prows() const { return (int64_t)nch * world * chpad; }
  int64_t pos(int r, int64_t i) const { return (i / chpad) * world * chpad + (int64_t)r * chpad + i % chpad; }
  DevBuf d_B;                    // fp64 [KP][KP] orthogonal basis on the device: original = X · Bᵀ
  DevBuf d_Gk;                   // fp64 [KP][KP] last Gram of this side (as src), in basis d_GB
  DevBuf d_GB;                   // fp64 [KP][KP] the side's basis when d_Gk was computed (G_orig = GB G GBᵀ)
  bool has_gram = false;
  bool has_factors = false;
  double t[ALS_T_COUNT] = {0};
  int64_t stats[4] = {0};
  int64_t solver[4] = {0};       // NNLS iterations: sum over rows, max, rows (last half-sweep)
  DevBuf d_orig;                 // [n][KP] original-basis factors, dense order (materialised)
  bool orig_valid = false;
  // split-K of the heavy tail: the first n_split heavy rows (degree > split chunk), their chunks
  int64_t n_split = 0, n_chunks = 0;
  DevBuf d_chunk_row, d_chunk_idx, d_slot0;
  // nonnegative: the first n_batch rows of the (degree-ascending) light list go to the lockstep
  // NNLS kernel, rows [bat_off[v], bat_off[v+1]) with BATCH_SLOTS[v] slots per workgroup
  int64_t n_batch = 0, n_batch_nnz = 0;
  int64_t bat_off[6] = {0};
  // solve chunks (world > 1, Cholesky path): chunk q's rows of bucket b are the list positions
  // [cb[b][q], cb[b][q + 1]); its split-K rows are the first split_n[q] of its heavy segment, their
  // chunk lists start at ck_off[q] and their (chunk-local) slot0 at sl_off[q]
  int nsolve = 1;
  int64_t cb[NBUCKET][9] = {{0}};
  int64_t c8[8] = {0};           // bucket B_L16, solve chunk q: its first c8[q] rows have degree <= 8 (paired)
  int64_t split_n[8] = {0}, ck_off[9] = {0}, sl_off[8] = {0};
};

}  // namespace

struct als_ctx {
  als_params p{};
  int KP = 0;
  int dev = 0;
  hipStream_t st = nullptr;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  // host transport (tests: several processes sharing one GPU exchange through the host)
  int (*h_allreduce)(void*, double*, int64_t) = nullptr;
  int (*h_allgather)(void*, float*, int64_t) = nullptr;
  void* h_user = nullptr;
  Side s[2];
  int64_t nnz = 0;
  bool has_ratings = false;
  bool model_only = false;
  DevBuf slab, d_G, d_P, d_lam, d_err, d_Gt, d_cs, d_csmax;
  DevBuf d_eig;                  // device eigensolver scratch (eig.hip)
  DevBuf d_partial, d_reduced;   // split-K partial / reduced A' records (shared by both sides)
  DevBuf d_Zhl;                  // pre-split src rows of the uniform-confidence heavy build
  DevBuf d_Pf;                   // P's bf16 parts in MFMA fragment order (rotate_bf)
  DevBuf d_iters;                // NNLS iteration counters (sum, max)
  DevBuf d_gfrag, d_counter;     // lockstep NNLS: G in MFMA operand order, row counter
  int n_cu = 256;
  // top-k counters, cumulative: [0] rows through the MFMA scan, [1] rows re-scored by the exact scan
  // (certification misses), [2] dst chunks scanned, [3] dst chunks a full scan would take
  int64_t topk_stats[4] = {0, 0, 0, 0};
  // top-k device time, cumulative (ms, HIP events on st): [0] order + mask, [1] MFMA scan, [2] select,
  // [3] exact rescans; [4] scan flops (2·KP per src x dst pair the scan's waves scored)
  double topk_ms[5] = {0, 0, 0, 0, 0};
  hipEvent_t evt[5] = {};
  // src ids the last als_recommend / als_evaluate_ndcg sent to the exact rescan, built on demand
  // (als_topk_last_rescan) from the device flags of that call: position p of the call's rows was
  // rescanned when d_last_need[p] != 0; its src row is p (last_rows_dense) or last_rows[p]
  mutable std::vector<int32_t> last_rescan;
  DevBuf d_last_need;
  double* h_plan = nullptr;      // pinned: the top-k plan's dst Gram [KP][KP] + two max row norms
  int64_t last_need_n = 0;
  std::vector<int32_t> last_rows;
  mutable bool last_rescan_ready = true;
  bool last_rows_dense = false;
  int last_src = 0;
  int split_len = 0;             // ratings per split-K chunk (0: no split)
  int slab_blocks = 0;
  hipEvent_t ev[8] = {};
  hipStream_t st2 = nullptr;     // world > 1: factor-chunk gathers behind the solve
  // als_fork: a fork views its parent's ingest buffers; the parent is freed after its last fork
  als_ctx* parent = nullptr;
  int forks = 0;
  bool doomed = false;
  hipEvent_t evc[9] = {};        // per solve chunk: done on st; [8]: gathers done on st2
};

namespace {

int set_device(als_ctx* c) {
  HIPCHK(hipSetDevice(c->dev));
  return ALS_OK;
}

// Copies and fills between the host and the context's buffers go through the engine stream c->st and
// complete before returning.  c->st is a non-blocking stream: it does not order itself after the null
// stream, so a plain hipMemcpy / hipMemset could overlap the engine's kernels (a host-to-device
// hipMemcpy from pageable memory may return before its DMA lands, a device-to-device one does not
// wait at all, and neither waits for kernels still running on c->st).
hipError_t copy_st(const als_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  if (bytes == 0) return hipSuccess;
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c->st);
  return e != hipSuccess ? e : hipStreamSynchronize(c->st);
}
hipError_t fill_st(const als_ctx* c, void* dst, int v, size_t bytes) {
  if (bytes == 0) return hipSuccess;
  const hipError_t e = hipMemsetAsync(dst, v, bytes, c->st);
  return e != hipSuccess ? e : hipStreamSynchronize(c->st);
}

// world > 1: the factor-chunk gathers of the last half-sweep run on st2 behind the solve.  Anything
// that rewrites factor buffers with default-stream copies, or returns to the caller as "done",
// first waits for both streams.
int drain(als_ctx* c) {
  if (c->st2) HIPCHK(hipStreamSynchronize(c->st2));
  if (c->st) HIPCHK(hipStreamSynchronize(c->st));
  return ALS_OK;
}

int validate(const als_params* p) {
  auto bad = [](const char* name, double v) {
    char buf[160];
    snprintf(buf, sizeof buf, "als parameter %s given invalid value %g.", name, v);
    return fail(ALS_E_INVALID_ARGUMENT, buf);
  };
  if (p->rank < 1) return bad("rank", p->rank);
  if (p->max_iter < 0) return bad("maxIter", p->max_iter);
  if (!(p->reg_param >= 0)) return bad("regParam", p->reg_param);
  if (!(p->alpha >= 0)) return bad("alpha", p->alpha);
  if (p->num_user_blocks < 1) return bad("numUserBlocks", p->num_user_blocks);
  if (p->num_item_blocks < 1) return bad("numItemBlocks", p->num_item_blocks);
  if (padded_rank(p->rank) == 0)
    return fail(ALS_E_UNSUPPORTED, "rank " + std::to_string(p->rank) + " exceeds the compiled maximum (256)");
  return ALS_OK;
}

// Rows of degree <= light_limit take the push-through solve (a d x d system).  d <= 64 by default;
// light_max_degree up to 96 (KP = 128) routes rows of degree 65..96 through the d x d path too
// (solve_light_kernel<128, 96>), measured against the explicit k x k wave kernel in DESIGN §4.
int64_t light_limit(const als_ctx* c) {
  if (c->p.light_max_degree >= 0) return std::min<int64_t>(c->p.light_max_degree, c->KP == 128 ? 96 : 64);
  return c->KP >= 128 ? 64 : 32;
}

int bucket_of(int64_t d, int64_t lmax) {
  if (d <= lmax) {
    if (d <= 16) return B_L16;
    if (d <= 32) return B_L32;
    return d <= 64 ? B_L64 : B_L96;
  }
  return B_HEAVY;
}

// ---- collectives ------------------------------------------------------------------------------
int allreduce_G(als_ctx* c) {
  const int64_t n = (int64_t)c->KP * c->KP;
  if (c->world == 1) return ALS_OK;
  if (c->comm) {
    NCCLCHK(ncclAllReduce(c->d_G.p, c->d_G.p, n, ncclDouble, ncclSum, c->comm, c->st));
    return ALS_OK;
  }
  std::vector<double> h(n);
  HIPCHK(hipMemcpyAsync(h.data(), c->d_G.p, n * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  if (c->h_allreduce(c->h_user, h.data(), n) != 0) return fail(ALS_E_RCCL, "host all-reduce callback failed");
  HIPCHK(hipMemcpyAsync(c->d_G.p, h.data(), n * 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return ALS_OK;
}

// in-place all-gather on stream s: rank r's rows_per_rank rows at buf + r·rows_per_rank·KP
int allgather_rows(als_ctx* c, float* buf, int64_t rows_per_rank, hipStream_t s) {
  if (c->world == 1) return ALS_OK;
  const int64_t per = rows_per_rank * c->KP;
  if (c->comm) {
    NCCLCHK(ncclAllGather(buf + (int64_t)c->rank * per, buf, per, ncclFloat, c->comm, s));
    return ALS_OK;
  }
  std::vector<float> h((size_t)per * c->world);
  HIPCHK(hipMemcpyAsync(h.data() + (size_t)c->rank * per, buf + (int64_t)c->rank * per, per * 4,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (c->h_allgather(c->h_user, h.data(), per) != 0) return fail(ALS_E_RCCL, "host all-gather callback failed");
  HIPCHK(hipMemcpyAsync(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return ALS_OK;
}

// all-gather of host blocks: buf holds world blocks of n floats (this rank's filled); bytes are
// moved, never combined (ids travel as float bit patterns)
int allgather_host(als_ctx* c, float* buf, int64_t n) {
  if (c->world == 1) return ALS_OK;
  if (c->comm) {
    DevBuf d;
    HIPCHK(d.ensure((size_t)n * c->world * 4));
    float* dp = d.as<float>();
    HIPCHK(hipMemcpyAsync(dp + (int64_t)c->rank * n, buf + (int64_t)c->rank * n, n * 4, hipMemcpyHostToDevice, c->st));
    NCCLCHK(ncclAllGather(dp + (int64_t)c->rank * n, dp, n, ncclFloat, c->comm, c->st));
    HIPCHK(hipMemcpyAsync(buf, dp, (size_t)n * c->world * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return ALS_OK;
  }
  if (c->h_allgather(c->h_user, buf, n) != 0) return fail(ALS_E_RCCL, "host all-gather callback failed");
  return ALS_OK;
}

// Gathers layout chunks [q0, q1) of the own rows `own` ([nch·chpad][KP], zero past own_n) into
// `full` ([prows][KP]) on stream s: chunk q of every rank is one contiguous all-gather.
int gather_chunks(als_ctx* c, const Side& S, const float* own, float* full, int q0, int q1, hipStream_t s) {
  const int64_t per = S.chpad * c->KP;
  for (int q = q0; q < q1; ++q) {
    float* base = full + (int64_t)q * c->world * per;
    HIPCHK(hipMemcpyAsync(base + (int64_t)c->rank * per, own + (int64_t)q * per, per * 4, hipMemcpyDeviceToDevice, s));
    TRYC(allgather_rows(c, base, S.chpad, s));
  }
  return ALS_OK;
}

// Ratings per split-K chunk.  One workgroup gathering a 10^6-star row is the launch's tail (45.9
// ms for 1.05M stars at rank 128, more than a whole c4 half-sweep at 8 GPUs), and a partial of 8192
// ratings keeps every fp32 MFMA accumulation to 256 steps before the fp64 sum (a 1.05M-star row then
// matches the fp64 solve to 7e-7, tests/test_gpu_heavy_tail.py).  ALBEDO_SPLIT_CHUNK overrides it
// for tuning (0 disables the split): 2048 / 4096 / 16384 measured 338 / 324 / 311 ms per c4 sweep
// against 316 ms.
int split_chunk_len() {
  const char* e = std::getenv("ALBEDO_SPLIT_CHUNK");
  if (e && *e) return std::max(0, std::atoi(e));
  return 8192;
}

// nonnegative = true: light rows run in lockstep (nnls_batch.hip), BATCH_SLOTS[v] rows per workgroup
// for degrees up to nnls_batch_max_degree(KP, slots).  A lockstep iteration costs about the same for
// any slot count, so the variants pay off down to 8 slots (KP = 256 per row-iteration, tools/probe/
// batchtime: 16 slots 1.3 us, 8 slots 2.2 us, 4 slots 4.7 us against 4.5 us for solve_nnls_kernel);
// rows of higher degree take solve_nnls_kernel.
constexpr int BATCH_SLOTS[5] = {16, 8, 4, 2, 1};
constexpr int BATCH_MIN_SLOTS = 8;
int nnls_min_slots() {  // ALBEDO_NNLS_MIN_SLOTS: A/B knob (16, 8, 4, 2 or 1)
  const char* e = std::getenv("ALBEDO_NNLS_MIN_SLOTS");
  const int v = e && *e ? std::atoi(e) : BATCH_MIN_SLOTS;
  return (v == 16 || v == 8 || v == 4 || v == 2 || v == 1) ? v : BATCH_MIN_SLOTS;
}
int64_t nnls_batch_rows_limit(const als_ctx* c, int v) {
  if (BATCH_SLOTS[v] < nnls_min_slots()) return 0;
  return std::min<int64_t>(nnls_batch_max_degree(c->KP, BATCH_SLOTS[v]), light_limit(c));
}

// world > 1: the solve runs in this many row chunks, each gathered on a second stream while the
// next one solves
int gather_chunk_count() { return 4; }

// Heavy rows at padded rank <= 128 run one wave per row (heavy_wave.hip); rank 256 uses the 4-wave
// workgroup kernel (solve_heavy_kernel).
bool use_wave_kernel(const als_ctx* c);

int factor_buffers(als_ctx* c);

// Everything that depends on the rank / light-row limit rather than on the ratings: degree buckets
// (the light limit follows KP), split-K lists, then factor_buffers.  Called after ingest and again by
// als_set_params, so several fits (a CV grid) share one ingest.
int rank_layout(als_ctx* c) {
  TRYC(drain(c));
  const int64_t lmax = light_limit(c);
  c->split_len = split_chunk_len();
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    // degree buckets (heavy rows longest first for the tail)
    std::vector<int32_t> rows[NBUCKET];
    for (int b = 0; b < NBUCKET; ++b) S.bnnz[b] = 0;
    for (int64_t r = 0; r < S.own_n; ++r) {
      const int b = bucket_of(S.h_deg[r], lmax);
      rows[b].push_back((int32_t)r);
      S.bnnz[b] += S.h_deg[r];
    }
    std::stable_sort(rows[B_HEAVY].begin(), rows[B_HEAVY].end(),
                     [&](int32_t a, int32_t b) { return S.h_deg[a] > S.h_deg[b]; });
    S.n_batch = S.n_batch_nnz = 0;
    for (int v = 0; v < 6; ++v) S.bat_off[v] = 0;
    if (c->p.nonnegative) {  // light rows by ascending degree: the lockstep NNLS kernel's rows first
      for (int b = 0; b < B_HEAVY; ++b)
        std::stable_sort(rows[b].begin(), rows[b].end(), [&](int32_t x, int32_t y) { return S.h_deg[x] < S.h_deg[y]; });
      // variant v takes the degrees (limit of v-1, limit of v]; the light list is one ascending run
      int64_t pos = 0;
      std::vector<int32_t> light;
      for (int b = 0; b < B_HEAVY; ++b) light.insert(light.end(), rows[b].begin(), rows[b].end());
      for (int v = 0; v < 5; ++v) {
        const int64_t dl = nnls_batch_rows_limit(c, v);
        while (pos < (int64_t)light.size() && S.h_deg[light[pos]] <= dl) S.n_batch_nnz += S.h_deg[light[pos++]];
        S.bat_off[v + 1] = pos;
      }
      S.n_batch = pos;
    }
    // world > 1 (Cholesky path): each bucket's rows grouped by solve chunk (= gathered-layout
    // chunk, local row / chpad), stably, so a chunk's rows of a bucket are one contiguous run
    const int nsolve = (c->world > 1 && !c->p.nonnegative) ? S.nch : 1;
    S.nsolve = nsolve;
    auto chunk_of = [&](int32_t r) { return nsolve == 1 ? 0 : (int)std::min<int64_t>(r / S.chpad, nsolve - 1); };
    std::vector<int32_t> all;
    all.reserve(S.own_n);
    for (int b = 0; b < NBUCKET; ++b) {
      S.boff[b] = (int64_t)all.size();
      // grouped by solve chunk; B_L16: within a chunk the rows of degree <= 8 first (light16 pairs them)
      const bool pairs = b == B_L16;
      std::stable_sort(rows[b].begin(), rows[b].end(), [&](int32_t x, int32_t y) {
        const int cx = chunk_of(x), cy = chunk_of(y);
        if (cx != cy || !pairs) return cx < cy;
        return (S.h_deg[x] <= 8) > (S.h_deg[y] <= 8);
      });
      int64_t p = 0;
      for (int q = 0; q <= nsolve; ++q) {
        while (q < nsolve && p < (int64_t)rows[b].size() && chunk_of(rows[b][p]) < q) ++p;
        S.cb[b][q] = S.boff[b] + (q == nsolve ? (int64_t)rows[b].size() : p);
      }
      if (pairs)
        for (int q = 0; q < nsolve; ++q) {
          int64_t k = 0;
          for (int64_t i = S.cb[b][q] - S.boff[b]; i < S.cb[b][q + 1] - S.boff[b] && S.h_deg[rows[b][i]] <= 8; ++i) ++k;
          S.c8[q] = k;
        }
      all.insert(all.end(), rows[b].begin(), rows[b].end());
    }
    S.boff[NBUCKET] = (int64_t)all.size();
    HIPCHK(S.d_rows.ensure(all.size() * 4));
    HIPCHK(copy_st(c, S.d_rows.p, all.data(), all.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(S.d_desc.ensure(all.size() * 16));
    HIPCHK(launch_row_desc(S.d_rows.as<int32_t>(), (int64_t)all.size(), S.d_ptr.as<int64_t>(), S.d_desc.as<int32_t>(), c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    // split-K chunks of each solve chunk's heaviest rows (a prefix of its heavy run: by degree);
    // slot0 is chunk-local (starts at 0 for every solve chunk)
    const int64_t CH = c->split_len;
    std::vector<int32_t> crow, cidx, slot0;
    S.n_split = 0;
    for (int q = 0; q < nsolve; ++q) {
      S.ck_off[q] = (int64_t)crow.size();
      S.sl_off[q] = (int64_t)slot0.size();
      slot0.push_back(0);
      int64_t n = 0;
      for (int64_t p = S.cb[B_HEAVY][q]; p < S.cb[B_HEAVY][q + 1]; ++p) {
        const int32_t r = all[p];
        if (CH <= 0 || S.h_deg[r] <= CH) break;
        const int64_t nch = (S.h_deg[r] + CH - 1) / CH;
        for (int64_t k = 0; k < nch; ++k) {
          crow.push_back(r);
          cidx.push_back((int32_t)k);
        }
        slot0.push_back((int32_t)((int64_t)crow.size() - S.ck_off[q]));
        ++n;
      }
      S.split_n[q] = n;
      S.n_split += n;
    }
    S.ck_off[nsolve] = (int64_t)crow.size();
    S.n_chunks = (int64_t)crow.size();
    if (S.n_split > 0) {
      HIPCHK(S.d_chunk_row.ensure(crow.size() * 4));
      HIPCHK(S.d_chunk_idx.ensure(cidx.size() * 4));
      HIPCHK(S.d_slot0.ensure(slot0.size() * 4));
      HIPCHK(copy_st(c, S.d_chunk_row.p, crow.data(), crow.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(copy_st(c, S.d_chunk_idx.p, cidx.data(), cidx.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(copy_st(c, S.d_slot0.p, slot0.data(), slot0.size() * 4, hipMemcpyHostToDevice));
    }
  }
  return factor_buffers(c);
}

// Per-fit device state: split-K records, factor / rotated-factor buffers, Gram slabs and scratch;
// the factors are dropped (the next fit initialises them).
int factor_buffers(als_ctx* c) {
  {
    const size_t rec = (size_t)split_rec_floats(c->KP) * 4;
    const int64_t mc = std::max(c->s[0].n_chunks, c->s[1].n_chunks);
    const int64_t ms = std::max(c->s[0].n_split, c->s[1].n_split);
    if (mc > 0) {
      HIPCHK(c->d_partial.ensure(mc * rec));
      HIPCHK(c->d_reduced.ensure(ms * rec));
    }
  }
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    // X padded to whole layout chunks (zero rows past own_n: they travel in the chunk gathers)
    HIPCHK(S.d_X.ensure((size_t)std::max<int64_t>(std::max<int64_t>(S.own_n, (int64_t)S.nch * S.chpad), 1) * c->KP * 4));
    // + one zero row at prows(): the gather target of masked light-row entries (never written)
    HIPCHK(S.d_Z.ensure((size_t)(S.prows() + 1) * c->KP * 4));
    HIPCHK(fill_st(c, S.d_X.p, 0, S.d_X.bytes));
    HIPCHK(fill_st(c, S.d_Z.p, 0, S.d_Z.bytes));
    if (c->world > 1) {
      HIPCHK(S.d_Xfull.ensure((size_t)std::max<int64_t>(S.prows(), 1) * c->KP * 4));
      HIPCHK(fill_st(c, S.d_Xfull.p, 0, S.d_Xfull.bytes));
    }
    S.full_valid = false;
    HIPCHK(S.d_B.ensure((size_t)c->KP * c->KP * 8));
    HIPCHK(S.d_Gk.ensure((size_t)c->KP * c->KP * 8));
    HIPCHK(S.d_GB.ensure((size_t)c->KP * c->KP * 8));
    HIPCHK(launch_identity(S.d_B.as<double>(), c->KP, c->st));
    S.has_gram = false;
    S.has_factors = false;
    S.orig_valid = false;
    S.full_valid = false;
  }
  const int64_t maxsrc = std::max(c->s[0].own_n, c->s[1].own_n);
  c->slab_blocks = gram_slab_blocks(c->KP, maxsrc);
  HIPCHK(c->slab.ensure(gram_slab_doubles(c->KP, c->slab_blocks) * 8));
  HIPCHK(c->d_G.ensure((size_t)c->KP * c->KP * 8));
  HIPCHK(c->d_P.ensure((size_t)c->KP * c->KP * 4));
  HIPCHK(c->d_eig.ensure(eig_scratch_doubles(c->KP) * 8));
  HIPCHK(c->d_lam.ensure((size_t)c->KP * 4));
  HIPCHK(c->d_err.ensure(16));
  HIPCHK(c->d_cs.ensure((size_t)2 * c->KP * 4));
  HIPCHK(c->d_csmax.ensure((size_t)c->KP * 4));
  return ALS_OK;
}

// ---- ingest -------------------------------------------------------------------------------------
// A fork views its parent's ingest, and a parent's ingest is viewed by its live forks: neither may
// rebuild it (a re-ingest would write through the views or free buffers the forks still read).
int ingest_allowed(als_ctx* c) {
  std::lock_guard<std::mutex> lk(g_fork_mu);
  if (c->parent) return fail(ALS_E_STATE, "new ratings on a fork (set them on a fresh context instead)");
  if (c->forks > 0) return fail(ALS_E_STATE, "new ratings while forks view this context's ingest");
  return ALS_OK;
}

int ingest_device(als_ctx* c, int64_t n, const int32_t* d_user, const int32_t* d_item, const float* d_rating) {
  TRYC(ingest_allowed(c));
  if (n <= 0)
    return fail(ALS_E_INVALID_ARGUMENT, "No ratings available from the input dataset (empty ratings).");
  TRYC(set_device(c));
  // the previous top-k call's rescan flags index the old id tables: drop them before S.ids changes
  c->last_rescan.clear();
  c->last_need_n = 0;
  c->last_rows.clear();
  c->last_rescan_ready = true;
  hipStream_t st = c->st;
  DevBuf ud, id;
  HIPCHK(ud.ensure(n * 4));
  HIPCHK(id.ensure(n * 4));
  int32_t *uu = nullptr, *ii = nullptr;
  int64_t nu = 0, ni = 0;
  HIPCHK(remap_ids(d_user, n, ud.as<int32_t>(), &uu, &nu, st));
  HIPCHK(remap_ids(d_item, n, id.as<int32_t>(), &ii, &ni, st));
  Side& U = c->s[ALS_USER];
  Side& I = c->s[ALS_ITEM];
  U.n = nu;
  I.n = ni;
  U.ids.resize(nu);
  I.ids.resize(ni);
  HIPCHK(copy_st(c, U.ids.data(), uu, nu * 4, hipMemcpyDeviceToHost));
  HIPCHK(copy_st(c, I.ids.data(), ii, ni * 4, hipMemcpyDeviceToHost));
  (void)hipFree(uu);
  (void)hipFree(ii);
  c->nnz = n;
  // both orientations, full, then sliced to this rank's rows
  struct Full { DevBuf ptr, col, val; std::vector<int64_t> hptr; } full[2];
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    Full& F = full[side];
    HIPCHK(F.ptr.ensure((S.n + 1) * 8));
    HIPCHK(F.col.ensure(n * 4));
    HIPCHK(F.val.ensure(n * 4));
    const int32_t* dst = side == ALS_USER ? ud.as<int32_t>() : id.as<int32_t>();
    const int32_t* src = side == ALS_USER ? id.as<int32_t>() : ud.as<int32_t>();
    HIPCHK(build_csr(dst, src, d_rating, n, S.n, c->s[1 - side].n, F.ptr.as<int64_t>(), F.col.as<int32_t>(),
                     F.val.as<float>(), st));
    F.hptr.resize(S.n + 1);
    HIPCHK(copy_st(c, F.hptr.data(), F.ptr.p, (S.n + 1) * 8, hipMemcpyDeviceToHost));
    S.starts.assign(c->world + 1, 0);
    plan_shards(F.hptr.data(), S.n, c->world, S.starts.data());
    S.maxrows = 0;
    for (int r = 0; r < c->world; ++r) S.maxrows = std::max<int64_t>(S.maxrows, S.starts[r + 1] - S.starts[r]);
    S.own0 = S.starts[c->rank];
    S.own_n = S.starts[c->rank + 1] - S.own0;
    S.world = c->world;
    S.nch = c->world > 1 ? gather_chunk_count() : 1;
    S.chpad = std::max<int64_t>(1, (S.maxrows + S.nch - 1) / S.nch);
  }
  ud.release();
  id.release();
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    Side& Src = c->s[1 - side];
    Full& F = full[side];
    const int64_t e0 = F.hptr[S.own0], e1 = F.hptr[S.own0 + S.own_n];
    S.own_nnz = e1 - e0;
    std::vector<int64_t> lp(S.own_n + 1);
    for (int64_t r = 0; r <= S.own_n; ++r) lp[r] = F.hptr[S.own0 + r] - e0;
    HIPCHK(S.d_ptr.ensure((S.own_n + 1) * 8));
    HIPCHK(copy_st(c, S.d_ptr.p, lp.data(), (S.own_n + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(S.d_col.ensure(S.own_nnz * 4));
    HIPCHK(S.d_val.ensure(S.own_nnz * 4));
    HIPCHK(copy_st(c, S.d_val.p, F.val.as<float>() + e0, S.own_nnz * 4, hipMemcpyDeviceToDevice));
    if (c->world == 1) {
      HIPCHK(copy_st(c, S.d_col.p, F.col.as<int32_t>() + e0, S.own_nnz * 4, hipMemcpyDeviceToDevice));
    } else {  // dense src index -> padded src position, on the device
      ShardStarts ss{};
      ss.world = c->world;
      for (int r = 0; r <= c->world; ++r) ss.s[r] = Src.starts[r];
      HIPCHK(padded_remap(F.col.as<int32_t>() + e0, S.own_nnz, ss, Src.chpad, S.d_col.as<int32_t>(), st));
      HIPCHK(hipStreamSynchronize(st));
    }
    S.h_deg.resize(S.own_n);
    for (int64_t r = 0; r < S.own_n; ++r) S.h_deg[r] = lp[r + 1] - lp[r];
  }
  TRYC(rank_layout(c));
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    unsigned bits[2] = {0, 0};
    HIPCHK(launch_absmax(S.d_val.as<float>(), S.own_nnz, c->d_csmax.as<unsigned>(), st));
    HIPCHK(launch_absmin(S.d_val.as<float>(), S.own_nnz, c->d_csmax.as<unsigned>() + 1, st));
    HIPCHK(hipMemcpyAsync(bits, c->d_csmax.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(&S.vmax, &bits[0], 4);
    std::memcpy(&S.vmin, &bits[1], 4);
  }
  c->has_ratings = true;
  return ALS_OK;
}

// upload host factors (dense order, [n][rank]) for this rank's own rows
int upload_factors(als_ctx* c, int side, const float* f, int64_t ld) {
  TRYC(drain(c));
  Side& S = c->s[side];
  std::vector<float> h((size_t)std::max<int64_t>(S.own_n, 1) * c->KP, 0.f);
  for (int64_t r = 0; r < S.own_n; ++r)
    std::memcpy(&h[(size_t)r * c->KP], f + (size_t)(S.own0 + r) * ld, sizeof(float) * c->p.rank);
  HIPCHK(copy_st(c, S.d_X.p, h.data(), (size_t)S.own_n * c->KP * 4, hipMemcpyHostToDevice));
  HIPCHK(launch_identity(S.d_B.as<double>(), c->KP, c->st));
  S.has_factors = true;
  S.orig_valid = false;
  S.full_valid = false;
  return ALS_OK;
}

// Spark's initialize for every side that has no factors yet.  Both side seeds are always drawn
// (seedGen.nextLong twice, user first), so a side initialised here gets the same rows whether or
// not the other side was injected by the caller.
int spark_init(als_ctx* c) {
  int64_t su, si;
  spark_side_seeds(c->p.seed, &su, &si);
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    if (S.has_factors) continue;
    std::vector<float> f((size_t)S.n * c->p.rank);
    spark_initialize(S.ids.data(), S.n, c->p.rank, side == ALS_USER ? su : si,
                     side == ALS_USER ? c->p.num_user_blocks : c->p.num_item_blocks, f.data(), c->p.rank);
    TRYC(upload_factors(c, side, f.data(), c->p.rank));
  }
  return ALS_OK;
}

// the solve paths named by the bits of a not-positive-definite flag word (kernels.h ALBEDO_EF_*)
std::string err_paths(int err) {
  std::string r;
  const std::pair<int, const char*> names[] = {{ALBEDO_EF_LIGHT16, "light16"}, {ALBEDO_EF_LIGHT_REG, "light-d16"},
                                               {ALBEDO_EF_LIGHT_ACC, "light"}, {ALBEDO_EF_WAVE, "wave"},
                                               {ALBEDO_EF_HEAVY, "heavy"}};
  for (const auto& n : names)
    if (err & n.first) r += std::string(r.empty() ? ": " : ",") + n.second;
  return r;
}

float event_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

// fp16 column scales of the heavy build for dst side T over the gathered src rows Z
// have_max: the rotation left the column maxima of Z in d_csmax (rotate_kernel's epilogue)
int column_scales(als_ctx* c, const Side& S, const Side& T, bool have_max = false) {
  const float cmax = c->p.implicit_prefs ? (float)c->p.alpha * T.vmax : 1.0f;
  HIPCHK(launch_colscale(c->KP, S.d_Z.as<float>(), S.prows(), cmax, c->d_csmax.as<unsigned>(),
                         c->d_cs.as<float>(), c->st, have_max));
  return ALS_OK;
}

int heavy_launches(als_ctx* c, const Side& T, SolveArgs a, int64_t h0, int64_t hn, bool nnls, int q = 0);
bool use_wave_kernel(const als_ctx* c);

// KP = 128: the rotation on bf16 MFMA with the fused operand split (rotate_bf); KP = 64 / 256 keep the
// fp32 MFMA rotation + colmax epilogue + separate presplit pass
bool rotate_bf_on(const als_ctx* c) { return c->KP == 128; }

// One confidence c for every rating of dst side T (explicit: c = 1; implicit: all |r| equal): the
// heavy build's operand split z·√c·colscale -> fp16 hi + lo is then the same for every gather of a
// src row, so it runs once per src row here (launch_presplit) instead of once per gathered rating
// inside the wave kernel.
// presplit_wanted: whether the split applies to this half (and its √c); split_done: the rotation
// already wrote it (rotate_bf)
bool presplit_wanted(const als_ctx* c, const Side& T, float* sw) {
  const bool uniform = !c->p.implicit_prefs || (T.vmin == T.vmax && T.vmax > 0.f);
  if (!uniform || !use_wave_kernel(c) || T.boff[NBUCKET] == T.boff[B_HEAVY]) return false;
  const float cw = c->p.implicit_prefs ? (float)c->p.alpha * T.vmax : 1.0f;
  if (!(cw > 0.f)) return false;
  *sw = std::sqrt(cw);
  return true;
}

int presplit(als_ctx* c, const Side& S, const Side& T, const void** zhl, float* wsc, float* inv_sw,
             bool split_done = false) {
  *zhl = nullptr;
  float sw = 1.f;
  if (!presplit_wanted(c, T, &sw)) return ALS_OK;
  const float cw = c->p.implicit_prefs ? (float)c->p.alpha * T.vmax : 1.0f;
  HIPCHK(c->d_Zhl.ensure((size_t)(S.prows() + 1) * c->KP * 4));
  if (!split_done)
    HIPCHK(launch_presplit(c->KP, S.d_Z.as<float>(), S.prows(), c->d_cs.as<float>(), sw, c->d_Zhl.p, c->st));
  // b' weights w = 1 + c (implicit, r > 0) or r (explicit), scaled by a power of two below 2^13
  const double wmax = c->p.implicit_prefs ? 1.0 + (double)cw : (double)T.vmax;
  int e = 0;
  std::frexp(wmax > 0.0 ? wmax : 1.0, &e);  // wmax < 2^e
  *wsc = (float)std::ldexp(1.0, std::max(-60, std::min(60, 13 - e)));
  *inv_sw = 1.0f / sw;
  *zhl = c->d_Zhl.p;
  return ALS_OK;
}

// nonnegative = true: Spark's NNLSSolver in the original basis (no rotation; B stays I)
int half_sweep_nnls(als_ctx* c, int t) {
  const int sidx = 1 - t;
  Side& S = c->s[sidx];
  Side& T = c->s[t];
  const int KP = c->KP, k = c->p.rank;
  hipStream_t st = c->st;
  hipEvent_t* ev = c->ev;
  const int ngt = nnls_gtile_floats(KP);
  std::vector<float> gt(ngt, 0.f);
  float gscale = 1.0f;
  if (c->p.implicit_prefs) {
    HIPCHK(launch_gram(KP, S.d_X.as<float>(), S.own_n, c->slab.as<double>(), c->slab_blocks, c->d_G.as<double>(), st));
    TRYC(allreduce_G(c));
    std::vector<double> Gf((size_t)KP * KP);
    HIPCHK(hipMemcpyAsync(Gf.data(), c->d_G.p, Gf.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(S.d_Gk.p, c->d_G.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(S.d_GB.p, S.d_B.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    S.has_gram = true;
    for (int i = 0; i < KP; ++i)
      for (int j = 0; j < 16 * ((i >> 4) + 1); ++j) gt[nnls_gtile_index(i, j)] = (float)Gf[(size_t)i * KP + j];
    double gmax = 0.0;
    for (double v : Gf) gmax = std::max(gmax, std::fabs(v));
    if (gmax > 0.0) {  // lockstep kernel's fp16 split of G: max|G|·gscale < 2^15
      int ex = 0;
      (void)std::frexp(gmax, &ex);
      gscale = (float)std::ldexp(1.0, std::max(-120, std::min(120, 15 - ex)));
    }
  }
  HIPCHK(hipEventRecord(ev[1], st));
  HIPCHK(c->d_Gt.ensure((size_t)ngt * 4));
  HIPCHK(hipMemcpyAsync(c->d_Gt.p, gt.data(), (size_t)ngt * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(c->d_lam.p, 0, KP * 4, st));
  HIPCHK(hipEventRecord(ev[2], st));
  if (c->world == 1) HIPCHK(hipMemcpyAsync(S.d_Z.p, S.d_X.p, (size_t)S.own_n * KP * 4, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipEventRecord(ev[3], st));
  if (c->world > 1) TRYC(gather_chunks(c, S, S.d_X.as<float>(), S.d_Z.as<float>(), 0, S.nch, st));
  HIPCHK(hipEventRecord(ev[4], st));
  HIPCHK(hipMemsetAsync(c->d_err.p, 0, 4, st));
  TRYC(column_scales(c, S, T));
  HIPCHK(hipEventRecord(ev[5], st));
  SolveArgs a{};
  a.Z = S.d_Z.as<float>();
  a.ptr = T.d_ptr.as<int64_t>();
  a.col = T.d_col.as<int32_t>();
  a.val = T.d_val.as<float>();
  a.lam = c->d_lam.as<float>();
  a.X = T.d_X.as<float>();
  a.kreal = k;
  a.implicit = c->p.implicit_prefs;
  a.alpha = (float)c->p.alpha;
  a.reg = (float)c->p.reg_param;
  a.err = c->d_err.as<int>();
  a.colscale = c->d_cs.as<float>();
  HIPCHK(c->d_iters.ensure(32));  // [sum, max] of every row, then [sum, max] of the lockstep rows
  HIPCHK(hipMemsetAsync(c->d_iters.p, 0, 32, st));
  a.iters = c->d_iters.as<unsigned long long>();
  const int64_t nb = std::min<int64_t>(T.n_batch, T.boff[B_HEAVY]);
  if (nb > 0) {
    HIPCHK(c->d_gfrag.ensure((size_t)KP * KP * 4));
    HIPCHK(c->d_counter.ensure(64));
    HIPCHK(launch_nnls_gfrag(KP, c->d_Gt.as<float>(), gscale, c->d_gfrag.p, st));
    // ALBEDO_NNLS_BATCH_WGS caps the persistent grid (tests: force many slot refills per workgroup)
    const char* ew = std::getenv("ALBEDO_NNLS_BATCH_WGS");
    const int wgs = (ew && std::atoi(ew) > 0) ? std::min(c->n_cu, std::atoi(ew)) : c->n_cu;
    for (int v = 0; v < 5; ++v) {
      SolveArgs b = a;
      b.rows = T.d_rows.as<int32_t>() + T.bat_off[v];
      b.n_rows = T.bat_off[v + 1] - T.bat_off[v];
      b.iters = a.iters + 2;
      HIPCHK(launch_nnls_batch(KP, BATCH_SLOTS[v], b, c->d_gfrag.p, gscale, c->d_counter.as<unsigned int>(), wgs, st));
    }
  }
  HIPCHK(hipEventRecord(ev[7], st));
  TRYC(heavy_launches(c, T, a, nb, T.boff[B_HEAVY] - nb, true));
  TRYC(heavy_launches(c, T, a, T.boff[B_HEAVY], T.boff[NBUCKET] - T.boff[B_HEAVY], true));
  a.n_rows = T.boff[NBUCKET];
  T.stats[0] = nb;  // the lockstep kernel's rows and stars, then every other row
  T.stats[1] = nb > 0 ? T.n_batch_nnz : 0;
  T.stats[2] = a.n_rows - T.stats[0];
  T.stats[3] = T.own_nnz - T.stats[1];
  HIPCHK(hipEventRecord(ev[6], st));
  int err = 0;
  unsigned long long it[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(&err, c->d_err.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(it, c->d_iters.p, 32, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  T.solver[0] = (int64_t)(it[0] + it[2]);
  T.solver[1] = (int64_t)std::max(it[1], it[3]);
  T.solver[2] = T.boff[NBUCKET];
  T.solver[3] = (int64_t)it[2];
  T.t[ALS_T_GRAM] = event_ms(ev[0], ev[1]);
  T.t[ALS_T_EIG] = 0.0;
  T.t[ALS_T_ROTATE] = event_ms(ev[2], ev[3]);
  T.t[ALS_T_COMM] = event_ms(ev[3], ev[4]);
  T.t[ALS_T_SOLVE_LIGHT] = event_ms(ev[5], ev[7]);  // lockstep kernel
  T.t[ALS_T_SOLVE_HEAVY] = event_ms(ev[7], ev[6]);  // per-row kernels (split-K included)
  T.t[ALS_T_HALF_TOTAL] = event_ms(ev[0], ev[6]);
  if (err & 4) return fail(ALS_E_STATE, "lockstep NNLS row above its degree limit (row layout out of date)");
  if (err) return fail(ALS_E_NOT_POSITIVE_DEFINITE, "NNLS solve produced a non-finite result");
  HIPCHK(hipMemcpyAsync(T.d_B.p, S.d_B.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));  // no rotation
  T.has_factors = true;
  T.orig_valid = false;
  T.full_valid = false;
  return ALS_OK;
}

// Heavy launch over rows [h0, h0 + hn) of T's bucket-ordered row list, the first split_n[q] of which
// (when h0 starts solve chunk q's heavy run) are the split-K rows: chunk partials + fp64 reduce, then
// the factor (or NNLS) from the reduced records, then the remaining rows as usual.
int heavy_launches(als_ctx* c, const Side& T, SolveArgs a, int64_t h0, int64_t hn, bool nnls, int q) {
  const int KP = c->KP;
  const int32_t* rows = T.d_rows.as<int32_t>();
  int64_t ns = (h0 == T.cb[B_HEAVY][q]) ? std::min<int64_t>(T.split_n[q], hn) : 0;
  if (ns > 0) {
    SplitArgs sp{};
    sp.chunk_row = T.d_chunk_row.as<int32_t>() + T.ck_off[q];
    sp.chunk_idx = T.d_chunk_idx.as<int32_t>() + T.ck_off[q];
    sp.n_chunks = T.ck_off[q + 1] - T.ck_off[q];
    sp.chunk_len = c->split_len;
    sp.slot0 = T.d_slot0.as<int32_t>() + T.sl_off[q];
    sp.n_split = ns;
    sp.partial = c->d_partial.as<float>();
    sp.reduced = c->d_reduced.as<float>();
    HIPCHK(launch_heavy_split(KP, a, sp, use_wave_kernel(c), c->st));
    SolveArgs b = a;
    b.rows = rows + h0;
    b.n_rows = ns;
    b.prebuilt = c->d_reduced.as<float>();
    if (nnls) HIPCHK(launch_solve_nnls(KP, b, c->d_Gt.as<float>(), c->st));
    else HIPCHK(launch_solve_heavy(KP, b, c->st));
  }
  a.rows = rows + h0 + ns;
  a.n_rows = hn - ns;
  a.prebuilt = nullptr;
  if (nnls) HIPCHK(launch_solve_nnls(KP, a, c->d_Gt.as<float>(), c->st));
  else if (use_wave_kernel(c)) HIPCHK(launch_solve_wave(KP, a, c->st));
  else HIPCHK(launch_solve_heavy(KP, a, c->st));
  return ALS_OK;
}

bool use_wave_kernel(const als_ctx* c) { return c->KP <= 128; }

// After a failed solve: what the half's inputs and outputs held (non-finite counts, first bad index,
// max |value|), so a failure that does not repeat still names where it started
std::string failure_diag(als_ctx* c, const Side& S, const Side& T, int64_t ns, const void* zhl) {
  const int KP = c->KP;
  struct Item {
    const char* name;
    const void* p;
    int64_t n;
    bool f16;
  } items[] = {{"src X", S.d_X.p, S.own_n * KP, false},
               {"src Z", S.d_Z.p, ns * KP, false},
               {"Z zero row", S.d_Z.as<float>() + S.prows() * KP, KP, false},
               {"Zhl", zhl, zhl ? (S.prows() + 1) * KP * 2 : 0, true},
               {"lam", c->d_lam.p, KP, false},
               {"colscale", c->d_cs.p, KP, false},
               {"dst X", T.d_X.p, T.own_n * KP, false}};
  const int ni = (int)(sizeof(items) / sizeof(items[0]));
  DevBuf out;
  std::vector<unsigned long long> h((size_t)ni * 3, 0ull);
  for (int i = 0; i < ni; ++i) h[(size_t)i * 3 + 1] = ~0ull;
  // an early return drains the stream first: the queued upload reads h and the scans write out
  auto unavailable = [&]() { (void)hipStreamSynchronize(c->st); return std::string(" [diagnostics unavailable]"); };
  if (out.ensure(h.size() * 8) != hipSuccess ||
      hipMemcpyAsync(out.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, c->st) != hipSuccess)
    return unavailable();
  for (int i = 0; i < ni; ++i)
    if (items[i].p && launch_diag_scan(items[i].p, items[i].n, items[i].f16, out.as<unsigned long long>() + 3 * i, c->st) != hipSuccess)
      return unavailable();
  std::vector<float> lam(KP), cs(KP);
  if (hipMemcpyAsync(h.data(), out.p, h.size() * 8, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
      hipMemcpyAsync(lam.data(), c->d_lam.p, KP * 4, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
      hipMemcpyAsync(cs.data(), c->d_cs.p, KP * 4, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
      hipStreamSynchronize(c->st) != hipSuccess)
    return unavailable();
  std::string r = " [";
  char buf[160];
  for (int i = 0; i < ni; ++i) {
    if (!items[i].p) continue;
    const unsigned mx = (unsigned)h[(size_t)i * 3 + 2];
    float fmx;
    std::memcpy(&fmx, &mx, 4);
    if (h[(size_t)i * 3])
      std::snprintf(buf, sizeof buf, "%s: %llu non-finite (first at %llu, row %llu), max %.3g; ", items[i].name,
                    h[(size_t)i * 3], h[(size_t)i * 3 + 1], h[(size_t)i * 3 + 1] / (items[i].f16 ? 2 * KP : KP), fmx);
    else std::snprintf(buf, sizeof buf, "%s: finite, max %.3g; ", items[i].name, fmx);
    r += buf;
  }
  const auto lm = std::minmax_element(lam.begin(), lam.begin() + c->p.rank);
  const auto cm = std::minmax_element(cs.begin(), cs.begin() + c->p.rank);
  std::snprintf(buf, sizeof buf, "lam %.4g..%.4g, colscale %.4g..%.4g]", *lm.first, *lm.second, *cm.first, *cm.second);
  return r + buf;
}

int half_sweep(als_ctx* c, int t) {
  const int sidx = 1 - t;
  Side& S = c->s[sidx];
  Side& T = c->s[t];
  if (!S.has_factors) return fail(ALS_E_STATE, "source factors are not initialised");
  const int KP = c->KP, k = c->p.rank;
  hipStream_t st = c->st;
  hipEvent_t* ev = c->ev;
  const bool multi = c->world > 1;
  bool have_cmax = false, cs_done = false, split_done = false;
  bool force_heavy = c->p.light_max_degree == 0;
  // world > 1: the previous half's factor gathers (second stream) finish before any collective or
  // rotation of this one is issued -- two RCCL operations of one communicator must never overlap
  if (multi) HIPCHK(hipStreamWaitEvent(st, c->evc[8], 0));
  HIPCHK(hipEventRecord(ev[0], st));
  if (c->p.nonnegative) return half_sweep_nnls(c, t);
  if (multi && !S.full_valid) {  // src factors set outside a half-sweep (init / injection): gather now
    TRYC(gather_chunks(c, S, S.d_X.as<float>(), S.d_Xfull.as<float>(), 0, S.nch, st));
    S.full_valid = true;
  }
  if (c->p.implicit_prefs) {
    HIPCHK(launch_gram(KP, S.d_X.as<float>(), S.own_n, c->slab.as<double>(), c->slab_blocks, c->d_G.as<double>(), st));
    TRYC(allreduce_G(c));
    HIPCHK(hipEventRecord(ev[1], st));
    // eigenbasis of the src Gram on the device (eig.hip): warm-started cyclic Jacobi in fp64, no host
    // round trip; the dst side's new basis B_t = B_s·P is formed there too
    HIPCHK(hipMemcpyAsync(S.d_Gk.p, c->d_G.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(S.d_GB.p, S.d_B.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));
    S.has_gram = true;
    HIPCHK(launch_device_eig(KP, k, c->d_G.as<double>(), S.d_B.as<double>(), T.d_B.as<double>(), T.d_B.as<double>(),
                             c->d_eig.as<double>(), c->d_P.as<float>(), c->d_lam.as<float>(), c->d_csmax.as<unsigned>(), st));
    if (c->p.reg_param == 0.0) {
      // the push-through light solve needs Λ + λn > 0 for every row; with λ = 0 a singular Gram sends
      // every row to the explicit path (the only host round trip left, and only at regParam = 0)
      double wmm[2] = {0.0, 0.0};
      HIPCHK(hipMemcpyAsync(wmm, eig_minmax(c->d_eig.as<double>(), KP), 16, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (!(wmm[0] > 1e-12 * wmm[1])) force_heavy = true;
    }
    HIPCHK(hipEventRecord(ev[2], st));
    // world > 1: every rank rotates the whole gathered src (no collective on the critical path)
    const float* Xs = multi ? S.d_Xfull.as<float>() : S.d_X.as<float>();
    const int64_t ns = multi ? S.prows() : S.own_n;
    if (rotate_bf_on(c)) {
      // bf16 MFMA rotation with the heavy build's split in the same pass.  Its column scales come
      // first, from a bound: Σ_i Z_ij² = p_jᵀ G p_j, which is λ_j up to the fp32 rounding of P and of
      // the product (≤ 1e-6 λ_max), so max_i |Z_ij| ≤ √(λ_j + 1e-6 λ_max).  The split's fp16 range
      // needs the scaled maxima below 2^16; the scales put the bound at 2^13 (colscale_kernel).
      // (the bound itself came from the eigensolver: launch_device_eig left it in d_csmax)
      TRYC(column_scales(c, S, T, true));
      cs_done = true;
      float sw = 1.f;
      split_done = presplit_wanted(c, T, &sw);
      if (split_done) HIPCHK(c->d_Zhl.ensure((size_t)(S.prows() + 1) * KP * 4));
      HIPCHK(c->d_Pf.ensure((size_t)rotate_bf_pfrag_bytes(KP)));
      HIPCHK(launch_rotate_bf(KP, Xs, c->d_P.as<float>(), c->d_Pf.p, S.d_Z.as<float>(), ns, c->d_cs.as<float>(), sw,
                              split_done ? c->d_Zhl.p : nullptr, S.prows(), c->n_cu, st));
    } else {
      // the rotation also leaves the column maxima of Z for the heavy build's column scales
      HIPCHK(hipMemsetAsync(c->d_csmax.p, 0, KP * sizeof(unsigned), st));
      HIPCHK(launch_rotate(KP, Xs, c->d_P.as<float>(), S.d_Z.as<float>(), ns, st, c->d_csmax.as<unsigned>()));
      have_cmax = true;
    }
  } else {
    HIPCHK(hipEventRecord(ev[1], st));
    HIPCHK(hipMemsetAsync(c->d_lam.p, 0, KP * 4, st));
    HIPCHK(hipMemcpyAsync(T.d_B.p, S.d_B.p, (size_t)KP * KP * 8, hipMemcpyDeviceToDevice, st));
    if (c->p.reg_param == 0.0) force_heavy = true;
    HIPCHK(hipEventRecord(ev[2], st));
    if (multi) HIPCHK(hipMemcpyAsync(S.d_Z.p, S.d_Xfull.p, (size_t)S.prows() * KP * 4, hipMemcpyDeviceToDevice, st));
    else HIPCHK(hipMemcpyAsync(S.d_Z.p, S.d_X.p, (size_t)S.own_n * KP * 4, hipMemcpyDeviceToDevice, st));
  }
  HIPCHK(hipEventRecord(ev[3], st));
  if (!cs_done) TRYC(column_scales(c, S, T, have_cmax));
  const void* zhl = nullptr;
  float wsc = 1.f, inv_sw = 1.f;
  TRYC(presplit(c, S, T, &zhl, &wsc, &inv_sw, split_done));
  HIPCHK(hipEventRecord(ev[4], st));
  HIPCHK(hipMemsetAsync(c->d_err.p, 0, 4, st));
  SolveArgs a{};
  a.Zhl = zhl;
  a.zero_row = S.prows();
  a.wsc = wsc;
  a.inv_sw = inv_sw;
  a.Z = S.d_Z.as<float>();
  a.ptr = T.d_ptr.as<int64_t>();
  a.col = T.d_col.as<int32_t>();
  a.val = T.d_val.as<float>();
  a.lam = c->d_lam.as<float>();
  a.X = T.d_X.as<float>();
  a.kreal = k;
  a.implicit = c->p.implicit_prefs;
  a.alpha = (float)c->p.alpha;
  a.reg = (float)c->p.reg_param;
  a.err = c->d_err.as<int>();
  a.colscale = c->d_cs.as<float>();
  a.n_cu = c->n_cu;
  const int32_t* rows = T.d_rows.as<int32_t>();
  static const int Dof[B_HEAVY] = {16, 32, 64, 96};
  T.stats[0] = T.stats[1] = T.stats[2] = T.stats[3] = 0;
  for (int b = 0; b < B_HEAVY; ++b) {
    T.stats[force_heavy ? 2 : 0] += T.boff[b + 1] - T.boff[b];
    T.stats[force_heavy ? 3 : 1] += T.bnnz[b];
  }
  T.stats[2] += T.boff[B_HEAVY + 1] - T.boff[B_HEAVY];
  T.stats[3] += T.bnnz[B_HEAVY];
  // Solve chunk by chunk (one chunk unless world > 1); world > 1: each finished chunk of the new
  // factors is gathered on the second stream while the next chunk solves
  for (int q = 0; q < T.nsolve; ++q) {
    for (int b = 0; b < B_HEAVY; ++b) {
      a.rows = rows + T.cb[b][q];
      a.desc = T.d_desc.as<int32_t>() + 4 * T.cb[b][q];
      a.n_rows = T.cb[b][q + 1] - T.cb[b][q];
      if (force_heavy && use_wave_kernel(c)) HIPCHK(launch_solve_wave(KP, a, st));
      else if (force_heavy) HIPCHK(launch_solve_heavy(KP, a, st));
      else if (b == B_L16) {  // light16.hip: degree <= 8 two rows per wave unit, then the rest
        SolveArgs p8 = a, p16 = a;
        p8.n_rows = T.c8[q];
        p16.rows += T.c8[q];
        p16.desc += 4 * T.c8[q];
        p16.n_rows -= T.c8[q];
        HIPCHK(launch_solve_light16(KP, p8, st, true));
        HIPCHK(launch_solve_light16(KP, p16, st, false));
      } else HIPCHK(launch_solve_light(KP, Dof[b], a, st));
    }
    if (T.nsolve == 1) HIPCHK(hipEventRecord(ev[5], st));
    TRYC(heavy_launches(c, T, a, T.cb[B_HEAVY][q], T.cb[B_HEAVY][q + 1] - T.cb[B_HEAVY][q], false, q));
    if (multi) {
      HIPCHK(hipEventRecord(c->evc[q], st));
      HIPCHK(hipStreamWaitEvent(c->st2, c->evc[q], 0));
      TRYC(gather_chunks(c, T, T.d_X.as<float>(), T.d_Xfull.as<float>(), q, q + 1, c->st2));
    }
  }
  if (T.nsolve > 1) HIPCHK(hipEventRecord(ev[5], st));  // chunked: the whole solve is timed as heavy
  if (multi) {
    if (T.nsolve == 1) TRYC(gather_chunks(c, T, T.d_X.as<float>(), T.d_Xfull.as<float>(), 0, T.nch, c->st2));
    HIPCHK(hipEventRecord(c->evc[8], c->st2));
  }
  HIPCHK(hipEventRecord(ev[6], st));
  int err = 0, sweeps = 0;
  HIPCHK(hipMemcpyAsync(&err, c->d_err.p, 4, hipMemcpyDeviceToHost, st));
  if (c->p.implicit_prefs) HIPCHK(hipMemcpyAsync(&sweeps, eig_sweeps(c->d_eig.as<double>(), KP), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // Cholesky path: the device eigensolver's Jacobi sweeps (als_solver_stats), decoded like
  // als_device_eigh (eig.hip stores -(sweeps + 1) when the budget ran out)
  T.solver[0] = sweeps < 0 ? -sweeps - 1 : sweeps;
  T.solver[1] = T.solver[2] = T.solver[3] = 0;
  T.t[ALS_T_GRAM] = event_ms(ev[0], ev[1]);
  T.t[ALS_T_EIG] = event_ms(ev[1], ev[2]);  // device eigensolver + the new basis
  T.t[ALS_T_ROTATE] = event_ms(ev[2], ev[3]);
  T.t[ALS_T_COMM] = event_ms(ev[3], ev[4]);
  if (T.nsolve > 1) {
    T.t[ALS_T_SOLVE_LIGHT] = 0.0;
    T.t[ALS_T_SOLVE_HEAVY] = event_ms(ev[4], ev[5]);
  } else {
    T.t[ALS_T_SOLVE_LIGHT] = event_ms(ev[4], ev[5]);
    T.t[ALS_T_SOLVE_HEAVY] = event_ms(ev[5], ev[6]);
  }
  T.t[ALS_T_HALF_TOTAL] = event_ms(ev[0], ev[6]);
  if (sweeps < 0)  // eig.hip: the Jacobi sweep budget ran out (the host eigensolver's "did not converge")
    return fail(ALS_E_NOT_POSITIVE_DEFINITE, "eigensolver did not converge (device Jacobi: " +
                                                 std::to_string(-sweeps - 1) + " sweeps without meeting the tolerance)");
  if (err & 3)
    return fail(ALS_E_NOT_POSITIVE_DEFINITE,
                "LAPACK.dppsv-equivalent Cholesky met a non-positive pivot because A is not positive "
                "definite. Is A derived from a singular matrix (e.g. collinear column values)? (flags " +
                    std::to_string(err) + err_paths(err) + ", " + std::to_string(sweeps) + " eigensolver sweeps, " +
                    (t == ALS_USER ? "user" : "item") + " half)" +
                    failure_diag(c, S, T, c->p.implicit_prefs ? (multi ? S.prows() : S.own_n) : S.own_n, zhl));
  T.has_factors = true;
  T.orig_valid = false;
  T.full_valid = multi;  // gathered behind the solve (st2); the next half waits for it
  return ALS_OK;
}

// original-basis factors of `side`, dense order, on device: d_orig [n][KP]
int materialize(als_ctx* c, int side) {
  Side& S = c->s[side];
  if (S.orig_valid) return ALS_OK;
  if (!S.has_factors) return fail(ALS_E_STATE, "factors are not available (call fit first)");
  const int KP = c->KP;
  HIPCHK(c->d_P.ensure((size_t)KP * KP * 4));
  HIPCHK(launch_basis_t32(S.d_B.as<double>(), c->d_P.as<float>(), KP, c->st));
  HIPCHK(S.d_orig.ensure((size_t)std::max<int64_t>(S.n, 1) * KP * 4));
  if (c->world == 1) {
    HIPCHK(launch_rotate(KP, S.d_X.as<float>(), c->d_P.as<float>(), S.d_orig.as<float>(), S.own_n, c->st));
  } else {  // rotate the own chunks, gather them, unpack the chunk-major layout into dense order
    if (c->st2) HIPCHK(hipStreamWaitEvent(c->st, c->evc[8], 0));
    DevBuf own, padded;
    const int64_t nown = (int64_t)S.nch * S.chpad;
    HIPCHK(own.ensure((size_t)nown * KP * 4));
    HIPCHK(padded.ensure((size_t)std::max<int64_t>(S.prows(), 1) * KP * 4));
    HIPCHK(launch_rotate(KP, S.d_X.as<float>(), c->d_P.as<float>(), own.as<float>(), nown, c->st));
    TRYC(gather_chunks(c, S, own.as<float>(), padded.as<float>(), 0, S.nch, c->st));
    for (int r = 0; r < c->world; ++r) {
      const int64_t nr = S.starts[r + 1] - S.starts[r];
      for (int q = 0; q < S.nch && (int64_t)q * S.chpad < nr; ++q) {
        const int64_t l0 = (int64_t)q * S.chpad, cnt = std::min<int64_t>(S.chpad, nr - l0);
        HIPCHK(hipMemcpyAsync(S.d_orig.as<float>() + (size_t)(S.starts[r] + l0) * KP,
                              padded.as<float>() + (size_t)S.pos(r, l0) * KP, (size_t)cnt * KP * 4,
                              hipMemcpyDeviceToDevice, c->st));
      }
    }
    HIPCHK(hipStreamSynchronize(c->st));
  }
  HIPCHK(hipStreamSynchronize(c->st));
  S.orig_valid = true;
  return ALS_OK;
}

int64_t find_row(const Side& S, int32_t id) {
  auto it = std::lower_bound(S.ids.begin(), S.ids.end(), id);
  if (it == S.ids.end() || *it != id) return -1;
  return it - S.ids.begin();
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

const char* als_last_error(void) { return g_err.c_str(); }
int als_abi_version(void) { return ALBEDO_ALS_ABI_VERSION; }

int als_device_count(int* out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  int good = 0;
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, d) == hipSuccess && std::strncmp(pr.gcnArchName, "gfx950", 6) == 0) ++good;
  }
  *out = good;
  return ALS_OK;
}

int als_params_default(als_params* p) {
  if (!p) return fail(ALS_E_INVALID_ARGUMENT, "null params");
  p->rank = 10;
  p->max_iter = 10;
  p->implicit_prefs = 0;
  p->nonnegative = 0;
  p->num_user_blocks = 10;
  p->num_item_blocks = 10;
  p->reg_param = 0.1;
  p->alpha = 1.0;
  p->seed = 0;
  p->device = -1;
  p->light_max_degree = -1;
  return ALS_OK;
}

static int ctx_common(const als_params* p, als_ctx** out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(ALS_E_NO_DEVICE, "no HIP device visible: the ALS engine runs on MI355X (gfx950) only");
  auto* c = new als_ctx();
  c->p = *p;
  c->KP = padded_rank(p->rank);
  if (p->device >= 0) c->dev = p->device;
  else if (hipGetDevice(&c->dev) != hipSuccess) c->dev = 0;
  if (c->dev >= ndev) {
    delete c;
    return fail(ALS_E_NO_DEVICE, "device ordinal out of range");
  }
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, c->dev) != hipSuccess || std::strncmp(pr.gcnArchName, "gfx950", 6) != 0) {
    delete c;
    return fail(ALS_E_NO_DEVICE, "device is not gfx950 (MI355X)");
  }
  c->n_cu = pr.multiProcessorCount;
  if (hipSetDevice(c->dev) != hipSuccess || hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(ALS_E_HIP, "failed to create a HIP stream");
  }
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  for (auto& e : c->evt) (void)hipEventCreate(&e);
  for (auto& e : c->evc) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(ALS_E_HIP, "failed to create a HIP stream");
  }
  *out = c;
  return ALS_OK;
}

int als_create(const als_params* p, als_ctx** out) {
  if (!p || !out) return fail(ALS_E_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  TRYC(validate(p));
  return ctx_common(p, out);
}

int als_set_params(als_ctx* c, const als_params* p) {
  if (!c || !p) return fail(ALS_E_INVALID_ARGUMENT, "null argument");
  if (c->model_only) return fail(ALS_E_STATE, "als_set_params on a model-only context");
  if (c->parent) return fail(ALS_E_STATE, "als_set_params on a fork (fork the parent again instead)");
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    if (c->forks > 0) return fail(ALS_E_STATE, "als_set_params while forks view this context's layout");
  }
  TRYC(validate(p));
  TRYC(set_device(c));
  const int dev = c->dev;
  c->p = *p;
  c->p.device = dev;  // the context stays on its device
  c->KP = padded_rank(p->rank);
  if (c->has_ratings) TRYC(rank_layout(c));  // factors are dropped: the next fit re-initialises
  return ALS_OK;
}

int als_fork(als_ctx* parent, const als_params* p, als_ctx** out) {
  if (!parent || !p || !out) return fail(ALS_E_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (!parent->has_ratings || parent->model_only) return fail(ALS_E_STATE, "als_fork needs a context holding ratings");
  if (parent->world > 1) return fail(ALS_E_UNSUPPORTED, "als_fork of a sharded (multi-rank) context");
  TRYC(validate(p));
  if (p->rank != parent->p.rank || p->nonnegative != parent->p.nonnegative ||
      p->light_max_degree != parent->p.light_max_degree)
    return fail(ALS_E_INVALID_ARGUMENT, "a fork keeps its parent's rank, nonnegative and light_max_degree");
  als_params q = *p;
  q.device = parent->dev;
  als_ctx* c = nullptr;
  TRYC(ctx_common(&q, &c));
  // the ingest and the rank layout are the parent's (read-only during a fit): views, not copies
  c->nnz = parent->nnz;
  c->split_len = parent->split_len;
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    const Side& P = parent->s[side];
    S.n = P.n;
    S.ids = P.ids;
    S.starts = P.starts;
    S.maxrows = P.maxrows;
    S.nch = P.nch;
    S.world = P.world;
    S.chpad = P.chpad;
    S.own0 = P.own0;
    S.own_n = P.own_n;
    S.own_nnz = P.own_nnz;
    S.h_deg = P.h_deg;
    S.vmax = P.vmax;
    S.vmin = P.vmin;
    S.d_ptr.share(P.d_ptr);
    S.d_col.share(P.d_col);
    S.d_val.share(P.d_val);
    S.d_rows.share(P.d_rows);
    S.d_desc.share(P.d_desc);
    S.d_chunk_row.share(P.d_chunk_row);
    S.d_chunk_idx.share(P.d_chunk_idx);
    S.d_slot0.share(P.d_slot0);
    std::memcpy(S.boff, P.boff, sizeof S.boff);
    std::memcpy(S.bnnz, P.bnnz, sizeof S.bnnz);
    S.n_split = P.n_split;
    S.n_chunks = P.n_chunks;
    S.n_batch = P.n_batch;
    S.n_batch_nnz = P.n_batch_nnz;
    std::memcpy(S.bat_off, P.bat_off, sizeof S.bat_off);
    S.nsolve = P.nsolve;
    std::memcpy(S.cb, P.cb, sizeof S.cb);
    std::memcpy(S.c8, P.c8, sizeof S.c8);
    std::memcpy(S.split_n, P.split_n, sizeof S.split_n);
    std::memcpy(S.ck_off, P.ck_off, sizeof S.ck_off);
    std::memcpy(S.sl_off, P.sl_off, sizeof S.sl_off);
  }
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    ++parent->forks;
  }
  c->parent = parent;
  c->has_ratings = true;
  if (int rc = set_device(c); rc != ALS_OK || (rc = factor_buffers(c)) != ALS_OK) {
    const std::string msg = g_err;
    als_destroy(c);
    return fail(rc, msg);
  }
  *out = c;
  return ALS_OK;
}

static void destroy_now(als_ctx* c);

void als_destroy(als_ctx* c) {
  if (!c) return;
  als_ctx* parent_to_free = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    if (c->forks > 0) {  // forks still view this context's ingest: freed with the last of them
      c->doomed = true;
      return;
    }
    if (c->parent && --c->parent->forks == 0 && c->parent->doomed) parent_to_free = c->parent;
  }
  destroy_now(c);
  if (parent_to_free) destroy_now(parent_to_free);
}

static void destroy_now(als_ctx* c) {
  (void)hipSetDevice(c->dev);
  if (c->st) (void)hipStreamSynchronize(c->st);
  if (c->st2) (void)hipStreamSynchronize(c->st2);  // no RCCL gather may be in flight at the destroy
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->evc)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->evt)
    if (e) (void)hipEventDestroy(e);
  if (c->h_plan) (void)hipHostFree(c->h_plan);
  if (c->st2) (void)hipStreamDestroy(c->st2);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

int als_comm_unique_id(void* out128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof id);
  return ALS_OK;
}

int als_comm_init(als_ctx* c, int32_t rank, int32_t world, const void* id128) {
  if (!c || !id128 || world < 1 || rank < 0 || rank >= world) return fail(ALS_E_INVALID_ARGUMENT, "bad comm args");
  if (world > 16) return fail(ALS_E_UNSUPPORTED, "at most 16 ranks (one node)");
  if (c->has_ratings) return fail(ALS_E_STATE, "als_comm_init must precede als_set_ratings");
  TRYC(set_device(c));
  c->rank = rank;
  c->world = world;
  if (world > 1) {
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof id);
    NCCLCHK(ncclCommInitRank(&c->comm, world, id, rank));
  }
  return ALS_OK;
}

int als_comm_init_host(als_ctx* c, int32_t rank, int32_t world, int (*allreduce)(void*, double*, int64_t),
                       int (*allgather)(void*, float*, int64_t), void* user) {
  if (!c || world < 1 || rank < 0 || rank >= world || !allreduce || !allgather)
    return fail(ALS_E_INVALID_ARGUMENT, "bad comm args");
  if (world > 16) return fail(ALS_E_UNSUPPORTED, "at most 16 ranks (one node)");
  if (c->has_ratings) return fail(ALS_E_STATE, "als_comm_init_host must precede als_set_ratings");
  c->rank = rank;
  c->world = world;
  c->h_allreduce = allreduce;
  c->h_allgather = allgather;
  c->h_user = user;
  return ALS_OK;
}

int als_set_ratings(als_ctx* c, int64_t n, const int32_t* user, const int32_t* item, const float* rating) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  if (n <= 0) return fail(ALS_E_INVALID_ARGUMENT, "No ratings available from the input dataset (empty ratings).");
  if (!user || !item || !rating) return fail(ALS_E_INVALID_ARGUMENT, "null ratings");
  TRYC(ingest_allowed(c));
  TRYC(set_device(c));
  DevBuf du, di, dr;
  HIPCHK(du.ensure(n * 4));
  HIPCHK(di.ensure(n * 4));
  HIPCHK(dr.ensure(n * 4));
  HIPCHK(copy_st(c, du.p, user, n * 4, hipMemcpyHostToDevice));
  HIPCHK(copy_st(c, di.p, item, n * 4, hipMemcpyHostToDevice));
  HIPCHK(copy_st(c, dr.p, rating, n * 4, hipMemcpyHostToDevice));
  return ingest_device(c, n, du.as<int32_t>(), di.as<int32_t>(), dr.as<float>());
}

int als_set_ratings_device(als_ctx* c, int64_t n, const int32_t* du, const int32_t* di, const float* dr) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  return ingest_device(c, n, du, di, dr);
}

int64_t als_num_rows(const als_ctx* c, int side) {
  if (!c || (side != 0 && side != 1)) return -1;
  return c->s[side].n;
}
int64_t als_num_ratings(const als_ctx* c) { return c ? c->nnz : -1; }
int als_rank(const als_ctx* c) { return c ? c->p.rank : -1; }

int als_get_ids(const als_ctx* c, int side, int32_t* out) {
  if (!c || (side != 0 && side != 1) || !out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  std::memcpy(out, c->s[side].ids.data(), c->s[side].ids.size() * 4);
  return ALS_OK;
}

int als_set_initial_factors(als_ctx* c, int side, int64_t n, const int32_t* ids, const float* f) {
  if (!c || (side != 0 && side != 1) || !ids || !f) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings before injecting factors");
  TRYC(set_device(c));
  Side& S = c->s[side];
  const int k = c->p.rank;
  std::vector<float> dense((size_t)S.n * k, 0.f);
  std::vector<char> seen(S.n, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = find_row(S, ids[i]);
    if (r < 0) continue;  // ids absent from the ratings are ignored, like Spark's join
    std::memcpy(&dense[(size_t)r * k], f + (size_t)i * k, sizeof(float) * k);
    seen[r] = 1;
  }
  for (int64_t r = 0; r < S.n; ++r)
    if (!seen[r]) return fail(ALS_E_INVALID_ARGUMENT, "initial factors missing for id " + std::to_string(S.ids[r]));
  return upload_factors(c, side, dense.data(), k);
}

int als_init_factors(als_ctx* c) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  TRYC(set_device(c));
  c->s[0].has_factors = c->s[1].has_factors = false;  // explicit request: both sides
  return spark_init(c);
}

int als_init_factors_random(als_ctx* c, uint64_t seed) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  TRYC(set_device(c));
  TRYC(drain(c));
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    HIPCHK(launch_init_random(c->KP, c->p.rank, S.d_X.as<float>(), S.own_n, seed + 0x51ED270B27u * (side + 1),
                              S.own0, c->st));
    HIPCHK(launch_identity(S.d_B.as<double>(), c->KP, c->st));
    S.has_factors = true;
    S.orig_valid = false;
    S.full_valid = false;
  }
  HIPCHK(hipStreamSynchronize(c->st));
  return ALS_OK;
}

int als_half_sweep(als_ctx* c, int dst_side) {
  if (!c || (dst_side != 0 && dst_side != 1)) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  TRYC(set_device(c));
  return half_sweep(c, dst_side);
}

int als_run_sweeps(als_ctx* c, int32_t n) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  TRYC(set_device(c));
  for (int it = 0; it < n; ++it) {
    TRYC(half_sweep(c, ALS_ITEM));
    TRYC(half_sweep(c, ALS_USER));
  }
  return ALS_OK;
}

int als_fit(als_ctx* c) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  if (!c->has_ratings)
    return fail(ALS_E_INVALID_ARGUMENT, "No ratings available from the input dataset (empty ratings).");
  TRYC(set_device(c));
  TRYC(spark_init(c));  // only the sides the caller did not inject
  return als_run_sweeps(c, c->p.max_iter);
}

int als_get_basis(als_ctx* c, int side, double* out) {
  if (!c || (side != 0 && side != 1) || !out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  const Side& S = c->s[side];
  if (!S.d_B.p) return fail(ALS_E_STATE, "no factors yet");
  TRYC(set_device(c));
  const int k = c->p.rank, KP = c->KP;
  std::vector<double> B((size_t)KP * KP);
  HIPCHK(hipMemcpyAsync(B.data(), S.d_B.p, B.size() * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) out[(size_t)i * k + j] = B[(size_t)i * KP + j];
  return ALS_OK;
}

int als_get_gram(als_ctx* c, int src_side, double* out) {
  if (!c || (src_side != 0 && src_side != 1) || !out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  const Side& S = c->s[src_side];
  if (!S.has_gram) return fail(ALS_E_STATE, "no Gram computed yet");
  TRYC(set_device(c));
  // G was formed from the factors in the side's basis at that time (original = X·GBᵀ):
  // YᵀY = GB G GBᵀ, restricted to the model rank (GB is the identity on the padding)
  const int k = c->p.rank, KP = c->KP;
  std::vector<double> Gf((size_t)KP * KP), GB((size_t)KP * KP), G((size_t)k * k);
  HIPCHK(hipMemcpyAsync(Gf.data(), S.d_Gk.p, Gf.size() * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(GB.data(), S.d_GB.p, GB.size() * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) G[(size_t)i * k + j] = Gf[(size_t)i * KP + j];
  std::vector<double> T((size_t)k * k, 0.0);  // T = GB_k G
  for (int i = 0; i < k; ++i)
    for (int m = 0; m < k; ++m) {
      const double b = GB[(size_t)i * KP + m];
      if (b == 0.0) continue;
      for (int j = 0; j < k; ++j) T[(size_t)i * k + j] += b * G[(size_t)m * k + j];
    }
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) {
      double acc = 0.0;
      for (int m = 0; m < k; ++m) acc += T[(size_t)i * k + m] * GB[(size_t)j * KP + m];
      out[(size_t)i * k + j] = acc;
    }
  return ALS_OK;
}

int als_get_factors(als_ctx* c, int side, int32_t* ids_out, float* f_out) {
  if (!c || (side != 0 && side != 1)) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  TRYC(set_device(c));
  TRYC(materialize(c, side));
  Side& S = c->s[side];
  if (ids_out) std::memcpy(ids_out, S.ids.data(), S.n * 4);
  if (f_out) {
    const int KP = c->KP, k = c->p.rank;
    std::vector<float> h((size_t)S.n * KP);
    HIPCHK(copy_st(c, h.data(), S.d_orig.p, h.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < S.n; ++r) std::memcpy(f_out + (size_t)r * k, &h[(size_t)r * KP], sizeof(float) * k);
  }
  return ALS_OK;
}

int als_model_create(int32_t rank, int64_t nu, const int32_t* uids, const float* uf, int64_t ni,
                     const int32_t* iids, const float* ifac, int32_t device, als_ctx** out) {
  if (!out) return fail(ALS_E_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  als_params p;
  als_params_default(&p);
  p.rank = rank;
  p.device = device;
  TRYC(validate(&p));
  if (nu < 0 || ni < 0 || (nu && (!uids || !uf)) || (ni && (!iids || !ifac)))
    return fail(ALS_E_INVALID_ARGUMENT, "bad factor arrays");
  als_ctx* c = nullptr;
  TRYC(ctx_common(&p, &c));
  c->model_only = true;
  const int64_t ns[2] = {nu, ni};
  const int32_t* ids[2] = {uids, iids};
  const float* fs[2] = {uf, ifac};
  for (int side = 0; side < 2; ++side) {
    Side& S = c->s[side];
    std::vector<int64_t> ord(ns[side]);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return ids[side][a] < ids[side][b]; });
    S.n = ns[side];
    S.ids.resize(S.n);
    std::vector<float> h((size_t)std::max<int64_t>(S.n, 1) * c->KP, 0.f);
    for (int64_t r = 0; r < S.n; ++r) {
      S.ids[r] = ids[side][ord[r]];
      if (r > 0 && S.ids[r] == S.ids[r - 1]) {
        als_destroy(c);
        return fail(ALS_E_INVALID_ARGUMENT, "duplicate id in factors");
      }
      std::memcpy(&h[(size_t)r * c->KP], fs[side] + (size_t)ord[r] * rank, sizeof(float) * rank);
    }
    if (S.d_orig.ensure(h.size() * 4) != hipSuccess ||
        copy_st(c, S.d_orig.p, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      als_destroy(c);
      return fail(ALS_E_OUT_OF_MEMORY, "failed to upload factors");
    }
    S.orig_valid = true;
    S.has_factors = true;
    S.starts = {0, S.n};
    S.maxrows = S.n;
    S.chpad = std::max<int64_t>(1, S.n);
  }
  *out = c;
  return ALS_OK;
}

// One recommendForAll* call's prepared dst side (topk.hip): max row norms (the pre-selection's error
// bound), fp16 power-of-two scales, the descending-norm fp16 image with chunk head norms, dst ids on
// the device; plus the per-chunk scratch reused by every src chunk.
struct TopkPlan {
  int src = 0, k = 0;
  bool exact_only = false;
  double tmax = 0.0, smax = 0.0, ssc = 1.0, tsc = 1.0;
  int CH = 0;
  int64_t n_chunks = 0, n_super = 0;
  bool prune = false;
  DevBuf d_th, d_keys, d_perm, d_nperm, d_tp, d_tmp, d_dstids, d_VP, d_cfeat, d_supf, d_probe, d_slab, d_G;
  DevBuf d_scan;
  // a pass's device buffers; two sets, so that a pass's select / rescans (on the post stream) can run
  // while the next pass orders and scans with the other set (r06)
  struct PassBufs {
    DevBuf d_src, d_ls, d_lc, d_flag, d_okeys, d_order, d_srcs, d_otmp, d_thr, d_sf, d_mask, d_kth, d_inv;
    DevBuf d_cnt;  // int [4]: the range's flagged count, the rescan work counter, the set's flagged total
  } pb[2];
  // per call (topk_begin .. topk_finish): the passes run back to back with no host round trip; their
  // event pairs, scan counters (d_scan[pass]) and rows per scan workgroup are read at the end
  // per pass: start, order + mask done, scan done, then per output range: select done, rescans done
  std::vector<hipEvent_t> evs;
  struct PassRec { int rpw; size_t e0; int ranges; };
  std::vector<PassRec> passes;
  int64_t n_passes = 0;
  hipError_t event(size_t i, hipEvent_t* e) {  // the i-th event of the pool (created on demand)
    while (evs.size() <= i) {
      hipEvent_t x;
      const hipError_t r = hipEventCreate(&x);
      if (r != hipSuccess) return r;
      evs.push_back(x);
    }
    *e = evs[i];
    return hipSuccess;
  }
  ~TopkPlan() {
    for (hipEvent_t e : evs)
      if (e) (void)hipEventDestroy(e);
  }
};

// The dst side's Gram Σ t tᵀ (original basis) on the device, copied into c->h_plan ([KP][KP] fp64)
// on st; `done` is recorded behind the copy, so the host can wait for it alone.
int topk_dst_gram(als_ctx* c, const Side& T, TopkPlan& P, hipEvent_t done) {
  const int KP = c->KP;
  const int nblk = gram_slab_blocks(KP, T.n);
  double* slab = c->slab.as<double>();  // the sweeps' Gram scratch (idle here, same stream) when it fits
  if (c->slab_blocks < nblk || !slab) {
    HIPCHK(P.d_slab.ensure(gram_slab_doubles(KP, nblk) * 8));
    slab = P.d_slab.as<double>();
  }
  HIPCHK(P.d_G.ensure((size_t)KP * KP * 8));
  HIPCHK(launch_gram(KP, T.d_orig.as<float>(), T.n, slab, nblk, P.d_G.as<double>(), c->st));
  // into pinned memory: a pageable copy would block the host here until the stream drains
  HIPCHK(hipMemcpyAsync(c->h_plan, P.d_G.p, (size_t)KP * KP * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipEventRecord(done, c->st));
  return ALS_OK;
}

// The leading TOPK_M eigenvectors of that Gram, fp64 [TOPK_M][KP]: the directions the top-k chunk
// bound keeps exactly (topk.hip).  Runs on the host while the row norms are computed on the device.
int topk_dst_basis(als_ctx* c, const double* Gf, std::vector<double>& VP) {
  const int KP = c->KP, k = c->p.rank;
  std::vector<double> Gk((size_t)k * k), w(k), V((size_t)k * k);
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) Gk[(size_t)i * k + j] = Gf[(size_t)i * KP + j];
  if (!sym_eig(k, Gk.data(), w.data(), V.data()))
    return fail(ALS_E_NOT_POSITIVE_DEFINITE, "eigendecomposition of the dst Gram matrix did not converge");
  std::vector<int> idx(k);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return w[a] > w[b]; });
  VP.assign((size_t)TOPK_M * KP, 0.0);
  for (int d = 0; d < TOPK_M && d < k; ++d)
    for (int i = 0; i < k; ++i) VP[(size_t)d * KP + i] = V[(size_t)i * k + idx[d]];
  return ALS_OK;
}

// The scan prunes against the kt-th best candidate so far, not the 64th: certification needs a gap
// between the k-th exact score and the kt-th approximate one (~1e-3 relative), and k + 16 leaves one
// while the threshold rises faster than at 64 (fewer dst chunks scanned once the factors converge).
// The lists still hold 64 and the best 64 are rescored.
// the running threshold's rank in the candidate lists: k + 16 (c4 all users after 25 sweeps: k + 8 /
// 12 / 16 / 24 -> 33.6 / 47.6 / 50.7 / 46.9M users/s; fewer leave more rows to the exact rescan)
int topk_threshold_rank(int k) { return std::max(k, std::min(TOPK_KC, k + ALBEDO_TOPK_KT_EXTRA)); }

int topk_plan(als_ctx* c, int src, int k, TopkPlan& P, const std::function<void(const char*)>& stamp = nullptr) {
  auto st = [&](const char* w) {
    if (stamp) stamp(w);
  };
  P.src = src;
  P.k = k;
  P.exact_only = k > TOPK_KC;  // no MFMA pre-selection: exact full scan of every row
  TRYC(materialize(c, src));
  TRYC(materialize(c, 1 - src));
  st("  plan: materialize dst");
  Side& S = c->s[src];
  Side& T = c->s[1 - src];
  const int KP = c->KP;
  // the dst Gram first; its host eigensolve overlaps the row-norm launches behind it
  std::vector<double> VP;
  hipEvent_t ev_gram;
  HIPCHK(P.event(0, &ev_gram));
  if (!c->h_plan) HIPCHK(hipHostMalloc((void**)&c->h_plan, ((size_t)KP * KP + 2) * 8, hipHostMallocDefault));
  {
    DevBuf d_nrm;
    HIPCHK(d_nrm.ensure(16));
    TRYC(topk_dst_gram(c, T, P, ev_gram));
    HIPCHK(launch_rownorm_max(T.d_orig.as<float>(), T.n, KP, c->p.rank, d_nrm.as<unsigned long long>(), c->st));
    HIPCHK(launch_rownorm_max(S.d_orig.as<float>(), S.n, KP, c->p.rank, d_nrm.as<unsigned long long>() + 1, c->st));
    double* nr = c->h_plan + (size_t)KP * KP;
    HIPCHK(hipMemcpyAsync(nr, d_nrm.p, 16, hipMemcpyDeviceToHost, c->st));
    st("  plan: dst Gram + row norms enqueued");
    HIPCHK(hipEventSynchronize(ev_gram));
    st("  plan: dst Gram");
    TRYC(topk_dst_basis(c, c->h_plan, VP));
    st("  plan: host eigensolve (row norms on the device)");
    HIPCHK(hipStreamSynchronize(c->st));
    P.tmax = nr[0];
    P.smax = nr[1];
  }
  // |entry| <= row norm, so scaling by 2^(13 - ceil(log2 max norm)) keeps every fp16 value < 2^13
  auto pow2_scale = [](double m) {
    if (!(m > 0.0) || !std::isfinite(m)) return 1.0;
    int e = 0;
    std::frexp(m, &e);  // m < 2^e
    e = std::max(-60, std::min(60, 13 - e));
    return std::ldexp(1.0, e);
  };
  P.ssc = pow2_scale(P.smax);
  P.tsc = pow2_scale(P.tmax);
  // dst side in descending-norm order, fp16 rows + chunk head norms (also for k > 64: the exact scan
  // visits the dst rows in this norm order and stops early)
  P.CH = topk_chunk_rows(KP);
  P.n_chunks = (T.n + P.CH - 1) / P.CH;
  P.n_super = (P.n_chunks + TOPK_SUPER - 1) / TOPK_SUPER;
  // the chunk bound prunes only catalogues larger than the candidate lists (smaller ones are scanned
  // whole: the lists then hold every dst row, which select's n_dst <= TOPK_KC shortcut relies on)
  P.prune = T.n > TOPK_KC;
  st("  plan: row norms");
  HIPCHK(P.d_VP.ensure(VP.size() * 8));
  HIPCHK(hipMemcpyAsync(P.d_VP.p, VP.data(), VP.size() * 8, hipMemcpyHostToDevice, c->st));
  const int64_t nn = std::max<int64_t>(T.n, 1);
  HIPCHK(P.d_th.ensure((size_t)std::max<int64_t>(P.n_chunks, 1) * P.CH * KP * 2));
  HIPCHK(P.d_keys.ensure((size_t)nn * 16));
  HIPCHK(P.d_perm.ensure((size_t)nn * 8));
  HIPCHK(P.d_nperm.ensure((size_t)nn * 8));
  HIPCHK(P.d_tp.ensure((size_t)nn * TOPK_M * 8));
  HIPCHK(P.d_cfeat.ensure((size_t)std::max<int64_t>(P.n_chunks, 1) * TOPK_CF * 4));
  HIPCHK(P.d_supf.ensure((size_t)std::max<int64_t>(P.n_super, 1) * TOPK_CF * 4));
  HIPCHK(P.d_probe.ensure((size_t)TOPK_NPROBE * KP * 2));
  const size_t tb = topk_sort_temp_bytes(T.n);
  HIPCHK(P.d_tmp.ensure(std::max<size_t>(tb, 16)));
  if (T.n > 0)
    HIPCHK(topk_prepare(KP, c->p.rank, T.d_orig.as<float>(), T.n, (float)P.tsc, P.d_VP.as<double>(), P.d_tmp.p, tb,
                        P.d_keys.as<uint32_t>(), P.d_perm.as<uint32_t>(), P.d_nperm.as<uint32_t>(),
                        P.d_tp.as<double>(), P.d_th.p, P.d_cfeat.as<float>(), P.d_supf.as<float>(), P.d_probe.p,
                        c->st));
  st("  plan: dst sort + fp16 pack + chunk features");
  HIPCHK(P.d_dstids.ensure(std::max<int64_t>(T.n, 1) * 4));
  HIPCHK(hipMemcpyAsync(P.d_dstids.p, T.ids.data(), T.n * 4, hipMemcpyHostToDevice, c->st));
  HIPCHK(P.d_scan.ensure(8));
  st("  plan: dst ids");
  return ALS_OK;
}

// Src rows per top-k pass: 2^25 (candidate lists 32 GiB of the 288 GB), or what half of the free
// device memory holds at ~1.5 KiB per src row (the TOPK_CAP-entry candidate list plus the row's
// features, order keys and output slots), so a smaller GPU or ranks sharing one fall back to more passes
static int64_t topk_pass_rows(als_ctx* c) {
  size_t fr = 0, tot = 0;
  int64_t cap = (int64_t)1 << 25;
  if (set_device(c) == ALS_OK && hipMemGetInfo(&fr, &tot) == hipSuccess) {
    const int64_t fit = (int64_t)(fr / 2 / 1536);
    cap = std::min<int64_t>(cap, std::max<int64_t>((int64_t)1 << 16, fit & ~(int64_t)0xFFFF));
  }
  return cap;
}

// A call's top-k passes: topk_begin (n_rows positions, at most n_passes passes; the rescan flags of
// position p land in c->d_last_need[p]), topk_run_rows per pass, topk_finish (one synchronisation:
// timers and counters).
int topk_begin(als_ctx* c, TopkPlan& P, int64_t n_rows, int64_t n_passes, const int32_t* rows) {
  HIPCHK(P.d_scan.ensure((size_t)std::max<int64_t>(n_passes, 1) * 8));
  HIPCHK(hipMemsetAsync(P.d_scan.p, 0, (size_t)std::max<int64_t>(n_passes, 1) * 8, c->st));
  for (auto& B : P.pb) {
    HIPCHK(B.d_cnt.ensure(16));
    HIPCHK(hipMemsetAsync(B.d_cnt.p, 0, 16, c->st));
  }
  HIPCHK(c->d_last_need.ensure((size_t)std::max<int64_t>(n_rows, 1) * 4));
  HIPCHK(hipMemsetAsync(c->d_last_need.p, 0, (size_t)std::max<int64_t>(n_rows, 1) * 4, c->st));
  c->last_need_n = n_rows;
  c->last_src = P.src;
  c->last_rows_dense = rows == nullptr;
  if (rows) c->last_rows.assign(rows, rows + n_rows);
  else c->last_rows.clear();
  c->last_rescan.clear();
  c->last_rescan_ready = false;
  P.n_passes = n_passes;
  P.passes.clear();
  return ALS_OK;
}

int topk_finish(als_ctx* c, TopkPlan& P, hipStream_t sp = nullptr) {
  if (sp) HIPCHK(hipStreamSynchronize(sp));
  HIPCHK(hipStreamSynchronize(c->st));
  const int64_t np = (int64_t)P.passes.size();
  std::vector<unsigned long long> scanned((size_t)std::max<int64_t>(np, 1), 0ull);
  int cnt[4] = {0, 0, 0, 0}, cnt1[4] = {0, 0, 0, 0};
  if (np > 0) HIPCHK(copy_st(c, scanned.data(), P.d_scan.p, np * 8, hipMemcpyDeviceToHost));
  HIPCHK(copy_st(c, cnt, P.pb[0].d_cnt.p, 16, hipMemcpyDeviceToHost));
  HIPCHK(copy_st(c, cnt1, P.pb[1].d_cnt.p, 16, hipMemcpyDeviceToHost));
  cnt[2] += cnt1[2];
  for (int64_t q = 0; q < np; ++q) {
    const TopkPlan::PassRec& R = P.passes[q];
    const hipEvent_t* e = P.evs.data() + R.e0;
    c->topk_ms[0] += event_ms(e[0], e[1]);
    c->topk_ms[1] += event_ms(e[1], e[2]);
    for (int r = 0; r < R.ranges; ++r) {
      c->topk_ms[2] += event_ms(r == 0 ? e[2] : e[3 + 2 * r - 1], e[3 + 2 * r]);
      c->topk_ms[3] += event_ms(e[3 + 2 * r], e[4 + 2 * r]);
    }
    c->topk_stats[2] += (int64_t)scanned[q];
    c->topk_ms[4] += (double)scanned[q] * (R.rpw / 4) * 2.0 * c->KP;  // per wave: rpw / 4 src rows x each dst row
  }
  c->topk_stats[1] += cnt[2];
  return ALS_OK;
}

// One pass: the nc src rows `rows` (host, dense row indices; nullptr: rows row0 .. row0 + nc - 1,
// generated on the device) at positions pos0 .. pos0 + nc - 1 of the call, into the device lists
// d_oid / d_osc ([nc][k], score desc, id asc).  Rows that fail certification are compacted on the
// device and re-scored by a persistent exact scan in the same stream: nothing here waits for the GPU.
// After the scan the results are finished in output ranges of `range` rows (select, then the
// rescans of the range); ready(o0, o1), when given, is called once a range's work is enqueued, so
// the caller can copy those rows out while the next range computes.
using TopkReady = std::function<int(int64_t, int64_t)>;
int topk_run_rows(als_ctx* c, TopkPlan& P, const int32_t* rows, int64_t row0, int64_t pos0, int64_t nc, int32_t* d_oid,
                  float* d_osc, int64_t range = INT64_MAX, const TopkReady& ready = nullptr, int par = 0,
                  hipStream_t sp = nullptr) {
  // buffer set `par`; with a post stream sp the select / rescans wait for the scan on sp, so the
  // caller's next pass (the other set) can order and scan meanwhile
  TopkPlan::PassBufs& B = P.pb[par];
  hipStream_t ps = sp ? sp : c->st;
  Side& S = c->s[P.src];
  Side& T = c->s[1 - P.src];
  const int KP = c->KP, k = P.k;
  if (nc <= 0) return ALS_OK;
  HIPCHK(B.d_src.ensure(nc * 4));
  if (!P.exact_only) {
    HIPCHK(B.d_ls.ensure(nc * TOPK_CAP * 8));
    HIPCHK(B.d_lc.ensure(nc * 4));
  }
  if (rows) HIPCHK(hipMemcpyAsync(B.d_src.p, rows, nc * 4, hipMemcpyHostToDevice, c->st));
  else HIPCHK(launch_iota_i32(B.d_src.as<int32_t>(), nc, row0, c->st));
  (void)S;
  TopkArgs a{};
  a.S = S.d_orig.as<float>();
  a.T = T.d_orig.as<float>();
  a.src_rows = B.d_src.as<int32_t>();
  a.n_src = nc;
  a.n_dst = T.n;
  a.dst_ids = P.d_dstids.as<int32_t>();
  a.kreal = c->p.rank;
  a.k = k;
  a.kt = topk_threshold_rank(k);
  a.tmax_norm = (float)(P.tmax * (1.0 + 1e-6));
  a.Th = P.d_th.p;
  a.perm = P.d_perm.as<uint32_t>();
  a.n_chunks = P.n_chunks;
  a.VP = P.d_VP.as<double>();
  a.cfeat = P.prune ? P.d_cfeat.as<float>() : nullptr;
  a.probe = P.d_probe.p;
  a.ssc = (float)P.ssc;
  a.tsc = (float)P.tsc;
  a.unscale = (float)(1.0 / (P.ssc * P.tsc));
  a.scaled = (float)(P.ssc * P.tsc);
  a.lent = B.d_ls.as<uint2>();
  a.lcnt = B.d_lc.as<int32_t>();
  // scan order: 12 bits of depth, then 7 / 7 / 6 bits of direction (topk_order_key_kernel; c4 all
  // users: scan 260 -> 193 ms, order + mask 56 -> 39 ms against the depth-only key; 18 / 22 / 24
  // direction bits 206 / 206 / 276 ms, other splits of 20 the same 193)
  a.order_dir_bits = 7 | (7 << 8) | (6 << 16);
  a.out_ids = d_oid;
  a.out_scores = d_osc;
  int32_t* d_need = c->d_last_need.as<int32_t>() + pos0;
  a.need_exact = d_need;
  if (!P.exact_only) {
    HIPCHK(B.d_kth.ensure(nc * 4));
    a.kth0 = B.d_kth.as<float>();
  }
  const int64_t pass = (int64_t)P.passes.size();
  if (pass >= P.n_passes) return fail(ALS_E_STATE, "top-k: more passes than planned");
  a.scanned = P.d_scan.as<unsigned long long>() + pass;
  if (P.exact_only) {
    HIPCHK(launch_topk_exact(KP, a, nullptr, nc, c->st));
    if (ready) TRYC(ready(0, nc));
    return ALS_OK;
  }
  const int64_t nr = std::max<int64_t>(1, (nc + range - 1) / range);  // output ranges
  const size_t e0 = P.evs.size();
  hipEvent_t ev[3];
  for (int i = 0; i < 3; ++i) HIPCHK(P.event(e0 + i, &ev[i]));
  // scan order: rows that stop at similar depths share a workgroup (topk_order); the select writes
  // each row's results back to its own slot
  TopkArgs b = a;
  HIPCHK(hipEventRecord(ev[0], c->st));
  HIPCHK(B.d_okeys.ensure(nc * 8));
  HIPCHK(B.d_order.ensure(nc * 8));
  HIPCHK(B.d_srcs.ensure(nc * 4));
  const size_t otb = topk_order_temp_bytes(nc);
  HIPCHK(B.d_otmp.ensure(std::max<size_t>(otb, 16)));
  HIPCHK(B.d_thr.ensure(nc * 8));
  HIPCHK(B.d_sf.ensure((size_t)nc * TOPK_SF * 8));
  float* sf_tmp = B.d_sf.as<float>();
  float* sf_sorted = sf_tmp + (size_t)nc * TOPK_SF;
  HIPCHK(topk_order(KP, a, B.d_otmp.p, otb, B.d_okeys.as<uint32_t>(), B.d_order.as<uint32_t>(), B.d_srcs.as<int32_t>(),
                    B.d_thr.as<float>(), B.d_thr.as<float>() + nc, sf_tmp, sf_sorted, c->st));
  b.src_rows = B.d_srcs.as<int32_t>();
  b.out_pos = B.d_order.as<uint32_t>();
  b.thr0 = B.d_thr.as<float>() + nc;
  b.sfeat = sf_sorted;
  const int rpw = topk_rows_per_workgroup(KP, nc, c->n_cu);
  if (P.prune) {  // per scan workgroup, the chunks its rows can need against the starting thresholds
    const int64_t n_wg = (nc + rpw - 1) / rpw;
    b.mask_words = (P.n_super + 1) / 2;
    HIPCHK(B.d_mask.ensure((size_t)n_wg * b.mask_words * 4));
    b.mask = B.d_mask.as<uint32_t>();
    HIPCHK(launch_topk_mask(b, rpw, P.d_supf.as<float>(), P.n_super, B.d_mask.as<uint32_t>(), c->st));
  }
  HIPCHK(hipEventRecord(ev[1], c->st));
  HIPCHK(launch_topk(KP, b, c->n_cu, c->st));
  HIPCHK(hipEventRecord(ev[2], c->st));
  HIPCHK(B.d_flag.ensure(nc * 4));
  if (nr > 1) HIPCHK(B.d_inv.ensure(nc * 4));
  if (sp) HIPCHK(hipStreamWaitEvent(sp, ev[2], 0));  // the select needs this pass's scan
  if (nr > 1) {  // select by output slot: slot -> scan position
    HIPCHK(launch_invert_perm(b.out_pos, nc, B.d_inv.as<uint32_t>(), ps));
  }
  P.passes.push_back(TopkPlan::PassRec{rpw, e0, 0});
  for (int64_t r = 0; r < nr; ++r) {
    const int64_t o0 = r * range, n = std::min<int64_t>(range, nc - o0);
    hipEvent_t es, ex;
    HIPCHK(P.event(e0 + 3 + 2 * r, &es));
    HIPCHK(P.event(e0 + 4 + 2 * r, &ex));
    TopkArgs bs = b;
    if (nr > 1) {
      bs.in_pos = B.d_inv.as<uint32_t>();
      bs.slot0 = o0;
      bs.n_slots = n;
    }
    HIPCHK(launch_topk_select(KP, bs, ps));
    HIPCHK(hipEventRecord(es, ps));
    // certification failures of the range: compacted on the device (range-local positions), re-scored
    // in place
    TopkArgs ar = a;
    ar.src_rows = a.src_rows + o0;
    ar.out_ids = a.out_ids + o0 * k;
    ar.out_scores = a.out_scores + o0 * k;
    ar.kth0 = a.kth0 + o0;
    ar.n_src = n;
    HIPCHK(hipMemsetAsync(B.d_cnt.p, 0, 8, ps));  // this range's count and work counter
    HIPCHK(launch_topk_exact_flagged(KP, ar, d_need + o0, n, B.d_flag.as<int32_t>(), B.d_cnt.as<int>(), c->n_cu, ps));
    HIPCHK(hipEventRecord(ex, ps));
    P.passes.back().ranges = (int)(r + 1);
    if (ready) TRYC(ready(o0, o0 + n));
  }
  c->topk_stats[0] += nc;
  c->topk_stats[3] += (nc + rpw - 1) / rpw * 4 * P.n_chunks * P.CH;  // dst rows x waves
  return ALS_OK;
}

int als_recommend(als_ctx* c, int side, int32_t k, const int32_t* subset, int64_t n_subset, int32_t* src_ids_out,
                  int32_t* dst_ids_out, float* scores_out) {
  if (!c || (side != 0 && side != 1) || !dst_ids_out || !scores_out)
    return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (k <= 0) return fail(ALS_E_INVALID_ARGUMENT, "num must be positive");
  if (k > TOPK_MAX)
    return fail(ALS_E_UNSUPPORTED, "num above " + std::to_string(TOPK_MAX) + " is not supported by this engine");
  TRYC(set_device(c));
  // ALBEDO_TOPK_TRACE (diagnostic): wall-clock stamps of the call's phases on stderr, the stream
  // synchronised at each (so the stamps bracket device work)
  static const bool trace = [] {
    const char* e = std::getenv("ALBEDO_TOPK_TRACE");
    return e && *e && *e != '0';
  }();
  const auto t_start = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (!trace) return;
    (void)hipStreamSynchronize(c->st);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    std::fprintf(stderr, "[topk] %9.2f ms  %s\n", ms, what);
  };
  const int src = side;
  TRYC(materialize(c, src));
  stamp("materialize src");
  Side& S = c->s[src];
  const Side& T = c->s[1 - src];
  const int64_t nq = subset ? n_subset : S.n;
  // recommendForAll*: every src row, in row order -- no host index arrays (the device generates the
  // row indices of each pass); a subset: id -> row by a merge walk when ascending (the usual case),
  // binary search otherwise, unknown ids padded here
  const bool all_rows = subset == nullptr;
  std::vector<int32_t> known;
  std::vector<int64_t> pos;
  if (!all_rows) {
    std::vector<int32_t> qrow(nq);
    if (std::is_sorted(subset, subset + nq)) {
      int64_t r = 0;
      for (int64_t i = 0; i < nq; ++i) {
        while (r < S.n && S.ids[r] < subset[i]) ++r;
        qrow[i] = (r < S.n && S.ids[r] == subset[i]) ? (int32_t)r : -1;
      }
    } else {
      for (int64_t i = 0; i < nq; ++i) qrow[i] = (int32_t)find_row(S, subset[i]);
    }
    known.reserve(nq);
    pos.reserve(nq);
    for (int64_t i = 0; i < nq; ++i)
      if (qrow[i] >= 0) {
        known.push_back(qrow[i]);
        pos.push_back(i);
      } else {
        std::fill(dst_ids_out + i * k, dst_ids_out + (i + 1) * k, -1);
        std::fill(scores_out + i * k, scores_out + (i + 1) * k, NAN);
      }
  }
  if (src_ids_out) {
    if (all_rows) std::memcpy(src_ids_out, S.ids.data(), (size_t)nq * 4);
    else std::memcpy(src_ids_out, subset, (size_t)nq * 4);
  }
  const int64_t n_known = all_rows ? nq : (int64_t)known.size();
  auto posf = [&](int64_t i) { return all_rows ? i : pos[i]; };           // output slot of known row i
  auto rowsf = [&](int64_t q0) { return all_rows ? nullptr : known.data() + q0; };  // null: rows q0 ..
  const bool dense_out = n_known == nq;  // results land in place, no scatter
  c->last_rescan.clear();
  c->last_rescan_ready = true;
  if (n_known == 0 || T.n == 0) return ALS_OK;
  stamp("host id mapping");
  // Src rows per pass: up to 2^25 (candidate lists 32 GiB of the 288 GB).  One scan launch over every
  // row dispatches the heaviest workgroups (lowest relative thresholds) first and fills in behind
  // them; split into 4M-row passes, each pass paid its own heavy tail (c4 all users: scan 436 ms in
  // five passes, 260 ms in one; profiles/r05_bench_c4_topk_pass{4M,10M,20M}.json).  The results are
  // finished and copied out in ranges of pass / 8 rows (at most 4M) while the next range computes.
  // ALBEDO_TOPK_PASS (test knob): rows per pass.
  // ALBEDO_TOPK_OVERLAP=1 (r06 experiment, off by default): with the lists written in place the select
  // is link-bound (~40 GB/s of lists) and the scan compute-bound, so a call of >= 2M rows runs as two
  // passes whose first select / rescans (post stream, second buffer set) overlap the second order +
  // scan.  Measured slower (c4 all users 0.318 vs 0.293 s, profiles/r06_bench_c4_topk_overlap_REJECTED
  // .json): the store-bound select waves slow the concurrent scan, and the second pass adds its own
  // order, sort and mask.
  const bool want_overlap = [] {
    const char* e = std::getenv("ALBEDO_TOPK_OVERLAP");
    return e && std::atoi(e) == 1;
  }();
  const int64_t chunk = [&] {
    const char* e = std::getenv("ALBEDO_TOPK_PASS");
    if (e && *e) return std::max<int64_t>(1 << 16, std::atoll(e));
    const int64_t cap = topk_pass_rows(c);
    const int64_t n_here = (std::min<int64_t>(n_known, ((int64_t)c->rank + 1) * ((n_known + c->world - 1) / c->world)) -
                            std::min<int64_t>(n_known, (int64_t)c->rank * ((n_known + c->world - 1) / c->world)));
    if (want_overlap && n_here >= ((int64_t)1 << 21)) return std::min<int64_t>(cap, (n_here + 1) / 2);
    return cap;
  }();
  const int64_t range = std::min<int64_t>((int64_t)1 << 22, std::max<int64_t>(chunk / 8, 1 << 16));
  // world > 1 (SURVEY §8(e) "Top-k: shard users"): rank r scores the r-th contiguous slice of the
  // known src rows against the replicated dst factors; the lists are all-gathered afterwards
  const int64_t per_rank = (n_known + c->world - 1) / c->world;
  const int64_t lo = std::min<int64_t>(n_known, (int64_t)c->rank * per_rank);
  const int64_t hi = std::min<int64_t>(n_known, lo + per_rank);
  std::vector<int64_t> pstart;  // pass starts
  {
    int64_t q = lo;
    while (hi - q > chunk) {
      pstart.push_back(q);
      q += chunk;
    }
    if (q < hi) {
      pstart.push_back(q);
    }
  }
  const int64_t n_pass = (int64_t)pstart.size();
  // dense output (every row of the side, the recommendForAll* case): the caller's arrays are pinned
  // in place (by a helper thread, while the plan runs) and each range's lists go down on a copy stream
  // while the next range computes (two device buffers across passes); elsewise (or if pinning fails)
  // each pass is copied back before the next starts
  int pin_state = 0;  // bit 0: ids registered, bit 1: scores registered
  const size_t pin_bytes = (size_t)(hi - lo) * k * 4;
  // Zero-copy results (r06, default): the select / exact kernels write the lists straight into the
  // mapped caller arrays over PCIe.  The DMA pipeline (device buffers, copies of each finished range
  // on a copy stream) moved the 4.8 GB of an all-users c4 call at ~29 GB/s and finished ~110 ms after
  // the last kernel; written in place, the select runs at the link's rate with nothing behind it.
  // Mode 2 (default) selects in output-slot ranges, so a workgroup's four lists leave as one block of
  // 16-B stores (c4 all users: DMA 0.339 s, mode 1 (scan order) 0.298-0.318 s, mode 2 0.291 s on the
  // box that ran mode 1 at 0.318); ALBEDO_TOPK_ZEROCOPY=0: the DMA pipeline.
  const int zmode = [] {
    const char* e = std::getenv("ALBEDO_TOPK_ZEROCOPY");
    return e ? std::atoi(e) : 2;
  }();
  bool zcopy = zmode == 1 || zmode == 2;
  auto pin = [&, dev = c->dev]() {
    if (hipSetDevice(dev) != hipSuccess) return;
    const unsigned fl = zcopy ? hipHostRegisterMapped : hipHostRegisterDefault;
    if (hipHostRegister(dst_ids_out + lo * k, pin_bytes, fl) != hipSuccess) return;
    pin_state |= 1;
    if (hipHostRegister(scores_out + lo * k, pin_bytes, fl) == hipSuccess) pin_state |= 2;
  };
  std::thread pin_thr;
  const bool want_pin = dense_out && hi - lo > range;
  if (want_pin) {
    try {
      pin_thr = std::thread(pin);
    } catch (const std::system_error&) {
      pin();  // no thread: pin here
    }
  }
  TopkPlan P;
  const int plan_rc = topk_plan(c, src, k, P, trace ? std::function<void(const char*)>(stamp) : nullptr);
  if (pin_thr.joinable()) pin_thr.join();
  (void)hipGetLastError();  // a refused registration is not an error: the synchronous path runs
  if (pin_state == 1) (void)hipHostUnregister(dst_ids_out + lo * k);
  bool async_out = pin_state == 3;
  if (plan_rc != ALS_OK) {
    if (async_out) {
      (void)hipHostUnregister(dst_ids_out + lo * k);
      (void)hipHostUnregister(scores_out + lo * k);
    }
    return plan_rc;
  }
  stamp("plan (materialize dst, Gram + host eig, dst sort + fp16 pack) + pin the output arrays");
  int32_t* zids = nullptr;
  float* zsc = nullptr;
  if (async_out && zcopy) {
    void* pi = nullptr;
    void* ps = nullptr;
    if (hipHostGetDevicePointer(&pi, dst_ids_out + lo * k, 0) == hipSuccess &&
        hipHostGetDevicePointer(&ps, scores_out + lo * k, 0) == hipSuccess) {
      zids = static_cast<int32_t*>(pi);
      zsc = static_cast<float*>(ps);
    } else {
      zcopy = false;
      (void)hipGetLastError();
    }
  }
  hipStream_t cs = nullptr;
  hipEvent_t ev_copy[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> ev_rng;  // one per finished range: the copy stream waits for it
  DevBuf d_oid2[2], d_osc2[2];
  // releases everything the async path holds (null-safe: also after a partial set-up)
  hipStream_t sp = nullptr;                   // the post stream of overlapped passes (zero-copy)
  hipEvent_t ev_post[2] = {nullptr, nullptr};  // buffer set b's last select / rescans are done
  auto end_post = [&]() {
    if (sp) (void)hipStreamSynchronize(sp);
    for (auto& e : ev_post)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    if (sp) (void)hipStreamDestroy(sp);
    sp = nullptr;
  };
  auto end_async = [&]() {
    end_post();
    if (!async_out) return;
    if (cs) (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(c->st);
    (void)hipHostUnregister(dst_ids_out + lo * k);
    (void)hipHostUnregister(scores_out + lo * k);
    for (int b = 0; b < 2; ++b) {
      if (ev_copy[b]) (void)hipEventDestroy(ev_copy[b]);
      ev_copy[b] = nullptr;
    }
    for (hipEvent_t e : ev_rng) (void)hipEventDestroy(e);
    ev_rng.clear();
    if (cs) (void)hipStreamDestroy(cs);
    cs = nullptr;
    async_out = false;
  };
  if (async_out) {  // the copy stream and its events; if any cannot be created, the synchronous path runs
    bool ok = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) == hipSuccess;
    if (!ok) cs = nullptr;
    for (int b = 0; b < 2 && ok; ++b)
      if (!(ok = hipEventCreateWithFlags(&ev_copy[b], hipEventDisableTiming) == hipSuccess)) ev_copy[b] = nullptr;
    if (!ok) {
      end_async();
      (void)hipGetLastError();
    }
  }
  if (async_out && zcopy && n_pass > 1) {  // a failure here leaves the passes sequential
    bool ok = hipStreamCreateWithFlags(&sp, hipStreamNonBlocking) == hipSuccess;
    if (!ok) sp = nullptr;
    for (int b = 0; b < 2 && ok; ++b)
      if (!(ok = hipEventCreateWithFlags(&ev_post[b], hipEventDisableTiming) == hipSuccess)) ev_post[b] = nullptr;
    if (!ok) {
      end_post();
      (void)hipGetLastError();
    }
  }
  DevBuf d_oid, d_osc;
  {
    const int rc = topk_begin(c, P, n_known, n_pass, all_rows ? nullptr : known.data());
    if (rc != ALS_OK) {
      end_async();
      return rc;
    }
  }
  for (int64_t it = 0; it < n_pass; ++it) {
    const int64_t q0 = pstart[it], nc = (it + 1 < n_pass ? pstart[it + 1] : hi) - q0;
    if (async_out && zcopy) {  // results written in place by the kernels
      // mode 2: select in output-slot order by ranges (consecutive waves write consecutive lists);
      // with a post stream, buffer set it & 1, reused once its previous select / rescans are done
      const int par = sp ? (int)(it & 1) : 0;
      int rc = ALS_OK;
      if (sp && it >= 2 && hipStreamWaitEvent(c->st, ev_post[par], 0) != hipSuccess) rc = fail(ALS_E_HIP, "stream wait");
      if (rc == ALS_OK)
        rc = topk_run_rows(c, P, rowsf(q0), q0, q0, nc, zids + (q0 - lo) * k, zsc + (q0 - lo) * k,
                           zmode == 2 ? range : INT64_MAX, nullptr, par, sp);
      if (rc == ALS_OK && sp && hipEventRecord(ev_post[par], sp) != hipSuccess) rc = fail(ALS_E_HIP, "post event");
      if (rc != ALS_OK) {
        end_async();
        return rc;
      }
      stamp("pass");
      continue;
    }
    if (async_out) {
      const int b = (int)(it & 1);
      int rc = ALS_OK;
      if (it >= 2 && hipStreamWaitEvent(c->st, ev_copy[b], 0) != hipSuccess) rc = fail(ALS_E_HIP, "stream wait");
      if (rc == ALS_OK && (d_oid2[b].ensure(nc * k * 4) != hipSuccess || d_osc2[b].ensure(nc * k * 4) != hipSuccess))
        rc = fail(ALS_E_OUT_OF_MEMORY, "top-k output buffers");
      // each finished range of the pass goes down on the copy stream
      const TopkReady copy_out = [&, b, q0](int64_t o0, int64_t o1) -> int {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(ALS_E_HIP, "top-k copy event");
        ev_rng.push_back(e);
        if (hipEventRecord(e, c->st) != hipSuccess || hipStreamWaitEvent(cs, e, 0) != hipSuccess ||
            hipMemcpyAsync(dst_ids_out + (q0 + o0) * k, d_oid2[b].as<int32_t>() + o0 * k, (o1 - o0) * k * 4,
                           hipMemcpyDeviceToHost, cs) != hipSuccess ||
            hipMemcpyAsync(scores_out + (q0 + o0) * k, d_osc2[b].as<float>() + o0 * k, (o1 - o0) * k * 4,
                           hipMemcpyDeviceToHost, cs) != hipSuccess)
          return fail(ALS_E_HIP, "top-k result copy");
        return ALS_OK;
      };
      if (rc == ALS_OK)
        rc = topk_run_rows(c, P, rowsf(q0), q0, q0, nc, d_oid2[b].as<int32_t>(), d_osc2[b].as<float>(), range, copy_out);
      if (rc == ALS_OK && hipEventRecord(ev_copy[b], cs) != hipSuccess) rc = fail(ALS_E_HIP, "top-k result copy");
      if (rc != ALS_OK) {
        end_async();
        return rc;
      }
      stamp("pass");
      continue;
    }
    HIPCHK(d_oid.ensure(nc * k * 4));
    HIPCHK(d_osc.ensure(nc * k * 4));
    TRYC(topk_run_rows(c, P, rowsf(q0), q0, q0, nc, d_oid.as<int32_t>(), d_osc.as<float>()));
    if (dense_out) {
      HIPCHK(hipMemcpyAsync(dst_ids_out + q0 * k, d_oid.p, nc * k * 4, hipMemcpyDeviceToHost, c->st));
      HIPCHK(hipMemcpyAsync(scores_out + q0 * k, d_osc.p, nc * k * 4, hipMemcpyDeviceToHost, c->st));
      HIPCHK(hipStreamSynchronize(c->st));
    } else {
      std::vector<int32_t> oid(nc * k);
      std::vector<float> osc(nc * k);
      HIPCHK(hipMemcpyAsync(oid.data(), d_oid.p, oid.size() * 4, hipMemcpyDeviceToHost, c->st));
      HIPCHK(hipMemcpyAsync(osc.data(), d_osc.p, osc.size() * 4, hipMemcpyDeviceToHost, c->st));
      HIPCHK(hipStreamSynchronize(c->st));
      for (int64_t i = 0; i < nc; ++i) {
        std::memcpy(dst_ids_out + posf(q0 + i) * k, &oid[i * k], k * 4);
        std::memcpy(scores_out + posf(q0 + i) * k, &osc[i * k], k * 4);
      }
    }
  }
  {
    const int rc = topk_finish(c, P, sp);
    if (rc != ALS_OK) {
      end_async();
      return rc;
    }
  }
  end_async();
  stamp("last copies + unpin");
  if (c->world > 1 && per_rank > 0) {  // every rank ends with every list: one all-gather of the slices
    std::vector<float> blk((size_t)c->world * per_rank * k * 2, 0.f);
    float* mine = blk.data() + (size_t)c->rank * per_rank * k * 2;
    for (int64_t i = lo; i < hi; ++i) {
      std::memcpy(mine + (size_t)(i - lo) * k * 2, dst_ids_out + posf(i) * k, k * 4);
      std::memcpy(mine + (size_t)(i - lo) * k * 2 + k, scores_out + posf(i) * k, k * 4);
    }
    TRYC(allgather_host(c, blk.data(), per_rank * k * 2));
    for (int r = 0; r < c->world; ++r) {
      if (r == c->rank) continue;
      const int64_t rl = std::min<int64_t>(n_known, (int64_t)r * per_rank), rh = std::min<int64_t>(n_known, rl + per_rank);
      const float* bb = blk.data() + (size_t)r * per_rank * k * 2;
      for (int64_t i = rl; i < rh; ++i) {
        std::memcpy(dst_ids_out + posf(i) * k, bb + (size_t)(i - rl) * k * 2, k * 4);
        std::memcpy(scores_out + posf(i) * k, bb + (size_t)(i - rl) * k * 2 + k, k * 4);
      }
    }
  }
  return ALS_OK;
}

int als_evaluate_ndcg(als_ctx* c, int32_t k, int64_t n, const int32_t* user, const int32_t* item, const int64_t* key,
                      double* ndcg_out, int64_t* n_users_out, int32_t* users_out, double* per_user_out, int64_t cap) {
  if (!c || !ndcg_out || !n_users_out || (n > 0 && (!user || !item || !key)))
    return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (k <= 0) return fail(ALS_E_INVALID_ARGUMENT, "ranking position k should be positive");
  if (k > TOPK_KC) return fail(ALS_E_UNSUPPORTED, "NDCG@k on the device supports k <= " + std::to_string(TOPK_KC));
  TRYC(set_device(c));
  TRYC(materialize(c, ALS_USER));
  Side& S = c->s[ALS_USER];
  *ndcg_out = NAN;
  *n_users_out = 0;
  c->last_rescan.clear();
  c->last_rescan_ready = true;
  if (n <= 0 || S.n == 0) return ALS_OK;
  hipStream_t st = c->st;
  // 1. intoUserActualItems on the device: group by model user (inner join), top-k by (key desc, item asc)
  DevBuf d_user, d_item, d_key, d_ids, d_row, d_rows, d_idx, d_idxs, d_runs, d_cnt, d_off, d_nr, d_tmp;
  HIPCHK(d_user.ensure(n * 4));
  HIPCHK(d_item.ensure(n * 4));
  HIPCHK(d_key.ensure(n * 8));
  HIPCHK(d_ids.ensure(S.n * 4));
  HIPCHK(hipMemcpyAsync(d_user.p, user, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_item.p, item, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_key.p, key, n * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_ids.p, S.ids.data(), S.n * 4, hipMemcpyHostToDevice, st));
  for (DevBuf* b : {&d_row, &d_rows, &d_idx, &d_idxs, &d_runs, &d_cnt}) HIPCHK(b->ensure(n * 4));
  HIPCHK(d_off.ensure(n * 8));
  HIPCHK(d_nr.ensure(8));
  const size_t tb = eval_sort_temp_bytes(n);
  HIPCHK(d_tmp.ensure(std::max<size_t>(tb, 16)));
  HIPCHK(eval_group_users(d_user.as<int32_t>(), n, d_ids.as<int32_t>(), S.n, d_tmp.p, tb, d_row.as<uint32_t>(),
                          d_rows.as<uint32_t>(), d_idx.as<uint32_t>(), d_idxs.as<uint32_t>(), d_runs.as<uint32_t>(),
                          d_cnt.as<int32_t>(), d_off.as<int64_t>(), d_nr.as<int64_t>(), st));
  int64_t nr = 0;
  HIPCHK(hipMemcpyAsync(&nr, d_nr.p, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::vector<int32_t> rows(nr);
  HIPCHK(hipMemcpyAsync(rows.data(), d_runs.p, nr * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (nr > 0 && (uint32_t)rows[nr - 1] == 0xFFFFFFFFu) --nr;  // ids unknown to the model: dropped
  rows.resize(nr);
  *n_users_out = nr;
  if (nr == 0) return ALS_OK;
  DevBuf d_act, d_actn, d_gain, d_vals;
  HIPCHK(d_act.ensure(nr * k * 4));
  HIPCHK(d_actn.ensure(nr * 4));
  HIPCHK(eval_actual_lists(d_idxs.as<uint32_t>(), d_off.as<int64_t>(), d_cnt.as<int32_t>(), nr, d_key.as<int64_t>(),
                           d_item.as<int32_t>(), k, d_act.as<int32_t>(), d_actn.as<int32_t>(), st));
  // ndcgAt's gains from the host's libm: the host evaluator's table (1.0 / math.log(i + 2))
  std::vector<double> gain(k);
  for (int i = 0; i < k; ++i) gain[i] = 1.0 / std::log((double)(i + 2));
  HIPCHK(d_gain.ensure(k * 8));
  HIPCHK(hipMemcpyAsync(d_gain.p, gain.data(), k * 8, hipMemcpyHostToDevice, st));
  HIPCHK(d_vals.ensure(nr * 8));
  // 2. intoUserPredictedItems: the users' top-k lists stay on the device; 3. ndcgAt per user
  TopkPlan P;
  TRYC(topk_plan(c, ALS_USER, k, P));
  const int64_t per_rank = (nr + c->world - 1) / c->world;
  const int64_t lo = std::min<int64_t>(nr, (int64_t)c->rank * per_rank), hi = std::min<int64_t>(nr, lo + per_rank);
  const int64_t chunk = topk_pass_rows(c);  // one pass for any realistic user count (see als_recommend)
  DevBuf d_oid, d_osc;
  TRYC(topk_begin(c, P, nr, (hi - lo + chunk - 1) / chunk, rows.data()));
  for (int64_t q0 = lo; q0 < hi; q0 += chunk) {
    const int64_t nc = std::min<int64_t>(chunk, hi - q0);
    HIPCHK(d_oid.ensure(nc * k * 4));
    HIPCHK(d_osc.ensure(nc * k * 4));
    TRYC(topk_run_rows(c, P, rows.data() + q0, 0, q0, nc, d_oid.as<int32_t>(), d_osc.as<float>()));
    HIPCHK(eval_ndcg(d_oid.as<int32_t>(), d_act.as<int32_t>() + q0 * k, d_actn.as<int32_t>() + q0, nc, k,
                     d_gain.as<double>(), d_vals.as<double>() + q0, st));
  }
  TRYC(topk_finish(c, P));
  std::vector<double> vals((size_t)std::max<int64_t>(per_rank, 1) * c->world, 0.0);
  if (hi > lo)
    HIPCHK(hipMemcpyAsync(vals.data() + (size_t)c->rank * per_rank, d_vals.as<double>() + lo, (hi - lo) * 8,
                          hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (c->world > 1) TRYC(allgather_host(c, reinterpret_cast<float*>(vals.data()), per_rank * 2));
  double sum = 0.0;  // mean over users in ascending id order (RankingMetrics: RDD mean)
  for (int64_t i = 0; i < nr; ++i) sum += vals[i];
  *ndcg_out = sum / (double)nr;
  if (nr <= cap) {
    if (users_out)
      for (int64_t i = 0; i < nr; ++i) users_out[i] = S.ids[rows[i]];
    if (per_user_out) std::memcpy(per_user_out, vals.data(), nr * 8);
  }
  return ALS_OK;
}

int als_predict(als_ctx* c, int64_t n, const int32_t* user, const int32_t* item, float* out) {
  if (!c || (n > 0 && (!user || !item || !out))) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (n <= 0) return ALS_OK;
  TRYC(set_device(c));
  TRYC(materialize(c, ALS_USER));
  TRYC(materialize(c, ALS_ITEM));
  std::vector<int32_t> u(n), v(n);
  for (int64_t i = 0; i < n; ++i) {
    u[i] = (int32_t)find_row(c->s[ALS_USER], user[i]);
    v[i] = (int32_t)find_row(c->s[ALS_ITEM], item[i]);
  }
  DevBuf du, dv, dout;
  HIPCHK(du.ensure(n * 4));
  HIPCHK(dv.ensure(n * 4));
  HIPCHK(dout.ensure(n * 4));
  HIPCHK(copy_st(c, du.p, u.data(), n * 4, hipMemcpyHostToDevice));
  HIPCHK(copy_st(c, dv.p, v.data(), n * 4, hipMemcpyHostToDevice));
  HIPCHK(launch_predict(c->KP, c->p.rank, c->s[ALS_USER].d_orig.as<float>(), c->s[ALS_ITEM].d_orig.as<float>(),
                        du.as<int32_t>(), dv.as<int32_t>(), dout.as<float>(), n, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(copy_st(c, out, dout.p, n * 4, hipMemcpyDeviceToHost));
  return ALS_OK;
}

int als_get_row_ratings(als_ctx* c, int side, int32_t id, int64_t cap, int32_t* src_ids, float* ratings,
                        int64_t* n_out) {
  if (!c || (side != 0 && side != 1) || !n_out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  TRYC(set_device(c));
  Side& S = c->s[side];
  const Side& Src = c->s[1 - side];
  const int64_t r = find_row(S, id);
  if (r < 0) return fail(ALS_E_INVALID_ARGUMENT, "unknown id " + std::to_string(id));
  if (r < S.own0 || r >= S.own0 + S.own_n) return fail(ALS_E_STATE, "row not owned by this rank");
  int64_t pr[2];
  HIPCHK(copy_st(c, pr, S.d_ptr.as<int64_t>() + (r - S.own0), 16, hipMemcpyDeviceToHost));
  const int64_t n = pr[1] - pr[0];
  *n_out = n;
  if (n > cap) return ALS_OK;
  std::vector<int32_t> col(n);
  if (n) {
    HIPCHK(copy_st(c, col.data(), S.d_col.as<int32_t>() + pr[0], n * 4, hipMemcpyDeviceToHost));
    if (ratings) HIPCHK(copy_st(c, ratings, S.d_val.as<float>() + pr[0], n * 4, hipMemcpyDeviceToHost));
  }
  if (src_ids)
    for (int64_t e = 0; e < n; ++e) {
      const int64_t p = col[e];
      const int64_t span = (int64_t)Src.world * Src.chpad;  // invert the chunk-major gathered layout
      const int64_t q = p / span, rem = p % span, rk = rem / Src.chpad;
      src_ids[e] = Src.ids[Src.starts[rk] + q * Src.chpad + rem % Src.chpad];
    }
  return ALS_OK;
}

int als_get_degrees(const als_ctx* c, int side, int64_t* out) {
  if (!c || (side != 0 && side != 1) || !out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!c->has_ratings) return fail(ALS_E_STATE, "set ratings first");
  const Side& S = c->s[side];
  for (int64_t r = 0; r < S.n; ++r) out[r] = -1;
  for (int64_t r = 0; r < S.own_n; ++r) out[S.own0 + r] = S.h_deg[r];
  return ALS_OK;
}

int als_last_timings(const als_ctx* c, int dst_side, double* out, int n) {
  if (!c || (dst_side != 0 && dst_side != 1) || !out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  for (int i = 0; i < n && i < ALS_T_COUNT; ++i) out[i] = c->s[dst_side].t[i];
  return ALS_OK;
}

int als_path_stats(const als_ctx* c, int dst_side, int64_t* out4) {
  if (!c || (dst_side != 0 && dst_side != 1) || !out4) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  for (int i = 0; i < 4; ++i) out4[i] = c->s[dst_side].stats[i];
  return ALS_OK;
}

int als_solver_stats(const als_ctx* c, int dst_side, int64_t* out4) {
  if (!c || (dst_side != 0 && dst_side != 1) || !out4) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  for (int i = 0; i < 4; ++i) out4[i] = c->s[dst_side].solver[i];
  return ALS_OK;
}

int als_topk_stats(const als_ctx* c, int64_t* out4) {
  if (!c || !out4) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  for (int i = 0; i < 4; ++i) out4[i] = c->topk_stats[i];
  return ALS_OK;
}

int als_topk_timing(const als_ctx* c, double* out5) {
  if (!c || !out5) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  for (int i = 0; i < 5; ++i) out5[i] = c->topk_ms[i];
  return ALS_OK;
}

int als_topk_last_rescan(const als_ctx* c, int32_t* src_ids_out, int64_t cap, int64_t* n_out) {
  if (!c || !n_out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!c->last_rescan_ready) {  // first query after a top-k call: read its device flags
    TRYC(set_device(const_cast<als_ctx*>(c)));
    std::vector<int32_t> need((size_t)c->last_need_n);
    if (c->last_need_n > 0) {
      HIPCHK(hipStreamSynchronize(c->st));
      HIPCHK(copy_st(c, need.data(), c->d_last_need.p, need.size() * 4, hipMemcpyDeviceToHost));
    }
    const Side& S = c->s[c->last_src];
    c->last_rescan.clear();
    const int64_t nrow = (int64_t)S.ids.size();
    for (int64_t p = 0; p < c->last_need_n; ++p) {
      if (!need[p]) continue;
      const int64_t r = c->last_rows_dense ? p : (p < (int64_t)c->last_rows.size() ? c->last_rows[p] : -1);
      if (r < 0 || r >= nrow) return fail(ALS_E_STATE, "top-k rescan flags out of range of the src rows");
      c->last_rescan.push_back(S.ids[r]);
    }
    c->last_rescan_ready = true;
  }
  *n_out = (int64_t)c->last_rescan.size();
  if (src_ids_out && *n_out <= cap) std::memcpy(src_ids_out, c->last_rescan.data(), c->last_rescan.size() * 4);
  return ALS_OK;
}

int als_synchronize(als_ctx* c) {
  if (!c) return fail(ALS_E_INVALID_ARGUMENT, "null context");
  TRYC(set_device(c));
  return drain(c);  // both streams: the bench barrier covers the trailing factor gathers
}

int als_synth_generate(int32_t device, uint64_t seed, int32_t rounds, int64_t n_users, int64_t n_items,
                       const int64_t* deg_prefix, const double* cw, const int32_t* perm, int32_t* user_out,
                       int32_t* item_out, float* rating_out, int64_t* n_out) {
  if (!deg_prefix || !cw || !perm || !n_out || n_users <= 0 || n_items <= 0)
    return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(ALS_E_NO_DEVICE, "no HIP device");
  if (device >= 0) HIPCHK(hipSetDevice(device));
  const int64_t n = deg_prefix[n_users];
  DevBuf dp, dcw, dperm, du, di, dr;
  HIPCHK(dp.ensure((n_users + 1) * 8));
  HIPCHK(dcw.ensure(n_items * 8));
  HIPCHK(dperm.ensure(n_items * 4));
  HIPCHK(du.ensure(n * 4));
  HIPCHK(di.ensure(n * 4));
  HIPCHK(dr.ensure(n * 4));
  HIPCHK(hipMemcpy(dp.p, deg_prefix, (n_users + 1) * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dcw.p, cw, n_items * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dperm.p, perm, n_items * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  HIPCHK(hipStreamCreate(&st));
  hipError_t e = synth_fill(seed, rounds, n_users, n_items, dp.as<int64_t>(), dcw.as<double>(), dperm.as<int32_t>(),
                            du.as<int32_t>(), di.as<int32_t>(), dr.as<float>(), n, n_out, st);
  (void)hipStreamDestroy(st);
  HIPCHK(e);
  if (user_out) HIPCHK(hipMemcpy(user_out, du.p, *n_out * 4, hipMemcpyDeviceToHost));
  if (item_out) HIPCHK(hipMemcpy(item_out, di.p, *n_out * 4, hipMemcpyDeviceToHost));
  if (rating_out) HIPCHK(hipMemcpy(rating_out, dr.p, *n_out * 4, hipMemcpyDeviceToHost));
  return ALS_OK;
}

int als_set_ratings_synthetic(als_ctx* c, uint64_t seed, int32_t rounds, int64_t n_users, int64_t n_items,
                              const int64_t* deg_prefix, const double* cw, const int32_t* perm) {
  if (!c || !deg_prefix || !cw || !perm || n_users <= 0 || n_items <= 0)
    return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  TRYC(ingest_allowed(c));
  TRYC(set_device(c));
  const int64_t n = deg_prefix[n_users];
  DevBuf dp, dcw, dperm, du, di, dr;
  HIPCHK(dp.ensure((n_users + 1) * 8));
  HIPCHK(dcw.ensure(n_items * 8));
  HIPCHK(dperm.ensure(n_items * 4));
  HIPCHK(du.ensure(n * 4));
  HIPCHK(di.ensure(n * 4));
  HIPCHK(dr.ensure(n * 4));
  HIPCHK(copy_st(c, dp.p, deg_prefix, (n_users + 1) * 8, hipMemcpyHostToDevice));
  HIPCHK(copy_st(c, dcw.p, cw, n_items * 8, hipMemcpyHostToDevice));
  HIPCHK(copy_st(c, dperm.p, perm, n_items * 4, hipMemcpyHostToDevice));
  int64_t nout = 0;
  HIPCHK(synth_fill(seed, rounds, n_users, n_items, dp.as<int64_t>(), dcw.as<double>(), dperm.as<int32_t>(),
                    du.as<int32_t>(), di.as<int32_t>(), dr.as<float>(), n, &nout, c->st));
  dp.release();
  dcw.release();
  dperm.release();
  return ingest_device(c, nout, du.as<int32_t>(), di.as<int32_t>(), dr.as<float>());
}

// ---- host-only utilities (no GPU needed; used by the CPU test suite) ------------------------
int als_host_eigh(int32_t n, const double* a, double* w, double* v) {
  if (n <= 0 || !a || !w || !v) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (!sym_eig(n, a, w, v)) return fail(ALS_E_NOT_POSITIVE_DEFINITE, "eigensolver did not converge");
  return ALS_OK;
}

int als_device_eigh(int32_t device, int32_t k, const double* g, const double* w0, double* w, double* v,
                    int32_t* sweeps) {
  if (k <= 0 || k > 256 || !g || !w || !v) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  if (hipSetDevice(device) != hipSuccess) return fail(ALS_E_NO_DEVICE, "no such device");
  const int KP = padded_rank(k);
  std::vector<double> G((size_t)KP * KP, 0.0), B((size_t)KP * KP, 0.0), W((size_t)KP * KP, 0.0);
  for (int i = 0; i < KP; ++i) B[(size_t)i * KP + i] = W[(size_t)i * KP + i] = 1.0;
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) {
      G[(size_t)i * KP + j] = g[(size_t)i * k + j];
      if (w0) W[(size_t)i * KP + j] = w0[(size_t)i * k + j];
    }
  DevBuf dG, dB, dW, dOut, dS, dP, dl, du;
  HIPCHK(dG.ensure(G.size() * 8));
  HIPCHK(dB.ensure(B.size() * 8));
  HIPCHK(dW.ensure(W.size() * 8));
  HIPCHK(dOut.ensure(W.size() * 8));
  HIPCHK(dS.ensure(eig_scratch_doubles(KP) * 8));
  HIPCHK(dP.ensure((size_t)KP * KP * 4));
  HIPCHK(dl.ensure((size_t)KP * 4));
  HIPCHK(du.ensure((size_t)KP * 4));
  HIPCHK(hipMemcpy(dG.p, G.data(), G.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dB.p, B.data(), B.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dW.p, W.data(), W.size() * 8, hipMemcpyHostToDevice));
  // B_s = I, B_t = W0: the warm start is W0 itself; B_t_out = P
  HIPCHK(launch_device_eig(KP, k, dG.as<double>(), dB.as<double>(), dW.as<double>(), dOut.as<double>(), dS.as<double>(),
                           dP.as<float>(), dl.as<float>(), du.as<unsigned>(), nullptr));
  std::vector<double> wk(KP), P(W.size());
  int sw = 0;
  HIPCHK(hipMemcpy(P.data(), dOut.p, P.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(wk.data(), dS.as<double>() + (size_t)3 * KP * KP, KP * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(&sw, eig_sweeps(dS.as<double>(), KP), 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < k; ++i) {
    w[i] = wk[i];
    for (int j = 0; j < k; ++j) v[(size_t)i * k + j] = P[(size_t)i * KP + j];
  }
  if (sweeps) *sweeps = sw < 0 ? -sw - 1 : sw;
  if (sw < 0) return fail(ALS_E_NOT_POSITIVE_DEFINITE, "eigensolver did not converge");
  return ALS_OK;
}

int als_host_spark_side_seeds(int64_t seed, int64_t* user_seed, int64_t* item_seed) {
  if (!user_seed || !item_seed) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  spark_side_seeds(seed, user_seed, item_seed);
  return ALS_OK;
}

int als_host_spark_init(const int32_t* ids_sorted, int64_t n, int32_t rank, int64_t side_seed, int32_t num_blocks,
                        float* out) {
  if ((n > 0 && (!ids_sorted || !out)) || rank < 1 || num_blocks < 1) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  spark_initialize(ids_sorted, n, rank, side_seed, num_blocks, out, rank);
  return ALS_OK;
}

int als_host_plan_shards(const int64_t* ptr, int64_t n, int32_t world, int64_t* starts_out) {
  if (!ptr || n < 0 || world < 1 || !starts_out) return fail(ALS_E_INVALID_ARGUMENT, "bad args");
  plan_shards(ptr, n, world, starts_out);
  return ALS_OK;
}

}  // extern "C"
