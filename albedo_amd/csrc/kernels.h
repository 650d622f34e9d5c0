// Internal launch interface between the host engine (als_engine.cpp) and the HIP kernels.
// Not part of the public C ABI (include/albedo_als.h).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace albedo {

// Padded rank used on device: factor rows are KP floats (zero beyond `rank`).
int padded_rank(int rank);  // 64, 128 or 256 (0 if unsupported)

// *SolveArgs::err bits: 1 = a non-positive diagonal (λn + Λ), 2 = a collapsed pivot / non-finite
// solution; with 2 the path that met it (reported in the not-positive-definite message)
constexpr int ALBEDO_EF_LIGHT16 = 16, ALBEDO_EF_LIGHT_REG = 32, ALBEDO_EF_LIGHT_ACC = 64, ALBEDO_EF_WAVE = 128,
              ALBEDO_EF_HEAVY = 256;

struct SolveArgs {
  const float* Z;          // src factors in the eigenbasis of the src Gram, [*][KP]
  const int64_t* ptr;      // dst CSR row pointer (global dst row index)
  const int32_t* col;      // src row index (into Z)
  const float* val;        // rating
  const int32_t* rows;     // dst rows handled by this launch
  int64_t n_rows;
  const float* lam;        // [KP] eigenvalues of the src Gram (implicit) or zeros (explicit)
  float* X;                // out: dst factors in that eigenbasis, [*][KP]
  int kreal;               // the model rank (<= KP)
  int implicit;
  float alpha;
  float reg;
  int* err;                // device flag: set to 1 when a solve meets a non-positive pivot
  const float* colscale;   // [2*KP] heavy-build fp16 column scales 2^e and their inverses
  const float* prebuilt;   // split rows: reduced A' records [n_rows][split_rec_floats] (else null)
  unsigned long long* iters;  // NNLS: [0] += iterations of every row, [1] = max over rows (or null)
  // uniform confidence (every rating of the side has the same c: binary implicit data, or explicit):
  // the heavy build gathers pre-split rows instead of Z (launch_presplit), null otherwise
  const void* Zhl;         // [*][2·KP] fp16: hi of √c·colscale·z, then lo
  int64_t zero_row;        // an all-zero row of Zhl (the gather target of ratings past a row's end)
  float wsc;               // power-of-two scale of the rating weights w in the b' MFMA (max|w|·wsc < 2^13)
  float inv_sw;            // 1 / √c
  const int32_t* desc;     // light launches: int4 {row, p0 lo, p0 hi, degree} per entry of `rows` (or null)
  int n_cu;                // compute units (persistent launches)
};

// Split-K of the heavy tail (rows with more ratings than one chunk): every chunk of chunk_len
// ratings is built by its own workgroup into an fp32 partial record (packed A' tiles + b' + the
// positive-rating count), the partials of a row are summed in fp64 in chunk order (deterministic),
// and the row is factored from the reduced record (SolveArgs::prebuilt).
struct SplitArgs {
  const int32_t* chunk_row;  // [n_chunks] dst row (CSR row index) of each chunk
  const int32_t* chunk_idx;  // [n_chunks] chunk number within its row
  int64_t n_chunks;
  int chunk_len;
  const int32_t* slot0;      // [n_split + 1] first chunk of each split row (rows in factor order)
  int64_t n_split;
  float* partial;            // [n_chunks][split_rec_floats]
  float* reduced;            // [n_split][split_rec_floats]
};
int split_rec_floats(int KP);
// partial builds of every chunk (wave: one wave per chunk, heavy_wave.hip, KP <= 128; else one
// 4/16-wave workgroup per chunk), then the fp64 reduction into s.reduced
hipError_t launch_heavy_split(int KP, const SolveArgs& a, const SplitArgs& s, bool wave, hipStream_t st);
hipError_t launch_wave_partial(int KP, const SolveArgs& a, const SplitArgs& s, hipStream_t st);

// G (fp64 [KP][KP], full symmetric) = Σ_rows Xᵀ X over rows [0, n) of X ([n][KP]).
hipError_t launch_gram(int KP, const float* X, int64_t n, double* slab, int slab_blocks, double* G,
                       hipStream_t s);
int gram_slab_blocks(int KP, int64_t n);
size_t gram_slab_doubles(int KP, int slab_blocks);

// Z = X · M for n rows ([n][KP] · [KP][KP], row-major M); cmax (optional, zeroed by the caller):
// atomicMax of the bits of max |Z[.][c]| per column (launch_colscale(..., have_max = true) reads it)
hipError_t launch_rotate(int KP, const float* X, const float* M, float* Z, int64_t n, hipStream_t s,
                         unsigned* cmax = nullptr);

// Per-row solves. light: rows with degree <= D (D in {16,32,64}); heavy: any degree.
hipError_t launch_solve_light(int KP, int D, const SolveArgs& a, hipStream_t s);
// light rows of degree <= 16 (light16.hip): the push-through solve written for VALU instruction count
hipError_t launch_solve_light16(int KP, const SolveArgs& a, hipStream_t s, bool pair = false);
// desc[4i .. 4i+3] = {rows[i], ptr[rows[i]] lo, hi, degree}: one scalar load per row for light16
hipError_t launch_row_desc(const int32_t* rows, int64_t n, const int64_t* ptr, int32_t* desc, hipStream_t s);
hipError_t launch_solve_heavy(int KP, const SolveArgs& a, hipStream_t s);
// heavy rows, one wave per row (heavy_wave.hip), KP <= 128; rows of any degree (split rows excepted)
hipError_t launch_solve_wave(int KP, const SolveArgs& a, hipStream_t s);

// nonnegative = true: Spark NNLS per row; Gt = the src Gram in the NNLS tile layout (fp32).
hipError_t launch_solve_nnls(int KP, const SolveArgs& a, const float* Gt, hipStream_t s);
// KP = 256 per-row NNLS on 512-thread workgroups, two per CU (nnls_row.hip); launch_solve_nnls
// routes KP = 256 here unless ALBEDO_NNLS_ROW=1024 (the register kernel of als_kernels.hip)
hipError_t launch_solve_nnls_row256(const SolveArgs& a, const float* Gt, hipStream_t s);
int nnls_gtile_floats(int KP);
// NNLS rows of low degree, `slots` (16/8/4/2/1) per workgroup in lockstep (nnls_batch.hip); a slot
// holds rows of degree <= nnls_batch_max_degree(KP, slots).  A persistent grid of at most n_cu
// workgroups takes rows from *counter (zeroed by the launch).  Gfrag: KP*KP*4 bytes holding G·gscale
// in MFMA operand order as fp16 hi + lo, filled by launch_nnls_gfrag (gscale a power of two with
// max|G|·gscale < 2^15).
int nnls_batch_max_degree(int KP, int slots);
hipError_t launch_nnls_gfrag(int KP, const float* Gt, float gscale, void* Gfrag, hipStream_t s);
hipError_t launch_nnls_batch(int KP, int slots, const SolveArgs& a, const void* Gfrag, float gscale,
                             unsigned int* counter, int n_cu, hipStream_t s);
// colscale[c] = 2^e_c with max_rows |Z[.][c]|·√cmax < 2^13, colscale[KP+c] = 2^-e_c (tmp: KP uints)
hipError_t launch_colscale(int KP, const float* Z, int64_t n, float cmax, unsigned* tmp, float* colscale,
                           hipStream_t s, bool have_max = false);
// Zhl[r] = fp16 hi and lo of Z[r][c]·(sw·colscale[c]) (the heavy build's operand split, done once per
// src row instead of once per gathered rating); row n (the zero row) is cleared
hipError_t launch_presplit(int KP, const float* Z, int64_t n, const float* colscale, float sw, void* Zhl, hipStream_t s);
// Z = X·P on bf16 MFMA (three-part split of both operands, KP = 128 only); Pf: rotate_bf_pfrag_bytes
// of scratch for P's parts; Zhl (or null): the heavy build's operand split written in the same pass
// (colscale cs and √c sw as launch_presplit, which it replaces), row zrow of Zhl zeroed
hipError_t launch_rotate_bf(int KP, const float* X, const float* P, void* Pf, float* Z, int64_t n, const float* cs, float sw,
                            void* Zhl, int64_t zrow, int n_cu, hipStream_t s);
int rotate_bf_pfrag_bytes(int KP);
// *out = bits of max |v[i]| (non-negative float, compared as unsigned)
hipError_t launch_absmax(const float* v, int64_t n, unsigned* out, hipStream_t s);
// *out = bits of min |v[i]| (0x7f800000 when n = 0)
hipError_t launch_absmin(const float* v, int64_t n, unsigned* out, hipStream_t s);
int nnls_gtile_index(int r, int c);  // block(r) >= block(c): NNLS tile layout, diagonal tiles full

// Eigenbasis of the src Gram on the device (eig.hip): W = B_sᵀ·B_t_in (warm start), M = Wᵀ G W, cyclic
// Jacobi in fp64 -> P (eigenvectors, in scratch), P32 (fp32 [KP][KP]), lam32 = max(Λ, 0), ub = the
// rotation's column-scale bound (float bits), B_t_out = B_s·P.  G, B_s, B_t: fp64 [KP][KP] row-major
// (B_t_in may alias B_t_out: it is read before the last GEMM writes).  scratch: eig_scratch_doubles.
size_t eig_scratch_doubles(int KP);
hipError_t launch_device_eig(int KP, int k, const double* G, const double* Bs, const double* Bt_in, double* Bt_out,
                             double* scratch, float* P32, float* lam32, unsigned* ub, hipStream_t s);
const double* eig_minmax(const double* scratch, int KP);  // device {min Λ, max Λ} of the last call
const int* eig_sweeps(const double* scratch, int KP);     // device Jacobi sweep count of the last call
hipError_t launch_identity(double* B, int KP, hipStream_t s);
hipError_t launch_basis_t32(const double* B, float* Bt, int KP, hipStream_t s);  // Bt = (float) Bᵀ

// Seeded unit-norm Gaussian rows (global row index row0 + r) for large synthetic runs.
hipError_t launch_init_random(int KP, int kreal, float* X, int64_t n, uint64_t seed, int64_t row0, hipStream_t s);

// ALSModel.transform: out[p] = F2J sdot(U[u[p]], V[v[p]]) (NaN when u[p] < 0 or v[p] < 0).
hipError_t launch_predict(int KP, int kreal, const float* U, const float* V, const int32_t* u,
                          const int32_t* v, float* out, int64_t n, hipStream_t s);

// Top-k (topk.hip): dst rows ordered by descending ‖t_⊥‖ in the dst Gram's eigenbasis and packed as
// fp16 with per-chunk bound boxes (topk_prepare), a probe pass for the starting thresholds and the src
// features (topk_order), per-workgroup chunk masks (launch_topk_mask), an MFMA scan over the masked
// chunks, then exact F2J rescoring of the best TOPK_KC candidates with a certification bound (rows
// that fail it: topk_exact).
constexpr int TOPK_M = 4;       // leading eigen-directions of the dst Gram in the pruning bound
constexpr int TOPK_CF = 12;     // floats per chunk feature record: lo[M], hi[M], R = max ‖t_⊥‖, pad
constexpr int TOPK_SF = 8;      // floats per src feature record: s_P[M], ‖s_⊥‖, margin, ‖s‖, pad
constexpr int TOPK_SUPER = 16;  // chunks per super-chunk (mask pre-pass)
struct TopkArgs {
  const float* S;          // src factors (original basis) [*][KP]
  const float* T;          // dst factors (original basis) [n_dst][KP]
  const int32_t* src_rows; // src rows to score
  int64_t n_src;
  int64_t n_dst;
  const int32_t* dst_ids;  // raw ids of dst rows (ascending with the row index)
  int kreal;
  int k;                   // requested top-k
  int kt;                  // rank of the running threshold in the candidate lists (k <= kt <= TOPK_KC)
  float tmax_norm;         // max_j ||T_j||_2 (for the error bound)
  const void* Th;          // [n_chunks * chunk rows][KP] fp16: T[perm[p]]·tsc, zero rows past n_dst
  const uint32_t* perm;    // [n_dst] dst row of scan position p
  int64_t n_chunks;
  const double* VP;        // [TOPK_M][KP] leading eigenvectors of the dst Gram (fp64)
  const float* cfeat;      // [n_chunks][TOPK_CF] chunk bound boxes (null: no pruning)
  const void* probe;       // [256][KP] fp16 probe rows (the largest norms), ·tsc, zero rows past n_dst
  const float* sfeat;      // [n_src][TOPK_SF] src features by scan position (order kernel output)
  const uint32_t* mask;    // [n_wg][mask_words] needed chunks per scan workgroup (null: every chunk)
  int64_t mask_words;
  float ssc, tsc;          // src / dst fp16 scales (powers of two)
  float unscale;           // 1 / (ssc·tsc): exact rescaling of the MFMA scores
  float scaled;            // ssc·tsc
  uint2* lent;             // [n_src][TOPK_CAP] candidate lists: (approx score bits, scan position) pairs
  int32_t* lcnt;           // [n_src] list lengths
  int32_t* out_ids;        // [n_src][k] raw dst ids
  float* out_scores;       // [n_src][k]
  int32_t* need_exact;     // [n_src] set when the candidate set could not be certified
  float* kth0;             // [n_src] select -> exact rescan: the certification pass's k-th exact score (or null)
  unsigned long long* scanned;  // += dst chunks scanned by each scan workgroup (or null)
  const uint32_t* out_pos;      // select: results of scan position i go to slot out_pos[i] (or i)
  const float* thr0;            // scan: starting threshold of each src position (topk_order; or null)
  // select over output slots slot0 .. slot0 + n_slots - 1 (in_pos != null: slot -> scan position,
  // the inverse of out_pos), so a pass's results can be finished and copied out range by range
  const uint32_t* in_pos;
  int64_t slot0, n_slots;
  int order_dir_bits;           // order: key bits of the direction s_P / ‖s‖ (bytes: u1, u2, u3; 0: depth only)
};
constexpr int TOPK_KC = 64;     // candidates rescored exactly per src row (k <= 64)
#ifndef ALBEDO_TOPK_NPROBE
#define ALBEDO_TOPK_NPROBE 512
#endif
constexpr int TOPK_NPROBE = ALBEDO_TOPK_NPROBE;  // probe rows of the starting thresholds (largest norms)
#ifndef ALBEDO_TOPK_BISECT
#define ALBEDO_TOPK_BISECT 16
#endif
// bisection steps of the probe threshold: the top bits of the order-preserving key; fewer than 32 leave
// a lower bound of the kt-th probe score (valid, coarser by the undecided bits)
constexpr int TOPK_BISECT = ALBEDO_TOPK_BISECT;
#ifndef ALBEDO_TOPK_KT_EXTRA
#define ALBEDO_TOPK_KT_EXTRA 16
#endif
constexpr int TOPK_CAP = 128;   // candidate list capacity per src row (compacted to 64 above TOPK_TRIG)
constexpr int TOPK_TRIG = 112;  // compaction trigger: frequent enough that thresholds follow the running kt-th best
constexpr int TOPK_MAX = 512;   // k above TOPK_KC: exact full scan (topk_exact_kernel)
int topk_chunk_rows(int KP);    // dst rows per scan chunk (Th / cfeat are padded to whole chunks)
size_t topk_sort_temp_bytes(int64_t n_dst);
// VP: [TOPK_M][KP] fp64 (device); keys: 4·n uint32, perm / nperm: 2·n uint32 ([0, n) is the result:
// scan order / descending norm), tp: [n][TOPK_M] fp64 scratch, Th / cfeat / supf (super-chunk boxes)
// as above, probe: [256][KP] fp16
hipError_t topk_prepare(int KP, int kreal, const float* T, int64_t n_dst, float tsc, const double* VP, void* temp,
                        size_t temp_bytes, uint32_t* keys, uint32_t* perm, uint32_t* nperm, double* tp, void* Th,
                        float* cfeat, float* supf, void* probe, hipStream_t s);
hipError_t launch_topk(int KP, const TopkArgs& a, int n_cu, hipStream_t s);
hipError_t launch_topk_select(int KP, const TopkArgs& a, hipStream_t s);  // after launch_topk (the scan)
// starting thresholds + features + scan order of the src rows: keys / order 2·n_src uint32,
// thr_tmp / thr_sorted n_src floats, sf_tmp / sf_sorted n_src·TOPK_SF floats
size_t topk_order_temp_bytes(int64_t n_src);
hipError_t topk_order(int KP, const TopkArgs& a, void* temp, size_t temp_bytes, uint32_t* keys, uint32_t* order,
                      int32_t* src_sorted, float* thr_tmp, float* thr_sorted, float* sf_tmp, float* sf_sorted,
                      hipStream_t s);
// mask[wg][a.mask_words]: the chunks scan workgroup wg (rows_per_wg rows from position wg·rows_per_wg)
// can need against the starting thresholds (a.thr0, a.sfeat in scan order)
hipError_t launch_topk_mask(const TopkArgs& a, int rows_per_wg, const float* supf, int64_t n_super, uint32_t* mask,
                            hipStream_t s);
int topk_rows_per_workgroup(int KP, int64_t n_src, int n_cu);
// exact full scan for the given src-row indices (rows == null: rows 0 .. n_rows-1), any k <= TOPK_MAX
hipError_t launch_topk_exact(int KP, const TopkArgs& a, const int32_t* rows, int64_t n_rows, hipStream_t s);
// inv[perm[i]] = i for i < n
hipError_t launch_invert_perm(const uint32_t* perm, int64_t n, uint32_t* inv, hipStream_t s);
hipError_t launch_iota_i32(int32_t* out, int64_t n, int64_t start, hipStream_t s);  // out[i] = start + i
// the certification rescans without a host round trip: need[0 .. n) compacted into flags (cnt[0]: their
// count, cnt[1]: the persistent grid's work counter, both zero on entry; cnt[2] += the count), then a
// persistent exact scan over them
hipError_t launch_topk_exact_flagged(int KP, const TopkArgs& a, const int32_t* need, int64_t n, int32_t* flags, int* cnt,
                                     int n_cu, hipStream_t s);
// ---- evaluation (eval.hip): RankingEvaluator.scala:83-139 on the device ----------------------------
size_t eval_sort_temp_bytes(int64_t n);
// user ids -> rows of the ascending `ids`, grouped: runs[r] (row) with counts[r] entries at
// idx_sorted[offsets[r] ..]; *n_runs on the device (host copy synchronised inside); the unknown-id run
// (row 0xFFFFFFFF) is the last one when present
hipError_t eval_group_users(const int32_t* user, int64_t n, const int32_t* ids, int64_t n_ids, void* temp,
                            size_t temp_bytes, uint32_t* row, uint32_t* row_sorted, uint32_t* idx, uint32_t* idx_sorted,
                            uint32_t* runs, int32_t* counts, int64_t* offsets, int64_t* n_runs, hipStream_t s);
// per run: the first min(k, count) items by (key desc, item asc) -> act [n_runs][k] (-1 padded), act_n
hipError_t eval_actual_lists(const uint32_t* idx_sorted, const int64_t* offsets, const int32_t* counts, int64_t n_runs,
                             const int64_t* key, const int32_t* item, int k, int32_t* act, int32_t* act_n,
                             hipStream_t s);
// ndcgAt(k) per user of pred [n][k] (raw ids, -1 tail) against act; gain[i] = 1 / ln(i + 2)
hipError_t eval_ndcg(const int32_t* pred, const int32_t* act, const int32_t* act_n, int64_t n_users, int k,
                     const double* gain, double* out, hipStream_t s);
// *out = bits of max_r ||T[r][0..kreal)||_2 computed in fp64
hipError_t launch_rownorm_max(const float* T, int64_t n, int KP, int kreal, unsigned long long* out, hipStream_t s);

// Ingest (ingest.hip): COO -> remap + CSR.
struct DeviceBuf;
hipError_t remap_ids(const int32_t* d_ids, int64_t n, int32_t* d_dense, int32_t** d_unique,
                     int64_t* n_unique, hipStream_t s);
hipError_t build_csr(const int32_t* d_dst, const int32_t* d_src, const float* d_val, int64_t n,
                     int64_t n_dst, int64_t n_src, int64_t* d_ptr, int32_t* d_col, float* d_valout,
                     hipStream_t s);
// Shard row starts of one side (world + 1 entries, world <= 16), passed by value to kernels.
struct ShardStarts {
  int64_t s[17];
  int world;
};
// out[e] = gathered-layout position of dense src row in[e]: local row l of rank r at
// (l / chpad)·world·chpad + r·chpad + l % chpad (chunk-major: one chunk of every rank is contiguous)
hipError_t padded_remap(const int32_t* d_in, int64_t n, const ShardStarts& st, int64_t chpad, int32_t* d_out,
                        hipStream_t s);
// Failure diagnostics (not on the hot path): over n values of p (fp32, or fp16 when f16),
// out[0] += non-finite count, out[1] = min index of a non-finite value (atomicMin; caller sets it to
// ~0), out[2] = max |finite value| as float bits (atomicMax; caller zeroes it)
hipError_t launch_diag_scan(const void* p, int64_t n, bool f16, unsigned long long* out, hipStream_t s);
// Synthetic generator (synth.hip)
hipError_t synth_fill(uint64_t seed, int rounds, int64_t n_users, int64_t n_items,
                      const int64_t* d_deg_prefix, const double* d_cw, const int32_t* d_perm,
                      int32_t* d_user, int32_t* d_item, float* d_rating, int64_t n_slots,
                      int64_t* n_out, hipStream_t s);

}  // namespace albedo
