/*
 * albedo_als.h — C ABI of libalbedo_als.so, the MI355X implicit-ALS engine.
 *
 * Drop-in boundary: this library replaces Spark MLlib 2.2.0's
 * `ml.recommendation.ALS` / `ALSModel` as reached from albedo:
 *   - estimator params + fit  : ALSRecommenderBuilder.scala:46-58  (new ALS().setX(...).fit(ds))
 *                               ALSRecommenderCV.scala:46-52, Playground.scala:54-65,
 *                               src/main/python/train_als.py:55-61
 *   - model factors / rank    : ALSRecommender.scala:16-19,33-36  (alsModel.userFactors/itemFactors/rank)
 *   - top-k recommendation    : ALSRecommender.scala:28-65 (+ BoundedPriorityQueue.scala:30-53),
 *                               Spark ALSModel.recommendForAllUsers / recommendForUserSubset
 *   - per-pair prediction     : Spark ALSModel.transform (LogisticRegressionRanker.scala:167-174,229)
 * A JVM would bind these through JNI / Panama; Python binds them via ctypes
 * (albedo_amd/als.py).  No C++ or torch types cross this boundary: plain pointers and sizes.
 *
 * Conventions
 *   - Every function returning int returns ALS_OK (0) or an ALS_E_* code; the message is in
 *     als_last_error() (thread-local, valid until the next failing call on the same thread).
 *   - Host inputs are caller-owned and copied in.  Outputs go to caller-allocated buffers sized
 *     with als_num_rows()/als_rank().  The context owns all device memory.
 *   - A context is not re-entrant; separate contexts may be used from separate threads.
 *   - side: ALS_USER (0) or ALS_ITEM (1).  Factor rows are returned in ascending raw-id order,
 *     row-major [n][rank] float32, exactly like ALSModel.userFactors sorted by id.
 */
#ifndef ALBEDO_ALS_H
#define ALBEDO_ALS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALBEDO_ALS_ABI_VERSION 1

enum {
  ALS_OK = 0,
  ALS_E_INVALID_ARGUMENT = 1, /* Spark: IllegalArgumentException (ParamValidators, "No ratings available") */
  ALS_E_NOT_POSITIVE_DEFINITE = 2, /* Spark: IllegalArgumentException from CholeskyDecomposition (dppsv info>0) */
  ALS_E_STATE = 3,            /* call out of order (e.g. recommend before fit) -> IllegalStateException */
  ALS_E_HIP = 4,              /* HIP runtime failure                -> SparkException/RuntimeException */
  ALS_E_RCCL = 5,             /* RCCL failure */
  ALS_E_OUT_OF_MEMORY = 6,
  ALS_E_NO_DEVICE = 7,        /* no gfx950 device visible: the engine has no CPU fallback */
  ALS_E_UNSUPPORTED = 8       /* e.g. rank above the compiled maximum */
};

enum { ALS_USER = 0, ALS_ITEM = 1 };

/* Spark ALS params (ml/recommendation/ALS.scala ALSParams), defaults as Spark 2.2.0. */
typedef struct als_params {
  int32_t rank;            /* setRank, default 10, >= 1 */
  int32_t max_iter;        /* setMaxIter, default 10, >= 0 */
  int32_t implicit_prefs;  /* setImplicitPrefs, default 0 */
  int32_t nonnegative;     /* setNonnegative, default 0 */
  int32_t num_user_blocks; /* setNumUserBlocks, default 10, >= 1 (only shapes the Spark-style init) */
  int32_t num_item_blocks; /* setNumItemBlocks, default 10, >= 1 */
  double reg_param;        /* setRegParam, default 0.1, >= 0 */
  double alpha;            /* setAlpha, default 1.0, >= 0 */
  int64_t seed;            /* setSeed, default = hash of the class name in Spark; here 0 if unset */
  int32_t device;          /* HIP device ordinal; -1 = current device */
  int32_t light_max_degree;/* rows with <= this many ratings take the rotated push-through solve (capped at
                              96 at rank 65..128, 64 otherwise);
                              -1 = engine default, 0 = every row takes the explicit Cholesky solve */
} als_params;

typedef struct als_ctx als_ctx;

/* ---- lifecycle ---------------------------------------------------------------------------- */
int als_params_default(als_params* p);
int als_create(const als_params* p, als_ctx** out);
void als_destroy(als_ctx* ctx);
/* Replace the params of a context that already holds ratings (Spark Estimator.fit(dataset, paramMaps),
 * ALSRecommenderCV.scala:67-90): the ingest (remap, both CSRs, shards) is kept, rank-dependent
 * buffers and degree buckets are rebuilt and the factors are dropped, so the next als_fit starts
 * from the new seed's initialisation.  Validated like als_create; the device is kept. */
int als_set_params(als_ctx* ctx, const als_params* p);
/* A context that shares `parent`'s ingest (both CSRs, degree buckets, split-K lists: read-only views)
 * with factors, streams and scratch of its own, for concurrent fits of a CV grid
 * (ALSRecommenderCV.scala:67-90: several ParamMaps of one rank fitted at once from separate host
 * threads).  regParam, alpha, maxIter, implicitPrefs and seed may differ from the parent's; rank,
 * nonnegative and light_max_degree may not.  Single-process contexts only.  The parent's memory stays
 * allocated until its last fork is destroyed; als_set_params is refused on a fork and on a parent with
 * live forks. */
int als_fork(als_ctx* parent, const als_params* p, als_ctx** out);
const char* als_last_error(void);
int als_abi_version(void);
/* number of visible gfx950 devices (0 when no GPU; never initialises a context) */
int als_device_count(int* out);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI --------------------------------------- */
/* 128-byte ncclUniqueId produced on rank 0 and broadcast by the host (e.g. torch.distributed). */
int als_comm_unique_id(void* out128);
/* Must be called before als_set_ratings*; all ranks pass identical ratings. Rows of both sides are
 * sharded by nnz across ranks; each half-sweep all-reduces the partial Gram and all-gathers the
 * rotated factor shard. */
int als_comm_init(als_ctx* ctx, int32_t rank, int32_t world, const void* unique_id128);

/* ---- ingest (DatasetUtils.scala:111-123 input contract: (user Int, item Int, rating Float)) -- */
int als_set_ratings(als_ctx* ctx, int64_t n, const int32_t* user, const int32_t* item, const float* rating);
/* same, inputs already resident in device memory of ctx's device (not modified) */
int als_set_ratings_device(als_ctx* ctx, int64_t n, const int32_t* d_user, const int32_t* d_item,
                           const float* d_rating);
int64_t als_num_rows(const als_ctx* ctx, int side);
int64_t als_num_ratings(const als_ctx* ctx);
int als_rank(const als_ctx* ctx);
int als_get_ids(const als_ctx* ctx, int side, int32_t* ids_out); /* ascending */

/* ---- factors --------------------------------------------------------------------------------- */
/* Parity path: inject initial factors ([n][rank], any id order; every side id must be present). */
int als_set_initial_factors(als_ctx* ctx, int side, int64_t n, const int32_t* ids, const float* factors);
/* Spark-style initialisation (ALS.initialize with XORShiftRandom; best effort). */
int als_init_factors(als_ctx* ctx);
/* Seeded unit-norm Gaussian rows generated on device (large synthetic runs; not Spark's RNG). */
int als_init_factors_random(als_ctx* ctx, uint64_t seed);
int als_get_factors(als_ctx* ctx, int side, int32_t* ids_out, float* factors_out);

/* ---- fit --------------------------------------------------------------------------------------- */
/* Full ALS.train: init (if not injected) + max_iter x (item half-sweep, user half-sweep). Blocking. */
int als_fit(als_ctx* ctx);
/* Run n more full sweeps on the current factors (bench / incremental use). Blocking. */
int als_run_sweeps(als_ctx* ctx, int32_t n);
/* One half-sweep solving `dst_side` from the other side's current factors. Blocking. */
int als_half_sweep(als_ctx* ctx, int dst_side);
/* The ratings of one dst row (by raw id) as (src raw ids, ratings); *n_out = row length, arrays
 * are filled only when n_out <= cap.  Rows of other ranks are not available (ALS_E_STATE). */
int als_get_row_ratings(als_ctx* ctx, int side, int32_t id, int64_t cap, int32_t* src_ids, float* ratings,
                        int64_t* n_out);
/* Ratings per row of `side` in ascending id order (this rank's rows; -1 for rows other ranks own).
 * Observability for the power-law skew (the per-row work of Spark's computeFactors). */
int als_get_degrees(const als_ctx* ctx, int side, int64_t* out);
/* The orthogonal basis B of side's factors (rank x rank, row-major): original factors = X·Bᵀ, X the
 * factors as the engine holds them (als_get_factors returns the original ones).  Implicit fits
 * rotate every half-sweep's solution into the eigenbasis of the src Gram (B_t = B_s·P). */
int als_get_basis(als_ctx* ctx, int side, double* out);
/* Debug/parity: the last Gram matrix YᵀY of `src_side` in the original basis (fp64, [rank][rank];
 * Spark computeYtY of the src factors the last half-sweep solved from). */
int als_get_gram(als_ctx* ctx, int src_side, double* out);

/* ---- model (ALSModel) ------------------------------------------------------------------------ */
/* Build a model-only context from saved factors (ALSModel.load); ids need not be sorted. */
int als_model_create(int32_t rank, int64_t n_users, const int32_t* user_ids, const float* user_factors,
                     int64_t n_items, const int32_t* item_ids, const float* item_factors, int32_t device,
                     als_ctx** out);
/* recommendForAllUsers / recommendForUserSubset (side=ALS_USER) or ...Items (side=ALS_ITEM):
 * for each requested src id (all src rows when subset==NULL, ascending) the top-k dst ids by the
 * F2J-order fp32 dot product (ALSRecommender.scala:51), sorted (score desc, id asc).
 * Outputs [n_src][k]; rows with fewer than k dst entries are padded with id -1 / score NaN.
 * Unknown subset ids produce an all-padding row.  src_ids_out may be NULL.
 * k <= 64: MFMA pre-selection + exact rescoring; 64 < k <= 512: exact full scan per src row (slower);
 * k > 512: ALS_E_UNSUPPORTED. */
int als_recommend(als_ctx* ctx, int side, int32_t k, const int32_t* subset, int64_t n_subset,
                  int32_t* src_ids_out, int32_t* dst_ids_out, float* scores_out);
/* RankingEvaluator (RankingEvaluator.scala:83-139) on the device, the albedo protocol of
 * ALSRecommenderBuilder.scala:92-104: actual lists = intoUserActualItems(user, item, key desc, k) of
 * the given (user, item, key) rows (key = starred_at; rank() <= k, collect_list, slice(0, k) = the
 * first k by (key desc, item asc)), restricted to the model's users (inner join); predicted lists =
 * the users' top-k recommendations (als_recommend, kept on the device); mllib RankingMetrics.ndcgAt(k)
 * per user and the mean over users (*ndcg_out; NaN when no user is left).  users_out (ascending ids)
 * and per_user_out are filled when non-null and *n_users_out <= cap.  1 <= k <= 64. */
int als_evaluate_ndcg(als_ctx* ctx, int32_t k, int64_t n, const int32_t* user, const int32_t* item, const int64_t* key,
                      double* ndcg_out, int64_t* n_users_out, int32_t* users_out, double* per_user_out, int64_t cap);
/* ALSModel.transform: F2J sdot per (user, item) pair; NaN when either id is unknown. */
int als_predict(als_ctx* ctx, int64_t n, const int32_t* user, const int32_t* item, float* out);

/* ---- observability ---------------------------------------------------------------------------- */
/* Per-stage device time (ms) of the last half-sweeps: see ALS_T_* indices. n = array length. */
enum {
  ALS_T_GRAM = 0, ALS_T_EIG = 1, ALS_T_ROTATE = 2, ALS_T_COMM = 3, ALS_T_SOLVE_LIGHT = 4,
  ALS_T_SOLVE_HEAVY = 5, ALS_T_HALF_TOTAL = 6, ALS_T_COUNT = 8
};
int als_last_timings(const als_ctx* ctx, int dst_side, double* out, int n);
/* Rows / nnz handled by each solve path in the last half-sweep of dst_side:
 * out[0]=light rows, out[1]=light nnz, out[2]=heavy rows, out[3]=heavy nnz.  With nonnegative =
 * true "light" is the lockstep NNLS kernel (16 low-degree rows per workgroup) and "heavy" every
 * other row (one workgroup per row). */
int als_path_stats(const als_ctx* ctx, int dst_side, int64_t* out4);
/* Solver counters of the last half-sweep of dst_side.
 * nonnegative = true (NNLS): out[0] = iterations summed over rows, out[1] = max over rows,
 *   out[2] = rows, out[3] = the part of out[0] spent by the lockstep kernel's rows (als_path_stats out[0]).
 * nonnegative = false (Cholesky path): out[0] = Jacobi sweeps the device eigensolver took on the src
 *   Gram (0 without implicitPrefs), out[1..3] = 0.  A half-sweep whose eigensolver spends its sweep
 *   budget without converging fails with ALS_E_NOT_POSITIVE_DEFINITE. */
int als_solver_stats(const als_ctx* ctx, int dst_side, int64_t* out4);
/* Top-k counters since als_create (als_recommend with k <= 64): out[0] = src rows through the MFMA
 * scan, out[1] = rows whose candidate set failed certification and were re-scored by the exact scan,
 * out[2] = dst rows the scan waves scored (a wave skips a chunk none of its rows can use), out[3] = the same without the chunk
 * early exit. */
int als_topk_stats(const als_ctx* ctx, int64_t* out4);
/* Top-k device time since als_create, from HIP events on the context's stream (ms): out[0] = scan
 * order + chunk masks, out[1] = the MFMA scan, out[2] = select + certification, out[3] = exact
 * rescans; out[4] = the flops the scan's MFMAs performed (2·KP per scored src x dst pair), so
 * out[4] / out[1] is the scan's achieved matrix rate. */
int als_topk_timing(const als_ctx* ctx, double* out5);
/* The src ids whose candidate set failed certification in the last als_recommend call (k <= 64) and
 * were re-scored by the exact scan, in output order; *n_out = their count, ids filled when
 * n_out <= cap.  Parity tests check exactly these rows against the oracle. */
int als_topk_last_rescan(const als_ctx* ctx, int32_t* src_ids_out, int64_t cap, int64_t* n_out);
/* Synchronise the context's streams (bench barrier helper). */
int als_synchronize(als_ctx* ctx);

/* ---- synthetic workloads (BASELINE configs; same algorithm as albedo_amd/synthetic.py) -------- */
/* Run the device twin of synthetic.generate() and copy the COO to host buffers (n_out entries;
 * buffers sized deg_prefix[n_users]).  deg_prefix: per-user degree prefix (n_users+1, host),
 * cw: cumulative popularity weights (n_items, host), perm: popularity rank -> item position. */
int als_synth_generate(int32_t device, uint64_t seed, int32_t rounds, int64_t n_users, int64_t n_items,
                       const int64_t* deg_prefix, const double* cw, const int32_t* perm, int32_t* user_out,
                       int32_t* item_out, float* rating_out, int64_t* n_out);
/* Same, generated straight into the context's device ingest (inputs resident in HBM). */
int als_set_ratings_synthetic(als_ctx* ctx, uint64_t seed, int32_t rounds, int64_t n_users, int64_t n_items,
                              const int64_t* deg_prefix, const double* cw, const int32_t* perm);

/* ---- multi-process exchange through the host (tests: ranks sharing one GPU) -------------------- */
/* allreduce: in-place sum of n doubles over ranks; allgather: buf holds world*n_per_rank floats with
 * this rank's block filled; on return every block is filled.  Return 0 on success. */
int als_comm_init_host(als_ctx* ctx, int32_t rank, int32_t world, int (*allreduce)(void*, double*, int64_t),
                       int (*allgather)(void*, float*, int64_t), void* user);

/* ---- host-only utilities (no GPU; exercised by the CPU test suite) ----------------------------- */
int als_host_eigh(int32_t n, const double* a, double* w, double* v);  /* a = v diag(w) vᵀ, w ascending */
/* The engine's device eigensolver (warm-started cyclic Jacobi, eig.hip) on one k x k symmetric g:
 * a = v diag(w) vᵀ, w unordered; w0 (or NULL = identity) the orthogonal warm start; sweeps: Jacobi
 * sweeps taken.  Test hook, like als_host_eigh. */
int als_device_eigh(int32_t device, int32_t k, const double* g, const double* w0, double* w, double* v,
                    int32_t* sweeps);
int als_host_spark_side_seeds(int64_t seed, int64_t* user_seed, int64_t* item_seed);
int als_host_spark_init(const int32_t* ids_sorted, int64_t n, int32_t rank, int64_t side_seed,
                        int32_t num_blocks, float* out);
int als_host_plan_shards(const int64_t* ptr, int64_t n, int32_t world, int64_t* starts_out);

#ifdef __cplusplus
}
#endif
#endif /* ALBEDO_ALS_H */
