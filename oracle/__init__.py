"""CPU oracle for the implicit-ALS hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import, call or
link anything under `oracle/`, and only as the checker (or the timed CPU baseline), never as the
thing measured or shipped.  The product path (`albedo_amd`, `libalbedo_als.so`) never imports it.

What it restates:
* `spark_als.py`  — Spark MLlib 2.2.0 `ml.recommendation.ALS` implicit/explicit fit in fp64
  (`computeYtY`, `NormalEquation.add/merge`, `CholeskySolver` -> LAPACK `dppsv`,
  `NNLSSolver` -> `mllib.optimization.NNLS`), reached from `ALSRecommenderBuilder.scala:46-58`;
  albedo's scorer `ALSRecommender.scala:28-65` (F2J `sdot` order) with
  `BoundedPriorityQueue.scala:30-53`; `RankingMetrics.ndcgAt` used at `RankingEvaluator.scala:96-98`.
* `c/als_cpu.c`   — the same half-sweep in C/OpenMP (fp64 packed `dspr` + packed Cholesky),
  used as the timed CPU baseline ("port") and cross-checked against the numpy restatement.

Pinning: Spark itself cannot run here (no JVM, no pyspark) and the reference
has no tests, so the ALS loop is **parity unpinned** against Spark.  What is pinned:
* the Cholesky solve IS LAPACK `dppsv` (scipy's LAPACK, the routine netlib-java calls);
* `ndcgAt` reproduces Spark's `RankingMetricsSuite` known answers (tests/test_oracle.py);
* NNLS reaches scipy's active-set NNLS optimum on well-conditioned systems;
* the F2J `sdot` association order is restated from netlib BLAS `sdot.f`.
"""
