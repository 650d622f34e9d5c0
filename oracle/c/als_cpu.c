/*
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): C/OpenMP restatement of one Spark MLlib 2.2.0
 * ALS half-sweep (ml/recommendation/ALS.scala computeFactors, reached from
 * ALSRecommenderBuilder.scala:58), in fp64 like Spark:
 *   computeYtY           G = Σ y yᵀ over all src rows (NormalEquation.add(y, 0) = dspr + merge)
 *   per dst row j        A = G (implicit) ; for each rating: c1 = α|r|, A += c1 y yᵀ (dspr),
 *                        b += (r > 0 ? 1 + c1 : 0) y (daxpy), n += (r > 0)
 *                        explicit: A += y yᵀ, b += r y, n += 1
 *   CholeskySolver       A += λ n I ; dppsv (Cholesky A = Uᵀ U + two triangular solves) ; to float
 *   NNLSSolver           (nonnegative = true) fillAtA (full symmetric, A += λ n I) ; NNLS.solve
 *                        (mllib/optimization/NNLS.scala: projected gradient with CG acceleration,
 *                        restated in oracle/spark_als.py:nnls) ; to float
 * Used (a) by tests to cross-check the numpy restatement and (b) by bench.py as the timed
 * `cpu_baseline` ("port": Spark-algorithm CPU restatement, not Spark).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Upper-packed (column-major, LAPACK 'U') index of (i, j), i <= j */
#define UP(i, j) ((i) + (int64_t)(j) * ((j) + 1) / 2)

static void dspr_upper(int k, double alpha, const double* x, double* ap) {
  for (int j = 0; j < k; ++j) {
    const double t = alpha * x[j];
    if (x[j] != 0.0)
      for (int i = 0; i <= j; ++i) ap[UP(i, j)] += x[i] * t;
  }
}

/* dppsv('U'): returns 0 or the order of the first non-positive leading minor */
static int dppsv_upper(int k, double* ap, double* b) {
  /* dpptrf: U column by column */
  for (int j = 0; j < k; ++j) {
    for (int i = 0; i < j; ++i) {  /* solve Uᵀ u_j = a_j for the off-diagonal part of column j */
      double s = ap[UP(i, j)];
      for (int m = 0; m < i; ++m) s -= ap[UP(m, i)] * ap[UP(m, j)];
      ap[UP(i, j)] = s / ap[UP(i, i)];
    }
    double d = ap[UP(j, j)];
    for (int m = 0; m < j; ++m) d -= ap[UP(m, j)] * ap[UP(m, j)];
    if (!(d > 0.0)) return j + 1;
    ap[UP(j, j)] = sqrt(d);
  }
  /* dpptrs: Uᵀ y = b, U x = y */
  for (int i = 0; i < k; ++i) {
    double s = b[i];
    for (int m = 0; m < i; ++m) s -= ap[UP(m, i)] * b[m];
    b[i] = s / ap[UP(i, i)];
  }
  for (int i = k - 1; i >= 0; --i) {
    double s = b[i];
    for (int m = i + 1; m < k; ++m) s -= ap[UP(i, m)] * b[m];
    b[i] = s / ap[UP(i, i)];
  }
  return 0;
}

int oracle_gram(int64_t n_src, int k, const float* Y, double* G_full, int nthreads) {
  const int64_t tk = (int64_t)k * (k + 1) / 2;
  double* acc = calloc((size_t)tk * (nthreads > 0 ? nthreads : 1), sizeof(double));
  if (!acc) return -1;
#pragma omp parallel num_threads(nthreads)
  {
    double* ap = acc + (size_t)tk * omp_get_thread_num();
    double* x = malloc(sizeof(double) * k);
#pragma omp for schedule(static)
    for (int64_t r = 0; r < n_src; ++r) {
      for (int c = 0; c < k; ++c) x[c] = Y[r * k + c];
      dspr_upper(k, 1.0, x, ap);
    }
    free(x);
  }
  for (int i = 0; i < k; ++i)
    for (int j = i; j < k; ++j) {
      double s = 0.0;
      for (int t = 0; t < nthreads; ++t) s += acc[(size_t)tk * t + UP(i, j)];
      G_full[i * k + j] = G_full[j * k + i] = s;
    }
  free(acc);
  return 0;
}

/* Solve dst rows given the src Gram G (k x k, used when implicit). rows: which dst rows (NULL = all
 * n_dst); X_out indexed by dst row. Returns 0 or the (1-based) dst row whose normal equation was not
 * positive definite. */
int oracle_solve_rows(int64_t n_dst, const int64_t* ptr, const int32_t* col, const float* val,
                      const float* Y, int k, int implicit, double alpha, double reg, const double* G,
                      const int32_t* rows, int64_t n_rows, float* X_out, int nthreads) {
  const int64_t tk = (int64_t)k * (k + 1) / 2;
  double* Gp = calloc((size_t)tk, sizeof(double));
  if (!Gp) return -1;
  if (implicit)
    for (int j = 0; j < k; ++j)
      for (int i = 0; i <= j; ++i) Gp[UP(i, j)] = G[i * k + j];
  if (!rows) n_rows = n_dst;
  int bad = 0;
#pragma omp parallel num_threads(nthreads)
  {
    double* ap = malloc(sizeof(double) * tk);
    double* b = malloc(sizeof(double) * k);
    double* y = malloc(sizeof(double) * k);
#pragma omp for schedule(dynamic, 64)
    for (int64_t q = 0; q < n_rows; ++q) {
      const int64_t j = rows ? rows[q] : q;
      if (implicit) memcpy(ap, Gp, sizeof(double) * tk);
      else memset(ap, 0, sizeof(double) * tk);
      memset(b, 0, sizeof(double) * k);
      int64_t n = 0;
      for (int64_t p = ptr[j]; p < ptr[j + 1]; ++p) {
        const float* yr = Y + (int64_t)col[p] * k;
        for (int c = 0; c < k; ++c) y[c] = yr[c];
        const double r = val[p];
        double cw, bw;
        if (implicit) {
          cw = alpha * fabs(r);
          bw = r > 0.0 ? 1.0 + cw : 0.0;
          if (r > 0.0) ++n;
        } else {
          cw = 1.0;
          bw = r;
          ++n;
        }
        if (cw != 0.0) dspr_upper(k, cw, y, ap);
        if (bw != 0.0)
          for (int c = 0; c < k; ++c) b[c] += bw * y[c];
      }
      const double lam = reg * (double)n;
      for (int c = 0; c < k; ++c) ap[UP(c, c)] += lam;
      if (dppsv_upper(k, ap, b) != 0) {
#pragma omp critical
        bad = (int)(j + 1);
      }
      for (int c = 0; c < k; ++c) X_out[j * k + c] = (float)b[c];
    }
    free(ap);
    free(b);
    free(y);
  }
  free(Gp);
  return bad;
}

/* mllib/optimization/NNLS.scala solve (Spark 2.2.0), the numpy restatement oracle/spark_als.py:nnls
 * (:247-299) line for line: ata full n x n (column-major = row-major, symmetric), ws = 5n doubles.
 * Returns the iterations taken. */
static int nnls_solve(int n, const double* ata, const double* atb, double* x, double* ws) {
  double *grad = ws, *dir = ws + n, *last_dir = ws + 2 * n, *res = ws + 3 * n, *scratch = ws + 4 * n;
  const int iter_max = n * 20 > 400 ? n * 20 : 400;
  double last_norm = 0.0;
  int iterno = 0, last_wall = 0;
  for (int i = 0; i < n; ++i) x[i] = last_dir[i] = 0.0;
#define NNLS_DOT(a, b) ({ double s_ = 0.0; for (int i_ = 0; i_ < n; ++i_) s_ += (a)[i_] * (b)[i_]; s_; })
#define NNLS_GEMV(v, out) for (int r_ = 0; r_ < n; ++r_) { double s_ = 0.0; \
    for (int c_ = 0; c_ < n; ++c_) s_ += ata[(int64_t)r_ * n + c_] * (v)[c_]; (out)[r_] = s_; }
  while (iterno < iter_max) {
    NNLS_GEMV(x, res);
    for (int i = 0; i < n; ++i) {
      res[i] -= atb[i];
      grad[i] = (res[i] > 0.0 && x[i] == 0.0) ? 0.0 : res[i];
    }
    const double ngrad = NNLS_DOT(grad, grad);
    for (int i = 0; i < n; ++i) dir[i] = grad[i];
    NNLS_GEMV(grad, scratch);
    double step = NNLS_DOT(grad, res) / (NNLS_DOT(scratch, grad) + 1e-20);
    double ndir;
    const double nx = NNLS_DOT(x, x);
#define NNLS_STOP(st, nd) (isnan(st) || (st) < 1e-7 || (st) > 1e40 || (nd) < 1e-12 * nx || (nd) < 1e-32)
    if (iterno > last_wall + 1) {
      const double alpha = ngrad / last_norm;
      for (int i = 0; i < n; ++i) dir[i] += alpha * last_dir[i];
      NNLS_GEMV(dir, scratch);
      const double dstep = NNLS_DOT(dir, res) / (NNLS_DOT(scratch, dir) + 1e-20);
      ndir = NNLS_DOT(dir, dir);
      if (NNLS_STOP(dstep, ndir)) {
        for (int i = 0; i < n; ++i) dir[i] = grad[i];
        ndir = NNLS_DOT(dir, dir);
      } else {
        step = dstep;
      }
    } else {
      ndir = NNLS_DOT(dir, dir);
    }
    if (NNLS_STOP(step, ndir)) break;
    for (int i = 0; i < n; ++i)
      if (step * dir[i] > x[i]) step = x[i] / dir[i];
    for (int i = 0; i < n; ++i) {
      if (step * dir[i] > x[i] * (1 - 1e-14)) {
        x[i] = 0.0;
        last_wall = iterno;
      } else {
        x[i] -= step * dir[i];
      }
    }
    ++iterno;
    for (int i = 0; i < n; ++i) last_dir[i] = dir[i];
    last_norm = ngrad;
  }
#undef NNLS_DOT
#undef NNLS_GEMV
#undef NNLS_STOP
  return iterno;
}

/* NNLS.solve on one dense system (ata full n x n with λ n already on its diagonal): x (n doubles) and the
 * iterations taken */
int oracle_nnls_dense(int n, const double* ata, const double* atb, double* x) {
  double* ws = malloc(sizeof(double) * 5 * n);
  if (!ws) return -1;
  const int it = nnls_solve(n, ata, atb, x, ws);
  free(ws);
  return it;
}

/* oracle_solve_rows with Spark's NNLSSolver in place of the CholeskySolver (ALS with
 * setNonnegative(true), ALSRecommenderBuilder.scala:46-56 surface): the same normal equation, then
 * fillAtA + NNLS.solve per row, OpenMP over rows.  iters_out (may be NULL): per solved row (indexed
 * like X_out) the NNLS iterations.  Returns 0. */
int oracle_solve_rows_nnls(int64_t n_dst, const int64_t* ptr, const int32_t* col, const float* val,
                           const float* Y, int k, int implicit, double alpha, double reg, const double* G,
                           const int32_t* rows, int64_t n_rows, float* X_out, int32_t* iters_out, int nthreads) {
  const int64_t tk = (int64_t)k * (k + 1) / 2;
  if (!rows) n_rows = n_dst;
#pragma omp parallel num_threads(nthreads)
  {
    double* ap = malloc(sizeof(double) * tk);
    double* A = malloc(sizeof(double) * k * k);
    double* b = malloc(sizeof(double) * k);
    double* y = malloc(sizeof(double) * k);
    double* x = malloc(sizeof(double) * k);
    double* ws = malloc(sizeof(double) * 5 * k);
#pragma omp for schedule(dynamic, 16)
    for (int64_t q = 0; q < n_rows; ++q) {
      const int64_t j = rows ? rows[q] : q;
      if (implicit) {
        for (int jj = 0; jj < k; ++jj)
          for (int i = 0; i <= jj; ++i) ap[UP(i, jj)] = G[i * k + jj];
      } else {
        memset(ap, 0, sizeof(double) * tk);
      }
      memset(b, 0, sizeof(double) * k);
      int64_t n = 0;
      for (int64_t p = ptr[j]; p < ptr[j + 1]; ++p) {
        const float* yr = Y + (int64_t)col[p] * k;
        for (int c = 0; c < k; ++c) y[c] = yr[c];
        const double r = val[p];
        double cw, bw;
        if (implicit) {
          cw = alpha * fabs(r);
          bw = r > 0.0 ? 1.0 + cw : 0.0;
          if (r > 0.0) ++n;
        } else {
          cw = 1.0;
          bw = r;
          ++n;
        }
        if (cw != 0.0) dspr_upper(k, cw, y, ap);
        if (bw != 0.0)
          for (int c = 0; c < k; ++c) b[c] += bw * y[c];
      }
      /* NNLSSolver.fillAtA: the full symmetric matrix, λ n on the diagonal */
      const double lam = reg * (double)n;
      for (int jj = 0; jj < k; ++jj)
        for (int i = 0; i <= jj; ++i) A[(int64_t)i * k + jj] = A[(int64_t)jj * k + i] = ap[UP(i, jj)];
      for (int c = 0; c < k; ++c) A[(int64_t)c * k + c] += lam;
      const int it = nnls_solve(k, A, b, x, ws);
      if (iters_out) iters_out[j] = it;
      for (int c = 0; c < k; ++c) X_out[j * k + c] = (float)x[c];
    }
    free(ap);
    free(A);
    free(b);
    free(y);
    free(x);
    free(ws);
  }
  return 0;
}

int oracle_half_sweep(int64_t n_dst, const int64_t* ptr, const int32_t* col, const float* val,
                      int64_t n_src, const float* Y, int k, int implicit, double alpha, double reg,
                      const int32_t* rows, int64_t n_rows, float* X_out, int nthreads) {
  double* G = calloc((size_t)k * k, sizeof(double));
  if (!G) return -1;
  if (implicit && oracle_gram(n_src, k, Y, G, nthreads) != 0) return -1;
  const int rc = oracle_solve_rows(n_dst, ptr, col, val, Y, k, implicit, alpha, reg, G, rows, n_rows, X_out,
                                   nthreads);
  free(G);
  return rc;
}

int oracle_max_threads(void) { return omp_get_max_threads(); }
