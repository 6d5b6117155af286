/* cg_oracle.c -- CPU restatement of the reference CG hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see cg_oracle.h).  Pinned bit-for-bit against the
 * compiled reference by tests/test_oracle.py + tests/golden/.
 *
 * Compile with -ffp-contract=off and without -march=native: the reference is
 * built -O0 (Makefile:2) and never fuses a multiply into an add.
 */
#include "cg_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>


/* mv_ops.c:160-201 (+ mat_get_row :99-113), CSR form. */
int oracle_spmv_csr(int n, const int *row_ptr, const int *col, const double *val,
                    const double *x, double *y)
{
  for (int i = 0; i < n; i++) {
    double acc = 0.0;                         /* mv_ops.c:190 dp_res = 0 */
    for (int k = row_ptr[i]; k < row_ptr[i + 1]; k++) {
      double prod = val[k] * x[col[k]];       /* rounded product */
      acc = acc + prod;                       /* mv_ops.c:193 */
    }
    y[i] = acc;                               /* mv_ops.c:196 */
  }
  return 0;
}

/* mv_ops.c:99-113 mat_get_row, greedy scan from row_ptr[row]. */
static void expand_row(int n, int nnz, const int *row_ptr, const int *col,
                       const double *val, int row, double *dense)
{
  int ci = row_ptr[row];
  for (int i = 0; i < n; i++) {
    if (ci < nnz && col[ci] == i)
      dense[i] = val[ci++];
    else
      dense[i] = 0.0;
  }
}

/* mv_ops.c:160-201, literal O(n^2) form. */
int oracle_spmv_dense_expand(int n, int nnz, const int *row_ptr, const int *col,
                             const double *val, const double *x, double *y)
{
  double *row = (double *)calloc((size_t)n, sizeof(double));
  if (!row)
    return -1;
  for (int i = 0; i < n; i++) {
    expand_row(n, nnz, row_ptr, col, val, i, row);
    double acc = 0.0;
    for (int j = 0; j < n; j++) {
      double prod = row[j] * x[j];
      acc = acc + prod;
    }
    y[i] = acc;
  }
  free(row);
  return 0;
}

/* mv_ops.c:117-132 */
double oracle_dot(int n, const double *a, const double *b)
{
  double acc = 0.0;
  for (int i = 0; i < n; i++) {
    double prod = a[i] * b[i];
    acc = acc + prod;
  }
  return acc;
}

/* mv_ops.c:134-158 */
void oracle_scale(int n, double s, const double *a, double *r)
{
  for (int i = 0; i < n; i++)
    r[i] = s * a[i];
}

/* mv_ops.c:203-230 */
void oracle_add(int n, const double *a, const double *b, double *r)
{
  for (int i = 0; i < n; i++)
    r[i] = a[i] + b[i];
}

/* mv_ops.c:232-259 */
void oracle_sub(int n, const double *a, const double *b, double *r)
{
  for (int i = 0; i < n; i++)
    r[i] = a[i] - b[i];
}

/* Shared HS-CG body: cg.c:88-141 with an optional tolerance stop placed at
 * the reference's break position (cg.c:125). */
static int hs_cg(int max_iter, double tol, int n, int nnz, const int *row_ptr,
                 const int *col, const double *val, const double *b, double *x,
                 int dense_expand, double *rr_hist)
{
  size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(double);
  double *r = (double *)malloc(bytes);
  double *p = (double *)malloc(bytes);
  double *s = (double *)malloc(bytes);
  double *t = (double *)malloc(bytes);
  if (!r || !p || !s || !t) {
    free(r); free(p); free(s); free(t);
    return -1;
  }
  memset(x, 0, (size_t)n * sizeof(double));      /* cg.c:104, x0 = 0 */
  memcpy(r, b, (size_t)n * sizeof(double));      /* cg.c:107 r = b   */
  memcpy(p, r, (size_t)n * sizeof(double));      /* cg.c:108 p = r   */
  double bb = oracle_dot(n, b, b);
  double rr = oracle_dot(n, r, r);
  double tol2bb = tol * tol * bb;
  int k = 0;
  for (;;) {                                                   /* cg.c:110 */
    if (dense_expand)
      oracle_spmv_dense_expand(n, nnz, row_ptr, col, val, p, s);
    else
      oracle_spmv_csr(n, row_ptr, col, val, p, s);             /* cg.c:111 */
    double alpha = rr / oracle_dot(n, p, s);                   /* cg.c:113 */
    oracle_scale(n, alpha, p, t);                              /* cg.c:115 */
    oracle_add(n, x, t, x);                                    /* cg.c:117-118 */
    oracle_scale(n, alpha, s, t);                              /* cg.c:122 */
    oracle_sub(n, r, t, r);                                    /* cg.c:123 */
    double rr_new = oracle_dot(n, r, r);                       /* cg.c:129 numerator */
    if (rr_hist)
      rr_hist[k] = rr_new;
    if (k == max_iter)                                         /* cg.c:125 */
      break;
    if (tol > 0.0 && rr_new <= tol2bb)
      break;
    double beta = rr_new / rr;                                 /* cg.c:129 */
    oracle_scale(n, beta, p, t);                               /* cg.c:131 */
    oracle_add(n, r, t, p);                                    /* cg.c:132 */
    rr = rr_new;
    k++;                                                       /* cg.c:134 */
  }
  free(r); free(p); free(s); free(t);
  return k + 1;
}

int oracle_conj_grad(int max_iter, int n, int nnz, const int *row_ptr,
                     const int *col, const double *val, const double *b,
                     double *x, int dense_expand, double *rr_hist)
{
  return hs_cg(max_iter, 0.0, n, nnz, row_ptr, col, val, b, x, dense_expand,
               rr_hist);
}

int oracle_solve(int maxit, double tol, int n, const int *row_ptr,
                 const int *col, const double *val, const double *b, double *x,
                 double *rr_hist)
{
  return hs_cg(maxit, tol, n, n > 0 ? row_ptr[n] : 0, row_ptr, col, val, b, x,
               0, rr_hist);
}

/* Chronopoulos-Gear CG: one fused reduction (gamma = r.r, delta = w.r) per
 * iteration.  p and s start at zero with beta = 0, so the first update gives
 * p = r, s = w exactly as the GPU kernels do. */
int oracle_solve_cg1(int maxit, double tol, int n, const int *row_ptr,
                     const int *col, const double *val, const double *b,
                     double *x, double *rr_hist)
{
  size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(double);
  double *r = (double *)malloc(bytes), *w = (double *)malloc(bytes);
  double *p = (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  double *s = (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  if (!r || !w || !p || !s) {
    free(r); free(w); free(p); free(s);
    return -1;
  }
  memset(x, 0, (size_t)n * sizeof(double));
  memcpy(r, b, (size_t)n * sizeof(double));
  double bb = oracle_dot(n, b, b);
  double tol2bb = tol * tol * bb;
  oracle_spmv_csr(n, row_ptr, col, val, r, w);
  double gamma = oracle_dot(n, r, r);
  double delta = oracle_dot(n, w, r);
  double alpha = gamma / delta, beta = 0.0;
  int k = 0;
  for (;;) {
    for (int i = 0; i < n; i++) {
      double bp = beta * p[i];
      p[i] = r[i] + bp;
      double bs = beta * s[i];
      s[i] = w[i] + bs;
      double ap = alpha * p[i];
      x[i] = x[i] + ap;
      double as = alpha * s[i];
      r[i] = r[i] - as;
    }
    double gamma_new = oracle_dot(n, r, r);
    if (rr_hist)
      rr_hist[k] = gamma_new;
    if (k == maxit)
      break;
    if (tol > 0.0 && gamma_new <= tol2bb)
      break;
    oracle_spmv_csr(n, row_ptr, col, val, r, w);
    delta = oracle_dot(n, w, r);
    beta = gamma_new / gamma;
    alpha = gamma_new / (delta - beta * gamma_new / alpha);
    gamma = gamma_new;
    k++;
  }
  free(r); free(w); free(p); free(s);
  return k + 1;
}

/* The single-reduction HS variant (CGX_ALG_SR, the N = 1 bench recurrence
 * and the partitioned solver's): cg.c:88-141's recurrence with p.s, s.s and
 * r.r computed together (one reduction / all-reduce on the GPUs).
 * alpha = r.r / p.s exactly as cg.c:113; beta (cg.c:129) uses
 * r_new.r_new = alpha (alpha s.s) - r.r (clamped at 0), which equals the
 * exact r_new.r_new in exact arithmetic because r.s = p.s.  The stop test
 * (cg.c:125 position) reads the EXACT r_new.r_new -- the reference's rule;
 * the GPUs get it from the next launch's reduction, one launch late -- and
 * the exact r_new.r_new is the next alpha's numerator.  rr_hist records the
 * exact r_new.r_new, as oracle_solve's. */
int oracle_solve_sr(int maxit, double tol, int n, const int *row_ptr,
                    const int *col, const double *val, const double *b,
                    double *x, double *rr_hist)
{
  size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(double);
  double *r = (double *)malloc(bytes), *p = (double *)malloc(bytes);
  double *s = (double *)malloc(bytes);
  if (!r || !p || !s) {
    free(r); free(p); free(s);
    return -1;
  }
  memset(x, 0, (size_t)n * sizeof(double));
  memcpy(r, b, (size_t)n * sizeof(double));
  memcpy(p, r, (size_t)n * sizeof(double));
  double bb = oracle_dot(n, b, b);
  double rr = bb;
  double tol2bb = tol * tol * bb;
  int k = 0;
  for (;;) {
    oracle_spmv_csr(n, row_ptr, col, val, p, s);
    double ps = oracle_dot(n, p, s), ss = oracle_dot(n, s, s);
    double alpha = rr / ps;
    for (int i = 0; i < n; i++) {
      double ap = alpha * p[i];
      x[i] = x[i] + ap;
      double as = alpha * s[i];
      r[i] = r[i] - as;
    }
    double as2 = alpha * ss;
    double est = alpha * as2 - rr;
    if (!(est > 0.0))
      est = 0.0;
    double rr_new = oracle_dot(n, r, r);
    if (rr_hist)
      rr_hist[k] = rr_new;
    if (k == maxit)
      break;
    if (tol > 0.0 && rr_new <= tol2bb)
      break;
    double beta = est / rr;
    for (int i = 0; i < n; i++) {
      double bp = beta * p[i];
      p[i] = r[i] + bp;
    }
    rr = rr_new;
    k++;
  }
  free(r); free(p); free(s);
  return k + 1;
}

int oracle_spmv_csr_f32(int n, const int *row_ptr, const int *col,
                        const float *val, const float *x, float *y)
{
  for (int i = 0; i < n; i++) {
    float acc = 0.0f;
    for (int k = row_ptr[i]; k < row_ptr[i + 1]; k++) {
      float prod = val[k] * x[col[k]];
      acc = acc + prod;
    }
    y[i] = acc;
  }
  return 0;
}

/* C5's iteration: cg.c:88-141 with fp32 matrix and vectors, as libcgx runs
 * it (the reference itself is fp64 only, mv_ops.h:20).
 * Row sums and products in float (oracle_spmv_csr_f32); every dot product
 * sums the EXACT double products of the float operands, sequentially from
 * 0.0 (the kernels' partials do the same in another grouping); alpha and
 * beta are formed in double (cg.c:113, 129) and rounded to float once for
 * the float vector updates, each a float product then a float add
 * (cg.c:115-132's two roundings). */
static double dot_f32(int n, const float *a, const float *b)
{
  double acc = 0.0;
  for (int i = 0; i < n; i++)
    acc = acc + (double)a[i] * (double)b[i];
  return acc;
}

int oracle_solve_f32(int maxit, double tol, int n, const int *row_ptr,
                     const int *col, const float *val, const float *b,
                     float *x, double *rr_hist)
{
  size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(float);
  float *r = (float *)malloc(bytes), *p = (float *)malloc(bytes);
  float *s = (float *)malloc(bytes);
  if (!r || !p || !s) {
    free(r); free(p); free(s);
    return -1;
  }
  memset(x, 0, (size_t)n * sizeof(float));          /* cg.c:104 */
  memcpy(r, b, (size_t)n * sizeof(float));          /* cg.c:107 */
  memcpy(p, b, (size_t)n * sizeof(float));          /* cg.c:108 */
  double bb = dot_f32(n, b, b), rr = bb, tol2bb = tol * tol * bb;
  int k = 0;
  for (;;) {
    oracle_spmv_csr_f32(n, row_ptr, col, val, p, s);          /* cg.c:111 */
    double alpha = rr / dot_f32(n, p, s);                     /* cg.c:113 */
    float af = (float)alpha;
    for (int i = 0; i < n; i++) {
      float ap = af * p[i];
      x[i] = x[i] + ap;                                       /* cg.c:115-118 */
      float as = af * s[i];
      r[i] = r[i] - as;                                       /* cg.c:122-123 */
    }
    double rr_new = dot_f32(n, r, r);
    if (rr_hist)
      rr_hist[k] = rr_new;
    if (k == maxit)                                           /* cg.c:125 */
      break;
    if (tol > 0.0 && rr_new <= tol2bb)
      break;
    float bf = (float)(rr_new / rr);                          /* cg.c:129 */
    for (int i = 0; i < n; i++) {
      float bp = bf * p[i];
      p[i] = r[i] + bp;                                       /* cg.c:131-132 */
    }
    rr = rr_new;
    k++;
  }
  free(r); free(p); free(s);
  return k + 1;
}

/* ---------------- multithreaded CPU baseline (pthreads) ---------------- */

typedef struct {
  int op, lo, hi;
  const int *row_ptr, *col;
  const double *val;
  double *x, *r, *p, *s;
  double alpha, beta;
  double part;
} mt_task;

enum { MT_SPMV_PS = 0, MT_UPDATE_XR = 1, MT_XPAY = 2 };

static void *mt_worker(void *arg)
{
  mt_task *t = (mt_task *)arg;
  double part = 0.0;
  if (t->op == MT_SPMV_PS) {
    for (int i = t->lo; i < t->hi; i++) {
      double acc = 0.0;
      for (int k = t->row_ptr[i]; k < t->row_ptr[i + 1]; k++) {
        double prod = t->val[k] * t->p[t->col[k]];
        acc = acc + prod;
      }
      t->s[i] = acc;
      double prod = t->p[i] * acc;
      part = part + prod;
    }
  } else if (t->op == MT_UPDATE_XR) {
    for (int i = t->lo; i < t->hi; i++) {
      double ap = t->alpha * t->p[i];
      t->x[i] = t->x[i] + ap;
      double as = t->alpha * t->s[i];
      double ri = t->r[i] - as;
      t->r[i] = ri;
      double prod = ri * ri;
      part = part + prod;
    }
  } else {
    for (int i = t->lo; i < t->hi; i++) {
      double bp = t->beta * t->p[i];
      t->p[i] = t->r[i] + bp;
    }
  }
  t->part = part;
  return NULL;
}

static double mt_run(mt_task *tasks, pthread_t *th, int threads, int op)
{
  for (int i = 0; i < threads; i++) {
    tasks[i].op = op;
    pthread_create(&th[i], NULL, mt_worker, &tasks[i]);
  }
  double sum = 0.0;
  for (int i = 0; i < threads; i++) {
    pthread_join(th[i], NULL);
    sum = sum + tasks[i].part;
  }
  return sum;
}

int oracle_solve_mt(int maxit, double tol, int n, const int *row_ptr,
                    const int *col, const double *val, const double *b,
                    double *x, int threads)
{
  if (threads < 1)
    threads = 1;
  size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(double);
  double *r = (double *)malloc(bytes), *p = (double *)malloc(bytes);
  double *s = (double *)malloc(bytes);
  mt_task *tasks = (mt_task *)calloc((size_t)threads, sizeof(mt_task));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  if (!r || !p || !s || !tasks || !th) {
    free(r); free(p); free(s); free(tasks); free(th);
    return -1;
  }
  memset(x, 0, (size_t)n * sizeof(double));
  memcpy(r, b, (size_t)n * sizeof(double));
  memcpy(p, b, (size_t)n * sizeof(double));
  for (int i = 0; i < threads; i++) {
    tasks[i].lo = (int)((long long)n * i / threads);
    tasks[i].hi = (int)((long long)n * (i + 1) / threads);
    tasks[i].row_ptr = row_ptr; tasks[i].col = col; tasks[i].val = val;
    tasks[i].x = x; tasks[i].r = r; tasks[i].p = p; tasks[i].s = s;
  }
  double bb = oracle_dot(n, b, b), rr = bb, tol2bb = tol * tol * bb;
  int k = 0;
  for (;;) {
    double ps = mt_run(tasks, th, threads, MT_SPMV_PS);
    double alpha = rr / ps;
    for (int i = 0; i < threads; i++) tasks[i].alpha = alpha;
    double rr_new = mt_run(tasks, th, threads, MT_UPDATE_XR);
    if (k == maxit || (tol > 0.0 && rr_new <= tol2bb))
      break;
    double beta = rr_new / rr;
    for (int i = 0; i < threads; i++) tasks[i].beta = beta;
    mt_run(tasks, th, threads, MT_XPAY);
    rr = rr_new;
    k++;
  }
  free(r); free(p); free(s); free(tasks); free(th);
  return k + 1;
}
