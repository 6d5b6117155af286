/* cg_oracle.h -- CPU restatement of the reference CG hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libcgx.so, the cg CLI)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the timed
 * CPU baseline.
 *
 * Every function restates the semantics of rnelias/Conjugate-Gradient
 * (cg.c, mv_ops.c); the reference file:line is cited on each declaration.
 * Parity is pinned: tests/test_oracle.py checks these functions bit-for-bit
 * against golden vectors produced by the compiled reference
 * (tests/golden/make_golden.py, oracle/Makefile target `ref`).
 *
 * Build rule: no FMA contraction (-ffp-contract=off, no -march=native).  The
 * reference's Makefile builds with `gcc -Wall -g` (-O0), which never contracts,
 * so x += alpha*p is two roundings there and must be two roundings here.
 */
#ifndef CG_ORACLE_H
#define CG_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* y = A x over CSR, each row summed sequentially from 0.0 in stored column
 * order, each product rounded before the add.  Equals the reference's
 * dense-row mv_mult (mv_ops.c:160-201 + mat_get_row mv_ops.c:99-113) bit for
 * bit on "chained" matrices (ascending columns, no empty row,
 * first_col(r+1) <= last_col(r)); see oracle_spmv_dense_expand for the literal
 * O(n^2) restatement.  Returns 0. */
int oracle_spmv_csr(int n, const int *row_ptr, const int *col, const double *val,
                    const double *x, double *y);

/* Literal restatement of mv_mult + mat_get_row (mv_ops.c:99-113, :160-201):
 * expands each row into a dense n-vector by the greedy scan starting at
 * row_ptr[row] (it never looks at row_ptr[row+1]), then a dense sequential
 * dot.  O(n^2).  nnz bounds the scan (the reference reads the zero tail of
 * its 18,020,000-entry calloc'd column buffer, cg.c:235-247, which behaves
 * as "no further match" for i > 0). */
int oracle_spmv_dense_expand(int n, int nnz, const int *row_ptr, const int *col,
                             const double *val, const double *x, double *y);

/* Sequential dot product from 0.0 (mv_ops.c:117-132). */
double oracle_dot(int n, const double *a, const double *b);

/* r = s*a (mv_ops.c:134-158), r = a+b (mv_ops.c:203-230), r = a-b
 * (mv_ops.c:232-259).  r may alias a or b. */
void oracle_scale(int n, double s, const double *a, double *r);
void oracle_add(int n, const double *a, const double *b, double *r);
void oracle_sub(int n, const double *a, const double *b, double *r);

/* conj_grad (cg.c:88-141): Hestenes-Stiefel CG, x0 = 0, max_iter+1 SpMVs,
 * break after the r-update when k == max_iter.  dense_expand != 0 uses the
 * literal O(n^2) mv_mult restatement; 0 uses oracle_spmv_csr.
 * rr_hist (optional, length >= max_iter+1) receives r.r after each r-update.
 * Returns the number of SpMVs performed (max_iter+1). */
int oracle_conj_grad(int max_iter, int n, int nnz, const int *row_ptr,
                     const int *col, const double *val, const double *b,
                     double *x, int dense_expand, double *rr_hist);

/* solve(A,b,x,tol,maxit) -- the north-star superset of conj_grad: same
 * recurrences; additionally stops after the r-update when
 * sqrt(r.r) <= tol*sqrt(b.b).  tol <= 0 is exactly conj_grad(maxit).
 * Returns the number of SpMVs performed (k+1). */
int oracle_solve(int maxit, double tol, int n, const int *row_ptr,
                 const int *col, const double *val, const double *b, double *x,
                 double *rr_hist);

/* Chronopoulos-Gear single-reduction CG (the multi-GPU recurrence), same
 * stopping rule as oracle_solve.  Mathematically equal to HS-CG, differs at
 * rounding level.  Used to check the partitioned solver within tolerance. */
int oracle_solve_cg1(int maxit, double tol, int n, const int *row_ptr,
                     const int *col, const double *val, const double *b,
                     double *x, double *rr_hist);

/* The single-reduction HS variant (CGX_ALG_SR): alpha as cg.c:113, beta
 * from alpha^2 s.s - r.r; the stop test on the exact r.r, the same stopping
 * rule as oracle_solve.  Rounding-level different from it. */
int oracle_solve_sr(int maxit, double tol, int n, const int *row_ptr,
                    const int *col, const double *val, const double *b,
                    double *x, double *rr_hist);

/* Same CSR SpMV with fp32 values and vectors, fp32 products and row sums
 * (the C5 fp32 configuration; the reference itself is fp64 only,
 * mv_ops.h:20). */
int oracle_spmv_csr_f32(int n, const int *row_ptr, const int *col,
                        const float *val, const float *x, float *y);

/* C5's HS-CG in fp32 (cg.c:88-141 with float matrix and vectors, as libcgx
 * runs it): float products and row sums in the SpMV, dot products as
 * sequential sums of the exact double products, alpha / beta in double
 * rounded once to float, float vector updates with two roundings each.
 * Same stopping rule as oracle_solve.  Returns SpMVs performed. */
int oracle_solve_f32(int maxit, double tol, int n, const int *row_ptr,
                     const int *col, const float *val, const float *b,
                     float *x, double *rr_hist);

/* Multithreaded CSR SpMV + HS-CG on `threads` host threads (pthreads) --
 * the "all host cores" CPU baseline mode of BASELINE.md.  Per-row sums are
 * sequential (bit-exact SpMV); dot products are reduced per thread chunk in
 * fixed order.  Returns SpMVs performed. */
int oracle_solve_mt(int maxit, double tol, int n, const int *row_ptr,
                    const int *col, const double *val, const double *b,
                    double *x, int threads);

#ifdef __cplusplus
}
#endif
#endif
