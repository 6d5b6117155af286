/* mv_ops.h -- drop-in replacement header for the reference's mv_ops.h
 * (rnelias/Conjugate-Gradient mv_ops.h:17-42), served by libcgx.so.
 *
 * Same struct, same 11 prototypes, same out-parameter and error conventions,
 * so cg.c-style callers (cg.c:42-85 main, cg.c:358-387 test_mv_ops) compile
 * and link against libcgx.so unchanged.  The arithmetic runs on the MI355X
 * (HIP kernels in conjugate-gradient_amd/csrc/); the struct always carries
 * HOST pointers -- device buffers are owned by libcgx and never exposed here.
 *
 * Semantics kept from the reference (file:line of the function each replaces):
 *   new_mv_struct            mv_ops.c:14-21   calloc'd shell
 *   new_mv_struct_with_size  mv_ops.c:23-37   n zeroed doubles, nnz = size
 *   free_mv_struct           mv_ops.c:39-42   frees the SHELL ONLY (arrays are
 *                                             not freed, as in the reference;
 *                                             cgx_free_mv_deep frees both)
 *   mv_deep_copy             mv_ops.c:44-74
 *   print_sparse             mv_ops.c:77-95   same stdout format
 *   mat_get_row              mv_ops.c:99-113  dense row expansion (see below)
 *   dot_product              mv_ops.c:117-132 returns -1.0 on NULL / size mismatch
 *   sv_mult                  mv_ops.c:134-158 r = s*a, allocate-or-realloc *r
 *   mv_mult                  mv_ops.c:160-201 r = A*b, allocate-or-realloc+zero *r
 *   vec_add / vec_sub        mv_ops.c:203-259 r = a +/- b, aliasing allowed
 * int functions return 0 on success and -1 on NULL or size mismatch; libcgx
 * additionally returns -2 when the GPU is unavailable or a HIP call fails
 * (cgx_last_error() says why).
 *
 * Numerics: mv_mult sums each row sequentially in column order from 0.0 with
 * separately rounded products (bit-identical to the reference on chained
 * matrices: ascending columns, no empty row, first_col(r+1) <= last_col(r)).
 * mat_get_row expands a row correctly from [row_ptr[r], row_ptr[r+1]); the
 * reference's greedy scan past row_ptr[r+1] is not reproduced.
 * dot_product in libcgx is a parallel two-stage reduction by default; after
 * cgx_ops_set_mode(CGX_MODE_EXACT, CGX_ALG_HS) (cgx.h) it is the reference's
 * sequential sum.  The library reads no configuration from outside the API.
 */
#ifndef CGX_MV_OPS_H
#define CGX_MV_OPS_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

/* mv_ops.h:17-23 -- a CSR matrix, or a dense vector when
 * col_indices == row_ptr == NULL and nnz == size.  LP64 layout: offsets
 * 0/4/8/16/24, sizeof 32. */
struct __mv_sparse {
  int size;
  int nnz;
  double *values;
  int *col_indices;
  int *row_ptr;
};

struct __mv_sparse *new_mv_struct();
struct __mv_sparse *new_mv_struct_with_size(int);
void free_mv_struct(struct __mv_sparse *);
struct __mv_sparse *mv_deep_copy(struct __mv_sparse *);

void print_sparse(struct __mv_sparse *);

int mat_get_row(struct __mv_sparse *, int, double *);

double dot_product(struct __mv_sparse *, struct __mv_sparse *);
int sv_mult(double, struct __mv_sparse *, struct __mv_sparse **);
int mv_mult(struct __mv_sparse *, struct __mv_sparse *, struct __mv_sparse **);
int vec_add(struct __mv_sparse *, struct __mv_sparse *, struct __mv_sparse **);
int vec_sub(struct __mv_sparse *, struct __mv_sparse *, struct __mv_sparse **);

#ifdef __cplusplus
}
#endif
#endif /* CGX_MV_OPS_H */
