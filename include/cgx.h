/* cgx.h -- C ABI of libcgx.so, the MI355X-native (gfx950) Conjugate-Gradient
 * solver that drops in for rnelias/Conjugate-Gradient's hot path
 * (cg.c:88-141 conj_grad + mv_ops.c:117-259).
 *
 * Plain C types only (pointers + sizes); every pointer argument is a HOST
 * pointer unless the name says otherwise.  All int-returning calls return
 * >= 0 on success and < 0 on failure; cgx_last_error() describes the last
 * failure of the calling thread.  There is no CPU fallback: without a usable
 * gfx950 device every compute call fails with CGX_ENODEV.
 */
#ifndef CGX_H
#define CGX_H

#include <stddef.h>
#include "mv_ops.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CGX_EINVAL  (-1) /* NULL argument or size mismatch (reference convention) */
#define CGX_ENODEV  (-2) /* no GPU / HIP failure                                  */
#define CGX_ENOMEM  (-3) /* device or host allocation failed                       */
#define CGX_ECOMM   (-4) /* RCCL failure                                          */

/* ------------------------------------------------------------------------
 * 1. Reference-compatible solver entry points
 * ------------------------------------------------------------------------ */

/* Replaces cg.c:88-141 (declared only at cg.c:24 in the reference).
 * Hestenes-Stiefel CG from x0 = 0, exactly max_iter+1 SpMVs, no tolerance;
 * *vec_x receives a freshly allocated host vector (any previous *vec_x is
 * ignored, as in the reference, cg.c:104,138).  Returns 0 (the reference
 * always returns 0) or < 0 on a device/argument failure.
 * Numerics and device: cgx_ops_set_mode / cgx_ops_set_device below. */
int conj_grad(int max_iter, struct __mv_sparse *mat_A,
              struct __mv_sparse *vec_b, struct __mv_sparse **vec_x);

/* The north-star entry point (BASELINE.json): a superset of conj_grad.
 * Same recurrences; stops after the r-update (the cg.c:125 position) when
 * k == maxit or r.r <= tol*tol*b.b.  tol <= 0 is exactly conj_grad(maxit).
 * Returns the number of x-updates performed (k+1 SpMVs), or < 0. */
int solve(const struct __mv_sparse *A, const struct __mv_sparse *b,
          struct __mv_sparse **x, double tol, int maxit);

/* Frees a struct and its arrays (the reference's free_mv_struct frees only
 * the shell, mv_ops.c:39-42, which libcgx keeps for drop-in safety). */
void cgx_free_mv_deep(struct __mv_sparse *m);

/* Numerics of the reference-compatible entry points (conj_grad, solve and
 * the mv_ops.h arithmetic), process-wide; the library is configured only
 * through these calls.
 *   mode CGX_MODE_FAST (default): two-stage parallel reductions, x within
 *        fp64 rounding of the reference (tests: 1e-12 relative)
 *   mode CGX_MODE_EXACT: the reference's sequential dot-product order, x
 *        bit-identical to cg.c on chained matrices (HS only)
 *   alg  CGX_ALG_HS (the reference recurrence, default), CGX_ALG_CG1, or
 *        CGX_ALG_SR (fast mode only: one reduction per iteration -- ONE
 *        launch where the matrix takes the plane-marched DIA step, the
 *        bench's N = 1 recurrence; two launches on any other matrix;
 *        cgx_ops_last_timing().alg reports what ran)
 * The drop-in CLI maps CGX_MODE=exact / CGX_ALG=cg1|sr onto this call. */
int cgx_ops_set_mode(int mode, int alg);
/* GPU of those entry points (default 0); before their first call only. */
int cgx_ops_set_device(int device);

/* Wall-clock split of the last conj_grad / solve call (what cg.c:71-75
 * times around conj_grad): setup = upload and layout encoding when A was
 * not resident (uploaded = 1) + hash_ms, the time spent waiting for the
 * content hash of A (it overlaps the device work when A is resident);
 * solve = device iterations incl. the rhs copy; download = x to the host. */
typedef struct {
  double total_ms, setup_ms, hash_ms, solve_ms, download_ms;
  int uploaded, iters;
  int breakdown;  /* as cgx_info.breakdown, for the last conj_grad / solve */
  int alg;        /* CGX_ALG_* that ran                                  */
} cgx_ops_timing;
int cgx_ops_last_timing(cgx_ops_timing *t);

/* Matrix residency of the mv_ops.h / conj_grad / solve entry points: the
 * last matrix stays on the device, keyed by the struct's array pointers and
 * sizes, and checked against a 64-bit content hash of row_ptr, col_indices
 * and values.  A call with the same struct starts on the resident matrix at
 * once while the hash runs on host threads beside the device work; if A was
 * edited in place since its upload the hash differs, A is uploaded again
 * and the call redone -- the result is always that of the A passed in.  A
 * cg.c caller linked at the op level (cg.c:111 -> mv_mult) thus uploads A
 * once, not once per iteration.
 * Counts since process start: uploads performed, reuses. */
int cgx_ops_counters(long long *uploads, long long *reuses);

const char *cgx_last_error(void);
int cgx_device_count(void);
/* Waits for all work on `device` (the solver's streams included). */
int cgx_device_synchronize(int device);
/* The HIP runtime the library runs on (hipRuntimeGetVersion), the HIP it
 * was compiled against (HIP_VERSION) and the RCCL it calls (ncclGetVersion).
 * A process that loads an older ROCm's libamdhip64.so.7 / librccl.so.1
 * before this library (PyTorch's bundled copies, `import torch` first) binds
 * the library to those: report, so a caller can tell. */
int cgx_runtime_versions(int *hip_runtime, int *hip_compiled, int *rccl);

/* On-box HBM ceilings (SURVEY.md 8d "STREAM-triad ceiling"), fp64 arrays of
 * n elements on `device`, best of `reps` timed launches, 16 B per lane:
 *   CGX_STREAM_TRIAD  a[i] = b[i] + s*c[i]      *gbs = 24 n B / time
 *   CGX_STREAM_READ   sum of a[i] (read only)   *gbs =  8 n B / time
 * and tuned read/write mixes (4 x 16 B per lane in flight before the first
 * store, grid = resident workgroup slots, grid-stride; _NT: non-temporal
 * stores), *gbs = (R + W) 8 n B / time:
 *   CGX_STREAM_COPY[_NT]         R = 1, W = 1 (a = b)
 *   CGX_STREAM_TRIAD_TUNED / _NT R = 2, W = 1 (a = b + s c)
 *   CGX_STREAM_MIX33[_NT]        R = 3, W = 3 (the one-launch SR step's
 *                                r, p, s read and written)
 * Measurement only (bench.py's roofline context). */
#define CGX_STREAM_TRIAD 0
#define CGX_STREAM_READ 1
#define CGX_STREAM_COPY 2
#define CGX_STREAM_COPY_NT 3
#define CGX_STREAM_TRIAD_TUNED 4
#define CGX_STREAM_TRIAD_NT 5
#define CGX_STREAM_MIX33 6
#define CGX_STREAM_MIX33_NT 7
int cgx_stream_bench(int device, int kind, long long n, int reps, double *gbs);

/* ------------------------------------------------------------------------
 * 2. Solver object: device-resident CSR, repeated solves, benchmarking
 * ------------------------------------------------------------------------ */

typedef struct cgx_solver cgx_solver;

enum { CGX_MODE_FAST = 0,    /* two-stage parallel reductions (default)      */
       CGX_MODE_EXACT = 1 }; /* sequential dots: reference bit order          */
enum { CGX_ALG_HS = 0,       /* Hestenes-Stiefel, the reference recurrence    */
       CGX_ALG_CG1 = 1,      /* Chronopoulos-Gear, one fused reduction/iter   */
       CGX_ALG_SR = 2 };     /* HS with one reduction/iter: one launch per
                                iteration where the plane-marched DIA step
                                applies (cgx_solver_set_march), else the SpMV
                                + one vector launch; ranks alike           */
enum { CGX_F64 = 0, CGX_F32 = 1 };

/* Device layout of the matrix the SpMV streams (the C ABI always takes the
 * reference's CSR; only the chosen layout's arrays are resident -- DIA keeps
 * just its per-row codes and value tables, and cgx_solver_get_matrix decodes
 * them back to CSR):
 *   AUTO     DIA where it applies, else DC, else CSR (PANEL for gathers with
 *            no locality, e.g. random SPD)                       (default)
 *   CSR      plain CSR, int32 columns: SURVEY.md 8d's B_spmv layout
 *   DC       dictionary-coded columns: <= 256 distinct col - row offsets,
 *            one code byte per nonzero + the value stream, rows <= 255
 *   DIA      value-indexed diagonal codes: nonzeros on <= 16 diagonals
 *            (col - row) with <= 15 distinct values each, every row's
 *            columns ascending; a 1-4 bit field per (row, diagonal) names
 *            the entry's value or "no entry" (a Laplacian: one byte per
 *            row) -- no column or value stream
 *            (stencils, banded matrices with few coefficients); on one
 *            GPU (and in a partition's one-launch SR matrix), values no
 *            table indexes on <= 8 diagonals are DIA-V: a presence bit per
 *            (row, diagonal) and the values streamed
 *            (cgx_info.dia_value_stream) when that is no more bytes than DC
 *   PANEL    CSR split into column panels (one SpMV pass per panel)
 *   STENCIL  matrix-free Laplacian (cgx_solver_set_stencil; info only)
 * A requested layout that does not apply falls back DIA -> DC -> CSR;
 * cgx_info.layout says which one runs.  Every layout sums each row in the
 * reference's order: y is bit-identical across layouts. */
enum { CGX_LAYOUT_AUTO = 0, CGX_LAYOUT_CSR = 1, CGX_LAYOUT_DC = 2, CGX_LAYOUT_DIA = 3,
       CGX_LAYOUT_PANEL = 4, CGX_LAYOUT_STENCIL = 5 };

typedef struct {
  int n, nnz, dtype, mode, alg;
  int layout;           /* CGX_LAYOUT_* the SpMV runs on                     */
  int n_items;          /* SpMV work items: 64-row blocks (CSR/DC/PANEL) or
                           512-row slices (DIA, STENCIL)                     */
  int spmv_grid;        /* workgroups of one SpMV launch (= its partials)    */
  int vec_grid;         /* 256-thread units of the vector-update launches    */
  double spmv_bytes;    /* algorithmic HBM bytes per SpMV, CSR basis
                           (SURVEY.md 8d B_spmv)                             */
  double iter_bytes;    /* algorithmic HBM bytes per CG iteration (8d)       */
  double spmv_iter_bytes; /* algorithmic bytes of one SpMV in the layout it
                             runs on (DIA: codes + x + y; DC: codes + values
                             + row lengths + x + y; PANEL: + P row_ptrs and
                             y round trips; fused HS step, average of its
                             two launch parities: + r, p_old read, p_new
                             written, x / p_{k-1} read and x written
                             every other launch: + 3.5 n vectors)                                 */
  size_t device_bytes;  /* device memory held by the solver                  */
  int n_panels;         /* column panels of the SpMV (1: none)               */
  int n_dict;           /* DC: distinct col - row offsets; DIA: diagonals;
                           0 otherwise                                      */
  int tile_bands;       /* L2-tiled item order: bands of the widest offset's
                           period swept one after another (0: natural)      */
  int nt;               /* 1: matrix stream and y store non-temporal        */
  int code_bytes_per_row; /* DIA: 1, 2, 4 or 8 (packed value-index fields)  */
  int encode_fallback;  /* 1: the sampled candidates missed one; an exact
                           host scan was needed                             */
  double setup_host_ms;   /* set_matrix: host time (checks, plan, submit)    */
  double setup_device_ms; /* set_matrix: device time after the last submit  */
  int n_values;         /* DIA: values over all diagonal tables             */
  int gathers_per_chunk; /* CSR / DC: x gathers issued per row chunk (7|8)  */
  int fused;            /* 1: the iteration runs fused (cgx_solver_set_fused) */
  int fuse_status;      /* CGX_FUSE_STATUS_*: why the fused step does or does
                           not run for the loaded matrix and settings       */
  int breakdown;        /* after a run: 1 + the first iteration whose p.s (HS)
                           or CG1 step denominator was <= 0 or not finite --
                           the point where the reference's iteration turns to
                           NaN (cg.c:113, 129) -- or 0.  Diagnostic only: the
                           iteration itself keeps the reference's IEEE
                           semantics (failure detection)        */
  int fuse_march;       /* > 0: the fused HS / SR step runs as a plane
                           march (cgx_solver_set_march), this many steps per
                           workgroup (the longest segment); 0: it does not  */
  int dia_value_stream; /* DIA: 1 = DIA-V, the values streamed per (row,
                           diagonal) beside one presence byte per row (one
                           GPU, general coefficients on <= 8 diagonals);
                           0 = DIA-VI (value-indexed codes, no value stream) */
} cgx_info;

/* cgx_info.fuse_status / cgx_dist_stats.fuse_status */
enum { CGX_FUSE_STATUS_RUNS = 0,        /* the fused step runs                   */
       CGX_FUSE_STATUS_OFF = 1,         /* CGX_FUSE_OFF requested                */
       CGX_FUSE_STATUS_NOT_DIA = 2,     /* the layout is not DIA                 */
       CGX_FUSE_STATUS_WIDE_CODES = 3,  /* DIA row words of 8 bytes (> 4)        */
       CGX_FUSE_STATUS_FAR_DIAGS = 4,   /* more than 4 diagonals with |d| > 1024
                                           (e.g. a slab not starting on a plane) */
       CGX_FUSE_STATUS_CACHED = 5,      /* AUTO: the working set fits the
                                           Infinity Cache (faster unfused)       */
       CGX_FUSE_STATUS_EXACT = 6,       /* exact mode runs the reference's order */
       CGX_FUSE_STATUS_PEER = 7,        /* partitioned: another rank's layout
                                           refused (all ranks or none)           */
       CGX_FUSE_STATUS_CG1_AUTO = 8,    /* partitioned CG1: fused only when
                                           forced on (slower on a rank's slab)   */
       CGX_FUSE_STATUS_NO_MARCH = 9,    /* CGX_ALG_SR on one GPU: the matrix has
                                           no plane-march plan, or
                                           cgx_solver_set_march(0)               */
       CGX_FUSE_STATUS_VALUE_STREAM = 10 }; /* DIA-V (cgx_info.dia_value_stream):
                                           only the one-launch SR step fuses;
                                           HS / CG1 run unfused                  */

int  cgx_solver_create(int device, cgx_solver **out);
void cgx_solver_destroy(cgx_solver *s);
int  cgx_solver_set_mode(cgx_solver *s, int mode, int alg);
/* The HS iteration in fast mode on a DIA layout (<= 4-byte row words, <= 4
 * diagonals with |d| > 1024) can fuse the vector update into the SpMV: one
 * launch does the previous iteration's p = r + beta p (cg.c:131-132) -- p of
 * its rows and their in-plane halo computed once into an LDS window -- then
 * s = A p; the next launch updates r (cg.c:118-123).  x += alpha p
 * (cg.c:115-116) runs every other launch for two iterations (same roundings,
 * in order).  Two launches per iteration instead of three, 12 B per row less
 * traffic; x and the r.r history are bit-identical to the unfused path.
 * mode: CGX_FUSE_OFF, CGX_FUSE_AUTO (default: where the layout takes it and
 * the working set exceeds the 256 MiB Infinity Cache -- cache-resident
 * systems are latency-bound and run faster unfused), CGX_FUSE_ON (wherever
 * the layout takes it). */
#define CGX_FUSE_OFF  0
#define CGX_FUSE_AUTO 1
#define CGX_FUSE_ON   2
int  cgx_solver_set_fused(cgx_solver *s, int mode);
/* The fused HS step as a plane march: where every diagonal with |d| > 1024 is
 * +F or -F and F lies within the in-plane halo of a multiple of 512 rows (a
 * 3-D stencil's +-nx*ny planes: C3, C4), a workgroup walks a chain of slices
 * F apart, keeping p of three consecutive slices (and their halos) in LDS, so
 * the +-F neighbours are read from LDS instead of recomputed from r / p
 * gathers.  Same values, same order: x and the r.r history are bit-identical
 * to the unfused path.  steps: -1 auto (default; HS: about 2,048 workgroups
 * per launch; CGX_ALG_SR's k_sr1_dia_m: each chain cut into the balanced
 * segment count that fills the device's resident workgroup slots), 0 off
 * (the per-slice fused kernel), > 0 slices of a chain per workgroup.
 * cgx_info.fuse_march reports what runs. */
int  cgx_solver_set_march(cgx_solver *s, int steps);
/* CGX_ALG_SR's one-launch plane march (k_sr1_dia_m): the width, in rows, of
 * the chains a step of the march is cut into.  0 auto (default): the width
 * and segment count whose chains x segments fill the device's resident
 * workgroup slots best; > 0 that width, the segment count still picked.
 * The width is made even and clamped to [128, 2,048] rows, and then to the
 * widest step that has a kernel for the matrix (1,024 rows on DIA-V, which
 * has no four-slice step; likewise when a wide halo rules four slices out).  Results do not depend on it beyond the grouping of the partial
 * sums (tolerance, as every SR launch shape). */
int  cgx_solver_set_sr_chain(cgx_solver *s, int rows);
/* Layout for the next set_matrix / gen_laplacian (CGX_LAYOUT_AUTO..PANEL). */
int  cgx_solver_set_layout(cgx_solver *s, int layout);
/* Host CSR (int32 row_ptr[n+1], col[nnz]; values f64 or f32) -> device.
 * Columns must be ascending within each row for bit-exact SpMV order. */
int  cgx_solver_set_matrix(cgx_solver *s, int n, int nnz, const int *row_ptr,
                           const int *col, const double *val);
int  cgx_solver_set_matrix_f32(cgx_solver *s, int n, int nnz,
                               const int *row_ptr, const int *col,
                               const float *val);

/* SURVEY.md 8f, on-device generators and the matrix-free stencil.  The
 * 5-point 2-D (dim 2; nz ignored) / 7-point 3-D Laplacian of an nx*ny*nz
 * grid, natural ordering -- the matrix of cgx_gen_laplacian2d/3d:
 *   gen_laplacian  fp64 CSR written straight into device memory (no host
 *                  arrays, no PCIe copy of col/val); row_ptr in closed form
 *   set_stencil    matrix-free operator: same rows, same column order, same
 *                  products, so the SpMV is bit-identical to the CSR one and
 *                  its CG an upper bound for the CSR runs (x and y only)
 *   get_matrix     the device CSR back to host arrays (plain fp64 CSR only)
 *   cgx_laplacian_row_ptr  the closed-form row_ptr of rows [row_begin,
 *                  row_end) (host; returns their nnz, or < 0) */
int  cgx_solver_gen_laplacian(cgx_solver *s, int dim, int nx, int ny, int nz);
int  cgx_solver_set_stencil(cgx_solver *s, int dim, int nx, int ny, int nz);
int  cgx_solver_get_matrix(cgx_solver *s, int *row_ptr, int *col, double *val);
long long cgx_laplacian_row_ptr(int dim, int nx, int ny, int nz, int row_begin,
                                int row_end, int *row_ptr);
/* Right-hand side, length n, in the matrix's dtype. */
int  cgx_solver_set_rhs(cgx_solver *s, const double *b);
int  cgx_solver_set_rhs_f32(cgx_solver *s, const float *b);
/* x0 = 0; stop rule as solve().  *iters = x-updates performed. */
int  cgx_solver_run(cgx_solver *s, int maxit, double tol, int *iters);
int  cgx_solver_get_x(cgx_solver *s, double *x);
int  cgx_solver_get_x_f32(cgx_solver *s, float *x);
/* r.r after each x-update of the last run (length >= iters). */
int  cgx_solver_get_history(cgx_solver *s, double *rr, int cap);
/* One y = A x with the loaded matrix (op-level parity). */
int  cgx_solver_spmv(cgx_solver *s, const double *x, double *y);
int  cgx_solver_spmv_f32(cgx_solver *s, const float *x, float *y);
int  cgx_solver_info(cgx_solver *s, cgx_info *info);

/* Benchmark hooks.  cgx_solver_bench_prepare: x0 = 0 prologue plus `warmup`
 * untimed CG iterations (tol = 0, no iteration limit), then a device sync.
 * cgx_solver_bench_run: `iters` further iterations of the same recurrence,
 * timed with HIP events on the solver's stream; returns after they finished.
 * flags & CGX_BENCH_GRAPH: replay the iteration loop as hipGraphs.
 * flags & CGX_BENCH_SPMV_EVENTS: also bracket every SpMV launch with events
 *   and report its average duration in *spmv_ms (else *spmv_ms = -1).
 * flags & CGX_BENCH_SPMV_ONLY: `iters` back-to-back SpMVs y = A p instead of
 *   CG iterations (the standard SpMV benchmark; the iteration state is not
 *   touched).
 * cgx_solver_bench = prepare + run. */
#define CGX_BENCH_GRAPH        1
#define CGX_BENCH_SPMV_EVENTS  2
#define CGX_BENCH_SPMV_ONLY    4
int  cgx_solver_bench_prepare(cgx_solver *s, int warmup);
int  cgx_solver_bench_run(cgx_solver *s, int iters, int flags, double *total_ms,
                          double *spmv_ms);
int  cgx_solver_bench(cgx_solver *s, int warmup, int iters, int flags,
                      double *total_ms, double *spmv_ms);

/* ------------------------------------------------------------------------
 * 3. Synthetic SPD generators (host, row range [row_begin, row_end))
 *    Two-pass: call with row_ptr == NULL to get the nnz of the range, then
 *    with arrays of that size.  row_ptr is local (starts at 0); columns are
 *    global indices.  Return nnz or < 0.
 * ------------------------------------------------------------------------ */
long long cgx_gen_laplacian2d(int nx, int ny, int row_begin, int row_end,
                              int *row_ptr, int *col, double *val);
long long cgx_gen_laplacian3d(int nx, int ny, int nz, int row_begin,
                              int row_end, int *row_ptr, int *col, double *val);
/* Random SPD: tridiagonal band + `partners` random partner columns per row
 * from a splitmix64 stream (seed), symmetrised, off-diagonals -U(0,1],
 * diagonal = sum|offdiag| + 1.  Values written as f32 when val32 != NULL. */
long long cgx_gen_random_spd(int n, int partners, unsigned long long seed,
                             int row_begin, int row_end, int *row_ptr,
                             int *col, double *val, float *val32);
/* The 7-point pattern of cgx_gen_laplacian3d with one random coefficient per
 * grid edge, a_ij = a_ji = -(0.5 + U(0,1]) from a splitmix64 hash of the
 * pair (seed), diagonal = sum |a_ij| + 0.01: SPD, every off-diagonal value
 * distinct -- the general-coefficient CSR case at a stencil's shape. */
long long cgx_gen_varcoef3d(int nx, int ny, int nz, unsigned long long seed,
                            int row_begin, int row_end, int *row_ptr, int *col,
                            double *val);
/* Reader for the reference's 4-line input format (replaces read_input_file,
 * cg.c:23,146-218): col_indices / row_ptr / values / b, comma separated.
 * Fills *A (CSR) and *b (vector) with freshly allocated host arrays.
 * Re-entrant, bounds-safe, accepts a missing final newline.  0 or -1. */
int cgx_read_input_file(const char *path, struct __mv_sparse *A,
                        struct __mv_sparse *b);
/* The same with a binary cache at cache_path, keyed on the text's size and
 * a 64-bit hash of its whole content: when they match, the text is hashed
 * but not parsed; otherwise it is parsed and the cache (re)written (best
 * effort: an unwritable cache_path only costs the next parse).  *from_cache
 * (may be NULL) = 1 when the cache was used.  0 or -1. */
int cgx_read_input_cached(const char *path, const char *cache_path,
                          struct __mv_sparse *A, struct __mv_sparse *b,
                          int *from_cache);

/* 1 if the CSR is "chained" (ascending cols, no empty row,
 * first_col(r+1) <= last_col(r)): the class on which the reference's
 * dense-row mv_mult equals CSR SpMV. */
int cgx_csr_is_chained(int n, const int *row_ptr, const int *col);

/* ------------------------------------------------------------------------
 * 4. Row partition layer (host only, no GPU)
 *    rank g of G owns rows [floor(g*n/G), floor((g+1)*n/G)); its local
 *    columns are owned rows -> [0, n_loc) and ghosts -> n_loc + position in
 *    the ghost list (sorted by global index, hence grouped by owner rank).
 * ------------------------------------------------------------------------ */
void cgx_partition_rows(long long n, int nranks, int rank, int *row_begin,
                        int *row_end);
int  cgx_partition_owner(long long n, int nranks, long long col);

typedef struct cgx_part cgx_part;
/* row_ptr (n_loc+1, local) and col_global (nnz) describe this rank's rows. */
int  cgx_part_create(long long n_global, int nranks, int rank, int n_loc,
                     int nnz, const int *row_ptr, const int *col_global,
                     cgx_part **out);
void cgx_part_destroy(cgx_part *p);
int  cgx_part_info(const cgx_part *p, int *n_loc, int *n_ghost,
                   int *row_begin, int *n_send);
int  cgx_part_local_cols(const cgx_part *p, int *col_local);   /* nnz     */
int  cgx_part_ghosts(const cgx_part *p, int *ghost_global);    /* n_ghost */
int  cgx_part_recv_counts(const cgx_part *p, int *counts);     /* nranks  */
/* Requests received from every rank (counts[nranks]; global row indices
 * concatenated by rank) -> this rank's halo send lists. */
int  cgx_part_set_requests(cgx_part *p, const int *req_counts,
                           const int *req_global);
int  cgx_part_send_counts(const cgx_part *p, int *counts);     /* nranks  */
int  cgx_part_send_local(const cgx_part *p, int *send_local);  /* n_send  */

/* ------------------------------------------------------------------------
 * 5. Multi-GPU solver: one rank per GPU, rows partitioned in contiguous
 *    blocks, halo x segments exchanged point to point (ncclSend/Recv on a
 *    high-priority stream, overlapped with the interior SpMV), dot products
 *    all-reduced over RCCL; batches of iterations replayed as hipGraphs.
 *    Stop rule as solve(); x0 = 0; every rank passes its own rows.
 * ------------------------------------------------------------------------ */
typedef struct cgx_dist cgx_dist;
typedef struct {
  long long n_global;
  int row_begin, n_loc, n_ghost, n_send, nnz;
  int interior_items, boundary_items;    /* SpMV work items (cgx_info)    */
  double spmv_bytes, iter_bytes;         /* algorithmic, CSR basis, rank  */
  double halo_bytes;                     /* sent + received per iteration */
  size_t device_bytes;
  double spmv_iter_bytes;                /* algorithmic bytes of the SpMV in
                                            the layout it runs on         */
  int layout;                            /* CGX_LAYOUT_* of the local rows */
  int n_dict;                            /* as cgx_info                   */
  int graph;                             /* 1 iterations replayed as a
                                            hipGraph, 0 not (yet), -1 the
                                            capture failed: eager        */
  int alg;                               /* CGX_ALG_* in use              */
  int fused;                             /* 1: the fused HS step runs (set
                                            once the ranks are connected) */
  int fuse_status;                       /* CGX_FUSE_STATUS_* (cgx_info)  */
  int breakdown;                         /* as cgx_info.breakdown         */
  int march;                             /* > 0: CGX_ALG_SR runs as ONE
                                            k_sr1_dia_m step per iteration
                                            (+ k_sr1_edge after the halo),
                                            this many steps per workgroup
                                            (the longest segment); 0: it
                                            does not                      */
  int inplace;                           /* 1: this rank's rows have the
                                            in-place ghost numbering the
                                            one-launch SR step needs      */
} cgx_dist_stats;

/* Rank 0 creates the id and distributes it (e.g. torch.distributed). */
int  cgx_dist_unique_id(unsigned char id[128]);
/* nranks == 1 needs no id and no communication. */
int  cgx_dist_create(int device, int nranks, int rank,
                     const unsigned char id[128], cgx_dist **out);
/* In-process transport: nparts partitions on one device driven by one host
 * thread (device copies for the halo, fixed-order sum for the all-reduce).
 * Run/bench through parts[0]; destroy through parts[0]. */
int  cgx_dist_create_local(int device, int nparts, cgx_dist **parts);
void cgx_dist_destroy(cgx_dist *d);
/* Layout of the local rows for the next set_matrix (AUTO, CSR, DC, DIA). */
int  cgx_dist_set_layout(cgx_dist *d, int layout);
int  cgx_dist_set_matrix(cgx_dist *d, long long n_global, int n_loc, int nnz,
                         const int *row_ptr, const int *col_global,
                         const double *val);
int  cgx_dist_set_rhs(cgx_dist *d, const double *b_local);
/* Recurrence: CGX_ALG_HS (default; the reference's cg.c:88-141 recurrence:
 * two all-reduces of one double per iteration, bit-identical to the
 * single-GPU solver at one rank), CGX_ALG_CG1 (Chronopoulos-Gear: ONE
 * all-reduce of two doubles, 8 bytes per row more vector traffic) or
 * CGX_ALG_SR (the HS recurrence with ONE all-reduce of three doubles and HS's
 * bytes: p.s, s.s and the exact r.r of the last r update are reduced
 * together; alpha = r.r / p.s as in cg.c:113, while beta (cg.c:129) and the
 * stop test use r_new.r_new = alpha^2 s.s - r.r, exact in exact arithmetic
 * since r.s = p.s; rounding-level different from HS, tolerance parity.
 * Needs the fused DIA step on every partition: run / bench_prepare return
 * CGX_EINVAL otherwise).  Every rank (every part of a local group) must use
 * the same one; on a local group, setting it on part 0 sets the group. */
int  cgx_dist_set_alg(cgx_dist *d, int alg);
/* The fused HS step (cgx_solver_set_fused modes) on all ranks or none --
 * agreed collectively at the next run / bench_prepare: the halo carries
 * p_new = r + beta p_old computed at the send rows, the interior and
 * boundary k_spmv_dia_h launches replace k_xpay_xf + the SpMV; x and the
 * history are bit-identical to the unfused path.  Call on every rank (on a
 * local group, part 0 sets the group). */
int  cgx_dist_set_fused(cgx_dist *d, int mode);
/* CGX_ALG_SR as ONE launch pair per iteration (the single-GPU k_sr1_dia_m
 * step: the r update of the previous iteration, p, x and s = A p in one plane
 * march) where every rank's ghost columns are the rows next to its own
 * (a banded matrix cut into row slabs, e.g. C4's planes): the ranks number
 * their rows in place (columns = global - row_begin, the neighbours' planes
 * below 0 and from n_loc), march every step while the halo of
 * p_k = (r - alpha s) + beta p is in flight, and recompute s of the edge rows
 * (those reaching a ghost column) after it.  steps: -1 auto (default: the
 * balanced segment count for the device), 0 off (the two-launch fused SR
 * step), > 0 steps per workgroup segment.  cgx_dist_stats.march reports it.
 * Call on every rank (on a local group, part 0 sets the group). */
int  cgx_dist_set_march(cgx_dist *d, int steps);
/* As cgx_solver_set_sr_chain, for the ranks' one-launch SR step.  Call on
 * every rank (on a local group, part 0 sets the group). */
int  cgx_dist_set_sr_chain(cgx_dist *d, int rows);
/* hipGraph replay of the iteration batches (RCCL calls included); on by
 * default; 0 runs every iteration eagerly.  Resets a failed capture. */
int  cgx_dist_set_graph(cgx_dist *d, int on);
/* Test hook: make this rank's next hipGraph captures fail.  mode 1: refused
 * before any RCCL call is recorded; mode 2: refused after the iteration's
 * RCCL calls were recorded.  When every rank is refused at the same point
 * the ranks agree (MIN / MAX all-reduce of the capture results) to drop
 * their graphs and run eager (cgx_dist_stats.graph -1), with the same
 * results; a mix -- ranks that recorded RCCL calls beside ranks that did
 * not -- makes every rank's run return CGX_ECOMM, the communicator unusable
 * from then on (the ranks' host-side RCCL state may be out of step).
 * mode 3: as 2, and this rank takes its peers to have captured (the mix,
 * testable on one rank).  0: off. */
int  cgx_dist_debug_refuse_capture(cgx_dist *d, int mode);
int  cgx_dist_run(cgx_dist *d, int maxit, double tol, int *iters);
int  cgx_dist_get_x(cgx_dist *d, double *x_local);
int  cgx_dist_get_history(cgx_dist *d, double *rr, int cap);
int  cgx_dist_bench_prepare(cgx_dist *d, int warmup);
/* flags: CGX_BENCH_SPMV_EVENTS brackets the interior and boundary SpMV
 * launches of partition 0 (one-launch SR: the march and the edge launch)
 * with events; *spmv_ms = their average sum. */
int  cgx_dist_bench_run(cgx_dist *d, int iters, int flags, double *total_ms,
                        double *spmv_ms);
/* Per-phase averages (ms per iteration) of the last bench_run with
 * CGX_BENCH_SPMV_EVENTS, from the events on partition 0's stream (eager
 * iterations): ms[0] the first SpMV launch (interior items; one-launch SR:
 * the march), ms[1] the gap until the second (the halo wait), ms[2] the
 * second launch (boundary items; SR: the edge rows), ms[3] the tail until
 * the next iteration's first launch (local sums, all-reduce(s), vector
 * updates, the next pack), ms[4] the iteration period; -1 before such a
 * run.  *iters (may be NULL): the iterations averaged. */
int  cgx_dist_bench_phases(cgx_dist *d, double *ms, int *iters);
int  cgx_dist_info(cgx_dist *d, cgx_dist_stats *s);

#ifdef __cplusplus
}
#endif
#endif /* CGX_H */
