// cgx_internal.h -- shared between the HIP kernels (cgx_kernels.hip) and the
// host orchestration (cgx_solver.cpp, cgx_mvops.cpp, cgx_dist.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "cgx.h"

namespace cgx {

// ---------------------------------------------------------------- errors
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define CGX_HIP(call)                                                        \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::cgx::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,    \
                       hipGetErrorString(e_));                               \
      return CGX_ENODEV;                                                     \
    }                                                                        \
  } while (0)

// ------------------------------------------------------- device CG state
// One per solve, device resident: every scalar of the recurrence lives here
// so an iteration never round-trips to the host (graph-replayable).
struct CgState {
  double rr;      // HS: r.r of the current r;  CG1: gamma = r.r
  double alpha;
  double beta;
  double bb;      // b.b
  double tol;     // requested tolerance (<= 0: none)
  double tol2bb;  // tol*tol*b.b
  double delta;   // CG1: w.r
  double ps;      // HS: p.s of the last SpMV (diagnostic)
  int k;          // index of the current iteration (x-updates done = k+1 at stop)
  int max_iter;
  int done;       // set by the finalize step; every kernel early-exits on it
  int use_tol;
  int hist_cap;
  // folded HS (CGX_FOLD): the scalar steps run inside the vector kernels, so
  // each kernel reads only what the previous one wrote: k_update_rf writes
  // rr_u / k_u (+ alpha), k_xpay_xf writes rr_x / k_x (+ rr, k, beta, done)
  int k_u;
  int k_x;
  int pad;
  double rr_u;
  double rr_x;
};
static_assert(sizeof(CgState) == 112, "CgState layout");

// -------------------------------------------------------------- geometry
// SpMV row block: bs (256 or 512) rows, one per lane, and at most
// spmv_cap(bs) products staged in LDS (16 KiB per 256 lanes).
inline int spmv_cap(int bs, bool f64) { return bs * (f64 ? 8 : 16); }
// Resident workgroups per CU of the engine SpMV's ring shapes (k_spmv_eng).
inline int eng_wg_per_cu(int shape) { return shape == 1 ? 4 : shape >= 2 ? 2 : 3; }
// Workgroups of one SpMV launch (= fused-dot partials it writes).
// k_spmv_vi's grid (and epilogue partial count)
inline int vi_grid(int nblk, int code_bits, int bpw) {
  if (code_bits != 8) bpw = 1;
  return (nblk + 4 * bpw - 1) / (4 * bpw);
}
inline int spmv_launch_grid(int bs, int wpb, int rbw, int nblk, int grid,
                            int dma = 0) {
  if (bs == 64 && dma == 2) return (nblk + 2 * rbw - 1) / (2 * rbw);
  if (bs == 64 && dma == 1 && wpb == 8) return (nblk + 7) / 8;
  if (bs == 64 && dma) return (nblk + 3) / 4;
  if (bs == 64) return (nblk + wpb * rbw - 1) / (wpb * rbw);
  return grid < 1 ? 1 : (grid > nblk ? nblk : grid);
}
constexpr int kVecBS = 256;
constexpr int kFinBS = 1024;
constexpr int kPad = 8;               // val/col padded to a multiple of this
constexpr int kWindowPad = 1024;      // + one SpMV window (LDS-DMA reads whole windows)
// Non-temporal matrix stream only when the matrix cannot stay resident in the
// 256 MiB Infinity Cache anyway (C3: 843 MB -> nt helps the vectors stay; C2:
// 60 MB -> nt would evict a matrix that otherwise never leaves the cache).
constexpr double kNtStreamBytes = 160.0 * 1024 * 1024;

// Finalize ops (single-workgroup scalar steps of the recurrence).
enum FinOp {
  FIN_INIT_HS = 0,  // bb = rr = sum(a)
  FIN_HS_ALPHA = 1, // alpha = rr / sum(a)            (cg.c:113)
  FIN_HS_ALPHA_X = 7, // as FIN_HS_ALPHA; deferred-x mode: a stop flag of 1
                      // (x update of the stop iteration pending) becomes 2
  FIN_HS_BETA = 2,  // rr_new = sum(a); stop test; beta = rr_new/rr (cg.c:125-129)
  FIN_INIT_CG1 = 3, // gamma = bb = sum(a), delta = sum(b), alpha = gamma/delta
  FIN_CG1 = 4,      // gamma' = sum(a), delta = sum(b); stop test; alpha, beta
  FIN_SUM = 5,      // out[0] = sum(a) (op-level dot)
  FIN_SUM2 = 6,     // out[0] = sum(a), out[1] = sum(b) (local sums to all-reduce)
};

// In-kernel two-level ticket reduction (see ticket_finish in
// cgx_kernels.hip): replaces a k_finalize launch.  cnt1 == nullptr: off.
constexpr int kTicketGroup = 64;
struct TicketArgs {
  double *part1;    // >= grid partials
  double *part2;    // >= ceil(grid / kTicketGroup)
  unsigned *cnt1;   // >= ceil(grid / kTicketGroup), zero-initialised
  unsigned *cnt2;   // 1, zero-initialised
  int op;           // FinOp applied by the final workgroup
  CgState *st;
  double *hist;
};

template <typename T>
struct SpmvArgs {
  const int *rp;       // row_ptr (local rows)
  const int *col;      // column indices into x (local numbering)
  const T *val;
  const T *x;
  T *y;
  const int *blk_row;  // row-block boundaries, nblk_total+1 entries
  const int *blk_k;    // rp[blk_row[i]]: nonzero offset of each row block
  const int *blk_rk;   // k_spmv_dc: (blk_row[i], blk_k[i]) pairs, so a block's
                       // whole descriptor is one 16-byte scalar load
  const int *blk_list; // optional subset of row blocks (nullptr: a contiguous
                       // run blk_first .. blk_first+nblk-1)
  int blk_first;
  int nblk;            // row blocks processed by this launch
  double *part;        // per-workgroup partial of x[row]*y[row] (nullptr: none)
  const int *done;     // early-exit flag (nullptr: never)
  int xcd;             // XCD-aware chunk mapping (speed only)
  int nt;              // non-temporal val/col stream loads (2: + CSR-VI y store)
  int bs;              // rows per row block: 256 | 512 (workgroup-wide block),
                       // 64 (one row block per wave, k_spmv_wave)
  int wpb;             // k_spmv_wave: waves per workgroup (4 | 8)
  int rbw;             // k_spmv_wave: row blocks per wave
  // fused p-update (k_spmv_wave only): x2 = p_old (nullptr: off); the gathered
  // operand is x + beta*x2 with beta = st->beta, and xout receives it for the
  // owned rows (p_new; must not alias x or x2).
  const T *x2;
  T *xout;
  const CgState *st;
  int tg;              // k_spmv_wave: transposed (row-per-lane) gather
  TicketArgs tk;       // k_spmv_wave + EPI: in-kernel finalize (cnt1 != 0)
  // SELL-64 layout (k_spmv_sell) when s_off != nullptr: val/col hold the
  // sliced arrays, s_off[i] = slice i's first element / 64, s_len[i] = width
  const int *s_off;
  const int *s_len;
  int nslices;
  int n;
  // column panels (k_spmv_dma): running row sums of the previous panels,
  // the row's sum starts from yacc[row] instead of 0 (nullptr: from 0).  The
  // entries of a row are ascending in column, so summing panel after panel
  // is the reference's sequential order.  May alias y.
  const T *yacc;
  int capw;            // k_spmv_dma fp64 window entries: 0 = 512, or 456 / 328
  int epi_last;        // k_spmv_dma: last-arriving wave writes the partial
  int dma;             // 1: k_spmv_dma (LDS-DMA stream, one block per wave)
                       // 2: k_spmv_pipe (persistent waves, rbw blocks each,
                       //    next block's stream prefetched by LDS-DMA)
  // dictionary-coded columns (k_spmv_dc) when code != nullptr: col[k] ==
  // row + dict[code[k]], one byte per nonzero instead of four (matrices with
  // <= 256 distinct column offsets col - row: stencils, banded matrices).
  // dict holds ndict_cap (64 | 256) entries, unused ones 0.
  const unsigned char *code;
  const int *dict;
  int ndict_cap;
  // k_spmv_dc: row lengths as one byte per row (every row <= 255 entries);
  // the kernel derives row bounds from blk_k and a wave prefix sum instead
  // of reading rp (nullptr: rp)
  const unsigned char *rlen;
  int code_bits;       // k_spmv_dc: 8 (byte codes) or 4 (nibbles, <= 16 offsets)
  int lds_pad;         // k_spmv_dc diagnostic: extra dynamic LDS bytes per workgroup
  // k_spmv_vi (value-indexed pairs, CSR-VI) when dval != nullptr: the
  // dictionary entries are (dict[c], dval[c]) pairs and val[k] ==
  // dval[code[k]] bit for bit, so val is not read (needs rlen, <= 64 pairs,
  // 4 waves per workgroup, every block's code window inside the kernel's)
  const T *dval;
  int bpw;             // k_spmv_vi: row blocks per wave (1 | 2 | 4; byte codes)
};

// Dictionary-coded columns (host side, cgx_solver.cpp): the distinct column
// offsets col[k] - row of a CSR matrix, first-seen order, and one code byte per
// nonzero.  Returns the dictionary size (1..256), or 0 when the matrix has
// more than 256 distinct offsets (or no nonzeros): then it stays plain CSR.
int build_col_codes(int n, const int *rp, const int *col, std::vector<int> &dict,
                    unsigned char *code);
// Value-indexed pairs (CSR-VI): from offset codes (dict = the offsets), the
// distinct (offset, value bit pattern) pairs, sorted by offset then bits.  On
// success (<= cap pairs) code is rewritten to pair codes, dict to the pairs'
// offsets, dval to their values, and the pair count returned; 0 (code, dict
// untouched) otherwise.
template <typename T>
int build_val_pairs(long long nnz, const T *val, unsigned char *code, std::vector<int> &dict,
                    std::vector<T> &dval, int cap);
// Nibble codes (dictionaries of <= 16 offsets): entry k in bits 4*(k&1) of
// byte k/2; out holds (nnz + 1) / 2 bytes.
void pack_nibbles(long long nnz, const unsigned char *code, unsigned char *out);
// Row lengths as bytes for k_spmv_dc; false (nothing written) when a row has
// more than 255 entries.
bool build_row_lengths(int n, const int *rp, unsigned char *rlen);
// Per-solver switch for coded columns at the next set_matrix (the op-level
// mv_mult turns it off: one product per upload).  Respects CGX_DC /
// CGX_LAYOUT: `on` restores the environment's choice.
void solver_want_dc(cgx_solver *s, bool on);
bool env_wants_dc();
// Dictionary capacity the SpMV kernel is instantiated for.
inline int dict_cap(int ndict) { return ndict <= 64 ? 64 : 256; }

inline int spmv_sell_grid(int nslices) { return (nslices + 3) / 4; }

// Row-block plan: consecutive rows, at most `rows` rows and `cap` nonzeros
// per block; a row longer than `cap` gets a block of its own (chunked path).
std::vector<int> plan_rowblocks(int n, const int *rp, int rows, int cap);

// ------------------------------------------------------------- launchers
// All launchers are graph-capturable (no sync, no allocation).
template <typename T>
hipError_t launch_spmv(const SpmvArgs<T> &a, int grid, int vec, hipStream_t st);

template <typename T>
hipError_t launch_init_hs(int n, const T *b, T *x, T *r, T *p, double *part,
                          int grid, hipStream_t st, bool p_zero = false,
                          const TicketArgs *tk = nullptr);
template <typename T>
hipError_t launch_init_cg1(int n, const T *b, T *x, T *r, T *p, T *s,
                           double *part, int grid, hipStream_t st);
template <typename T>
hipError_t launch_update_xr(int n, T *x, const T *p, T *r, const T *s,
                            const CgState *stt, double *part, int grid,
                            hipStream_t st, const TicketArgs *tk = nullptr);
hipError_t launch_triad(long long n2, double *a, const double *b, const double *c,
                        int grid, hipStream_t st);
hipError_t launch_stream_read(long long n2, const double *b, double *sink, int grid,
                              hipStream_t st);
// ---------------------------------------------------- Laplacian operators
// The 5-point 2-D (dim 2, nz = 1, diagonal 4) and 7-point 3-D (dim 3,
// diagonal 6) Laplacians of cgx_gen.cpp, natural ordering, -1 off-diagonals.
struct LapSpec {
  int dim, nx, ny, nz;
};

// Entries in rows [0, i): (2 dim + 1) i minus the missing neighbours of the
// boundary rows, counted per face in closed form (O(1), host and device).
__host__ __device__ inline long long lap_rp(long long i, const LapSpec &g) {
  const long long nx = g.nx, ny = g.ny, pl = nx * ny;
  long long miss = (i + nx - 1) / nx + i / nx;  // x == 0, x == nx-1
  if (g.dim == 3) {
    const long long f = i / pl, rem = i % pl;
    miss += f * nx + (rem < nx ? rem : nx);                        // y == 0
    miss += f * nx + (rem > (ny - 1) * nx ? rem - (ny - 1) * nx : 0);  // y == ny-1
    miss += i < pl ? i : pl;                                       // z == 0
    const long long top = ((long long)g.nz - 1) * pl;
    miss += i > top ? i - top : 0;                                 // z == nz-1
  } else {
    miss += i < nx ? i : nx;                                       // y == 0
    const long long top = (ny - 1) * nx;
    miss += i > top ? i - top : 0;                                 // y == ny-1
  }
  return (2LL * g.dim + 1) * i - miss;
}

hipError_t launch_gen_laplacian(const LapSpec &g, int n, int *col, double *val,
                                hipStream_t st);
// Device-side coded columns against a sorted dictionary (err |= 1 on a miss).
// With dval (value-indexed pairs, one value per offset): also err |= 1 when
// val[k] differs from dval[code] in any bit.
hipError_t launch_dc_encode(int n, const int *rp, const int *col, const int *dict, int nd,
                            unsigned char *code, int *err, hipStream_t st,
                            const double *val = nullptr, const double *dval = nullptr);
// The column offsets col - row a generated Laplacian can hold, sorted.
std::vector<int> lap_offsets(const LapSpec &g);
template <typename T>
hipError_t launch_stencil(const LapSpec &g, int n, const T *x, T *y, double *part,
                          const int *done, int grid, hipStream_t st);

template <typename T>
hipError_t launch_update_rf(int n, T *r, const T *s, CgState *stt, const double *ps_part,
                            int nps, double *rr_part, int grid, hipStream_t st, bool pf);
template <typename T>
hipError_t launch_xpay_xf(int n, T *x, T *p, const T *r, CgState *stt,
                          const double *rr_part, int nrr, double *hist, int grid,
                          hipStream_t st, bool pf);
template <typename T>
hipError_t launch_update_r(int n, T *r, const T *s, const CgState *stt,
                           double *part, int grid, hipStream_t st);
template <typename T>
hipError_t launch_xpay_x(int n, T *x, T *p, const T *r, const CgState *stt,
                         int grid, hipStream_t st);
template <typename T>
hipError_t launch_xpay(int n, T *p, const T *r, const CgState *stt, int grid,
                       hipStream_t st);
template <typename T>
hipError_t launch_cg1_update(int n, T *x, T *p, T *r, T *s, const T *w,
                             const CgState *stt, double *part, int grid,
                             hipStream_t st);
// Sequential dot (exact mode): out[0] = sum_i a[i]*b[i] in index order.
template <typename T>
hipError_t launch_dot_seq(int n, const T *a, const T *b, double *out,
                          const int *done, hipStream_t st);
// Two-stage dot, stage 1: part[blockIdx] = partial sums.
template <typename T>
hipError_t launch_dot_part(int n, const T *a, const T *b, double *part,
                           int grid, hipStream_t st);
hipError_t launch_finalize(int op, const double *pa, int na, const double *pb,
                           int nb, CgState *stt, double *hist, double *out,
                           hipStream_t st);
// Elementwise ops of the mv_ops API: op 0: r = s*a, 1: r = a+b, 2: r = a-b
template <typename T>
hipError_t launch_axpby(int op, int n, double s, const T *a, const T *b, T *r,
                        int grid, hipStream_t st);
// Halo pack: buf[i] = x[idx[i]]
template <typename T>
hipError_t launch_gather(int m, const int *idx, const T *x, T *buf,
                         hipStream_t st);

hipError_t launch_group_sum(const double *const *srcs, int P, int count,
                            double *dst, hipStream_t st, int off = 0);

int vec_grid_for(int n, int cus);
int env_int(const char *name, int dflt);

// Partition helpers (cgx_partition.cpp)
long long part_begin(long long n, int G, int g);
int part_owner(long long n, int G, long long c);

}  // namespace cgx
