// cgx_internal.h -- shared between the HIP kernels (cgx_kernels.hip), the
// device matrix (cgx_matrix.cpp) and the host orchestration (cgx_solver.cpp,
// cgx_dist.cpp, cgx_mvops.cpp).
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

// Checks that `device` exists and is a gfx950 (MI355X); CGX_ENODEV otherwise.
int check_device(int device, int *cus = nullptr);
// Device allocation (physically contiguous when the driver allows it: -1 to
// -2% per C3 iteration, r01), zero-size requests get 16 bytes.  Every
// buffer starts kGuardBytes (zeroed) after its allocation, so a pair load
// of x[-1], x[0] (DIA / stencil SpMV, an edge row without that neighbour)
// stays inside it.  Adds the size to *counter.  CGX_ENOMEM (with
// cgx_last_error set) on failure.  Free with dev_free only.
constexpr size_t kGuardBytes = 256;
int dev_alloc(void **p, size_t bytes, size_t *counter);
void dev_free_raw(void *p);
template <typename P>
inline int dev_alloc(P **p, size_t bytes, size_t *counter) {
  return dev_alloc((void **)p, bytes, counter);
}
template <typename P>
inline void dev_free(P **p) {
  dev_free_raw((void *)*p);
  *p = nullptr;
}

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
  int done;       // stop flag; every kernel early-exits on it
  int use_tol;
  int hist_cap;
  // folded HS: the scalar steps run inside the vector kernels, so each
  // kernel reads only what the previous one wrote: k_update_rf writes
  // rr_u / k_u (+ alpha), k_xpay_xf writes rr_x / k_x (+ rr, k, beta, done)
  int k_u;
  int k_x;
  int brk;        // breakdown: 1 + the first iteration whose p.s (HS) or CG1
                  // denominator was <= 0 or not finite (the reference then
                  // yields NaN, cg.c:113, 129); 0 = none.  Diagnostic only.
  double rr_u;
  double rr_x;
  // fused HS step (k_spmv_dia_h): k_update_rf's last workgroup writes the
  // canonical sum of its r.r partials here; k_u = -1 after the prologue
  // marks "no previous iteration" (p = r, no x update)
  double rr_new;
  // fused step: alpha of an even iteration whose x update is deferred to the
  // next (odd) one -- written by the launch that defers it
  double alpha_def;
  // partitioned one-launch SR: 1 when the all-reduced (p.s, s.s, r.r) of the
  // last launch pair are not yet applied to this state (every kernel of the
  // next iteration applies them to its own copy, FIN_SUM3_SR1 to the state)
  int sr_pend;
  // the one-launch SR step's x deferral depth (2, or 4 on one GPU: x +=
  // alpha p for four iterations in every fourth launch; 0 reads as 2) and
  // alpha_i of the pending iterations (alpha_q[i % 4], depth 4)
  int xdef;
  double alpha_q[4];
};
static_assert(sizeof(CgState) == 168, "CgState layout");

// Finalize ops (single-workgroup scalar steps of the recurrence).
enum FinOp {
  FIN_INIT_HS = 0,   // bb = rr = sum(a)
  FIN_HS_ALPHA = 1,  // alpha = rr / sum(a)                     (cg.c:113)
  FIN_HS_BETA = 2,   // rr_new = sum(a); stop test; beta        (cg.c:125-129)
  FIN_INIT_CG1 = 3,  // gamma = bb = sum(a), delta = sum(b), alpha = gamma/delta
  FIN_CG1 = 4,       // gamma' = sum(a), delta = sum(b); stop test; alpha, beta
  FIN_SUM = 5,       // out[0] = sum(a) (op-level dot, local sums)
  FIN_SUM2 = 6,      // out[0] = sum(a), out[1] = sum(b)
  FIN_SUM3 = 7,      // out[0..2] = sums of a's (x, y) pairs and of c (SR local sums)
  FIN_SR1 = 8,       // single-GPU SR step: (p.s, s.s) pairs + r.r -> alpha, estimate,
                     // stop test, beta (k_sr1_dia_m's partials)
  FIN_SUM3_SR1 = 9,  // partitioned one-launch SR: FIN_SR1 of the previous all-reduce
                     // (pb: the all-reduced sums, when st->sr_pend) applied to the
                     // state, then FIN_SUM3's local sums (sr_pend = 1)
};

constexpr int kVecBS = 256;
constexpr int kFinBS = 1024;
constexpr int kFoldBS = 1024;
constexpr int kPad = 8;            // val/col/vectors padded by this many entries
constexpr int kWindowPad = 1024;   // + one SpMV window (LDS-DMA reads 16-B pieces)
constexpr int kDiaSliceRows = 512; // DIA-VI work item: one workgroup, 2 rows per thread
constexpr int kDiaMax = 16;        // DIA-VI: diagonals (fields of a <= 64-bit row word)
constexpr int kDiaVals = 15;       // DIA-VI: values per diagonal (all-ones field = no entry)
constexpr int kDiaVMax = 8;        // DIA-V: diagonals (one-byte presence words)
constexpr int kHaloMax = 1024;     // fused step: diagonals |d| <= this read p from the LDS window
constexpr double kMallBytes = 256.0 * 1024 * 1024;  // Infinity Cache

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
// The column offsets col - row a generated Laplacian can hold, sorted.
std::vector<int> lap_offsets(const LapSpec &g);

// --------------------------------------------------------------- SpMV
// Device layouts of a matrix (cgx_matrix.cpp chooses one per matrix):
//   L_CSR      the reference's CSR (int32 columns), one 64-row block per wave,
//              val/col window staged in LDS by LDS-DMA       (k_spmv_csr)
//   L_DC       dictionary-coded columns: col = row + dict[code], one code
//              byte per nonzero + byte row lengths, value stream kept
//                                                            (k_spmv_dc)
//   L_DIA      value-indexed diagonal codes (DIA-VI): <= 16 diagonals
//              (col - row), <= 15 values each; per row a 1-4 bit field
//              per diagonal (value index, all ones = no entry) in a 1-8
//              byte word, no column or value stream; two rows per thread,
//              pair loads of x (k_spmv_dia; fused step k_spmv_dia_h)
//              DIA-V, its variant for values no table indexes (general
//              coefficients; one GPU and the ranks' one-launch SR matrix):
//              <= 8 diagonals, a one-bit presence field per diagonal, the
//              values streamed diagonal-major (SpmvArgs::dval; k_spmv_dia,
//              the one-launch SR step and its edge launch)
//   L_STENCIL  matrix-free 5/7-point Laplacian                (k_stencil)
// Every kernel sums each row sequentially in column order from 0.0 with
// separately rounded products: y is bit-identical across layouts and to the
// reference's mv_mult on chained matrices (mv_ops.c:187-197).
enum Layout : int { L_CSR = 0, L_DC = 1, L_DIA = 2, L_STENCIL = 3 };

// Work items of one launch (CSR/DC: row blocks; DIA: 512-row slices): list[0, count)
// when list != nullptr, else first, first+1, ..., first+count-1.
// The fused HS step (k_spmv_dia_h) with two slices per workgroup (wide
// halos, cgx_kernels.hip fuse_slices) runs super-items of <= 2 ADJACENT slices: pairs[2 w], pairs[2 w + 1] = (list position, 1 or 2) of
// super-item w (npairs of them); pairs == nullptr: the natural pairing
// (positions 2w, 2w + 1) -- a contiguous run, or a list of adjacent pairs.
struct Items {
  const int *list;
  int first;
  int count;
  const int *pairs = nullptr;
  int npairs = 0;
};
// Super-items of a list of slices on the host: greedy adjacent pairs, as
// Items::pairs (2 ints each).
std::vector<int> fuse_pairs(const std::vector<int> &slices);

// In-kernel local sums of k_update_rf ("last arriver"): every workgroup
// publishes its partials and takes a ticket on *cnt; the last one sums
// pa[0, na) in the canonical order -- sum_parts<1024>'s, the order k_finalize
// and the folded vector kernels use -- writes out[0] and re-arms the counter
// (the fused step's r.r, the partitioned solver's local r.r).  Only for
// grids of a few hundred workgroups: every workgroup drains its stores and
// takes a device-scope atomic before it retires (an SpMV of 15 K workgroups
// paid 70 us for it; its local sums are a k_finalize launch).  cnt ==
// nullptr: off.
// Tickets: two levels (cgx_kernels.hip take_ticket), cnt[0] for the launch
// and cnt[1 + g] per group of kTicketGroup workgroups; a ticket region holds
// kTickRegion counters (grids up to (kTickRegion - 1) * kTicketGroup).
constexpr int kTicketGroup = 128;
constexpr int kTickRegion = 4096;
struct FinArgs {
  unsigned *cnt;
  const double *pa;
  int na;
  double *out;
};

// DIA-VI candidates for the device encoder: diagonal offsets and the number
// of values in each diagonal's table.
struct DiaCand {
  int ndiag;
  int doff[kDiaMax];
  int nval[kDiaMax];
  // packed row codes: diagonal k's field is bits [csh[k], csh[k] + cbits[k])
  // of the row's word, value indices 0..nval-1, all ones = no entry; the
  // word is cbytes (1, 2, 4 or 8) bytes (dia_pack)
  int cbits[kDiaMax];
  int csh[kDiaMax];
  int cbytes;
};
// Field widths and word size from nval: 1 bit for one value (a Laplacian's
// diagonals), 2 for <= 3, 3 for <= 7, 4 for <= 15.
void dia_pack(DiaCand &c);

template <typename T>
struct SpmvArgs {
  int layout;
  const T *x;
  T *y;
  double *part;     // one x[row]*y[row] partial per workgroup (nullptr: none)
  const int *done;  // early-exit flag (nullptr: never)
  int nt;           // non-temporal matrix stream and y store
  Items items;
  // CSR / DC row blocks: (first row, first nonzero) of block i at 2i, 2i+1
  const int *blkrk;
  int capw;         // LDS window entries per wave (fp64 512 | 328, fp32 1024)
  // CSR
  const int *rp, *col;
  const T *val;
  const T *yacc;    // column panels: row sums continue from yacc[row] (may alias y)
  // DC
  const unsigned char *code, *rlen;
  const int *dict;  // 64 or 256 entries (ndict_cap)
  int ndict_cap;
  int gath;               // CSR / DC: x gathers per row chunk (7 or 8)
  // DIA
  const unsigned char *dcode;  // row r: bytes [cb r, cb (r + 1)) (DiaCand)
  int cb;                 // code bytes per row: 1, 2, 4, 8
  int csh[kDiaMax];       // diagonal k's field: (word >> csh[k]) & cmask[k]
  unsigned cmask[kDiaMax];  // == cmask[k]: no entry on diagonal k
  const T *vtab;          // [16][16] values, vtab[16 k + v]
  // DIA-V (value-streamed diagonals, <= kDiaVMax of them): diagonal k's
  // value of row r at dval[k dvs + r] (0 where the row has none; the code
  // field is then a one-bit presence flag); nullptr: DIA-VI
  const T *dval;
  int dvs;
  int ndiag;              // diagonals
  int kdiag;              // index of the main diagonal (offset 0), -1: none
  int doff[kDiaMax];      // diagonal offsets col - row, ascending
  int n;                  // rows (DIA, stencil)
  int ncols;              // entries of x (DIA pair loads stay inside)
  int xlo;                // lowest pair start the windows may load: -1 (the guard
                          // entry x[-1]), or below a partition's in-place ghost
                          // rows [col_lo, 0) (DevMatrix::col_lo)
  // fused step (k_spmv_dia_h): the slice's LDS window covers rows
  // [s0 - hl, s0 + 512 + hr); diagonal k is read from it when near bit k
  int hl, hr;
  unsigned near;
  int fark[4];      // the far (not near) diagonals, -1: unused slot
  // plane march of the fused step (k_spmv_dia_m; DevMatrix::plan_march):
  // every far diagonal is +-F, F within the halo of mq slices; chains of
  // msb-slice super-items j0, j0 + mq, ... (mchains of them, j0 = msb c);
  // mws: LDS ring slot stride (entries); mpos: slice -> position in mlist
  // (the item order its partial slots follow; nullptr: natural order)
  int mq, msb, mchains, mslices, mws, mlen;
  const int *mpos, *mlist;
  // stencil
  LapSpec lap;
  double inv_nx, inv_pl;  // 1 / nx, 1 / (nx ny): exact floor divisions (fdiv)
  // CGX_ALG_SR without the fused step: the epilogue stores the (p.s, s.s)
  // pair per workgroup (part[2 b], part[2 b + 1]) instead of p.s
  int pair = 0;
};

// The fused HS step (single GPU, DIA layout): one launch does the previous
// iteration's p_new = r + beta p_old (beta and the stop test from CgState;
// cg.c:125-132) and, every other launch, x += alpha p for two iterations
// (cg.c:115-116), then s = A p_new with the p_new.s partials.  p is
// double-buffered (the launch reads p_old while it stores p_new; the p_new
// buffer holds p_{k-1} until then).
template <typename T>
struct FuseArgs {
  T *x;
  const T *pold;
  T *pnew;
  const T *r;
  CgState *st;
  double *hist;
  const double *rr_new;  // r.r of the last r update (&st->rr_new, or all-reduced)
  int publish;           // this launch's workgroup 0 writes the scalar state back
  int ghost;             // columns >= n are ghosts: p_new from pnew's ghost tail
  double *ss;            // CGX_ALG_SR: one (p.s, s.s) pair per workgroup, ss[2 b],
                         // ss[2 b + 1], instead of a.part (nullptr: none)
  int march = 0;         // plane march (k_spmv_dia_m): steps per segment, 0: off
};

// The single-GPU SR iteration in ONE launch (k_sr1_dia_m, plane march): the
// previous iteration's r = r - alpha s and p = r + beta p (the window rows:
// r, s, p read from the _o buffers) and x += alpha p, then s = A p; the
// (p.s, s.s) pairs (pq[2 b], pq[2 b + 1]) and r.r (pc[b]) per workgroup b for
// k_finalize(FIN_SR1).  r, s, p are double-buffered (read _o, write _n; s_n
// = SpmvArgs::y).
// Partitioned (in-place ghost rows, DevMatrix::col_lo): the same launch over
// every step while the halo is in flight (a window's ghost rows hold no p_k
// yet), then k_sr1_edge after it: s of the edge rows [0, elo) and [ehi, n)
// (even bounds; rows whose row reaches a ghost column) from the p_new buffer
// (own rows as stored, ghost rows from the halo), and their (p.s, s.s) --
// k_sr1_dia_m leaves those rows out of its pairs.  A chain's steps are cut
// into nseg balanced segments, or (nseg 0) segments of `march` steps.
template <typename T>
struct Sr1Args {
  T *x;
  const T *pold;
  T *pnew;
  const T *rold;
  T *rnew;
  const T *sold;
  const CgState *st;
  double *pq, *pc;
  int march;  // steps per segment (nseg == 0)
  int nseg = 0;
  int cw = 0;  // chain width in rows (even, <= sb slices; 0: sb slices)
  // x deferral depth 4 (st->xdef == 4; single GPU): the p buffers holding
  // p_{k-2} (pa) and p_{k-1} (pb) -- pnew holds p_{k-3}, pold p_k; nullptr:
  // depth 2
  const T *pa = nullptr, *pb = nullptr;
  int sb = 0;  // rows per step in slices (1, 2, 4; 0: the matrix's plan)
  int elo = 0, ehi = 0x7fffffff;
  // partitioned: the all-reduced (p.s, s.s, r.r) of the last iteration,
  // applied (FIN_SR1's step) to a private copy of *st when st->sr_pend --
  // no scalar launch between the all-reduce and this one; nullptr: *st is
  // current (single GPU, transport-free)
  const double *g = nullptr;
  // single GPU, the scalar step folded into the launch (no k_finalize): the
  // state is read from *st and handed to the next launch in *st_out
  // (workgroup 0, with the history entry in hist); when st->sr_pend, every
  // workgroup first runs FIN_SR1's step on the last launch's pq_in / pc_in
  // (np_in workgroups) -- the launches alternate two states and two sets of
  // partials; nullptr: off
  CgState *st_out = nullptr;
  const double *pq_in = nullptr, *pc_in = nullptr;
  int np_in = 0;
  double *hist = nullptr;
};

// The fused CG1 step (Chronopoulos-Gear, DIA layout, k_cg1_dia_h): one
// launch does k_cg1_update's p / s / x / r recurrences (alpha, beta and the
// stop flag from CgState) and w = A r_new, writing the gamma = r.r (pg) and
// delta = w.r (SpmvArgs::part) partials of the iteration's single
// reduction.  r, s, w are double-buffered (read _o, write _n; w_n = a.y).
template <typename T>
struct Cg1Args {
  T *x, *p;
  const T *r_o, *s_o, *w_o;
  T *r_n, *s_n;
  const CgState *st;
  double *pg;
  int ghost;  // columns >= n are ghosts: r_new from r_n's ghost tail
};

// Optional kernel timing events of a launch (hipExtLaunchKernel: stamped at
// the kernel's own start and end).
struct LaunchEv {
  hipEvent_t start = nullptr, stop = nullptr;
};

// Workgroups of one launch (= epilogue partials it writes).
template <typename T>
int spmv_grid(const SpmvArgs<T> &a);
template <typename T>
hipError_t launch_spmv(const SpmvArgs<T> &a, hipStream_t st, const LaunchEv &ev = LaunchEv{});
// The fused HS step on a DIA layout (a.x unused, a.y = s, a.part the
// p_new.s partials).
// Workgroups of the fused launch (= SR (p.s, s.s) pairs it writes)
template <typename T>
int fused_grid(const SpmvArgs<T> &a);
template <typename T>
hipError_t launch_sr1_march(const SpmvArgs<T> &a, const Sr1Args<T> &f, hipStream_t st,
                            const LaunchEv &ev);
// workgroups (= partial pairs) of the plane march at `len` steps per segment
template <typename T>
int march_grid(const SpmvArgs<T> &a, int len);
// workgroups (= partial pairs) of one k_sr1_dia_m launch
template <typename T>
int sr1_grid(const SpmvArgs<T> &a, const Sr1Args<T> &f);
// Launch shape of k_sr1_dia_m on `cus` CUs: segments per chain and chain
// width (rows), the pair whose launch takes the fewest window-times in the
// resident-workgroup model (ceil(chains nseg / slots) rounds of ceil(L /
// nseg) + 2 windows, L the longest chain; slots from the kernel's
// occupancy; fold: the single GPU's kernel with the folded scalar step,
// Sr1Args::st_out).  cw_force > 0: that chain width, only nseg picked.  An
// explicit march length (> 0) is used as given instead (nseg 0).
struct Sr1Shape {
  int nseg, cw, sb;
};
// the most workgroups one k_sr1_dia_m launch may have (its partial pairs)
// for a matrix of `slices` 512-row slices: sr1_pick_shape and
// launch_sr1_march keep to it
inline int sr1_max_grid(int slices) { return 4 * slices + 64; }
template <typename T>
Sr1Shape sr1_pick_shape(const SpmvArgs<T> &a, int cus, int cw_force = 0, bool fold = false);
// workgroups (= partial pairs) of k_sr1_edge over f's edge rows of n rows
template <typename T>
int sr1_edge_grid(int n, const Sr1Args<T> &f);
// k_sr1_edge: s of the edge rows after the halo, their (p.s, s.s) pairs
// (a.y = s; f.pnew = p_k with ghost rows; f.pq / f.pc: this launch's slots)
template <typename T>
hipError_t launch_sr1_edge(const SpmvArgs<T> &a, const Sr1Args<T> &f, hipStream_t st,
                           const LaunchEv &ev);
// out[i] = p_k[idx[i]] = (r - alpha s) + beta p of the last iteration's
// buffers (the one-launch SR step's halo send rows; r itself on the first
// iteration) -- the roundings k_sr1_dia_m uses for its window rows
template <typename T>
hipError_t launch_pack_sr(int n_send, const int *idx, const T *rold, const T *pold,
                          const T *sold, T *out, const CgState *stt, hipStream_t st,
                          const double *g = nullptr);
template <typename T>
hipError_t launch_spmv_fused(const SpmvArgs<T> &a, const FuseArgs<T> &f, hipStream_t st,
                             const LaunchEv &ev = LaunchEv{});
template <typename T>
hipError_t launch_cg1_fused(const SpmvArgs<T> &a, const Cg1Args<T> &f, hipStream_t st,
                            const LaunchEv &ev = LaunchEv{});
// out[i] = r_new[idx[i]] = r - alpha (w + beta s) (the fused partitioned CG1
// step's halo send rows)
template <typename T>
hipError_t launch_pack_rnext(int n_send, const int *idx, const T *r, const T *w, const T *s,
                             T *out, const CgState *stt, hipStream_t st);
// out[i] = p_new[idx[i]] = r + beta p_old (the fused partitioned step's halo
// send rows; beta from *rr_new and st, r on the first iteration)
template <typename T>
hipError_t launch_pack_pnext(int n_send, const int *idx, const T *r, const T *pold, T *out,
                             const CgState *stt, const double *rr_new, hipStream_t st);

// ------------------------------------------------------------- vectors
// All launchers are graph-capturable (no sync, no allocation).
template <typename T>
hipError_t launch_init_hs(int n, const T *b, T *x, T *r, T *p, double *part, int grid,
                          hipStream_t st);
template <typename T>
hipError_t launch_init_cg1(int n, const T *b, T *x, T *r, T *p, T *s, double *part,
                           int grid, hipStream_t st);
// exact-mode HS steps (separate finalize launches)
template <typename T>
hipError_t launch_update_xr(int n, T *x, const T *p, T *r, const T *s, const CgState *stt,
                            double *part, int grid, hipStream_t st);
template <typename T>
hipError_t launch_xpay(int n, T *p, const T *r, const CgState *stt, int grid,
                       hipStream_t st);
// folded HS steps (alpha / beta computed inside from the producer's partials)
// fin (optional): the r.r partials' canonical sum to fin->out[0] by the last
// workgroup (fin->pa must be rr_part, fin->na = 4 * grid)
// sr (CGX_ALG_SR): the reduced (p.s, s.s, r.r) -- first the previous
// iteration's stop test on the exact r.r (its history entry to hist), then
// alpha = r.r / p.s from them instead of ps_part and rr_x, and the estimate
// r_new.r_new = alpha^2 s.s - r.r to st->rr_new for the next fused launch's
// beta
template <typename T>
hipError_t launch_update_rf(int n, T *r, const T *s, CgState *stt, const double *ps_part,
                            int nps, double *rr_part, int grid, hipStream_t st,
                            const FinArgs *fin = nullptr, const double *sr = nullptr,
                            double *hist = nullptr, bool nt = false);
// p -> pn (pn == p: in place, x every iteration; pn != p: x every other
// iteration, k_xpay_xf).  nt (update_rf's r, xpay_xf's x and p): non-temporal
// stores, for an unfused iteration whose working set exceeds the Infinity
// Cache (DevMatrix::nt): the lines go to HBM inside the vector kernel instead
// of lingering dirty until the next SpMV's matrix stream evicts them (C3 CSR:
// 192.9 -> 184.8 us per in-iteration SpMV, 3,355 -> 3,467 it/s; C4 1,252 ->
// 1,217 us)
template <typename T>
hipError_t launch_xpay_xf(int n, T *x, const T *p, T *pn, const T *r, CgState *stt,
                          const double *rr_part, int nrr, double *hist, int grid,
                          hipStream_t st, bool nt = false);
// CGX_ALG_SR without the fused step (k_update_sr): the rest of iteration j
// after its SpMV's (p.s, s.s) reduction -- r -= alpha s, p_new = r + beta p
// (pn: the other p buffer), x += alpha p every other iteration, the exact
// r.r partials (4 per workgroup of grid).  g: the all-reduced sums applied
// privately (sr1_now; a partition's ranks), nullptr: *stt is current.
// fo (the single-GPU solver): no k_finalize before it -- every workgroup
// sums the SpMV's (p.s, s.s) pairs and the previous r.r partials (fo->pc,
// not rr_part) and runs FIN_SR1's step privately; the last arriver (fo->tick)
// writes the state and the history.
struct SrFold {
  const double *pq;  // the SpMV's (p.s, s.s) pairs
  int nq;
  const double *pc;  // r.r partials of the previous update (or the init)
  int nc;
  unsigned *tick;
  double *hist;
};
template <typename T>
hipError_t launch_update_sr(int n, T *x, T *r, const T *sv, const T *p, T *pn, CgState *stt,
                            const double *g, double *rr_part, int grid, hipStream_t st, bool nt,
                            const SrFold *fo = nullptr);
template <typename T>
hipError_t launch_cg1_update(int n, T *x, T *p, T *r, T *s, const T *w,
                             const CgState *stt, double *part, int grid, hipStream_t st);
// Sequential dot (exact mode): out[0] = sum_i a[i]*b[i] in index order.
template <typename T>
hipError_t launch_dot_seq(int n, const T *a, const T *b, double *out, const int *done,
                          hipStream_t st);
// Two-stage dot, stage 1: part[blockIdx] = partial sums.
template <typename T>
hipError_t launch_dot_part(int n, const T *a, const T *b, double *part, int grid,
                           hipStream_t st);
hipError_t launch_finalize(int op, const double *pa, int na, const double *pb, int nb,
                           CgState *stt, double *hist, double *out, hipStream_t st,
                           const double *pc = nullptr, int nc = 0);
// Elementwise ops of the mv_ops API: op 0: r = s*a, 1: r = a+b, 2: r = a-b
template <typename T>
hipError_t launch_axpby(int op, int n, double s, const T *a, const T *b, T *r, int grid,
                        hipStream_t st);
// Halo pack: buf[i] = x[idx[i]]
template <typename T>
hipError_t launch_gather(int m, const int *idx, const T *x, T *buf, hipStream_t st);
// In-process all-reduce: dst[off+c] = sum_q srcs[q][off+c] (fixed order)
hipError_t launch_group_sum(const double *const *srcs, int P, int count, double *dst,
                            hipStream_t st, int off = 0);
hipError_t launch_triad(long long n2, double *a, const double *b, const double *c, int grid,
                        hipStream_t st);
hipError_t launch_stream_read(long long n2, const double *b, double *sink, int grid,
                              hipStream_t st);
// the tuned CGX_STREAM_COPY.. kinds: arrays read / written (-1: not one),
// and the launch over buf (R + W arrays of n2 16-B chunks, `stride` apart)
int stream_rw_arrays(int kind, int *r, int *w);
hipError_t launch_stream_rw(int kind, long long n2, long long stride, double *buf, int cus,
                            hipStream_t st);
hipError_t launch_gen_laplacian(const LapSpec &g, int n, int *col, double *val,
                                hipStream_t st);
// Offset codes of a device CSR against a sorted dictionary (err |= 1 on a
// miss); with dval (one value per offset) also err |= 1 when a value differs
// from its offset's in any bit.
hipError_t launch_dc_encode(int n, const int *rp, const int *col, const int *dict, int nd,
                            unsigned char *code, int *err, hipStream_t st,
                            const double *val = nullptr, const double *dval = nullptr);
// DIA-VI codes of a device CSR (rows [0, npad), rows >= n all "no entry"):
// err |= 1 when an entry's diagonal or value is not a candidate or a row's
// columns do not strictly ascend.
template <typename T>
hipError_t launch_dia_encode(int n, int npad, const int *rp, const int *col, const T *val,
                             const DiaCand &c, const T *vtab, unsigned char *code, int *err,
                             hipStream_t st);

int vec_grid_for(int n, int cus);
// Iterations to run before the next stop-flag poll of a solve with a
// tolerance, from r.r at this poll and the last (k = iteration index).
long long next_batch(double rr, double tol2bb, int k, double rr_prev, int k_prev, long long batch);

// Partition helpers (cgx_partition.cpp)
long long part_begin(long long n, int G, int g);
int part_owner(long long n, int G, long long c);

}  // namespace cgx
