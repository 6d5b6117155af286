// cgx_matrix.h -- the device-resident sparse matrix shared by the single-GPU
// solver, the partitioned (multi-GPU) solver and the op-level mv_mult:
// layout choice, encoding, upload, and the SpMV launch.
//
// The C ABI takes the reference's CSR (mv_ops.h:17-23: int32 row_ptr and
// col_indices, fp64 values; fp32 for SURVEY.md C5).  The matrix picks, once
// per upload, the layout the SpMV streams (cgx_internal.h, Layout); only
// that layout's arrays are resident (DIA: codes and value tables, no CSR):
//   auto: DIA-VI when the nonzeros lie on <= 16 diagonals (col - row) with
//         <= 15 distinct values each and every row's columns ascend; else
//         (allow_dv: one GPU, a partition's in-place SR matrix) DIA-V when
//         they lie on <= 8 diagonals and its 1 + 8 ndiag bytes per row
//         (fp64) do not exceed CSR-DC's; else CSR-DC when they use <= 256
//         distinct offsets (rows <= 255 entries); else plain CSR, with
//         column panels when the gathers have no locality (C5).
// Candidates (pairs / offsets) come from a sample of rows on the host; an
// encoder then checks every nonzero against them (DIA: host threads, so only
// the 1-8 code bytes per row cross PCIe; DC: the device, over the uploaded
// CSR), and a miss falls back to an exact host scan.
#pragma once

#include <vector>

#include "cgx_internal.h"

namespace cgx {

struct DevMatrix {
  int device = 0;
  hipStream_t st = nullptr;  // setup stream (owner's)
  int dtype = CGX_F64;
  int n = 0, nnz = 0;
  int ncols = 0;             // columns of x (n, or n_loc + ghosts when partitioned)
  // lowest column (0; a partition's in-place numbering: -(ghost rows below),
  // columns = global - row_begin, DIA only)
  int col_lo = 0;
  int layout = L_CSR;
  bool nt = false;           // matrix stream + y store non-temporal
  size_t dev_bytes = 0;
  // CSR (CSR / DC / panels; panels: P row_ptrs back to back, panel-major col/val)
  int *d_rp = nullptr, *d_col = nullptr;
  void *d_val = nullptr;
  // CSR / DC row blocks
  int *d_blkrk = nullptr;
  int nblk = 0, capw = 512;
  std::vector<int> blk_row;  // host: first row of each block, nblk + 1 entries
  int npanel = 1;
  std::vector<int> panel_first, panel_count;
  // DC
  unsigned char *d_code = nullptr, *d_rlen = nullptr;
  int *d_dict = nullptr;
  int ndict = 0;
  // DIA
  unsigned char *d_dcode = nullptr;  // per row dia.cbytes bytes of packed value indices
  void *d_vtab = nullptr;       // [16][16] values
  // DIA-V (general coefficients on <= kDiaVMax diagonals; upload's
  // allow_dv): the values diagonal-major, [ndiag][padded rows]; nullptr:
  // DIA-VI
  void *d_dval = nullptr;
  bool dv() const { return d_dval != nullptr; }
  DiaCand dia{};
  int kdiag = -1;               // main diagonal's index, -1: none
  int gath = 8;                 // CSR / DC: gathers per row chunk
  // L2-tiled order of the work items (DC / DIA / banded CSR, wide stencils;
  // nullptr: natural)
  int *d_order = nullptr;
  std::vector<int> order;    // host copy of the tiled order (empty: natural)
  int tile_bands = 0;
  long long csr_reach = 0;   // CSR: largest |col - row| of a banded matrix (0: not banded)
  // stencil
  LapSpec lap{};
  // setup record
  double setup_host_ms = 0, setup_dev_ms = 0;
  int encode_fallback = 0;   // 1: a sampled candidate set missed, exact host scan used

  // Host CSR -> device.  want: CGX_LAYOUT_* request (a layout that does not
  // apply falls back along DIA -> DC -> CSR).  ncols: columns of x (>= n for
  // the partitioned solver's ghost tail).  gen: col/val generated on the
  // device (rp is the host closed form).  allow_panels: single-GPU only.
  // col_lo < 0: columns in [col_lo, ncols) (a partition's in-place ghost
  // rows); DIA-VI only -- CGX_EINVAL when it does not apply.
  // allow_dv: DIA-V may be built (the single-GPU solver; a partition's
  // in-place matrix for the one-launch SR step)
  template <typename T>
  int upload(int n, int ncols, int nnz, const int *rp, const int *col, const T *val, int want,
             bool allow_panels, const LapSpec *gen = nullptr, int col_lo = 0,
             bool allow_dv = false);
  int finish_upload(double t0);
  int set_stencil(const LapSpec &g);
  // The matrix as CSR on the host (fp64; DIA decodes its codes).
  int download_csr(int *row_ptr, int *col, double *val) const;
  void release();

  int items() const;  // work items of the layout (blocks or slices)
  // host: first row of each item, items() + 1 entries
  std::vector<int> item_rows() const;
  // The fused HS step applies (DIA, <= 4 code bytes per row, at most 4
  // far diagonals, |d| > kHaloMax): k_spmv_dia_h's window and far slots.
  // sr1: the one-launch SR step (k_sr1_dia_m), which also runs on DIA-V.
  bool fusable(bool sr1 = false) const;
  // why not: 0 fusable, else CGX_FUSE_STATUS_NOT_DIA / _WIDE_CODES /
  // _FAR_DIAGS / _VALUE_STREAM
  int fuse_block(bool sr1 = false) const;
  bool near_diag(int k) const;  // read from k_spmv_dia_h's LDS window
  // rows covered by the items (DIA pads to whole 512-row slices)
  int padded_rows() const;
  // algorithmic HBM bytes of one SpMV in the layout it runs on
  double layout_bytes() const;
  // CSR-basis algorithmic bytes (SURVEY.md 8d B_spmv)
  double csr_bytes() const;

  template <typename T>
  SpmvArgs<T> args(const T *x, T *y, double *part, const int *done, Items it) const;
  // the fused step's super-items of the tiled order (d_order's adjacent pairs)
  int *d_fpairs = nullptr;
  int n_fpairs = 0;
  // plane march of the fused step (k_spmv_dia_m): chain stride mq slices
  // (0: no march), msb slices per super-item, mchains chains, LDS ring slot
  // stride mws, mlen steps per segment (the default), d_mpos: slice ->
  // position in d_order (nullptr: natural order)
  int mq = 0, msb = 1, mchains = 0, mws = 0, mlen = 0;
  // 1: the plan marches across far diagonals (+-F from the ring); 0 with mq >
  // 0: a near-only plan (every diagonal within the window's halo: 2-D grids,
  // small planes) -- steps mq slices apart share nothing, only the one-launch
  // SR step (single GPU) runs it
  int mfar = 0;
  int *d_mpos = nullptr;
  int plan_march();
  Items all_items() const { return Items{d_order, 0, items(), d_fpairs, n_fpairs}; }
  // One SpMV (panels: one launch per panel, rows continuing their sums;
  // the epilogue partials on the last panel).  Returns the partial count.
  // ev: timing events around the whole SpMV (start on its first launch,
  // stop on its last).  pair: (p.s, s.s) pairs instead of p.s partials
  // (SpmvArgs::pair; 2 doubles per partial).
  template <typename T>
  hipError_t spmv(const T *x, T *y, double *part, const int *done, Items it, hipStream_t s,
                  int *nparts = nullptr, LaunchEv ev = LaunchEv{}, bool pair = false) const;
  // The number of partials spmv() writes for the given items.
  int partials(Items it) const;
};

// Row-block plan: consecutive rows, at most `rows` rows and `cap` nonzeros
// per block; a row longer than `cap` gets a block of its own.
std::vector<int> plan_rowblocks(int n, const int *rp, int rows, int cap);

}  // namespace cgx
