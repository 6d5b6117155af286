// cgx_solver.cpp -- device-resident CG solver: HIP-stream orchestration of the
// iteration that replaces conj_grad's loop (rnelias/Conjugate-Gradient
// cg.c:88-141).  The whole recurrence state (alpha, beta, r.r, k, stop flag)
// lives on the device in a CgState, so an iteration is a fixed sequence of
// kernel launches with no host round trip; batches of iterations are replayed
// as hipGraphs, and the host only polls the stop flag between batches when a
// tolerance is set.
//
// Per HS iteration (the reference's recurrence; fast mode):
//   SpMV        s = A p, p.s partials                    cg.c:111 (+113 partials)
//   k_update_rf alpha = r.r / p.s; r -= alpha s; r.r partials   cg.c:113, 118-123
//   k_xpay_xf   beta, stop test; x += alpha p; p = r + beta p   cg.c:115-116, 125-132
// Exact mode replaces the partial sums by the reference's sequential dot
// products (k_dot_seq) and keeps the reference's update order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cgx_internal.h"
#include "cgx_matrix.h"

using cgx::CgState;
using cgx::DevMatrix;

namespace cgx {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

int check_device(int device, int *cus) {
  int cnt = 0;
  hipError_t e = hipGetDeviceCount(&cnt);
  if (e != hipSuccess || cnt == 0) {
    set_error("no HIP device available (%s)",
              e != hipSuccess ? hipGetErrorString(e) : "device count is 0");
    return CGX_ENODEV;
  }
  if (device < 0 || device >= cnt) {
    set_error("device %d out of range (%d devices)", device, cnt);
    return CGX_EINVAL;
  }
  hipDeviceProp_t prop;
  CGX_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("device %d is %s; libcgx is built for gfx950 (MI355X) only", device,
              prop.gcnArchName);
    return CGX_ENODEV;
  }
  if (cus) *cus = prop.multiProcessorCount;
  return 0;
}

int dev_alloc(void **p, size_t bytes, size_t *counter) {
  if (bytes == 0) bytes = 16;
  void *raw = nullptr;
  const size_t total = bytes + kGuardBytes;
  hipError_t e = hipExtMallocWithFlags(&raw, total, hipDeviceMallocContiguous);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipMalloc(&raw, total);
  }
  if (e == hipSuccess) e = hipMemset(raw, 0, kGuardBytes);  // the guard reads as 0.0
  if (e != hipSuccess) {
    set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    if (raw) (void)hipFree(raw);
    *p = nullptr;
    return CGX_ENOMEM;
  }
  *p = (char *)raw + kGuardBytes;
  if (counter) *counter += total;
  return 0;
}

void dev_free_raw(void *p) {
  if (p) (void)hipFree((char *)p - kGuardBytes);
}

int vec_grid_for(int n, int cus) {
  const long long vecs = (n + 1) / 2;
  long long g = (vecs + kVecBS - 1) / kVecBS;
  const long long cap = (long long)cus * 4;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

int public_layout(const DevMatrix &m) {
  switch (m.layout) {
    case L_DIA: return CGX_LAYOUT_DIA;
    case L_DC: return CGX_LAYOUT_DC;
    case L_STENCIL: return CGX_LAYOUT_STENCIL;
    default: return m.npanel > 1 ? CGX_LAYOUT_PANEL : CGX_LAYOUT_CSR;
  }
}

}  // namespace cgx

// ----------------------------------------------------------------- solver

struct cgx_solver {
  int device = 0;
  int cus = 256;
  hipStream_t stream = nullptr;
  int mode = CGX_MODE_FAST, alg = CGX_ALG_HS;
  int want_layout = CGX_LAYOUT_AUTO;
  DevMatrix A;
  int vec_grid = 0;
  int graph_batch = 16;
  bool use_graph = true;
  void *d_b = nullptr, *d_x = nullptr, *d_r = nullptr, *d_p = nullptr, *d_s = nullptr,
       *d_w = nullptr;
  void *d_p2 = nullptr;  // fused step: the second p buffer (p_old / p_new alternate)
  // fused CG1 step: the second r, s, w buffers (read one set, write the other)
  void *d_r2 = nullptr, *d_s2 = nullptr, *d_w2 = nullptr;
  int pbuf = 0;          // fused step: which buffer holds p_old (0: d_p) / r, s, w_old
  int fuse = CGX_FUSE_AUTO;  // cgx_solver_set_fused
  int march = -1;            // cgx_solver_set_march: -1 auto, 0 off, > 0 steps per segment
  int sr_chain = 0;          // cgx_solver_set_sr_chain: 0 auto, > 0 chain width (rows)
  unsigned *d_tick = nullptr;  // last-arriver counter of k_update_rf's r.r sum
  double *d_pa = nullptr, *d_pb = nullptr;
  double *d_pr2 = nullptr;   // unfused SR: the second r.r partial buffer
  void *d_p3 = nullptr, *d_p4 = nullptr;  // the one-launch SR step's third / fourth p
  int part_cap = 0;
  CgState *d_st = nullptr, *h_st = nullptr;
  double *d_hist = nullptr;
  int hist_alloc = 0;
  size_t vec_bytes = 0;
  bool have_matrix = false, have_rhs = false, bench_ready = false;
  int last_iters = 0;
  hipGraphExec_t gexec[4] = {};   // graph_batch iterations, per p-buffer rotation
  hipGraphExec_t gexec1[4] = {};  // one iteration (remainders), per rotation
  int gexec_key = -1;
  std::vector<hipEvent_t> events;
};

namespace {

using namespace cgx;

size_t tsize(int dtype) { return dtype == CGX_F32 ? 4 : 8; }

void drop_graph(cgx_solver *s) {
  for (int q = 0; q < 4; ++q) {
    if (s->gexec[q]) (void)hipGraphExecDestroy(s->gexec[q]);
    if (s->gexec1[q]) (void)hipGraphExecDestroy(s->gexec1[q]);
    s->gexec[q] = s->gexec1[q] = nullptr;
  }
  s->gexec_key = -1;
}

// The fused step (HS: k_spmv_dia_h + k_update_rf; CG1: k_cg1_dia_h +
// k_finalize) applies: fast mode, a fusable DIA layout and, in auto mode, a
// working set beyond the Infinity Cache (cache-resident systems are launch-
// and latency-bound: the heavier fused workgroup loses, C2 29.1 vs 26.8 us
// per HS iteration).
// CGX_ALG_SR on one GPU exists only as the single-launch plane march
// (k_sr1_dia_m): it needs a march plan, whatever the cache rule says.
bool fused(const cgx_solver *s) {
  if (s->alg == CGX_ALG_SR)
    return s->fuse != CGX_FUSE_OFF && s->mode == CGX_MODE_FAST && s->A.fusable(true) &&
           s->A.mq > 0 && s->march != 0;
  return s->fuse != CGX_FUSE_OFF && s->mode == CGX_MODE_FAST && s->A.fusable() &&
         (s->fuse == CGX_FUSE_ON || s->A.nt);
}

// Steps per segment of the fused HS step's plane march (k_spmv_dia_m), 0
// when it does not run: the matrix plans one (DevMatrix::plan_march) and
// cgx_solver_set_march has not turned it off.
int march_len(const cgx_solver *s) {
  if (!fused(s) || s->alg == CGX_ALG_CG1 || s->A.mq == 0 || s->march == 0) return 0;
  // a near-only plan (DevMatrix::mfar 0) is the one-launch SR step's alone
  if (!s->A.mfar && s->alg != CGX_ALG_SR) return 0;
  return s->march > 0 ? s->march : s->A.mlen;
}

// Buffers alternating per iteration: p for the fused HS step and the
// unfused folded HS step (k_xpay_xf's every-other-iteration x); r, s, w for
// the fused CG1 step.
bool alternating(const cgx_solver *s) {
  return (s->alg != CGX_ALG_CG1 && s->mode == CGX_MODE_FAST) || fused(s);
}

// The one-launch SR step defers x four iterations deep (round 5: x, p_{k-3},
// p_{k-2}, p_{k-1} read and x written in every fourth launch -- 10 B per row
// and iteration instead of 12; CgState::xdef): four p buffers rotate, p_i in
// buffer (i + 1) % 4.  Other recurrences alternate two (or keep one).
// Same box, alternating (profiles/r05_ab_sr_x4.log): C4 711.3-711.9 against
// 739.0 us per iteration (launch 694 against 730), C3 134.4-135.9 against
// 139.4-140.1.
bool sr_x4(const cgx_solver *s) { return fused(s) && s->alg == CGX_ALG_SR; }
// The one-launch SR step runs its scalar step folded into the next launch
// (round 6): no k_finalize between the launches; each launch
// sums the last one's (p.s, s.s) pairs and r.r partials under its
// prologue's window loads, and two CgState slots alternate (the launch
// reads one and hands the state over in the other).  Same box, alternating
// (profiles/r06_ab_sr1.log, box 5): C3 131.3-132.4 against 134.1-135.4 us
// per iteration, C4 even (712.7-713.2 against 710.0-718.3).
bool sr1_fold(const cgx_solver *s) { return sr_x4(s); }

int prot(const cgx_solver *s) { return sr_x4(s) ? 4 : alternating(s) ? 2 : 1; }

void free_system(cgx_solver *s) {
  drop_graph(s);
  s->A.release();
  dev_free(&s->d_b);
  dev_free(&s->d_x);
  dev_free(&s->d_r);
  dev_free(&s->d_p);
  dev_free(&s->d_s);
  dev_free(&s->d_w);
  dev_free(&s->d_p2);
  dev_free(&s->d_r2);
  dev_free(&s->d_s2);
  dev_free(&s->d_w2);
  dev_free(&s->d_pa);
  dev_free(&s->d_pb);
  dev_free(&s->d_pr2);
  dev_free(&s->d_p3);
  dev_free(&s->d_p4);
  dev_free(&s->d_hist);
  s->hist_alloc = 0;
  s->vec_bytes = 0;
  s->have_matrix = s->have_rhs = s->bench_ready = false;
}

// Vectors and partial buffers for the loaded matrix.
int alloc_vectors(cgx_solver *s) {
  const int n = s->A.n;
  const size_t nv = ((size_t)n + kPad) * tsize(s->A.dtype);
  s->vec_grid = vec_grid_for(n, s->cus);
  s->vec_grid = (std::max(s->vec_grid, 1) + 3) / 4 * 4;  // folded kernels: 4 x 256 threads
  s->part_cap = std::max(s->A.partials(s->A.all_items()), s->vec_grid) + 1;
  // CGX_ALG_SR: one (p.s, s.s) pair per march workgroup, at most
  // kSr1MaxGrid(items) (sr1_pick_shape keeps chains x segments within it)
  // (folded scalar step: two sets of pairs and r.r partials, 3 per workgroup)
  if (s->A.mq > 0) s->part_cap = std::max(s->part_cap, 3 * sr1_max_grid(s->A.items()) + 2);
  // unfused CGX_ALG_SR: the SpMV's (p.s, s.s) pair per workgroup
  s->part_cap = std::max(s->part_cap, 2 * s->A.partials(s->A.all_items()) + 2);
  int rc;
  if ((rc = dev_alloc(&s->d_b, nv, &s->vec_bytes)) || (rc = dev_alloc(&s->d_x, nv, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_r, nv, &s->vec_bytes)) || (rc = dev_alloc(&s->d_p, nv, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_s, nv, &s->vec_bytes)) || (rc = dev_alloc(&s->d_w, nv, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_p2, nv, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_pa, (size_t)s->part_cap * 8, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_pb, (size_t)s->part_cap * 8, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_pr2, (size_t)s->part_cap * 8, &s->vec_bytes))) {
    free_system(s);
    return rc;
  }
  // padding entries stay 0 (16-B vector loads read them)
  CGX_HIP(hipMemsetAsync(s->d_x, 0, nv, s->stream));
  CGX_HIP(hipMemsetAsync(s->d_p, 0, nv, s->stream));
  CGX_HIP(hipMemsetAsync(s->d_p2, 0, nv, s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  s->have_matrix = true;
  return 0;
}

// The second r, s (and w) buffers exist only while a recurrence that reads
// one set and writes the other runs (SR's one launch, the fused CG1 step):
// 3 n vectors HS never touches (1.5 GB at C4).  Allocated before
// the prologue and the graph capture of such a run.
bool needs_rsw2(const cgx_solver *s) {
  return fused(s) && (s->alg == CGX_ALG_SR || s->alg == CGX_ALG_CG1);
}

int ensure_rsw2(cgx_solver *s) {
  const size_t nv = ((size_t)s->A.n + kPad) * tsize(s->A.dtype);
  int rc;
  if (sr_x4(s) && !s->d_p3) {  // the one-launch SR step's four p buffers
    if ((rc = dev_alloc(&s->d_p3, nv, &s->vec_bytes)) || (rc = dev_alloc(&s->d_p4, nv, &s->vec_bytes))) {
      dev_free(&s->d_p3);
      dev_free(&s->d_p4);
      return rc;
    }
    for (void *v : {s->d_p3, s->d_p4}) CGX_HIP(hipMemsetAsync(v, 0, nv, s->stream));
  }
  if (!needs_rsw2(s) || s->d_r2) return 0;
  if ((rc = dev_alloc(&s->d_r2, nv, &s->vec_bytes)) || (rc = dev_alloc(&s->d_s2, nv, &s->vec_bytes)) ||
      (rc = dev_alloc(&s->d_w2, nv, &s->vec_bytes))) {
    dev_free(&s->d_r2);
    dev_free(&s->d_s2);
    dev_free(&s->d_w2);
    return rc;
  }
  for (void *v : {s->d_r2, s->d_s2, s->d_w2}) CGX_HIP(hipMemsetAsync(v, 0, nv, s->stream));
  return 0;
}

// A recurrence the loaded matrix cannot run is refused before anything is
// enqueued.  (CGX_ALG_SR runs on every layout since round 5: the one-launch
// plane march where the matrix plans one, else the unfused two-launch step
// -- SpMV with (p.s, s.s) pairs, then k_update_sr.)
int check_runnable(const cgx_solver *s) {
  if (s->alg == CGX_ALG_SR && s->mode != CGX_MODE_FAST) {
    set_error("CGX_ALG_SR is defined in fast mode only");
    return CGX_EINVAL;
  }
  return 0;
}

template <typename T>
int upload_matrix(cgx_solver *s, int n, int nnz, const int *rp, const int *col, const T *val,
                  const LapSpec *gen = nullptr) {
  CGX_HIP(hipSetDevice(s->device));
  free_system(s);
  int rc = s->A.upload<T>(n, n, nnz, rp, col, val, s->want_layout, true, gen, 0, true);
  if (rc) return rc;
  return alloc_vectors(s);
}

template <typename T>
int upload_rhs(cgx_solver *s, const T *b) {
  if (!s->have_matrix || (s->A.n > 0 && !b)) {
    set_error("set_rhs: no matrix loaded or NULL b");
    return CGX_EINVAL;
  }
  if ((sizeof(T) == 4) != (s->A.dtype == CGX_F32)) {
    set_error("set_rhs: dtype does not match the matrix");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  if (s->A.n > 0)
    CGX_HIP(hipMemcpy(s->d_b, b, (size_t)s->A.n * sizeof(T), hipMemcpyHostToDevice));
  s->have_rhs = true;
  return 0;
}

// Prologue: x = 0, r = b, p = b (HS) / p = s = 0, w = A r (CG1); b.b; state.
template <typename T>
int enqueue_init(cgx_solver *s) {
  hipStream_t st = s->stream;
  const int n = s->A.n;
  T *b = (T *)s->d_b, *x = (T *)s->d_x, *r = (T *)s->d_r, *p = (T *)s->d_p;
  s->pbuf = 0;  // the prologue writes p into d_p
  if (s->alg != CGX_ALG_CG1) {  // HS, SR: x = 0, r = p = b
    if (s->mode == CGX_MODE_EXACT) {
      CGX_HIP(launch_init_hs<T>(n, b, x, r, p, nullptr, s->vec_grid, st));
      CGX_HIP(launch_dot_seq<T>(n, b, b, s->d_pa, nullptr, st));
      CGX_HIP(launch_finalize(FIN_INIT_HS, s->d_pa, 1, nullptr, 0, s->d_st, s->d_hist, nullptr, st));
    } else {
      CGX_HIP(launch_init_hs<T>(n, b, x, r, p, s->d_pa, s->vec_grid, st));
      CGX_HIP(launch_finalize(FIN_INIT_HS, s->d_pa, s->vec_grid, nullptr, 0, s->d_st, s->d_hist,
                              nullptr, st));
    }
  } else {
    int np = 0;
    CGX_HIP(launch_init_cg1<T>(n, b, x, r, p, (T *)s->d_s, s->d_pa, s->vec_grid, st));
    CGX_HIP(s->A.spmv<T>(r, (T *)s->d_w, s->d_pb, nullptr, s->A.all_items(), st, &np));
    CGX_HIP(launch_finalize(FIN_INIT_CG1, s->d_pa, s->vec_grid, s->d_pb, np, s->d_st, s->d_hist,
                            nullptr, st));
  }
  return 0;
}

// The one-launch SR step's shape: set_march's length as given, else the
// balanced segment count; the chain width set_sr_chain gives, or the picked
// one (with the step width it needs)
template <typename T>
void sr1_shape(const cgx_solver *s, const SpmvArgs<T> &a, Sr1Args<T> &f) {
  const Sr1Shape sh = sr1_pick_shape(a, s->cus, s->sr_chain, true);
  if (s->march <= 0) f.nseg = sh.nseg;
  if (s->march <= 0 || s->sr_chain > 0) {
    f.cw = sh.cw;
    f.sb = sh.sb;
  }
}

// One CG iteration.  ev0/ev1 (optional): the SpMV kernel's start / end.
template <typename T>
int enqueue_iter(cgx_solver *s, hipEvent_t ev0, hipEvent_t ev1) {
  hipStream_t st = s->stream;
  const int n = s->A.n;
  T *x = (T *)s->d_x, *r = (T *)s->d_r, *p = (T *)s->d_p, *sv = (T *)s->d_s, *w = (T *)s->d_w;
  int np = 0;
  if (s->alg == CGX_ALG_SR && !fused(s)) {
    // unfused SR (any layout): s = A p with the (p.s, s.s) pair per
    // workgroup (cg.c:111), then k_update_sr with FIN_SR1 folded in (alpha
    // cg.c:113, the estimate's beta cg.c:129, the stop test of the previous
    // iteration on the exact r.r; round 5: no k_finalize launch between):
    // r, p, x of the iteration in one pass (cg.c:115-132) + the exact r.r
    // partials -- two launches and one reduction per iteration
    // (oracle_solve_sr)
    const int q = s->pbuf;
    T *pc = (T *)(q ? s->d_p2 : s->d_p), *pn = (T *)(q ? s->d_p : s->d_p2);
    CGX_HIP(s->A.spmv<T>(pc, sv, s->d_pb, &s->d_st->done, s->A.all_items(), st, &np,
                         LaunchEv{ev0, ev1}, true));
    if (2 * np > s->part_cap) return CGX_EINVAL;
    // FIN_SR1 folded into the update (round 5): its r.r partials alternate
    // between d_pa (the init's) and d_pr2
    double *rr_in = q ? s->d_pr2 : s->d_pa, *rr_out = q ? s->d_pa : s->d_pr2;
    const SrFold fo{s->d_pb, np, rr_in, s->vec_grid, s->d_tick, s->d_hist};
    CGX_HIP(launch_update_sr<T>(n, x, r, sv, pc, pn, s->d_st, nullptr, rr_out, s->vec_grid / 4,
                                st, s->A.nt, &fo));
    s->pbuf ^= 1;
    return 0;
  }
  if (s->alg == CGX_ALG_SR) {
    // k_sr1_dia_m: the scalar step of the last launch (FIN_SR1's:
    // oracle_solve_sr's recurrence, one reduction), r = r - alpha s, p = r +
    // beta p (window rows), x update, s = A p, (p.s, s.s) pairs + r.r per
    // workgroup -- ONE launch per iteration
    // p rotates over four buffers (sr_x4: p_{k-3}, p_{k-2}, p_{k-1} in pn,
    // pa, pb) or alternates over two; r and s alternate
    const int q = s->pbuf, rq = q & 1;
    T *pb4[4] = {(T *)s->d_p, (T *)s->d_p2, (T *)s->d_p3, (T *)s->d_p4};
    const int nr = sr_x4(s) ? 4 : 2;
    T *po = pb4[q % nr], *pn = pb4[(q + 1) % nr];
    T *ro = (T *)(rq ? s->d_r2 : s->d_r), *rn = (T *)(rq ? s->d_r : s->d_r2);
    T *so = (T *)(rq ? s->d_s2 : s->d_s), *sn = (T *)(rq ? s->d_s : s->d_s2);
    const SpmvArgs<T> a = s->A.args<T>(nullptr, sn, nullptr, &s->d_st->done, s->A.all_items());
    Sr1Args<T> f{x, po, pn, ro, rn, so, s->d_st, s->d_pa, s->d_pb, march_len(s)};
    if (nr == 4) {
      if (!pb4[2] || !pb4[3]) return CGX_EINVAL;
      f.pa = pb4[(q + 2) & 3];
      f.pb = pb4[(q + 3) & 3];
    }
    sr1_shape(s, a, f);
    const int g = sr1_grid(a, f);
    if (3 * g > s->part_cap) return CGX_EINVAL;
    // the scalar step folded into the next launch (sr1_fold): launch q reads
    // state slot q & 1 and the other parity's partials, writes its own
    // partials and hands the state over in slot (q + 1) & 1
    const int par = q & 1;
    double *pq[2] = {s->d_pa, s->d_pr2}, *pc[2] = {s->d_pb, s->d_pr2 + 2 * g};
    f.st = s->d_st + par;
    f.st_out = s->d_st + (par ^ 1);
    f.pq = pq[par];
    f.pc = pc[par];
    f.pq_in = pq[par ^ 1];
    f.pc_in = pc[par ^ 1];
    f.np_in = g;
    f.hist = s->d_hist;
    CGX_HIP(launch_sr1_march<T>(a, f, st, LaunchEv{ev0, ev1}));
    s->pbuf = (q + 1) % nr;
    return 0;
  }
  if (fused(s) && s->alg == CGX_ALG_CG1) {
    // k_cg1_dia_h: p, s, x, r recurrences + w = A r_new with the gamma /
    // delta partials; k_finalize: the single reduction's scalar step
    const int q = s->pbuf;
    T *ro = (T *)(q ? s->d_r2 : s->d_r), *rn = (T *)(q ? s->d_r : s->d_r2);
    T *so = (T *)(q ? s->d_s2 : s->d_s), *sn = (T *)(q ? s->d_s : s->d_s2);
    T *wo = (T *)(q ? s->d_w2 : s->d_w), *wn = (T *)(q ? s->d_w : s->d_w2);
    const SpmvArgs<T> a = s->A.args<T>(nullptr, wn, s->d_pb, &s->d_st->done, s->A.all_items());
    const Cg1Args<T> f{x, p, ro, so, wo, rn, sn, s->d_st, s->d_pa, 0};
    np = s->A.partials(s->A.all_items());
    CGX_HIP(launch_cg1_fused<T>(a, f, st, LaunchEv{ev0, ev1}));
    CGX_HIP(launch_finalize(FIN_CG1, s->d_pa, np, s->d_pb, np, s->d_st, s->d_hist, nullptr, st));
    s->pbuf ^= 1;
    return 0;
  }
  if (fused(s)) {
    // k_spmv_dia_h: the previous x / p update + s = A p_new (+ p_new.s
    // partials); k_update_rf: alpha, r -= alpha s, r.r partials and their
    // canonical sum (last workgroup) into st->rr_new for the next step
    // (cg.c:111-132)
    T *pold = (T *)(s->pbuf ? s->d_p2 : s->d_p), *pnew = (T *)(s->pbuf ? s->d_p : s->d_p2);
    const SpmvArgs<T> a = s->A.args<T>(nullptr, sv, s->d_pa, &s->d_st->done, s->A.all_items());
    FuseArgs<T> f{x, pold, pnew, r, s->d_st, s->d_hist, &s->d_st->rr_new, 1, 0, nullptr};
    f.march = march_len(s);
    np = s->A.partials(s->A.all_items());
    CGX_HIP(launch_spmv_fused<T>(a, f, st, LaunchEv{ev0, ev1}));
    const int gf = s->vec_grid / 4;
    const FinArgs fin{s->d_tick, s->d_pb, 4 * gf, &s->d_st->rr_new};
    CGX_HIP(launch_update_rf<T>(n, r, sv, s->d_st, s->d_pa, np, s->d_pb, gf, st, &fin));
    s->pbuf ^= 1;
    return 0;
  }
  if (s->alg == CGX_ALG_HS) {
    const bool exact = s->mode == CGX_MODE_EXACT;
    T *pn = p;  // exact mode: p in place
    if (alternating(s)) {
      p = (T *)(s->pbuf ? s->d_p2 : s->d_p);
      pn = (T *)(s->pbuf ? s->d_p : s->d_p2);
    }
    CGX_HIP(s->A.spmv<T>(p, sv, exact ? nullptr : s->d_pa, &s->d_st->done, s->A.all_items(), st,
                         &np, LaunchEv{ev0, ev1}));  // cg.c:111
    if (exact) {
      CGX_HIP(launch_dot_seq<T>(n, p, sv, s->d_pa, &s->d_st->done, st));
      CGX_HIP(launch_finalize(FIN_HS_ALPHA, s->d_pa, 1, nullptr, 0, s->d_st, s->d_hist, nullptr,
                              st));                                            // cg.c:113
      CGX_HIP(launch_update_xr<T>(n, x, p, r, sv, s->d_st, nullptr, s->vec_grid, st));  // :115-123
      CGX_HIP(launch_dot_seq<T>(n, r, r, s->d_pa, &s->d_st->done, st));
      CGX_HIP(launch_finalize(FIN_HS_BETA, s->d_pa, 1, nullptr, 0, s->d_st, s->d_hist, nullptr,
                              st));                                            // cg.c:125-129
      CGX_HIP(launch_xpay<T>(n, p, r, s->d_st, s->vec_grid, st));             // cg.c:131-132
    } else {
      const int gf = s->vec_grid / 4;  // 1024-thread workgroups, 4 partials each
      CGX_HIP(launch_update_rf<T>(n, r, sv, s->d_st, s->d_pa, np, s->d_pb, gf, st, nullptr,
                                  nullptr, nullptr, s->A.nt));
      CGX_HIP(launch_xpay_xf<T>(n, x, p, pn, r, s->d_st, s->d_pb, 4 * gf, s->d_hist, gf, st,
                                s->A.nt));
      s->pbuf ^= 1;
    }
  } else {
    CGX_HIP(launch_cg1_update<T>(n, x, p, r, sv, w, s->d_st, s->d_pa, s->vec_grid, st));
    CGX_HIP(s->A.spmv<T>(r, w, s->d_pb, &s->d_st->done, s->A.all_items(), st, &np,
                         LaunchEv{ev0, ev1}));
    CGX_HIP(launch_finalize(FIN_CG1, s->d_pa, s->vec_grid, s->d_pb, np, s->d_st, s->d_hist,
                            nullptr, st));
  }
  return 0;
}

template <typename T>
int capture_iters(cgx_solver *s, int count, int parity, hipGraphExec_t *out) {
  hipGraph_t g = nullptr;
  const int saved = s->pbuf;
  s->pbuf = parity;
  CGX_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  for (int i = 0; i < count && rc == 0; ++i) rc = enqueue_iter<T>(s, nullptr, nullptr);
  hipError_t e = hipStreamEndCapture(s->stream, &g);
  s->pbuf = saved;
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  CGX_HIP(e);
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  CGX_HIP(e);
  return 0;
}

// The replayed graphs of the current mode / recurrence: graph_batch
// iterations and one iteration (remainders), captured (not run) once -- for
// both p-buffer parities when the HS step alternates them (alternating()).
template <typename T>
int ensure_graphs(cgx_solver *s) {
  const int key = s->alg * 4 + s->mode * 2 + (fused(s) ? 1 : 0);
  const int nq = prot(s);
  if (s->gexec_key == key) return 0;
  drop_graph(s);
  int rc = 0;
  for (int q = 0; q < nq && rc == 0; ++q) {
    rc = capture_iters<T>(s, s->graph_batch, q, &s->gexec[q]);
    if (rc == 0) rc = capture_iters<T>(s, 1, q, &s->gexec1[q]);
  }
  if (rc) {
    drop_graph(s);
    return rc;
  }
  s->gexec_key = key;
  return 0;
}

template <typename T>
int enqueue_iters(cgx_solver *s, long long count) {
  if (s->use_graph && count > 0) {
    int rc = ensure_graphs<T>(s);
    if (rc) return rc;
    // the graph captured at the current buffer rotation; a batch advances
    // it by graph_batch, one iteration by one
    const int nr = prot(s);
    for (; count >= s->graph_batch; count -= s->graph_batch) {
      CGX_HIP(hipGraphLaunch(s->gexec[s->pbuf % nr], s->stream));
      s->pbuf = (s->pbuf + s->graph_batch) % nr;
    }
    for (; count > 0; --count) {
      CGX_HIP(hipGraphLaunch(s->gexec1[s->pbuf % nr], s->stream));
      s->pbuf = (s->pbuf + 1) % nr;
    }
    return 0;
  }
  for (long long i = 0; i < count; ++i) {
    int rc = enqueue_iter<T>(s, nullptr, nullptr);
    if (rc) return rc;
  }
  return 0;
}

}  // namespace

namespace cgx {

long long next_batch(double rr, double tol2bb, int k, double rr_prev, int k_prev, long long batch) {
  // iterations still needed if r.r keeps decaying at the rate seen since the
  // last poll, +25% and 4 of slack; 16..256, at most doubling per poll
  long long want = std::min<long long>(batch * 2, 256);
  if (k_prev >= 0 && k > k_prev && rr_prev > 0.0 && rr > 0.0 && rr < rr_prev && tol2bb > 0.0) {
    const double per_it = std::log(rr / rr_prev) / (double)(k - k_prev);  // < 0
    const double need = std::log(tol2bb / rr) / per_it;                    // >= 0 when rr > tol2bb
    if (std::isfinite(need) && need >= 0.0)
      want = std::min(want, (long long)(need * 1.25) + 4);
  }
  return std::max<long long>(16, want);
}

}  // namespace cgx

namespace {

int prepare_state(cgx_solver *s, int maxit, double tol, int hist_cap) {
  if (hist_cap > s->hist_alloc) {
    drop_graph(s);  // captured graphs hold the old history pointer
    CGX_HIP(hipStreamSynchronize(s->stream));
    dev_free(&s->d_hist);
    int rc = dev_alloc(&s->d_hist, (size_t)hist_cap * 8, nullptr);
    if (rc) return rc;
    s->hist_alloc = hist_cap;
  }
  memset(s->h_st, 0, sizeof(CgState));
  s->h_st->tol = tol;
  s->h_st->use_tol = tol > 0.0 ? 1 : 0;
  s->h_st->max_iter = maxit;
  s->h_st->hist_cap = std::min(hist_cap, s->hist_alloc);
  s->h_st->xdef = sr_x4(s) ? 4 : 2;
  CGX_HIP(hipMemcpyAsync(s->d_st, s->h_st, sizeof(CgState), hipMemcpyHostToDevice, s->stream));
  CGX_HIP(hipMemsetAsync(s->d_tick, 0, kTickRegion * sizeof(unsigned), s->stream));
  return 0;
}

int read_state(cgx_solver *s) {
  // the folded SR step: the state the next launch reads (slot pbuf & 1)
  const CgState *cur = s->d_st + (sr1_fold(s) ? (s->pbuf & 1) : 0);
  CGX_HIP(hipMemcpyAsync(s->h_st, cur, sizeof(CgState), hipMemcpyDeviceToHost, s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  return 0;
}

template <typename T>
int run_t(cgx_solver *s, int maxit, double tol, int *iters) {
  int rc;
  s->bench_ready = false;
  if ((rc = check_runnable(s)) || (rc = ensure_rsw2(s))) return rc;
  if ((rc = prepare_state(s, maxit, tol, maxit + 1))) return rc;
  if ((rc = enqueue_init<T>(s))) return rc;
  // the fused step does an iteration's x update in the next launch: one
  // more step carries the last one (and finds the stop); SR tests the stop
  // of iteration k on the exact r.r that launch k + 1 computes: one more
  // (the folded SR step: the launch after the finalize's would-be place
  // runs it -- one more)
  const long long total = (long long)maxit + 1 + (fused(s) && s->alg != CGX_ALG_CG1 ? 1 : 0) +
                          (s->alg == CGX_ALG_SR ? 1 : 0) + (sr1_fold(s) ? 1 : 0);
  // SR: complete once the finalize after the last x update marks done = 2
  const int fin_done = s->alg == CGX_ALG_SR ? 2 : 1;
  if (tol <= 0.0) {
    if ((rc = enqueue_iters<T>(s, total))) return rc;
    if ((rc = read_state(s))) return rc;
  } else {
    // poll the stop flag between batches; iterations after the stop
    // early-exit on the device flag, so the count is exactly the
    // reference's.  The batch follows the residual's observed decay rate
    // (next_batch), so few launches run past the stop.
    long long done_iters = 0, batch = 16;
    double rr_prev = 0.0;
    int k_prev = -1;
    for (;;) {
      const long long b = std::min(batch, total - done_iters);
      if ((rc = enqueue_iters<T>(s, b))) return rc;
      done_iters += b;
      if ((rc = read_state(s))) return rc;
      if (s->h_st->done >= fin_done || done_iters >= total) break;
      batch = next_batch(s->h_st->rr, s->h_st->tol2bb, s->h_st->k, rr_prev, k_prev, batch);
      rr_prev = s->h_st->rr;
      k_prev = s->h_st->k;
    }
  }
  if (!s->h_st->done) {
    set_error("solver did not reach its stop condition");
    return CGX_ENODEV;
  }
  s->last_iters = s->h_st->k + 1;
  if (iters) *iters = s->last_iters;
  return 0;
}

template <typename T>
int bench_prepare_t(cgx_solver *s, int warmup) {
  int rc;
  if ((rc = check_runnable(s)) || (rc = ensure_rsw2(s))) return rc;
  if ((rc = prepare_state(s, INT_MAX - 1, 0.0, 0))) return rc;
  if ((rc = enqueue_init<T>(s))) return rc;
  if ((rc = ensure_graphs<T>(s))) return rc;  // captured here, not in a timed region
  if ((rc = enqueue_iters<T>(s, warmup))) return rc;
  CGX_HIP(hipStreamSynchronize(s->stream));
  s->bench_ready = true;
  return 0;
}

template <typename T>
int bench_run_t(cgx_solver *s, int iters, int flags, double *total_ms, double *spmv_ms) {
  const bool per_spmv = (flags & CGX_BENCH_SPMV_EVENTS) != 0;
  const bool spmv_only = (flags & CGX_BENCH_SPMV_ONLY) != 0;
  const size_t need = 2 + (per_spmv ? 2 * (size_t)iters : 0);
  while (s->events.size() < need) {
    hipEvent_t e;
    CGX_HIP(hipEventCreate(&e));
    s->events.push_back(e);
  }
  hipEvent_t e0 = s->events[0], e1 = s->events[1];
  const bool graph_saved = s->use_graph;
  s->use_graph = (flags & CGX_BENCH_GRAPH) != 0;
  int rc = 0;
  CGX_HIP(hipEventRecord(e0, s->stream));
  if (spmv_only) {
    // back-to-back SpMVs y = A p (the standard SpMV benchmark), no iteration
    // and no epilogue partials: the plain y = A x kernel
    for (int i = 0; i < iters && !rc; ++i) {
      LaunchEv ev;
      if (per_spmv) ev = LaunchEv{s->events[2 + 2 * i], s->events[3 + 2 * i]};
      CGX_HIP(s->A.spmv<T>((T *)s->d_p, (T *)s->d_w, nullptr, nullptr, s->A.all_items(),
                           s->stream, nullptr, ev));
    }
  } else if (per_spmv) {
    for (int i = 0; i < iters && !rc; ++i)
      rc = enqueue_iter<T>(s, s->events[2 + 2 * i], s->events[3 + 2 * i]);
  } else {
    rc = enqueue_iters<T>(s, iters);
  }
  s->use_graph = graph_saved;
  if (rc) return rc;
  CGX_HIP(hipEventRecord(e1, s->stream));
  CGX_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  CGX_HIP(hipEventElapsedTime(&ms, e0, e1));
  *total_ms = ms;
  *spmv_ms = -1.0;
  if (per_spmv) {
    double sum = 0.0;
    for (int i = 0; i < iters; ++i) {
      float m = 0.f;
      CGX_HIP(hipEventElapsedTime(&m, s->events[2 + 2 * i], s->events[3 + 2 * i]));
      sum += m;
    }
    *spmv_ms = iters > 0 ? sum / iters : 0.0;
  }
  if ((rc = read_state(s))) return rc;
  if (s->h_st->done) {
    set_error("bench: solver stopped early");
    return CGX_EINVAL;
  }
  return 0;
}

template <typename T>
int spmv_t(cgx_solver *s, const T *x, T *y) {
  if (!s->have_matrix || (s->A.n > 0 && (!x || !y))) {
    set_error("spmv: no matrix or NULL vector");
    return CGX_EINVAL;
  }
  if ((sizeof(T) == 4) != (s->A.dtype == CGX_F32)) {
    set_error("spmv: dtype does not match the matrix");
    return CGX_EINVAL;
  }
  if (s->A.n == 0) return 0;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpyAsync(s->d_w, x, (size_t)s->A.n * sizeof(T), hipMemcpyHostToDevice,
                         s->stream));
  CGX_HIP(s->A.spmv<T>((const T *)s->d_w, (T *)s->d_s, nullptr, nullptr, s->A.all_items(),
                       s->stream));
  CGX_HIP(hipMemcpyAsync(y, s->d_s, (size_t)s->A.n * sizeof(T), hipMemcpyDeviceToHost,
                         s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  return 0;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" {

const char *cgx_last_error(void) { return cgx::g_err; }

int cgx_device_count(void) {
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess) return 0;
  return cnt;
}

int cgx_device_synchronize(int device) {
  int rc = check_device(device, nullptr);
  if (rc) return rc;
  CGX_HIP(hipSetDevice(device));
  CGX_HIP(hipDeviceSynchronize());
  return 0;
}

int cgx_stream_bench(int device, int kind, long long n, int reps, double *gbs) {
  int nr = 0, nw = 0;
  const bool rw = stream_rw_arrays(kind, &nr, &nw) == 0;
  if (!gbs || n < 2 || reps < 1 || (kind != CGX_STREAM_TRIAD && kind != CGX_STREAM_READ && !rw))
    return CGX_EINVAL;
  int cus = 256;
  int rc = check_device(device, &cus);
  if (rc) return rc;
  CGX_HIP(hipSetDevice(device));
  const long long n2 = n / 2;
  // arrays 4 KiB apart (each starts on its own page-aligned offset)
  const long long stride = (n2 + 255) / 256 * 256;
  const int narr = rw ? nr + nw : 3;
  double *buf = nullptr;
  if (hipMalloc((void **)&buf, (size_t)stride * 16 * narr) != hipSuccess) {
    set_error("stream_bench: out of device memory");
    return CGX_ENOMEM;
  }
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double *a = buf, *b = buf + 2 * stride, *c = buf + 4 * stride;
  float best = 1e30f;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMemsetAsync(buf, 0, (size_t)stride * 16 * narr, st);
  for (int r = -2; r < reps && e == hipSuccess; ++r) {  // two untimed warm-ups
    e = hipEventRecord(e0, st);
    if (e == hipSuccess)
      e = rw ? launch_stream_rw(kind, n2, stride, buf, cus, st)
          : kind == CGX_STREAM_TRIAD ? launch_triad(n2, a, b, c, cus * 16, st)
                                     : launch_stream_read(n2, b, a, cus * 16, st);
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && r >= 0) best = std::min(best, ms);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  (void)hipFree(buf);
  if (e != hipSuccess) {
    set_error("stream_bench: %s", hipGetErrorString(e));
    return CGX_ENODEV;
  }
  const double per = rw ? 16.0 * (nr + nw) : kind == CGX_STREAM_TRIAD ? 48.0 : 16.0;
  *gbs = per * (double)n2 / (best * 1e-3) / 1e9;
  return 0;
}

int cgx_solver_create(int device, cgx_solver **out) {
  if (!out) return CGX_EINVAL;
  *out = nullptr;
  int cus = 256;
  int rc = check_device(device, &cus);
  if (rc) return rc;
  CGX_HIP(hipSetDevice(device));
  cgx_solver *s = new cgx_solver();
  s->device = device;
  s->cus = cus;
  s->A.device = device;
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&s->d_st, 2 * sizeof(CgState)) != hipSuccess ||
      hipMalloc((void **)&s->d_tick, kTickRegion * sizeof(unsigned)) != hipSuccess ||
      hipMemset(s->d_tick, 0, kTickRegion * sizeof(unsigned)) != hipSuccess ||
      hipHostMalloc((void **)&s->h_st, sizeof(CgState), hipHostMallocDefault) != hipSuccess) {
    cgx::set_error("cgx_solver_create: stream/state allocation failed");
    cgx_solver_destroy(s);
    return CGX_ENODEV;
  }
  s->A.st = s->stream;
  *out = s;
  return 0;
}

void cgx_solver_destroy(cgx_solver *s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  free_system(s);
  for (hipEvent_t e : s->events) (void)hipEventDestroy(e);
  if (s->d_st) (void)hipFree(s->d_st);
  if (s->d_tick) (void)hipFree(s->d_tick);
  if (s->h_st) (void)hipHostFree(s->h_st);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

int cgx_solver_set_mode(cgx_solver *s, int mode, int alg) {
  if (!s || (mode != CGX_MODE_FAST && mode != CGX_MODE_EXACT) ||
      (alg != CGX_ALG_HS && alg != CGX_ALG_CG1 && alg != CGX_ALG_SR)) {
    cgx::set_error("set_mode: bad arguments");
    return CGX_EINVAL;
  }
  if (mode == CGX_MODE_EXACT && alg != CGX_ALG_HS) {
    cgx::set_error("exact mode is defined for the HS recurrence only");
    return CGX_EINVAL;
  }
  if (s->mode == mode && s->alg == alg) return 0;  // keeps the captured graphs
  s->mode = mode;
  s->alg = alg;
  drop_graph(s);
  s->bench_ready = false;  // the prepared state (buffers, prologue) was another recurrence's
  return 0;
}

int cgx_solver_set_fused(cgx_solver *s, int mode) {
  if (!s || mode < CGX_FUSE_OFF || mode > CGX_FUSE_ON) return CGX_EINVAL;
  if (s->fuse == mode) return 0;
  s->fuse = mode;
  drop_graph(s);
  s->bench_ready = false;
  return 0;
}

int cgx_solver_set_march(cgx_solver *s, int steps) {
  if (!s || steps < -1) return CGX_EINVAL;
  if (s->march == steps) return 0;
  s->march = steps;
  drop_graph(s);
  s->bench_ready = false;
  return 0;
}

int cgx_solver_set_sr_chain(cgx_solver *s, int rows) {
  if (!s || rows < 0) return CGX_EINVAL;
  if (s->sr_chain == rows) return 0;
  s->sr_chain = rows;
  drop_graph(s);
  s->bench_ready = false;
  return 0;
}

int cgx_solver_set_layout(cgx_solver *s, int layout) {
  if (!s || layout < CGX_LAYOUT_AUTO || layout > CGX_LAYOUT_PANEL) {
    cgx::set_error("set_layout: bad arguments");
    return CGX_EINVAL;
  }
  s->want_layout = layout;
  return 0;
}

int cgx_solver_set_matrix(cgx_solver *s, int n, int nnz, const int *row_ptr, const int *col,
                          const double *val) {
  if (!s) return CGX_EINVAL;
  return upload_matrix<double>(s, n, nnz, row_ptr, col, val);
}

int cgx_solver_set_matrix_f32(cgx_solver *s, int n, int nnz, const int *row_ptr, const int *col,
                              const float *val) {
  if (!s) return CGX_EINVAL;
  return upload_matrix<float>(s, n, nnz, row_ptr, col, val);
}

int cgx_solver_gen_laplacian(cgx_solver *s, int dim, int nx, int ny, int nz) {
  if (!s) return CGX_EINVAL;
  const LapSpec g{dim, nx, ny, dim == 3 ? nz : 1};
  const long long n = (long long)nx * ny * g.nz;
  if ((dim != 2 && dim != 3) || nx < 1 || ny < 1 || g.nz < 1 || n > INT32_MAX ||
      lap_rp(n, g) > INT32_MAX) {
    set_error("gen_laplacian: bad grid");
    return CGX_EINVAL;
  }
  std::vector<int> rp((size_t)n + 1);
  for (long long i = 0; i <= n; ++i) rp[(size_t)i] = (int)lap_rp(i, g);
  return upload_matrix<double>(s, (int)n, rp[(size_t)n], rp.data(), nullptr, nullptr, &g);
}

int cgx_solver_set_stencil(cgx_solver *s, int dim, int nx, int ny, int nz) {
  if (!s) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  free_system(s);
  int rc = s->A.set_stencil(LapSpec{dim, nx, ny, dim == 3 ? nz : 1});
  if (rc) return rc;
  return alloc_vectors(s);
}

int cgx_solver_get_matrix(cgx_solver *s, int *row_ptr, int *col, double *val) {
  if (!s || !s->have_matrix || s->A.layout == L_STENCIL || s->A.npanel > 1 ||
      s->A.dtype != CGX_F64 || (s->A.n > 0 && (!row_ptr || (s->A.nnz > 0 && (!col || !val))))) {
    set_error("get_matrix: needs an fp64 CSR-resident matrix and output arrays");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  return s->A.download_csr(row_ptr, col, val);
}

int cgx_solver_set_rhs(cgx_solver *s, const double *b) { return s ? upload_rhs<double>(s, b) : CGX_EINVAL; }

int cgx_solver_set_rhs_f32(cgx_solver *s, const float *b) {
  return s ? upload_rhs<float>(s, b) : CGX_EINVAL;
}

int cgx_solver_run(cgx_solver *s, int maxit, double tol, int *iters) {
  if (!s || !s->have_matrix || !s->have_rhs || maxit < 0) {
    cgx::set_error("run: need matrix + rhs and maxit >= 0");
    return CGX_EINVAL;
  }
  if (s->A.dtype == CGX_F32 && s->mode == CGX_MODE_EXACT) {
    cgx::set_error("exact mode is fp64 only");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  if (s->A.n == 0) {  // empty system: nothing to iterate, x is empty
    s->last_iters = maxit + 1;
    if (iters) *iters = s->last_iters;
    return 0;
  }
  return s->A.dtype == CGX_F32 ? run_t<float>(s, maxit, tol, iters)
                               : run_t<double>(s, maxit, tol, iters);
}

int cgx_solver_get_x(cgx_solver *s, double *x) {
  if (!s || !s->have_matrix || s->A.dtype != CGX_F64 || (s->A.n && !x)) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpy(x, s->d_x, (size_t)s->A.n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int cgx_solver_get_x_f32(cgx_solver *s, float *x) {
  if (!s || !s->have_matrix || s->A.dtype != CGX_F32 || (s->A.n && !x)) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpy(x, s->d_x, (size_t)s->A.n * 4, hipMemcpyDeviceToHost));
  return 0;
}

int cgx_solver_get_history(cgx_solver *s, double *rr, int cap) {
  if (!s || !rr || cap < 0) return CGX_EINVAL;
  const int m = std::min(cap, std::min(s->last_iters, s->hist_alloc));
  if (m <= 0) return 0;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpy(rr, s->d_hist, (size_t)m * 8, hipMemcpyDeviceToHost));
  return m;
}

int cgx_solver_spmv(cgx_solver *s, const double *x, double *y) {
  return s ? spmv_t<double>(s, x, y) : CGX_EINVAL;
}

int cgx_solver_spmv_f32(cgx_solver *s, const float *x, float *y) {
  return s ? spmv_t<float>(s, x, y) : CGX_EINVAL;
}

int cgx_solver_info(cgx_solver *s, cgx_info *info) {
  if (!s || !info) return CGX_EINVAL;
  const DevMatrix &A = s->A;
  const double sv = (double)tsize(A.dtype);
  memset(info, 0, sizeof *info);
  info->n = A.n;
  info->nnz = A.nnz;
  info->dtype = A.dtype;
  info->mode = s->mode;
  info->alg = s->alg;
  info->layout = s->have_matrix ? public_layout(A) : CGX_LAYOUT_AUTO;
  info->n_items = A.items();
  info->spmv_grid = s->have_matrix ? A.partials(A.all_items()) : 0;
  info->vec_grid = s->vec_grid;
  // B_spmv = nnz*(s_v+4) + 4*(n+1) + 2*n*s_v; B_iter = B_spmv + 9*n*s_v
  info->spmv_bytes = A.csr_bytes();
  info->iter_bytes = info->spmv_bytes + 9.0 * A.n * sv;
  info->spmv_iter_bytes = A.layout_bytes();
  // the fused step also reads r, p_old and writes p_new (the SpMV's own p
  // read becomes the r / p_old reads: +2 vectors); every other launch reads
  // x and p_{k-1}, writes x (+3 / 2): the average launch, +3.5 n vectors
  if (s->have_matrix && fused(s))
    // CG1: r, w, s, p, x read and p, s, r, w, x written, the SpMV's own x
    // read / y write included: + 8 n vectors
    // SR (one launch): r, s, p read and written, x / p_{k-2} every other
    // launch: + 5.5 n vectors
    // (SR with x four iterations deep, sr_x4: x, p_{k-3}, p_{k-2}, p_{k-1}
    // read and x written every fourth launch: + 5.25 n vectors)
    info->spmv_iter_bytes += (s->alg == CGX_ALG_CG1 ? 8.0
                              : s->alg == CGX_ALG_SR ? (sr_x4(s) ? 5.25 : 5.5)
                                                     : 3.5) * A.n * sv;
  info->device_bytes = A.dev_bytes + s->vec_bytes;
  info->n_panels = A.npanel;
  info->n_dict = A.layout == L_DC ? A.ndict : A.layout == L_DIA ? A.dia.ndiag : 0;
  info->tile_bands = A.tile_bands;
  info->nt = A.nt ? 1 : 0;
  info->code_bytes_per_row = A.layout == L_DIA ? A.dia.cbytes : 0;
  info->dia_value_stream = A.layout == L_DIA && A.dv() ? 1 : 0;
  for (int k = 0; k < A.dia.ndiag; ++k) info->n_values += A.dia.nval[k];
  info->gathers_per_chunk = A.layout == L_CSR || A.layout == L_DC ? A.gath : 0;
  info->setup_host_ms = A.setup_host_ms;
  info->setup_device_ms = A.setup_dev_ms;
  info->encode_fallback = A.encode_fallback;
  info->fused = s->have_matrix && fused(s) ? 1 : 0;
  // the conditions of fused(): SR needs the march plan and ignores the
  // Infinity Cache rule
  const bool sr = s->alg == CGX_ALG_SR;
  info->fuse_status = !s->have_matrix ? CGX_FUSE_STATUS_NOT_DIA
                      : s->mode == CGX_MODE_EXACT ? CGX_FUSE_STATUS_EXACT
                      : s->fuse == CGX_FUSE_OFF   ? CGX_FUSE_STATUS_OFF
                      : A.fuse_block(sr)          ? A.fuse_block(sr)
                      : sr && (A.mq == 0 || s->march == 0) ? CGX_FUSE_STATUS_NO_MARCH
                      : (!sr && s->fuse == CGX_FUSE_AUTO && !A.nt) ? CGX_FUSE_STATUS_CACHED
                                                                   : CGX_FUSE_STATUS_RUNS;
  info->breakdown = s->h_st ? s->h_st->brk : 0;
  info->fuse_march = s->have_matrix ? march_len(s) : 0;
  if (info->fuse_march > 0 && s->alg == CGX_ALG_SR && s->march <= 0) {
    // the balanced segments k_sr1_dia_m runs (enqueue_iter): the longest
    const SpmvArgs<double> a =
        s->A.args<double>(nullptr, nullptr, nullptr, nullptr, s->A.all_items());
    const long long QR = (long long)a.mq * kDiaSliceRows;
    const int steps = (int)((a.n + QR - 1) / QR);
    const int ns = sr1_pick_shape(a, s->cus, s->sr_chain, true).nseg;
    info->fuse_march = (steps + ns - 1) / std::max(1, ns);
  }
  return 0;
}

int cgx_solver_bench_prepare(cgx_solver *s, int warmup) {
  if (!s || !s->have_matrix || !s->have_rhs || s->A.n == 0 || warmup < 0) {
    cgx::set_error("bench_prepare: need a non-empty system and warmup >= 0");
    return CGX_EINVAL;
  }
  if (s->mode == CGX_MODE_EXACT && s->A.dtype == CGX_F32) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  return s->A.dtype == CGX_F32 ? bench_prepare_t<float>(s, warmup)
                               : bench_prepare_t<double>(s, warmup);
}

int cgx_solver_bench_run(cgx_solver *s, int iters, int flags, double *total_ms, double *spmv_ms) {
  if (!s || !s->bench_ready || iters < 1 || !total_ms || !spmv_ms) {
    cgx::set_error("bench_run: call cgx_solver_bench_prepare first; iters >= 1");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  return s->A.dtype == CGX_F32 ? bench_run_t<float>(s, iters, flags, total_ms, spmv_ms)
                               : bench_run_t<double>(s, iters, flags, total_ms, spmv_ms);
}

int cgx_solver_bench(cgx_solver *s, int warmup, int iters, int flags, double *total_ms,
                     double *spmv_ms) {
  int rc = cgx_solver_bench_prepare(s, warmup);
  if (rc) return rc;
  return cgx_solver_bench_run(s, iters, flags, total_ms, spmv_ms);
}

}  // extern "C"
