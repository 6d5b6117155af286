// cgx_dist.cpp -- the multi-GPU CG solver: one rank per GPU, rows partitioned
// into contiguous blocks (cgx_partition.cpp), halo x segments exchanged point
// to point, the iteration's dot products all-reduced over RCCL (SURVEY.md
// 8e; north star in BASELINE.json).  Each rank's rows live in a DevMatrix
// (cgx_matrix.h) with local column numbering: owned rows -> [0, n_loc),
// ghosts -> n_loc + position, so the halo exchange writes the gathered
// vector's ghost tail directly and every layout (CSR, CSR-DC, DIA-VI) works
// unchanged -- a slab's ghost columns are one more constant offset per face.
//
// Recurrences (cgx_dist_set_alg):
//   HS  (default; the reference's cg.c:88-141): per iteration
//       st_comm: (forked from st) pack p[send rows], halo of p
//                (ncclSend/Recv with each neighbour, into p's ghost tail),
//                created at the device's highest priority so its kernels
//                are dispatched ahead of the interior SpMV's workgroups
//       st:      SpMV s = A p over INTERIOR work items (no ghost columns)
//                || halo; wait; SpMV over BOUNDARY items; one finalize
//                workgroup sums the p.s partials (local p.s)
//                ncclAllReduce(p.s)
//                k_update_rf (alpha, r -= alpha s; its last workgroup sums
//                the r.r partials) -> ncclAllReduce(r.r)
//                k_xpay_xf (beta, stop test, x += alpha p, p = r + beta p)
//       fused (DIA layouts k_spmv_dia_h takes on every rank; cgx_dist_set_fused):
//       st_comm: pack p_new = r + beta p_old at the send rows (k_pack_pnext),
//                halo of p_new into the p_new buffer's ghost tail
//       st:      k_spmv_dia_h over INTERIOR items: beta, p_new, x (every
//                other iteration), s = A p_new || halo; wait; BOUNDARY items
//                (ghost diagonals read the received p_new) -> local p.s
//                ncclAllReduce(p.s); k_update_rf -> ncclAllReduce(r.r)
//                -- two launches and one pack per iteration instead of four
//   SR  (single reduction; the fused step only): the fused HS iteration with
//       the s.s partials beside p.s in the fused launch; ONE all-reduce of
//       (p.s, s.s, r.r) -- r.r the exact local sum of the last r update's
//       partials -- then k_update_rf takes alpha = r.r / p.s (cg.c:113) and
//       writes r_new.r_new = alpha^2 s.s - r.r (r.s = p.s) for beta
//       (cg.c:129) and the stop test: HS's bytes, one all-reduce latency per
//       iteration instead of two, rounding-level different from HS.
//       One launch per iteration (round 4; where every rank's rows take it,
//       cgx_dist_set_march): the single-GPU k_sr1_dia_m step on an IN-PLACE
//       numbering of the rank's rows -- columns = global - row_begin, the
//       neighbours' boundary planes at [-g_lo, 0) and [n_loc, n_loc + g_hi)
//       of every vector -- so the plane march runs across the slab edges:
//       st_comm: k_pack_sr (p_k = (r - alpha s) + beta p at the send rows),
//                halo into the p_new buffer's ghost rows
//       st:      k_sr1_dia_m over the INTERIOR steps (no window reaches a
//                ghost row) || halo; wait; the BOUNDARY steps (ghost rows'
//                p_k from the halo) -> local (p.s, s.s, r.r)
//                ncclAllReduce(3 doubles); k_finalize(FIN_SR1)
//       61 B/row instead of 69, no separate r-update launch.
//   CG1 (Chronopoulos-Gear): ONE all-reduce of (gamma, delta) per iteration,
//       rounding-level different from HS, 8 B per row more vector traffic;
//       fused (CGX_FUSE_ON only): k_cg1_dia_h does the vector recurrences
//       and w = A r_new in one launch, the halo carries r_new (k_pack_rnext).
// Every rank derives alpha, beta and the stop test from the same all-reduced
// sums, so they agree bit for bit.  With RCCL, batches of iterations --
// halo, all-reduces and kernels -- are captured once as a hipGraph and
// replayed (eager fallback if the capture fails).
//
// Transports: RCCL (one process per GPU; ncclCommInitRank from an id the
// caller distributes), or "local": P partitions driven by one host thread on
// one device (device copies for the halo, a fixed-order sum kernel for the
// all-reduce) -- the same phase code, used to validate the partitioned path
// on a single GPU.  The host driver runs each phase over all partitions it
// owns (one in RCCL mode), so every wait is on an already recorded event.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cgx_internal.h"
#include "cgx_matrix.h"

using cgx::CgState;
using cgx::DevMatrix;

struct cgx_dist;

namespace cgx {
int public_layout(const DevMatrix &m);
}

namespace {

struct Group {
  std::vector<cgx_dist *> parts;    // RCCL mode: just this rank
  const double **d_srcs = nullptr;  // local mode: every part's d_sums
  bool connected = false;
  bool fz_known = false;  // fz_all decided for the current matrices and fuse modes
};

}  // namespace

struct cgx_dist {
  int device = 0, nranks = 1, rank = 0;
  bool local = false;
  Group *group = nullptr;  // owned by part 0 in local mode, by self in RCCL
  bool owns_group = false;
  ncclComm_t comm = nullptr;
  int cus = 256;
  hipStream_t st = nullptr, st_comm = nullptr;
  hipEvent_t ev_fork = nullptr, ev_packed = nullptr, ev_halo = nullptr, ev_sums = nullptr,
             ev_sums2 = nullptr;
  hipEvent_t ev_red = nullptr;  // local transport: this part's last group sum has read d_sums
  cgx_part *part = nullptr;
  long long n_global = 0;
  int row_begin = 0, n_loc = 0, n_ghost = 0, nnz = 0;
  int alg = CGX_ALG_HS;
  int want_layout = CGX_LAYOUT_AUTO;
  DevMatrix A;
  cgx::Items it_int{}, it_bnd{};
  int *d_list_int = nullptr, *d_list_bnd = nullptr;
  int *d_pairs_int = nullptr, *d_pairs_bnd = nullptr;  // the fused step's super-items of a list
  int g_int = 0, g_bnd = 0;  // SpMV partials of each launch
  double *d_b = nullptr, *d_x = nullptr, *d_r = nullptr, *d_p = nullptr, *d_s = nullptr,
         *d_w = nullptr;
  double *d_p2 = nullptr;  // fused step: the second p buffer (with ghost tail)
  double *d_p3 = nullptr, *d_p4 = nullptr;  // one-launch SR: the third / fourth p (x4)
  // fused CG1 step: the second r, s, w buffers (with ghost tails)
  double *d_r2 = nullptr, *d_s2 = nullptr, *d_w2 = nullptr;  // lazily: ensure_rsw2
  size_t ng_alloc = 0;  // entries of a ghosted vector from element 0 (upload_local)
  int pbuf = 0;            // fused step: which buffer holds p_old (0: d_p) / r, s, w_old
  bool in_init = false;    // the CG1 prologue's phases (unfused SpMV w = A r)
  int fuse = CGX_FUSE_AUTO;  // cgx_dist_set_fused
  bool fz_all = false;     // every partition's layout takes the fused step (ensure_connected)
  int *d_send_idx = nullptr;
  double *d_sendbuf = nullptr;
  std::vector<int> send_count, send_off, recv_count, recv_off;
  int n_send = 0;
  double *d_pa = nullptr, *d_pb = nullptr;
  double *d_pss = nullptr;  // SR: the fused launches' (p.s, s.s) pairs, one per workgroup
  // the one-launch SR step (k_sr1_dia_m) on the in-place numbering
  DevMatrix Ai;              // columns = global - row_begin (DIA-VI, march plan)
  bool ai_ok = false;        // Ai built: contiguous ghost ranges, DIA, march plan
  int g_lo = 0, g_hi = 0;    // ghost rows below / above the own rows
  std::vector<int> recv_pos; // in-place position of each owner's first ghost row
  size_t vfront = 0;         // entries before element 0 of the ghosted vectors
  int march = -1;            // cgx_dist_set_march: -1 auto, 0 off, > 0 interior steps/segment
  int sr_chain = 0;          // cgx_dist_set_sr_chain: 0 auto, > 0 chain width (rows)
  bool mi_all = false;       // every partition runs the one-launch SR step (agreed)
  double *d_pq = nullptr, *d_pc = nullptr;  // its (p.s, s.s) pairs and r.r partials
  int gi1 = 0, gb1 = 0;      // workgroups of its interior / boundary launch
  double *d_sums = nullptr, *d_gsums = nullptr;  // [0, 4) local, [4, 8) all-reduced
  unsigned *d_tick = nullptr;                    // last-arriver counters
  int vec_grid = 1;
  CgState *d_st = nullptr, *h_st = nullptr;
  double *d_hist = nullptr;
  int hist_alloc = 0;
  size_t vec_bytes = 0;
  bool have_matrix = false, have_rhs = false, bench_ready = false;
  int last_iters = 0;
  // optional SpMV timing: 4 events per iteration (interior start/end,
  // boundary start/end) while rec_spmv is set (eager only)
  std::vector<hipEvent_t> spmv_ev;
  bool rec_spmv = false;
  size_t ev_i = 0;
  // per-phase averages of the last CGX_BENCH_SPMV_EVENTS run (cgx_dist_bench_phases)
  double phase_ms[5] = {-1.0, -1.0, -1.0, -1.0, -1.0};
  int phase_iters = 0;
  // batches of graph_batch iterations replayed as a hipGraph (solo and
  // RCCL; the in-process group runs eager)
  hipGraphExec_t gexec[4] = {};   // graph_batch iterations, per p-buffer rotation
  hipGraphExec_t gexec1[4] = {};  // one iteration (remainders), per rotation
  int gexec_alg = -1;
  int graph_batch = 16;
  bool use_graph = true;
  int graph_state = 0;  // 1 captured, -1 capture failed (eager from then on)
  // RCCL calls enqueued (or recorded under capture) by this rank: a capture
  // that fails after it recorded one leaves RCCL's host-side state advanced
  // for ops that will never run -- fatal for the communicator (comm_fatal)
  long long nccl_calls = 0;
  bool comm_fatal = false;
  int dbg_refuse = 0;  // cgx_dist_debug_refuse_capture: 1 before, 2 after the RCCL ops
};

namespace {

using namespace cgx;

// One rank with no transport: no halo, scalars straight from the partials.
// A 1-rank RCCL communicator (cgx_dist_create with an id at nranks 1) keeps
// the transport phases -- the multi-GPU code path, all-reduce included.
bool solo(const cgx_dist *d) { return !d->local && d->comm == nullptr; }

#define CGX_NCCL(call)                                                                  \
  do {                                                                                  \
    ncclResult_t r_ = (call);                                                           \
    if (r_ != ncclSuccess) {                                                            \
      set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call, ncclGetErrorString(r_)); \
      return CGX_ECOMM;                                                                 \
    }                                                                                   \
  } while (0)

void drop_graph(cgx_dist *d) {
  for (int q = 0; q < 4; ++q) {
    if (d->gexec[q]) (void)hipGraphExecDestroy(d->gexec[q]);
    if (d->gexec1[q]) (void)hipGraphExecDestroy(d->gexec1[q]);
    d->gexec[q] = d->gexec1[q] = nullptr;
  }
  d->gexec_alg = -1;
}

// The fused HS step (k_spmv_dia_h) runs when every partition's layout
// takes it (decided once per connection: the ranks' phase sequences match).
// SR is the fused step with one reduction.
// HS-shaped recurrences (HS, SR): s = A p, r -= alpha s, p = r + beta p
bool hs_like(const cgx_dist *d) { return d->alg == CGX_ALG_HS || d->alg == CGX_ALG_SR; }
bool sr(const cgx_dist *d) { return d->alg == CGX_ALG_SR; }
// SR as ONE k_sr1_dia_m launch pair per iteration on the in-place numbering
bool sr1(const cgx_dist *d) { return sr(d) && d->mi_all; }
bool fz(const cgx_dist *d) { return d->fz_all && hs_like(d) && !sr1(d); }
// SR without a fused step (round 5, VERDICT r04 #5: CSR, DC, wide-word DIA
// ranks): the SpMV stores (p.s, s.s) pairs, ONE all-reduce of (p.s, s.s,
// r.r), then k_update_sr does r, p (in place, its ghost tail refreshed by
// the next halo) and x in one pass with the sums applied privately
bool sru(const cgx_dist *d) { return sr(d) && !d->fz_all && !d->mi_all; }
// The fused CG1 step (k_cg1_dia_h): only when forced on (CGX_FUSE_ON) --
// on a rank's slab it loses to the unfused CG1 kernels (C4/8's 400 x 400 x
// 50 slab: 164 vs 144 us per iteration, tools/dist_probe.py: the unfused
// update's r and the SpMV's w are re-read from the Infinity Cache, the fused
// launch streams all ten vectors from HBM); not in the prologue.
bool fz1(const cgx_dist *d) {
  return d->fz_all && d->alg == CGX_ALG_CG1 && d->fuse == CGX_FUSE_ON && !d->in_init;
}

// this partition takes the fused step (cgx_solver.cpp fused(): auto needs a
// working set beyond the Infinity Cache; SR has no unfused form)
bool part_fusable(const cgx_dist *d) {
  return d->fuse != CGX_FUSE_OFF && d->A.fusable() &&
         (d->fuse == CGX_FUSE_ON || d->A.nt || sr(d));
}

// this partition can run the one-launch SR step (its in-place layout exists
// and the march is not switched off)
bool part_marchable(const cgx_dist *d) {
  return d->ai_ok && d->march != 0 && d->fuse != CGX_FUSE_OFF;
}

// the all-reduced sums the one-launch SR step's kernels apply themselves
// (FIN_SR1 folded into the next iteration's launches, FIN_SUM3_SR1 applies
// them to the state: no scalar launch between the all-reduce and the next
// SpMV, 3-4 us per iteration on the C4/8 slab); nullptr without a transport
// (FIN_SR1 on the partials)
const double *sr1_g(const cgx_dist *d);

bool has_peers(const cgx_dist *d);

// The one-launch SR step's launch shapes: segments (set_march's length, or
// the segment count and chain width sr1_pick_shape finds for the device) and, on a rank with
// neighbours, the edge rows k_sr1_edge recomputes after the halo -- [0, elo)
// below when there are ghost rows below (the rows that reach column < 0:
// -(lowest diagonal offset)), [ehi, n) above (n - the highest offset), both
// bounds even (row pairs); a slab too thin to have interior rows is all edge.
struct Sr1Plan {
  int nseg, len, elo, ehi, cw, sb;
};

Sr1Plan sr1_plan(const cgx_dist *d) {
  const SpmvArgs<double> a = d->Ai.args<double>(nullptr, nullptr, nullptr, nullptr, d->Ai.all_items());
  Sr1Plan p;
  const Sr1Shape sh = sr1_pick_shape(a, d->cus, d->sr_chain);
  p.nseg = d->march > 0 ? 0 : sh.nseg;
  p.len = d->march > 0 ? d->march : 0;
  const bool shaped = d->march <= 0 || d->sr_chain > 0;
  p.cw = shaped ? sh.cw : 0;
  p.sb = shaped ? sh.sb : 0;
  p.elo = 0;
  p.ehi = 0x7fffffff;
  if (has_peers(d) && a.ndiag > 0) {
    const int n = a.n;
    if (d->g_lo > 0) p.elo = std::min(n, std::max(0, -a.doff[0]));
    if (d->g_hi > 0) p.ehi = std::max(0, n - std::max(0, a.doff[a.ndiag - 1]));
    p.elo = (p.elo + 1) & ~1;
    if (p.ehi < n) p.ehi &= ~1;
    if (p.elo >= p.ehi) {  // every row an edge row
      p.elo = (n + 1) & ~1;
      p.ehi = 0x7fffffff;
    }
  }
  return p;
}

// the ghosted vectors start vfront entries into their allocation (the
// in-place numbering's ghost rows below element 0)
void free_ghosted(cgx_dist *d, double **p) {
  if (*p) dev_free_raw(*p - d->vfront);
  *p = nullptr;
}

void free_system(cgx_dist *d) {
  drop_graph(d);
  d->A.release();
  d->Ai.release();
  d->ai_ok = false;
  d->g_lo = d->g_hi = 0;
  d->recv_pos.clear();
  dev_free(&d->d_pq);
  dev_free(&d->d_pc);
  d->gi1 = d->gb1 = 0;
  dev_free(&d->d_list_int);
  dev_free(&d->d_list_bnd);
  dev_free(&d->d_pairs_int);
  dev_free(&d->d_pairs_bnd);
  dev_free(&d->d_b);
  dev_free(&d->d_x);
  for (double **v : {&d->d_r, &d->d_p, &d->d_s, &d->d_w, &d->d_p2, &d->d_r2, &d->d_s2, &d->d_w2,
                     &d->d_p3, &d->d_p4})
    free_ghosted(d, v);
  d->vfront = 0;
  dev_free(&d->d_send_idx);
  dev_free(&d->d_sendbuf);
  dev_free(&d->d_pa);
  dev_free(&d->d_pb);
  dev_free(&d->d_pss);
  dev_free(&d->d_hist);
  d->hist_alloc = 0;
  if (d->part) cgx_part_destroy(d->part);
  d->part = nullptr;
  d->have_matrix = d->have_rhs = d->bench_ready = false;
  d->vec_bytes = 0;
  if (d->group) d->group->connected = false;
}

int init_common(cgx_dist *d, int device) {
  int rc = check_device(device, &d->cus);
  if (rc) return rc;
  d->device = device;
  d->A.device = device;
  CGX_HIP(hipSetDevice(device));
  CGX_HIP(hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking));
  {
    // halo traffic on a high-priority stream: its RCCL kernel is dispatched
    // ahead of the interior SpMV's remaining workgroups, so the ghosts arrive
    // while the interior rows are still being summed
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    CGX_HIP(hipStreamCreateWithPriority(&d->st_comm, hipStreamNonBlocking, greatest));
  }
  d->A.st = d->st;
  CGX_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_packed, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_halo, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_sums, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_sums2, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_red, hipEventDisableTiming));
  CGX_HIP(hipMalloc((void **)&d->d_st, sizeof(CgState)));
  CGX_HIP(hipMalloc((void **)&d->d_sums, 8 * sizeof(double)));
  CGX_HIP(hipMemset(d->d_sums, 0, 8 * sizeof(double)));
  // the ticket region of k_update_rf's local r.r sums
  CGX_HIP(hipMalloc((void **)&d->d_tick, kTickRegion * sizeof(unsigned)));
  CGX_HIP(hipMemset(d->d_tick, 0, kTickRegion * sizeof(unsigned)));
  CGX_HIP(hipHostMalloc((void **)&d->h_st, sizeof(CgState), hipHostMallocDefault));
  d->d_gsums = d->d_sums + 4;
  return 0;
}

// ------------------------------------------------------------ system setup

// Interior / boundary work items (blocks or slices) of the local matrix:
// boundary = any row of the item references a ghost column.  In the
// matrix's (tiled) item order; one contiguous run needs no device list.
int split_items(cgx_dist *d, const int *rp, const std::vector<int> &col_local) {
  const std::vector<int> ir = d->A.item_rows();
  const int ni = (int)ir.size() - 1;
  std::vector<char> ghost((size_t)std::max(ni, 0), 0);
  for (int i = 0; i < ni; ++i)
    for (int k = rp[ir[(size_t)i]]; k < rp[ir[(size_t)i + 1]] && !ghost[(size_t)i]; ++k)
      ghost[(size_t)i] = col_local[(size_t)k] >= d->n_loc;
  std::vector<int> lint, lbnd;
  for (int j = 0; j < ni; ++j) {
    const int i = d->A.order.empty() ? j : d->A.order[(size_t)j];
    (ghost[(size_t)i] ? lbnd : lint).push_back(i);
  }
  auto make = [&](const std::vector<int> &l, int **dl, int **dp, Items &it) -> int {
    const bool run = !l.empty() && l.back() - l.front() + 1 == (int)l.size() &&
                     std::is_sorted(l.begin(), l.end());
    it = Items{nullptr, l.empty() ? 0 : l.front(), (int)l.size()};
    if (l.empty() || run) return 0;
    int rc = dev_alloc(dl, l.size() * 4, &d->vec_bytes);
    if (rc) return rc;
    CGX_HIP(hipMemcpy(*dl, l.data(), l.size() * 4, hipMemcpyHostToDevice));
    it.list = *dl;
    it.first = 0;
    if (d->A.layout == L_DIA) {  // the fused step's super-items of the list
      const std::vector<int> fp = fuse_pairs(l);
      if ((rc = dev_alloc(dp, fp.size() * 4, &d->vec_bytes))) return rc;
      CGX_HIP(hipMemcpy(*dp, fp.data(), fp.size() * 4, hipMemcpyHostToDevice));
      it.pairs = *dp;
      it.npairs = (int)fp.size() / 2;
    }
    return 0;
  };
  int rc;
  if ((rc = make(lint, &d->d_list_int, &d->d_pairs_int, d->it_int)) ||
      (rc = make(lbnd, &d->d_list_bnd, &d->d_pairs_bnd, d->it_bnd)))
    return rc;
  d->g_int = d->it_int.count ? d->A.partials(d->it_int) : 0;
  d->g_bnd = d->it_bnd.count ? d->A.partials(d->it_bnd) : 0;
  return 0;
}

// The in-place numbering of this rank's rows for the one-launch SR step:
// when its ghost columns are exactly the rows [row_begin - g_lo, row_begin)
// and [row_end, row_end + g_hi) (a banded matrix's neighbouring planes), the
// columns global - row_begin give a DIA-VI layout whose plane march runs
// across the slab edges (ghost rows in place, below 0 and from n_loc).
// Not applicable (scattered ghosts, no DIA, no march plan): ai_ok = false,
// and SR runs the two-launch fused step.
int build_inplace(cgx_dist *d, int n_loc, int nnz, const int *rp, const int *col_global,
                  const double *val) {
  d->ai_ok = false;
  // (the standard numbering's layout may be DC where thin slabs give it
  // ghost offsets beyond DIA's 16 diagonals; the in-place one has the
  // matrix's own offsets)
  if ((d->want_layout != CGX_LAYOUT_AUTO && d->want_layout != CGX_LAYOUT_DIA) || n_loc == 0)
    return 0;
  std::vector<int> gh((size_t)d->n_ghost);
  cgx_part_ghosts(d->part, gh.data());
  const long long rb = d->row_begin, re = rb + n_loc;
  int nb = 0;
  while (nb < d->n_ghost && gh[(size_t)nb] < rb) ++nb;
  for (int i = 0; i < d->n_ghost; ++i) {
    const long long want = i < nb ? rb - nb + i : re + (i - nb);
    if (gh[(size_t)i] != want) return 0;
  }
  std::vector<int> ci((size_t)nnz);
  for (size_t k = 0; k < (size_t)nnz; ++k) ci[k] = (int)(col_global[k] - rb);
  const int g_hi = d->n_ghost - nb;
  const int rc = d->Ai.upload<double>(n_loc, n_loc + g_hi, nnz, rp, ci.data(), val,
                                      CGX_LAYOUT_DIA, false, nullptr, -nb, true);
  // (a near-only plan, DevMatrix::mfar 0, is the single GPU's: ranks whose
  // slabs have no far diagonals keep the two-launch step)
  if (rc || d->Ai.layout != L_DIA || d->Ai.mq == 0 || !d->Ai.mfar) {
    d->Ai.release();
    set_error("%s", "");
    return 0;
  }
  d->g_lo = nb;
  d->g_hi = g_hi;
  d->recv_pos.assign((size_t)d->nranks, 0);
  for (int q = 0; q < d->nranks; ++q)
    if (d->recv_count[(size_t)q]) d->recv_pos[(size_t)q] = (int)(gh[(size_t)d->recv_off[q]] - rb);
  d->ai_ok = true;
  return 0;
}

int upload_local(cgx_dist *d, long long n_global, int n_loc, int nnz, const int *rp,
                 const int *col_global, const double *val) {
  CGX_HIP(hipSetDevice(d->device));
  free_system(d);
  cgx_part *pt = nullptr;
  int rc = cgx_part_create(n_global, d->nranks, d->rank, n_loc, nnz, rp, col_global, &pt);
  if (rc) return rc;
  d->part = pt;
  d->n_global = n_global;
  d->n_loc = n_loc;
  d->nnz = nnz;
  cgx_part_info(pt, nullptr, &d->n_ghost, &d->row_begin, nullptr);
  std::vector<int> col_local((size_t)nnz);
  cgx_part_local_cols(pt, col_local.data());
  d->recv_count.assign((size_t)d->nranks, 0);
  cgx_part_recv_counts(pt, d->recv_count.data());
  d->recv_off.assign((size_t)d->nranks, 0);
  for (int q = 1; q < d->nranks; ++q) d->recv_off[q] = d->recv_off[q - 1] + d->recv_count[q - 1];

  if ((rc = d->A.upload<double>(n_loc, n_loc + d->n_ghost, nnz, rp, col_local.data(), val,
                                d->want_layout, false))) {
    free_system(d);
    return rc;
  }
  if ((rc = split_items(d, rp, col_local))) {
    free_system(d);
    return rc;
  }
  if ((rc = build_inplace(d, n_loc, nnz, rp, col_global, val))) {
    free_system(d);
    return rc;
  }
  d->vec_grid = vec_grid_for(n_loc, d->cus);
  d->vec_grid = (std::max(d->vec_grid, 1) + 3) / 4 * 4;  // folded kernels: 4 x 256 threads
  const size_t nv = (size_t)n_loc + kPad;
  const size_t ng = nv + (size_t)std::max(d->n_ghost, d->g_hi + 2 * kPad);
  // the in-place numbering's ghost rows below element 0 (the windows may load
  // one pair below them, clamped: DevMatrix::col_lo - 1)
  d->vfront = d->ai_ok ? ((size_t)d->g_lo + 2 * kPad + 7) / 8 * 8 : 0;
  // d_pa: the vector kernels' partials, or the fused CG1 step's gamma partials
  const size_t npa = (size_t)std::max(d->vec_grid, d->g_int + d->g_bnd) + 8;
  size_t *cb = &d->vec_bytes;
  auto ghosted = [&](double **p) -> int {
    void *raw = nullptr;
    const int r = dev_alloc(&raw, (d->vfront + ng) * 8, cb);
    *p = r ? nullptr : (double *)raw + d->vfront;
    return r;
  };
  // r, p, s, w carry the ghost rows (s, w: the fused CG1 step's window /
  // far-slot loads reach them; only zeros are read there); the second r, s, w
  // buffers only the recurrences that alternate them allocate (ensure_rsw2)
  d->ng_alloc = ng;
  if ((rc = dev_alloc(&d->d_b, nv * 8, cb)) || (rc = dev_alloc(&d->d_x, nv * 8, cb)) ||
      (rc = ghosted(&d->d_r)) || (rc = ghosted(&d->d_p)) || (rc = ghosted(&d->d_s)) ||
      (rc = ghosted(&d->d_w)) || (rc = ghosted(&d->d_p2)) ||
      (rc = dev_alloc(&d->d_pa, npa * 8, cb)) ||
      (rc = dev_alloc(&d->d_pb, ((size_t)d->g_int + d->g_bnd + 8) * 16, cb)) ||  // SR pairs
      (rc = dev_alloc(&d->d_pss, ((size_t)d->g_int + d->g_bnd + 8) * 16, cb))) {
    free_system(d);
    return rc;
  }
  if (d->ai_ok) {
    // the one-launch SR step's partials: one (p.s, s.s) pair and one r.r per
    // workgroup of its launches (at most: sr1_max_grid for the march, and
    // one edge workgroup per 512 rows)
    const SpmvArgs<double> a = d->Ai.args<double>(nullptr, nullptr, nullptr, nullptr, d->Ai.all_items());
    const int cap = sr1_max_grid(a.mslices) + (d->n_loc + 511) / 512 + 8;
    if ((rc = dev_alloc(&d->d_pq, (size_t)cap * 16, cb)) || (rc = dev_alloc(&d->d_pc, (size_t)cap * 8, cb))) {
      free_system(d);
      return rc;
    }
  }
  for (double *v : {d->d_r, d->d_p, d->d_p2, d->d_s, d->d_w})
    CGX_HIP(hipMemsetAsync(v - d->vfront, 0, (d->vfront + ng) * 8, d->st));
  CGX_HIP(hipMemsetAsync(d->d_x, 0, nv * 8, d->st));
  CGX_HIP(hipStreamSynchronize(d->st));
  d->have_matrix = true;
  return 0;
}

// Send lists from the requests every peer sent us (global row indices).
int install_sends(cgx_dist *d, const std::vector<int> &req_counts,
                  const std::vector<int> &req_global) {
  int rc = cgx_part_set_requests(d->part, req_counts.data(), req_global.data());
  if (rc) return rc;
  d->send_count = req_counts;
  d->send_off.assign((size_t)d->nranks, 0);
  for (int q = 1; q < d->nranks; ++q) d->send_off[q] = d->send_off[q - 1] + d->send_count[q - 1];
  d->n_send = d->send_off[d->nranks - 1] + d->send_count[d->nranks - 1];
  std::vector<int> loc((size_t)d->n_send);
  cgx_part_send_local(d->part, loc.data());
  dev_free(&d->d_send_idx);
  dev_free(&d->d_sendbuf);
  if ((rc = dev_alloc(&d->d_send_idx, ((size_t)d->n_send + 1) * 4, &d->vec_bytes)) ||
      (rc = dev_alloc(&d->d_sendbuf, ((size_t)d->n_send + 1) * 8, &d->vec_bytes)))
    return rc;
  if (d->n_send > 0)
    CGX_HIP(hipMemcpy(d->d_send_idx, loc.data(), (size_t)d->n_send * 4, hipMemcpyHostToDevice));
  return 0;
}

// RCCL: exchange ghost requests (counts, then global indices) with grouped
// point-to-point calls; collective over the communicator.
int connect_rccl(cgx_dist *d) {
  const int P = d->nranks;
  std::vector<int> ghosts((size_t)d->n_ghost);
  cgx_part_ghosts(d->part, ghosts.data());
  std::vector<int> req_counts((size_t)P, 0);
  if (P > 1) {
    int *d_cnt = nullptr;
    CGX_HIP(hipMalloc((void **)&d_cnt, (size_t)P * 2 * 4));
    CGX_HIP(hipMemcpy(d_cnt, d->recv_count.data(), (size_t)P * 4, hipMemcpyHostToDevice));
    CGX_NCCL(ncclGroupStart());
    for (int q = 0; q < P; ++q) {
      if (q == d->rank) continue;
      CGX_NCCL(ncclSend(d_cnt + q, 1, ncclInt32, q, d->comm, d->st));
      CGX_NCCL(ncclRecv(d_cnt + P + q, 1, ncclInt32, q, d->comm, d->st));
    }
    CGX_NCCL(ncclGroupEnd());
    CGX_HIP(hipStreamSynchronize(d->st));
    CGX_HIP(hipMemcpy(req_counts.data(), d_cnt + P, (size_t)P * 4, hipMemcpyDeviceToHost));
    req_counts[d->rank] = 0;
    (void)hipFree(d_cnt);
  }
  std::vector<int> req_off((size_t)P, 0);
  for (int q = 1; q < P; ++q) req_off[q] = req_off[q - 1] + req_counts[q - 1];
  const int total = P > 0 ? req_off[P - 1] + req_counts[P - 1] : 0;
  std::vector<int> req_global((size_t)total);
  if (P > 1) {
    int *d_g = nullptr, *d_req = nullptr;
    CGX_HIP(hipMalloc((void **)&d_g, ((size_t)d->n_ghost + 1) * 4));
    CGX_HIP(hipMalloc((void **)&d_req, ((size_t)total + 1) * 4));
    if (d->n_ghost)
      CGX_HIP(hipMemcpy(d_g, ghosts.data(), (size_t)d->n_ghost * 4, hipMemcpyHostToDevice));
    CGX_NCCL(ncclGroupStart());
    for (int q = 0; q < P; ++q) {
      if (q == d->rank) continue;
      if (d->recv_count[q])
        CGX_NCCL(ncclSend(d_g + d->recv_off[q], d->recv_count[q], ncclInt32, q, d->comm, d->st));
      if (req_counts[q])
        CGX_NCCL(ncclRecv(d_req + req_off[q], req_counts[q], ncclInt32, q, d->comm, d->st));
    }
    CGX_NCCL(ncclGroupEnd());
    CGX_HIP(hipStreamSynchronize(d->st));
    if (total)
      CGX_HIP(hipMemcpy(req_global.data(), d_req, (size_t)total * 4, hipMemcpyDeviceToHost));
    (void)hipFree(d_g);
    (void)hipFree(d_req);
  }
  return install_sends(d, req_counts, req_global);
}

// Local transport: every partition reads its peers' ghost lists directly.
int connect_local(Group *g) {
  const int P = (int)g->parts.size();
  std::vector<std::vector<int>> ghosts((size_t)P);
  for (int q = 0; q < P; ++q) {
    ghosts[q].resize((size_t)g->parts[q]->n_ghost);
    cgx_part_ghosts(g->parts[q]->part, ghosts[q].data());
  }
  for (int p = 0; p < P; ++p) {
    cgx_dist *d = g->parts[p];
    CGX_HIP(hipSetDevice(d->device));
    std::vector<int> req_counts((size_t)P, 0), req_global;
    for (int q = 0; q < P; ++q) {
      const cgx_dist *o = g->parts[q];
      const int off = o->recv_off[p], cnt = o->recv_count[p];
      req_counts[q] = cnt;
      req_global.insert(req_global.end(), ghosts[q].begin() + off, ghosts[q].begin() + off + cnt);
    }
    int rc = install_sends(d, req_counts, req_global);
    if (rc) return rc;
  }
  if (!g->d_srcs) {
    std::vector<const double *> srcs((size_t)P);
    for (int q = 0; q < P; ++q) srcs[q] = g->parts[q]->d_sums;
    CGX_HIP(hipSetDevice(g->parts[0]->device));
    CGX_HIP(hipMalloc((void **)&g->d_srcs, (size_t)P * sizeof(double *)));
    CGX_HIP(hipMemcpy(g->d_srcs, srcs.data(), (size_t)P * sizeof(double *), hipMemcpyHostToDevice));
  }
  g->connected = true;
  return 0;
}

// MIN of an int over the ranks (RCCL): every rank's layout takes the fused
// step (ensure_fused_known), every rank's graph capture succeeded
// (ensure_graphs).  The value itself below two ranks.
int agree_min(cgx_dist *d, int mine, int *all) {
  *all = mine;
  if (d->comm == nullptr || d->nranks < 2) return 0;
  int *d_f = nullptr;
  CGX_HIP(hipMalloc((void **)&d_f, 2 * sizeof(int)));
  CGX_HIP(hipMemcpy(d_f, &mine, sizeof(int), hipMemcpyHostToDevice));
  ++d->nccl_calls;
  ncclResult_t r = ncclAllReduce(d_f, d_f + 1, 1, ncclInt32, ncclMin, d->comm, d->st);
  hipError_t e = r == ncclSuccess ? hipStreamSynchronize(d->st) : hipSuccess;
  if (r == ncclSuccess && e == hipSuccess) e = hipMemcpy(all, d_f + 1, sizeof(int), hipMemcpyDeviceToHost);
  (void)hipFree(d_f);
  CGX_NCCL(r);
  CGX_HIP(e);
  return 0;
}

// The fused step's group decision (all partitions or none), once per
// connection and after every cgx_dist_set_fused; collective over RCCL.
int ensure_fused_known(Group *g) {
  if (g->fz_known) return 0;
  if (g->parts[0]->local) {
    bool all = true, mall = true;
    for (cgx_dist *d : g->parts) {
      all = all && part_fusable(d);
      mall = mall && part_marchable(d);
    }
    for (cgx_dist *d : g->parts) {
      d->fz_all = all;
      d->mi_all = mall;
    }
  } else {
    cgx_dist *d = g->parts[0];
    int all = 0, mall = 0;
    int rc = agree_min(d, part_fusable(d) ? 1 : 0, &all);
    if (rc == 0) rc = agree_min(d, part_marchable(d) ? 1 : 0, &mall);
    if (rc) return rc;
    d->fz_all = all != 0;
    d->mi_all = mall != 0;
  }
  g->fz_known = true;
  return 0;
}

int ensure_connected_fz(Group *g);
bool sr1(const cgx_dist *d);
bool fz1(const cgx_dist *d);

// The second r, s, w buffers (ghosted, zeroed), allocated the first time a
// recurrence that alternates them runs -- the one-launch SR step, the fused
// CG1 step -- not for HS (3 n_loc doubles, 1.5 GB at C4 on one rank: ADVICE
// r03).  Before any graph capture (their pointers are captured).
int ensure_rsw2(Group *g) {
  for (cgx_dist *d : g->parts) {
    const bool x4 = sr1(d);  // the one-launch SR step's four p buffers
    if ((d->d_r2 && d->d_s2 && d->d_w2 && (!x4 || (d->d_p3 && d->d_p4))) || !(sr1(d) || fz1(d)))
      continue;
    CGX_HIP(hipSetDevice(d->device));
    int rc = 0;
    for (double **p : {&d->d_r2, &d->d_s2, &d->d_w2, &d->d_p3, &d->d_p4}) {
      if (!x4 && (p == &d->d_p3 || p == &d->d_p4)) continue;
      if (*p) continue;
      void *raw = nullptr;
      rc = dev_alloc(&raw, (d->vfront + d->ng_alloc) * 8, &d->vec_bytes);
      if (rc) break;
      *p = (double *)raw + d->vfront;
      if (hipMemsetAsync(raw, 0, (d->vfront + d->ng_alloc) * 8, d->st) != hipSuccess) {
        set_error("dist: zeroing the second r / s / w buffers failed");
        rc = CGX_ENODEV;
        break;
      }
    }
    if (!rc && hipStreamSynchronize(d->st) != hipSuccess) {
      set_error("dist: zeroing the second r / s / w buffers failed");
      rc = CGX_ENODEV;
    }
    if (rc) {  // none or all (a partial set ran with nulls)
      for (double **p : {&d->d_r2, &d->d_s2, &d->d_w2, &d->d_p3, &d->d_p4}) free_ghosted(d, p);
      return rc;
    }
  }
  return 0;
}

// connected, the fused step decided, the recurrence runnable on it and its
// buffers allocated
int ensure_connected(Group *g) {
  int rc = ensure_connected_fz(g);
  if (rc) return rc;
  return ensure_rsw2(g);
}

int ensure_connected_fz(Group *g) {
  if (!g->connected) {
    for (cgx_dist *d : g->parts)
      if (!d->have_matrix) {
        set_error("dist: every partition needs set_matrix before solving");
        return CGX_EINVAL;
      }
    int rc = g->parts[0]->local ? connect_local(g) : connect_rccl(g->parts[0]);
    if (rc) return rc;
    g->connected = true;
    g->fz_known = false;
  }
  return ensure_fused_known(g);
}

// ---------------------------------------------------------- phase helpers

// the vector the SpMV gathers (its ghost tail is the halo) and its output;
// fused: the p_new buffer
// the one-launch SR step rotates four p buffers (x deferred four iterations
// deep: p_{k-3}, p_{k-2}, p_{k-1} in p_new, p_rot(2), p_rot(3); CgState::xdef,
// as the single-GPU solver), every other recurrence alternates two; r, s, w
// alternate with pbuf's parity
int prot(const cgx_dist *d) { return sr1(d) ? 4 : 2; }
double *p_rot(cgx_dist *d, int i) {
  double *b[4] = {d->d_p, d->d_p2, d->d_p3, d->d_p4};
  return b[(d->pbuf + i) % prot(d)];
}
double *p_old(cgx_dist *d) { return p_rot(d, 0); }
double *p_new(cgx_dist *d) { return p_rot(d, 1); }
// fused CG1: r, s, w of the last iteration (read) and of this one (written)
double *r_old(cgx_dist *d) { return (d->pbuf & 1) ? d->d_r2 : d->d_r; }
double *r_new(cgx_dist *d) { return (d->pbuf & 1) ? d->d_r : d->d_r2; }
double *s_old(cgx_dist *d) { return (d->pbuf & 1) ? d->d_s2 : d->d_s; }
double *s_new(cgx_dist *d) { return (d->pbuf & 1) ? d->d_s : d->d_s2; }
double *w_old(cgx_dist *d) { return (d->pbuf & 1) ? d->d_w2 : d->d_w; }
double *w_new(cgx_dist *d) { return (d->pbuf & 1) ? d->d_w : d->d_w2; }
double *spmv_x(cgx_dist *d) {
  if (!hs_like(d)) return fz1(d) ? r_new(d) : d->d_r;
  return fz(d) ? p_new(d) : d->d_p;
}
// r.r of the last r update, as the fused step reads it (SR: k_update_rf's
// alpha^2 s.s - r.r)
const double *rr_new_src(cgx_dist *d) {
  return solo(d) || sr(d) ? &d->d_st->rr_new : d->d_gsums + 1;
}
double *spmv_y(cgx_dist *d) {
  return hs_like(d) ? d->d_s : fz1(d) ? w_new(d) : d->d_w;
}

// A rank with neighbours: ghost rows to receive or rows to send.  Without
// any (one rank, a rank the matrix does not couple) the halo phases are
// skipped entirely: no fork of the communication stream, no events.
bool has_peers(const cgx_dist *d) { return !solo(d) && (d->n_send > 0 || d->n_ghost > 0); }

// pack the send rows of the gathered vector (after its update; fused HS:
// p_new = r + beta p_old computed at the send rows; fused CG1: r_new) on the
// communication stream, forked from the iteration's stream here: the pack
// runs beside the interior SpMV instead of in front of it, and the halo
// send/recv follow it on the same stream.  The fork is a plain record on st
// + wait on st_comm; the join is phase_spmv's wait on ev_halo.  (Round 2's
// variant also waited, on st_comm, for an event recorded on st_comm itself,
// with nothing captured between: the 1-rank capture of that shape crashed
// the host process.  Neither a self-wait nor an empty fork remains.)
int phase_pack(cgx_dist *d) {
  if (!has_peers(d)) return 0;
  CGX_HIP(hipSetDevice(d->device));
  CGX_HIP(hipEventRecord(d->ev_fork, d->st));
  CGX_HIP(hipStreamWaitEvent(d->st_comm, d->ev_fork, 0));
  if (sr1(d))
    CGX_HIP(launch_pack_sr<double>(d->n_send, d->d_send_idx, r_old(d), p_old(d), s_old(d),
                                   d->d_sendbuf, d->d_st, d->st_comm, sr1_g(d)));
  else if (fz(d))
    CGX_HIP(launch_pack_pnext<double>(d->n_send, d->d_send_idx, d->d_r, p_old(d), d->d_sendbuf,
                                      d->d_st, rr_new_src(d), d->st_comm));
  else if (fz1(d))
    CGX_HIP(launch_pack_rnext<double>(d->n_send, d->d_send_idx, r_old(d), w_old(d), s_old(d),
                                      d->d_sendbuf, d->d_st, d->st_comm));
  else
    CGX_HIP(launch_gather<double>(d->n_send, d->d_send_idx, spmv_x(d), d->d_sendbuf, d->st_comm));
  // the local transport's peers copy from d_sendbuf on their own streams
  if (d->local) CGX_HIP(hipEventRecord(d->ev_packed, d->st_comm));
  return 0;
}

// halo exchange on the communication stream (after this rank's pack, in
// stream order), straight into the ghost tail; ev_halo joins it back
int phase_halo(cgx_dist *d) {
  if (!has_peers(d)) return 0;
  CGX_HIP(hipSetDevice(d->device));
  // owner q's ghost rows: the gathered vector's tail at recv_off[q], or (the
  // one-launch SR step's in-place numbering) p_new at recv_pos[q]
  const bool ip = sr1(d);
  double *ghost = ip ? p_new(d) : spmv_x(d) + d->n_loc;
  auto dst = [&](int q) { return ghost + (ip ? d->recv_pos[(size_t)q] : d->recv_off[q]); };
  if (d->local) {
    for (cgx_dist *o : d->group->parts) {
      if (o == d || d->recv_count[o->rank] == 0) continue;
      CGX_HIP(hipStreamWaitEvent(d->st_comm, o->ev_packed, 0));
      CGX_HIP(hipMemcpyAsync(dst(o->rank), o->d_sendbuf + o->send_off[d->rank],
                             (size_t)d->recv_count[o->rank] * 8, hipMemcpyDeviceToDevice,
                             d->st_comm));
    }
  } else {
    ++d->nccl_calls;
    CGX_NCCL(ncclGroupStart());
    for (int q = 0; q < d->nranks; ++q) {
      if (q == d->rank) continue;
      if (d->recv_count[q])
        CGX_NCCL(ncclRecv(dst(q), d->recv_count[q], ncclFloat64, q, d->comm, d->st_comm));
      if (d->send_count[q])
        CGX_NCCL(ncclSend(d->d_sendbuf + d->send_off[q], d->send_count[q], ncclFloat64, q,
                          d->comm, d->st_comm));
    }
    CGX_NCCL(ncclGroupEnd());
  }
  CGX_HIP(hipEventRecord(d->ev_halo, d->st_comm));
  return 0;
}

// SpMV over interior items (overlapping the halo), then boundary items; with
// a transport, one k_finalize workgroup sums the partials in the canonical
// order into the local sums (HS: p.s -> sums[0]; CG1: gamma, delta ->
// sums[0..1]).  (An in-kernel last-arriver sum costs every one of the
// SpMV's ~15 K workgroups a drained store and a device-scope atomic before
// it may retire: 70 us on an 8 M-row slab, against ~5 us for the launch.)
int allreduce(cgx_dist *d, int i, int count);

// The one-launch SR step (k_sr1_dia_m on the in-place numbering): every step
// while the halo of p_k is in flight, then (a rank with neighbours) the edge
// rows' s and (p.s, s.s) after it (k_sr1_edge); then the local (p.s, s.s,
// r.r) (FIN_SUM3_SR1), or with no transport the scalar step
// itself (FIN_SR1, as the single-GPU solver).
int phase_sr1(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const bool rec = d->rec_spmv && d->ev_i + 4 <= d->spmv_ev.size();
  const Sr1Plan pl = sr1_plan(d);
  const SpmvArgs<double> a =
      d->Ai.args<double>(nullptr, s_new(d), nullptr, &d->d_st->done, d->Ai.all_items());
  Sr1Args<double> f{d->d_x, p_old(d), p_new(d), r_old(d), r_new(d), s_old(d), d->d_st,
                    d->d_pq, d->d_pc, pl.len};
  if (!d->d_p3 || !d->d_p4) {
    set_error("dist: the one-launch SR step's p buffers are not allocated");
    return CGX_EINVAL;
  }
  f.pa = p_rot(d, 2);  // p_{k-2}, p_{k-1}: x four iterations deep
  f.pb = p_rot(d, 3);
  f.g = sr1_g(d);
  f.nseg = pl.nseg;
  f.cw = pl.cw;
  f.sb = pl.sb;
  f.elo = pl.elo;
  f.ehi = pl.ehi;
  const int gi = sr1_grid(a, f);
  Sr1Args<double> fe = f;
  fe.pq = d->d_pq + 2 * (size_t)gi;
  fe.pc = d->d_pc + gi;
  const bool edge = has_peers(d);
  const int ge = edge ? sr1_edge_grid(a.n, fe) : 0;
  d->gi1 = gi;
  d->gb1 = ge;
  auto ev = [&](int e) {
    return rec ? LaunchEv{d->spmv_ev[d->ev_i + e], d->spmv_ev[d->ev_i + e + 1]} : LaunchEv{};
  };
  CGX_HIP(launch_sr1_march<double>(a, f, d->st, ev(0)));
  if (edge) {
    CGX_HIP(hipStreamWaitEvent(d->st, d->ev_halo, 0));
    CGX_HIP(launch_sr1_edge<double>(a, fe, d->st, ev(2)));
  } else if (rec) {  // the second event pair brackets nothing
    CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i + 2], d->st));
    CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i + 3], d->st));
  }
  if (rec) d->ev_i += 4;
  const int np = gi + ge;
  if (solo(d)) {
    CGX_HIP(launch_finalize(FIN_SR1, d->d_pq, np, nullptr, 0, d->d_st, d->d_hist, nullptr, d->st,
                            d->d_pc, np));
    return 0;
  }
  if (d->local)  // as phase_spmv: every part's last group sum has read d_sums
    for (cgx_dist *o : d->group->parts)
      if (o != d) CGX_HIP(hipStreamWaitEvent(d->st, o->ev_red, 0));
  // the previous all-reduce applied to the state, then the local sums
  CGX_HIP(launch_finalize(FIN_SUM3_SR1, d->d_pq, np, d->d_gsums, 3, d->d_st, d->d_hist,
                          d->d_sums, d->st, d->d_pc, np));
  CGX_HIP(hipEventRecord(d->ev_sums, d->st));
  return 0;
}

const double *sr1_g(const cgx_dist *d) { return solo(d) ? nullptr : d->d_gsums; }

// the iteration's one all-reduce of (p.s, s.s, r.r) -- the next iteration's
// kernels apply it (the stop test of the previous iteration, alpha, the
// estimate, beta: sr1_g); the r, p, s buffers swap roles
int sr1_reduce(cgx_dist *d) {
  if (!solo(d)) {
    int rc = allreduce(d, 0, 3);
    if (rc) return rc;
  }
  d->pbuf = (d->pbuf + 1) % prot(d);
  return 0;
}

int phase_spmv(cgx_dist *d) {
  if (sr1(d)) return phase_sr1(d);
  CGX_HIP(hipSetDevice(d->device));
  const bool rec = d->rec_spmv && d->ev_i + 4 <= d->spmv_ev.size();
  const int np = d->g_int + d->g_bnd;
  // SR: the fused launches write one (p.s, s.s) pair per workgroup
  auto fgrid = [&](const Items &it) {
    return it.count ? fused_grid(d->A.args<double>(nullptr, nullptr, nullptr, nullptr, it)) : 0;
  };
  const bool pairs = sru(d);  // unfused SR: (p.s, s.s) pairs, 2 doubles per partial
  const int gi = sr(d) && !pairs ? fgrid(d->it_int) : 0;
  const int gb = sr(d) && !pairs ? fgrid(d->it_bnd) : 0;
  // rec: kernel timing events (hipExtLaunchKernel) of the two launches; an
  // empty launch records both of its events on the stream instead
  auto launch = [&](const Items &it, double *part, int e) -> hipError_t {
    LaunchEv ev;
    if (rec) ev = LaunchEv{d->spmv_ev[d->ev_i + e], d->spmv_ev[d->ev_i + e + 1]};
    if (it.count == 0) {
      if (rec) {
        hipError_t r = hipEventRecord(ev.start, d->st);
        return r != hipSuccess ? r : hipEventRecord(ev.stop, d->st);
      }
      return hipSuccess;
    }
    SpmvArgs<double> a = d->A.args<double>(spmv_x(d), spmv_y(d), part, &d->d_st->done, it);
    if (fz1(d)) {
      // gamma partials beside the delta ones (d_pa / d_pb, same offsets)
      const Cg1Args<double> f{d->d_x,   d->d_p,     r_old(d), s_old(d), w_old(d),
                              r_new(d), s_new(d),   d->d_st,  d->d_pa + (part - d->d_pb),
                              e == 2 ? 1 : 0};
      return launch_cg1_fused<double>(a, f, d->st, ev);
    }
    if (fz(d)) {
      // the first non-empty launch publishes the scalar step; boundary
      // items (e == 2) read ghost columns' p_new from the halo
      const int pub = (e == 0 || d->it_int.count == 0) ? 1 : 0;
      const FuseArgs<double> f{d->d_x, p_old(d), p_new(d), d->d_r, d->d_st, d->d_hist,
                               rr_new_src(d), pub, e == 2 ? 1 : 0,
                               sr(d) ? d->d_pss + (e == 2 ? 2 * gi : 0) : nullptr};
      return launch_spmv_fused<double>(a, f, d->st, ev);
    }
    a.pair = pairs ? 1 : 0;
    return launch_spmv<double>(a, d->st, ev);
  };
  CGX_HIP(launch(d->it_int, d->d_pb, 0));
  if (has_peers(d)) CGX_HIP(hipStreamWaitEvent(d->st, d->ev_halo, 0));
  CGX_HIP(launch(d->it_bnd, d->d_pb + (pairs ? 2 : 1) * d->g_int, 2));
  if (rec) d->ev_i += 4;
  if (pairs && solo(d)) {  // the scalar step itself (the single-GPU solver's FIN_SR1)
    CGX_HIP(launch_finalize(FIN_SR1, d->d_pb, np, nullptr, 0, d->d_st, d->d_hist, nullptr, d->st,
                            d->d_pa, d->vec_grid));
    return 0;
  }
  if (solo(d) && !sr(d)) return 0;
  // local transport: every part's group sum of the last reduction must have
  // read this part's local sums before they are overwritten.  The halo orders
  // this part only after its NEIGHBOURS' packs, so without the wait a part
  // could overwrite its prologue b.b (or last r.r) while a distant part was
  // still summing it: a race at P >= 3, seen on C4's 8 slabs (x wrong in the
  // first group of a process).  RCCL ranks reduce on their own stream.
  if (d->local)
    for (cgx_dist *o : d->group->parts)
      if (o != d) CGX_HIP(hipStreamWaitEvent(d->st, o->ev_red, 0));
  if (pairs)  // the previous all-reduce applied to the state, then the local sums
    CGX_HIP(launch_finalize(FIN_SUM3_SR1, d->d_pb, np, d->d_gsums, 3, d->d_st, d->d_hist,
                            d->d_sums, d->st, d->d_pa, d->vec_grid));
  else if (sr(d))  // p.s, s.s, and r.r of the last r update (the prologue's b.b at first)
    CGX_HIP(launch_finalize(FIN_SUM3, d->d_pss, gi + gb, nullptr, 0, d->d_st, d->d_hist,
                            d->d_sums, d->st, d->d_pa, d->vec_grid));
  else if (d->alg == CGX_ALG_HS)
    CGX_HIP(launch_finalize(FIN_SUM, d->d_pb, np, nullptr, 0, d->d_st, d->d_hist, d->d_sums,
                            d->st));
  else
    CGX_HIP(launch_finalize(FIN_SUM2, d->d_pa, fz1(d) ? np : d->vec_grid, d->d_pb, np, d->d_st,
                            d->d_hist, d->d_sums, d->st));
  CGX_HIP(hipEventRecord(d->ev_sums, d->st));
  return 0;
}

// the all-reduce of `count` local sums starting at sums[i] -> gsums[i]
int allreduce(cgx_dist *d, int i, int count) {
  if (d->local) {
    for (cgx_dist *o : d->group->parts)
      if (o != d) CGX_HIP(hipStreamWaitEvent(d->st, i == 0 ? o->ev_sums : o->ev_sums2, 0));
    CGX_HIP(launch_group_sum(d->group->d_srcs, (int)d->group->parts.size(), count, d->d_gsums,
                             d->st, i));
    CGX_HIP(hipEventRecord(d->ev_red, d->st));
  } else {
    ++d->nccl_calls;
    CGX_NCCL(ncclAllReduce(d->d_sums + i, d->d_gsums + i, count, ncclFloat64, ncclSum, d->comm,
                           d->st));
  }
  return 0;
}

// ---- HS
// prologue: x = 0, r = p = b, b.b (cg.c:104-107)
int hs_init(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  CGX_HIP(launch_init_hs<double>(d->n_loc, d->d_b, d->d_x, d->d_r, d->d_p, d->d_pa, d->vec_grid,
                                 d->st));
  if (solo(d)) {
    CGX_HIP(launch_finalize(FIN_INIT_HS, d->d_pa, d->vec_grid, nullptr, 0, d->d_st, d->d_hist,
                            nullptr, d->st));
    return 0;
  }
  CGX_HIP(launch_finalize(FIN_SUM, d->d_pa, d->vec_grid, nullptr, 0, d->d_st, d->d_hist,
                          d->d_sums, d->st));
  CGX_HIP(hipEventRecord(d->ev_sums, d->st));
  return 0;
}

int hs_init_reduce(cgx_dist *d) {
  if (solo(d)) return 0;
  int rc = allreduce(d, 0, 1);
  if (rc) return rc;
  CGX_HIP(launch_finalize(FIN_INIT_HS, d->d_gsums, 1, nullptr, 0, d->d_st, d->d_hist, nullptr,
                          d->st));
  return 0;
}

// alpha step: all-reduced p.s, r -= alpha s, local r.r (last workgroup)
int hs_alpha(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const int gf = d->vec_grid / 4;  // 1024-thread workgroups, 4 partials each
  if (sr(d)) {
    // the iteration's one all-reduce: (p.s, s.s, r.r); the r.r partials of
    // this update stay local until the next iteration's finalize
    if (!solo(d)) {
      int rc = allreduce(d, 0, 3);
      if (rc) return rc;
    }
    CGX_HIP(launch_update_rf<double>(d->n_loc, d->d_r, d->d_s, d->d_st, nullptr, 0, d->d_pa, gf,
                                     d->st, nullptr, solo(d) ? d->d_sums : d->d_gsums,
                                     d->d_hist));
    return 0;
  }
  if (solo(d)) {
    const FinArgs fin{d->d_tick, d->d_pa, 4 * gf, &d->d_st->rr_new};
    CGX_HIP(launch_update_rf<double>(d->n_loc, d->d_r, d->d_s, d->d_st, d->d_pb,
                                     d->g_int + d->g_bnd, d->d_pa, gf, d->st,
                                     fz(d) ? &fin : nullptr));
    return 0;
  }
  int rc = allreduce(d, 0, 1);
  if (rc) return rc;
  const FinArgs fin{d->d_tick, d->d_pa, 4 * gf, d->d_sums + 1};
  CGX_HIP(launch_update_rf<double>(d->n_loc, d->d_r, d->d_s, d->d_st, d->d_gsums, 1, d->d_pa, gf,
                                   d->st, &fin));  // cg.c:113, 118-123
  CGX_HIP(hipEventRecord(d->ev_sums2, d->st));
  return 0;
}

// beta step: all-reduced r.r, stop test, x += alpha p, p = r + beta p
int hs_beta(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const int gf = d->vec_grid / 4;
  const double *rr = d->d_pa;
  int nrr = 4 * gf;
  if (!solo(d)) {
    int rc = allreduce(d, 1, 1);
    if (rc) return rc;
    rr = d->d_gsums + 1;
    nrr = 1;
  }
  CGX_HIP(launch_xpay_xf<double>(d->n_loc, d->d_x, d->d_p, d->d_p, d->d_r, d->d_st, rr, nrr,
                                 d->d_hist, gf, d->st));  // cg.c:115-116, 125-132
  return 0;
}

// unfused SR: the iteration's one all-reduce, then r, p (in place) and x
// in one pass, the all-reduced sums applied privately (sr1_now)
int sru_update(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  if (!solo(d)) {
    int rc = allreduce(d, 0, 3);
    if (rc) return rc;
  }
  CGX_HIP(launch_update_sr<double>(d->n_loc, d->d_x, d->d_r, d->d_s, d->d_p, d->d_p, d->d_st,
                                   solo(d) ? nullptr : d->d_gsums, d->d_pa, d->vec_grid / 4,
                                   d->st, false));
  return 0;
}

// ---- CG1
// (fused CG1: the vector recurrences run inside the SpMV launch; only the
// halo rows of r_new are packed here)
int cg1_update(cgx_dist *d, bool init) {
  CGX_HIP(hipSetDevice(d->device));
  if (init)
    CGX_HIP(launch_init_cg1<double>(d->n_loc, d->d_b, d->d_x, d->d_r, d->d_p, d->d_s, d->d_pa,
                                    d->vec_grid, d->st));
  else if (!fz1(d))
    CGX_HIP(launch_cg1_update<double>(d->n_loc, d->d_x, d->d_p, d->d_r, d->d_s, d->d_w, d->d_st,
                                      d->d_pa, d->vec_grid, d->st));
  return phase_pack(d);
}

int cg1_reduce(cgx_dist *d, bool init) {
  CGX_HIP(hipSetDevice(d->device));
  const int op = init ? FIN_INIT_CG1 : FIN_CG1;
  const int np = d->g_int + d->g_bnd;
  if (solo(d)) {
    CGX_HIP(launch_finalize(op, d->d_pa, fz1(d) ? np : d->vec_grid, d->d_pb, np, d->d_st,
                            d->d_hist, nullptr, d->st));
    if (fz1(d)) d->pbuf ^= 1;
    return 0;
  }
  int rc = allreduce(d, 0, 2);
  if (rc) return rc;
  CGX_HIP(launch_finalize(op, d->d_gsums, 1, d->d_gsums + 1, 1, d->d_st, d->d_hist, nullptr, d->st));
  if (fz1(d)) d->pbuf ^= 1;
  return 0;
}

// fused: the all-reduce of the local r.r (the next iteration's beta), and
// the p buffers swap roles
int fz_close(cgx_dist *d) {
  if (!solo(d) && !sr(d)) {
    int rc = allreduce(d, 1, 1);
    if (rc) return rc;
  }
  d->pbuf ^= 1;
  return 0;
}

int run_phases_eager(Group *g, bool init, long long iters) {
  auto &P = g->parts;
  int rc;
  if (hs_like(P[0])) {
    if (init) {
      for (cgx_dist *d : P) d->pbuf = 0;  // the prologue writes p into d_p
      for (cgx_dist *d : P) if ((rc = hs_init(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_init_reduce(d))) return rc;
      return 0;
    }
    if (sr1(P[0])) {
      for (long long it = 0; it < iters; ++it) {
        for (cgx_dist *d : P) if ((rc = phase_pack(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_sr1(d))) return rc;
        for (cgx_dist *d : P) if ((rc = sr1_reduce(d))) return rc;
      }
      return 0;
    }
    if (sru(P[0])) {
      for (long long it = 0; it < iters; ++it) {
        for (cgx_dist *d : P) if ((rc = phase_pack(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_spmv(d))) return rc;
        for (cgx_dist *d : P) if ((rc = sru_update(d))) return rc;
      }
      return 0;
    }
    if (fz(P[0])) {
      for (long long it = 0; it < iters; ++it) {
        for (cgx_dist *d : P) if ((rc = phase_pack(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
        for (cgx_dist *d : P) if ((rc = phase_spmv(d))) return rc;
        for (cgx_dist *d : P) if ((rc = hs_alpha(d))) return rc;
        for (cgx_dist *d : P) if ((rc = fz_close(d))) return rc;
      }
      return 0;
    }
    // each iteration packs its own halo first, so a captured batch has no
    // dependency on work outside it
    for (long long it = 0; it < iters; ++it) {
      for (cgx_dist *d : P) if ((rc = phase_pack(d))) return rc;
      for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
      for (cgx_dist *d : P) if ((rc = phase_spmv(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_alpha(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_beta(d))) return rc;
    }
    return 0;
  }
  // the prologue (x = 0, r = b, w = A r) runs the unfused phases
  for (cgx_dist *d : P) {
    d->in_init = init;
    if (init) d->pbuf = 0;  // the prologue writes r, s, w into the first buffers
  }
  rc = 0;
  for (long long it = 0; it < (init ? 1 : iters) && rc == 0; ++it) {
    for (cgx_dist *d : P) if (rc == 0) rc = cg1_update(d, init);
    for (cgx_dist *d : P) if (rc == 0) rc = phase_halo(d);
    for (cgx_dist *d : P) if (rc == 0) rc = phase_spmv(d);
    for (cgx_dist *d : P) if (rc == 0) rc = cg1_reduce(d, init);
  }
  for (cgx_dist *d : P) d->in_init = false;
  return rc;
}

// CGX_DIST_TRACE=1: the capture / replay steps on stderr (diagnosis of a
// capture that fails inside the HIP runtime or RCCL)
bool dist_trace() {
  static const bool on = [] {
    const char *e = getenv("CGX_DIST_TRACE");
    return e && *e && *e != '0';
  }();
  return on;
}
#define DIST_TRACE(...)                          \
  do {                                           \
    if (dist_trace()) {                          \
      fprintf(stderr, "cgx_dist: " __VA_ARGS__); \
      fflush(stderr);                            \
    }                                            \
  } while (0)

// Capture `nit` iterations (kernels, halo send/recv on the comm stream
// forked and joined by events, all-reduces) into *out, without running them.
// Returns 1 when captured, 0 when the capture was refused before any RCCL
// call was recorded (nothing reached the communicator: eager is safe), -1
// when it was refused after RCCL calls were recorded.  Every outcome comes
// back as one of these (never as an early error return), so every rank
// reaches ensure_graphs' agreement.
int capture(cgx_dist *d, Group *g, int nit, int parity, hipGraphExec_t *out) {
  hipGraph_t gr = nullptr;
  *out = nullptr;
  DIST_TRACE("rank %d capture of %d iterations, parity %d\n", d->rank, nit, parity);
  if (hipSetDevice(d->device) != hipSuccess ||
      hipStreamBeginCapture(d->st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  const int saved = d->pbuf;
  const long long calls0 = d->nccl_calls;
  d->pbuf = parity;
  // cgx_dist_debug_refuse_capture(1): refused before the first phase
  const int rc = d->dbg_refuse == 1 ? CGX_ENODEV : run_phases_eager(g, false, nit);
  DIST_TRACE("rank %d phases recorded (rc %d)\n", d->rank, rc);
  // (modes 2 and 3: refused after the phases recorded their RCCL calls)
  const hipError_t e = hipStreamEndCapture(d->st, &gr);
  DIST_TRACE("rank %d end capture: %s\n", d->rank, hipGetErrorString(e));
  d->pbuf = saved;
  hipError_t ei = hipSuccess;
  const bool refused = rc || e != hipSuccess || d->dbg_refuse >= 2;
  if (!refused) ei = hipGraphInstantiate(out, gr, nullptr, nullptr, 0);
  DIST_TRACE("rank %d instantiate: %s\n", d->rank, hipGetErrorString(ei));
  if (gr) (void)hipGraphDestroy(gr);
  if (refused || ei != hipSuccess) {
    if (*out) (void)hipGraphExecDestroy(*out);
    *out = nullptr;
    (void)hipGetLastError();
    return d->nccl_calls > calls0 ? -1 : 0;
  }
  return 1;
}

bool graphs_on(const cgx_dist *d) {
  return !d->local && d->use_graph && d->graph_state >= 0 && d->graph_batch > 0 && !d->rec_spmv;
}

// The replayed graphs of the current recurrence: graph_batch iterations and
// one iteration (remainders), captured once -- by bench_prepare, so a timed
// region only replays.  Graph or eager is a COLLECTIVE decision: each rank's
// capture result (1 captured, 0 refused before any RCCL call was recorded,
// -1 refused after) is MIN- and MAX-all-reduced, and
//   every rank captured            -> every rank replays its graphs;
//   every rank refused at the same
//   point (all 0, or all -1)       -> every rank drops its graphs and runs
//                                     eager (graph_state -1 on all ranks:
//                                     the same RCCL calls, or none, were
//                                     recorded everywhere, so their send /
//                                     recv sequences stay equal -- e.g. a
//                                     refusal inside RCCL itself, which hits
//                                     every rank alike);
//   a mix (some ranks recorded RCCL
//   calls that others did not)     -> CGX_ECOMM on every rank, and the
//                                     communicator is marked unusable
//                                     (comm_fatal): the ranks' host-side
//                                     RCCL state may be out of step.
// Nothing captured is ever enqueued, so the decision costs two all-reduces
// of an int per capture (once per recurrence).
int ensure_graphs(Group *g) {
  cgx_dist *d = g->parts[0];
  if (!graphs_on(d)) return 0;
  const int key = d->alg * 8 + (fz(d) || fz1(d) ? 1 : 0) + (sr1(d) ? 2 : 0);
  if (d->gexec[0] && d->gexec1[0] && d->gexec_alg == key) return 0;
  drop_graph(d);
  const int nq = sr1(d) ? 4 : fz(d) || fz1(d) ? 2 : 1;
  int mine = 1;
  for (int q = 0; q < nq && mine == 1; ++q) {
    mine = capture(d, g, d->graph_batch, q, &d->gexec[q]);
    if (mine == 1) mine = capture(d, g, 1, q, &d->gexec1[q]);
  }
  int lo = mine, neg_hi = -mine;
  int rc = agree_min(d, mine, &lo);
  if (rc == 0) rc = agree_min(d, -mine, &neg_hi);
  // cgx_dist_debug_refuse_capture(3): as if the peers had captured (the mix)
  const int hi = d->dbg_refuse == 3 ? 1 : -neg_hi;
  if (rc || lo < 1) drop_graph(d);
  if (rc) return rc;
  if (lo < 1 && lo == hi) {
    d->graph_state = -1;  // every rank: eager from now on
    return 0;
  }
  if (lo < 1) {
    d->comm_fatal = true;
    d->graph_state = -1;
    set_error("dist: a rank's hipGraph capture failed after RCCL calls were recorded (or "
              "the ranks' captures disagree); the communicator is no longer usable");
    return CGX_ECOMM;
  }
  d->gexec_alg = key;
  d->graph_state = 1;
  DIST_TRACE("rank %d graphs agreed\n", d->rank);
  return 0;
}

int run_phases(Group *g, bool init, long long iters) {
  cgx_dist *d = g->parts[0];
  if (d->comm_fatal) {
    set_error("dist: the communicator is unusable after a failed capture (ensure_graphs)");
    return CGX_ECOMM;
  }
  if (!init && graphs_on(d)) {
    int rc = ensure_graphs(g);
    if (rc) return rc;
    if (d->gexec[0] && d->gexec1[0]) {
      // the graph captured at the current buffer rotation; a batch
      // advances it by graph_batch, one iteration by one
      const int nr = sr1(d) ? 4 : fz(d) || fz1(d) ? 2 : 1;
      DIST_TRACE("rank %d replay of %lld iterations\n", d->rank, iters);
      for (; iters >= d->graph_batch; iters -= d->graph_batch) {
        CGX_HIP(hipGraphLaunch(d->gexec[d->pbuf % nr], d->st));
        d->pbuf = (d->pbuf + d->graph_batch) % nr;
      }
      for (; iters > 0; --iters) {
        CGX_HIP(hipGraphLaunch(d->gexec1[d->pbuf % nr], d->st));
        d->pbuf = (d->pbuf + 1) % nr;
      }
      return 0;
    }
  }
  return run_phases_eager(g, init, iters);
}

int prepare_states(Group *g, int maxit, double tol, int hist_cap) {
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipSetDevice(d->device));
    CGX_HIP(hipMemsetAsync(d->d_tick, 0, kTickRegion * sizeof(unsigned), d->st));
    if (hist_cap > d->hist_alloc) {
      if (d->gexec[0]) {  // the captured graph holds the old history pointer
        CGX_HIP(hipStreamSynchronize(d->st));
        drop_graph(d);
      }
      dev_free(&d->d_hist);
      int rc = dev_alloc(&d->d_hist, (size_t)hist_cap * 8, nullptr);
      if (rc) return rc;
      d->hist_alloc = hist_cap;
    }
    memset(d->h_st, 0, sizeof(CgState));
    d->h_st->tol = tol;
    d->h_st->use_tol = tol > 0.0 ? 1 : 0;
    d->h_st->max_iter = maxit;
    d->h_st->hist_cap = std::min(hist_cap, d->hist_alloc);
    d->h_st->xdef = sr1(d) ? 4 : 2;
    CGX_HIP(hipMemcpyAsync(d->d_st, d->h_st, sizeof(CgState), hipMemcpyHostToDevice, d->st));
  }
  return 0;
}

int read_states(Group *g) {
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipSetDevice(d->device));
    CGX_HIP(hipMemcpyAsync(d->h_st, d->d_st, sizeof(CgState), hipMemcpyDeviceToHost, d->st));
  }
  for (cgx_dist *d : g->parts) CGX_HIP(hipStreamSynchronize(d->st));
  return 0;
}

int group_run(Group *g, int maxit, double tol, int *iters) {
  int rc;
  for (cgx_dist *d : g->parts)
    if (!d->have_matrix || !d->have_rhs) {
      set_error("dist run: every partition needs matrix and rhs");
      return CGX_EINVAL;
    }
  if (maxit < 0) return CGX_EINVAL;
  if ((rc = ensure_connected(g))) return rc;
  for (cgx_dist *d : g->parts) d->bench_ready = false;
  if ((rc = prepare_states(g, maxit, tol, maxit + 1))) return rc;
  if ((rc = run_phases(g, true, 1))) return rc;
  // the fused step does an iteration's x update in the next launch: one
  // more step carries the last one (and finds the stop); SR tests iteration
  // k's stop on the exact r.r of the next reduction: one more, and it is
  // complete at done = 2 (an even stop iteration's x update still pending
  // at 1)
  const bool sr0 = sr(g->parts[0]);
  // (the folded FIN_SR1 marks the stop one iteration later: one more)
  // (unfused SR: the stop of iteration maxit is known to update_sr(maxit + 1)
  // and reaches the state with the next FIN_SUM3_SR1: two more)
  const long long total = (long long)maxit + 1 + (fz(g->parts[0]) || sr1(g->parts[0]) ? 1 : 0) +
                          (sr0 ? 1 : 0) + (sr1(g->parts[0]) && sr1_g(g->parts[0]) ? 1 : 0) +
                          (sru(g->parts[0]) ? 2 : 0);
  const int fin_done = sr0 ? 2 : 1;
  if (tol <= 0.0) {
    if ((rc = run_phases(g, false, total))) return rc;
    if ((rc = read_states(g))) return rc;
  } else {
    long long done = 0, batch = 16;
    double rr_prev = 0.0;
    int k_prev = -1;
    for (;;) {
      const long long b = std::min(batch, total - done);
      if ((rc = run_phases(g, false, b))) return rc;
      done += b;
      if ((rc = read_states(g))) return rc;
      const CgState *h = g->parts[0]->h_st;
      if (h->done >= fin_done || done >= total) break;
      // every rank sees the same all-reduced r.r: the same batches everywhere
      batch = next_batch(h->rr, h->tol2bb, h->k, rr_prev, k_prev, batch);
      rr_prev = h->rr;
      k_prev = h->k;
    }
  }
  const CgState *s0 = g->parts[0]->h_st;
  for (cgx_dist *d : g->parts)
    if (!d->h_st->done || d->h_st->k != s0->k) {
      set_error("dist run: partitions disagree on the stop condition");
      return CGX_ECOMM;
    }
  for (cgx_dist *d : g->parts) d->last_iters = s0->k + 1;
  if (iters) *iters = s0->k + 1;
  return 0;
}

int group_bench_prepare(Group *g, int warmup) {
  int rc;
  for (cgx_dist *d : g->parts)
    if (!d->have_matrix || !d->have_rhs || d->n_loc == 0) return CGX_EINVAL;
  if ((rc = ensure_connected(g))) return rc;
  if ((rc = prepare_states(g, INT_MAX - 1, 0.0, 0))) return rc;
  if ((rc = run_phases(g, true, 1))) return rc;
  if ((rc = ensure_graphs(g))) return rc;  // captured here, not in the timed region
  if ((rc = run_phases(g, false, warmup))) return rc;
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipStreamSynchronize(d->st));
    d->bench_ready = true;
  }
  return 0;
}

int group_bench_run(Group *g, int iters, int flags, double *ms, double *spmv_ms) {
  for (cgx_dist *d : g->parts)
    if (!d->bench_ready) return CGX_EINVAL;
  cgx_dist *d0 = g->parts[0];
  const bool per_spmv = (flags & CGX_BENCH_SPMV_EVENTS) != 0;
  if (per_spmv) {
    CGX_HIP(hipSetDevice(d0->device));
    while (d0->spmv_ev.size() < 4 * (size_t)iters) {
      hipEvent_t e;
      CGX_HIP(hipEventCreate(&e));
      d0->spmv_ev.push_back(e);
    }
    d0->ev_i = 0;
    d0->rec_spmv = true;
  }
  const bool graph_saved = d0->use_graph;
  d0->use_graph = graph_saved && (flags & CGX_BENCH_GRAPH) != 0;
  hipEvent_t e0, e1;
  CGX_HIP(hipSetDevice(d0->device));
  CGX_HIP(hipEventCreate(&e0));
  CGX_HIP(hipEventCreate(&e1));
  CGX_HIP(hipEventRecord(e0, d0->st));
  int rc = run_phases(g, false, iters);
  d0->rec_spmv = false;
  d0->use_graph = graph_saved;
  if (rc) return rc;
  for (cgx_dist *d : g->parts)
    if (d != d0) {
      CGX_HIP(hipEventRecord(d->ev_sums, d->st));
      CGX_HIP(hipStreamWaitEvent(d0->st, d->ev_sums, 0));
    }
  CGX_HIP(hipEventRecord(e1, d0->st));
  CGX_HIP(hipEventSynchronize(e1));
  float f = 0.f;
  CGX_HIP(hipEventElapsedTime(&f, e0, e1));
  *ms = f;
  *spmv_ms = -1.0;
  if (per_spmv) {
    // per iteration on partition 0: the first launch (interior / march), the
    // gap to the second (the halo wait), the second (boundary / edge), and
    // the tail up to the next iteration's first launch (local sums, the
    // all-reduce(s), the vector updates, the next pack) -- averaged
    double sum = 0.0, ph[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < iters; ++i) {
      float a = 0.f, gap = 0.f, b = 0.f;
      CGX_HIP(hipEventElapsedTime(&a, d0->spmv_ev[4 * i], d0->spmv_ev[4 * i + 1]));
      CGX_HIP(hipEventElapsedTime(&gap, d0->spmv_ev[4 * i + 1], d0->spmv_ev[4 * i + 2]));
      CGX_HIP(hipEventElapsedTime(&b, d0->spmv_ev[4 * i + 2], d0->spmv_ev[4 * i + 3]));
      sum += (double)a + (double)b;
      ph[0] += a;
      ph[1] += gap;
      ph[2] += b;
      if (i + 1 < iters) {
        float tail = 0.f, per = 0.f;
        CGX_HIP(hipEventElapsedTime(&tail, d0->spmv_ev[4 * i + 3], d0->spmv_ev[4 * i + 4]));
        CGX_HIP(hipEventElapsedTime(&per, d0->spmv_ev[4 * i], d0->spmv_ev[4 * i + 4]));
        ph[3] += tail;
        ph[4] += per;
      }
    }
    *spmv_ms = sum / iters;
    for (int k = 0; k < 3; ++k) d0->phase_ms[k] = ph[k] / iters;
    for (int k = 3; k < 5; ++k) d0->phase_ms[k] = iters > 1 ? ph[k] / (iters - 1) : -1.0;
    d0->phase_iters = iters;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if ((rc = read_states(g))) return rc;
  if (d0->h_st->done) {
    set_error("dist bench: solver stopped early");
    return CGX_EINVAL;
  }
  return 0;
}

void destroy_one(cgx_dist *d) {
  (void)hipSetDevice(d->device);
  if (d->st) (void)hipStreamSynchronize(d->st);
  if (d->st_comm) (void)hipStreamSynchronize(d->st_comm);
  free_system(d);
  if (d->comm) ncclCommDestroy(d->comm);
  if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
  if (d->ev_packed) (void)hipEventDestroy(d->ev_packed);
  if (d->ev_halo) (void)hipEventDestroy(d->ev_halo);
  if (d->ev_sums) (void)hipEventDestroy(d->ev_sums);
  if (d->ev_sums2) (void)hipEventDestroy(d->ev_sums2);
  if (d->ev_red) (void)hipEventDestroy(d->ev_red);
  for (hipEvent_t e : d->spmv_ev) (void)hipEventDestroy(e);
  if (d->d_st) (void)hipFree(d->d_st);
  if (d->d_sums) (void)hipFree(d->d_sums);
  if (d->d_tick) (void)hipFree(d->d_tick);
  if (d->h_st) (void)hipHostFree(d->h_st);
  if (d->st) (void)hipStreamDestroy(d->st);
  if (d->st_comm) (void)hipStreamDestroy(d->st_comm);
  delete d;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" {

int cgx_runtime_versions(int *hip_runtime, int *hip_compiled, int *rccl) {
  if (hip_runtime) {
    *hip_runtime = 0;
    CGX_HIP(hipRuntimeGetVersion(hip_runtime));
  }
  if (hip_compiled) *hip_compiled = HIP_VERSION;
  if (rccl) {
    *rccl = 0;
    CGX_NCCL(ncclGetVersion(rccl));
  }
  return 0;
}

int cgx_dist_unique_id(unsigned char id[128]) {
  if (!id) return CGX_EINVAL;
  ncclUniqueId u;
  CGX_NCCL(ncclGetUniqueId(&u));
  memcpy(id, u.internal, sizeof u.internal);
  return 0;
}

int cgx_dist_create(int device, int nranks, int rank, const unsigned char id[128],
                    cgx_dist **out) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !id)) {
    set_error("cgx_dist_create: bad arguments");
    return CGX_EINVAL;
  }
  *out = nullptr;
  cgx_dist *d = new cgx_dist();
  d->nranks = nranks;
  d->rank = rank;
  int rc = init_common(d, device);
  if (rc) {
    destroy_one(d);
    return rc;
  }
  if (id) {  // nranks == 1 with an id: a 1-rank communicator (see solo())
    ncclUniqueId u;
    memcpy(u.internal, id, sizeof u.internal);
    ncclResult_t r = ncclCommInitRank(&d->comm, nranks, u, rank);
    if (r != ncclSuccess) {
      set_error("ncclCommInitRank(%d of %d) failed: %s", rank, nranks, ncclGetErrorString(r));
      destroy_one(d);
      return CGX_ECOMM;
    }
  }
  Group *g = new Group();
  g->parts.push_back(d);
  d->group = g;
  d->owns_group = true;
  *out = d;
  return 0;
}

int cgx_dist_create_local(int device, int nparts, cgx_dist **parts) {
  if (!parts || nparts < 1) return CGX_EINVAL;
  Group *g = new Group();
  for (int p = 0; p < nparts; ++p) {
    cgx_dist *d = new cgx_dist();
    d->nranks = nparts;
    d->rank = p;
    d->local = true;
    int rc = init_common(d, device);
    if (rc) {
      destroy_one(d);
      for (cgx_dist *o : g->parts) destroy_one(o);
      delete g;
      return rc;
    }
    d->group = g;
    g->parts.push_back(d);
  }
  g->parts[0]->owns_group = true;
  for (int p = 0; p < nparts; ++p) parts[p] = g->parts[p];
  return 0;
}

void cgx_dist_destroy(cgx_dist *d) {
  if (!d) return;
  Group *g = d->group;
  if (d->local) {
    if (!d->owns_group) return;  // local parts are destroyed through part 0
    std::vector<cgx_dist *> parts = g->parts;
    if (g->d_srcs) (void)hipFree((void *)g->d_srcs);
    for (cgx_dist *o : parts) destroy_one(o);
    delete g;
    return;
  }
  destroy_one(d);
  delete g;
}

int cgx_dist_set_layout(cgx_dist *d, int layout) {
  if (!d || layout < CGX_LAYOUT_AUTO || layout > CGX_LAYOUT_DIA) return CGX_EINVAL;
  d->want_layout = layout;
  return 0;
}

int cgx_dist_set_fused(cgx_dist *d, int mode) {
  if (!d || (d->local && !d->owns_group) || mode < CGX_FUSE_OFF || mode > CGX_FUSE_ON)
    return CGX_EINVAL;
  for (cgx_dist *o : d->group->parts) {
    if (o->gexec[0]) {
      (void)hipStreamSynchronize(o->st);
      drop_graph(o);
    }
    o->fuse = mode;
    o->bench_ready = false;
  }
  d->group->fz_known = false;
  return 0;
}

int cgx_dist_set_march(cgx_dist *d, int steps) {
  if (!d || (d->local && !d->owns_group) || steps < -1) return CGX_EINVAL;
  for (cgx_dist *o : d->group->parts) {
    if (o->gexec[0]) {
      (void)hipStreamSynchronize(o->st);
      drop_graph(o);
    }
    o->march = steps;
    o->bench_ready = false;
  }
  d->group->fz_known = false;
  return 0;
}

int cgx_dist_set_sr_chain(cgx_dist *d, int rows) {
  if (!d || (d->local && !d->owns_group) || rows < 0) return CGX_EINVAL;
  for (cgx_dist *o : d->group->parts) {
    if (o->gexec[0]) {
      (void)hipStreamSynchronize(o->st);
      drop_graph(o);
    }
    o->sr_chain = rows;
    o->bench_ready = false;
  }
  return 0;
}

int cgx_dist_set_graph(cgx_dist *d, int on) {
  if (!d) return CGX_EINVAL;
  d->use_graph = on != 0;
  d->graph_state = 0;  // (re)try a capture at the next run
  drop_graph(d);
  return 0;
}

int cgx_dist_debug_refuse_capture(cgx_dist *d, int mode) {
  if (!d || mode < 0 || mode > 3) return CGX_EINVAL;
  d->dbg_refuse = mode;
  d->graph_state = 0;  // the next run captures (and is refused) anew
  drop_graph(d);
  return 0;
}

int cgx_dist_set_matrix(cgx_dist *d, long long n_global, int n_loc, int nnz, const int *row_ptr,
                        const int *col_global, const double *val) {
  if (!d) return CGX_EINVAL;
  return upload_local(d, n_global, n_loc, nnz, row_ptr, col_global, val);
}

int cgx_dist_set_rhs(cgx_dist *d, const double *b_local) {
  if (!d || !d->have_matrix || (d->n_loc > 0 && !b_local)) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(d->device));
  if (d->n_loc) CGX_HIP(hipMemcpy(d->d_b, b_local, (size_t)d->n_loc * 8, hipMemcpyHostToDevice));
  d->have_rhs = true;
  return 0;
}

int cgx_dist_run(cgx_dist *d, int maxit, double tol, int *iters) {
  if (!d || (d->local && !d->owns_group)) {
    set_error("cgx_dist_run: pass partition 0 of a local group");
    return CGX_EINVAL;
  }
  return group_run(d->group, maxit, tol, iters);
}

int cgx_dist_get_x(cgx_dist *d, double *x_local) {
  if (!d || !d->have_matrix || (d->n_loc > 0 && !x_local)) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(d->device));
  if (d->n_loc) CGX_HIP(hipMemcpy(x_local, d->d_x, (size_t)d->n_loc * 8, hipMemcpyDeviceToHost));
  return 0;
}

int cgx_dist_get_history(cgx_dist *d, double *rr, int cap) {
  if (!d || !rr || cap < 0) return CGX_EINVAL;
  const int m = std::min(cap, std::min(d->last_iters, d->hist_alloc));
  if (m <= 0) return 0;
  CGX_HIP(hipSetDevice(d->device));
  CGX_HIP(hipMemcpy(rr, d->d_hist, (size_t)m * 8, hipMemcpyDeviceToHost));
  return m;
}

int cgx_dist_bench_prepare(cgx_dist *d, int warmup) {
  if (!d || warmup < 0 || (d->local && !d->owns_group)) return CGX_EINVAL;
  return group_bench_prepare(d->group, warmup);
}

int cgx_dist_bench_phases(cgx_dist *d, double *ms, int *iters) {
  if (!d || !ms || (d->local && !d->owns_group)) return CGX_EINVAL;
  const cgx_dist *d0 = d->group->parts[0];
  for (int k = 0; k < 5; ++k) ms[k] = d0->phase_ms[k];
  if (iters) *iters = d0->phase_iters;
  return 0;
}

int cgx_dist_bench_run(cgx_dist *d, int iters, int flags, double *total_ms, double *spmv_ms) {
  if (!d || iters < 1 || !total_ms || !spmv_ms || (d->local && !d->owns_group)) return CGX_EINVAL;
  return group_bench_run(d->group, iters, flags, total_ms, spmv_ms);
}

int cgx_dist_set_alg(cgx_dist *d, int alg) {
  if (!d || (alg != CGX_ALG_HS && alg != CGX_ALG_CG1 && alg != CGX_ALG_SR) ||
      (d->local && !d->owns_group))
    return CGX_EINVAL;
  for (cgx_dist *o : d->group->parts) {
    if (o->alg != alg && o->gexec[0]) {  // a captured graph holds the other recurrence
      (void)hipStreamSynchronize(o->st);
      drop_graph(o);
    }
    o->alg = alg;
    o->bench_ready = false;
  }
  d->group->fz_known = false;  // part_fusable depends on the recurrence (SR)
  return 0;
}

int cgx_dist_info(cgx_dist *d, cgx_dist_stats *s) {
  if (!d || !s) return CGX_EINVAL;
  memset(s, 0, sizeof *s);
  s->n_global = d->n_global;
  s->row_begin = d->row_begin;
  s->n_loc = d->n_loc;
  s->n_ghost = d->n_ghost;
  s->n_send = d->n_send;
  s->nnz = d->nnz;
  s->interior_items = d->it_int.count;
  s->boundary_items = d->it_bnd.count;
  s->spmv_bytes = (double)d->nnz * 12.0 + 4.0 * (d->n_loc + 1) + 16.0 * d->n_loc;
  s->iter_bytes = s->spmv_bytes + 72.0 * d->n_loc;
  s->halo_bytes = 8.0 * (d->n_ghost + d->n_send);
  s->device_bytes = d->A.dev_bytes + d->Ai.dev_bytes + d->vec_bytes;
  s->spmv_iter_bytes = d->have_matrix ? d->A.layout_bytes() : 0.0;
  // the one-launch SR step: its layout, + r, s, p read and written, x /
  // p_{k-2} every other launch (cgx_info)
  // (x four iterations deep: x, p_{k-3}, p_{k-2}, p_{k-1} read and x
  // written every fourth launch)
  if (d->have_matrix && sr1(d)) s->spmv_iter_bytes = d->Ai.layout_bytes() + 5.25 * d->n_loc * 8.0;
  // fused: + r, p_old read and p_new written, x / p_{k-1} read and x
  // written every other launch (cgx_info)
  if (d->have_matrix && fz(d)) s->spmv_iter_bytes += 3.5 * d->n_loc * 8.0;
  // fused CG1: + r, w, s, p, x read and p, s, r, w, x written (cgx_info)
  if (d->have_matrix && fz1(d)) s->spmv_iter_bytes += 8.0 * d->n_loc * 8.0;
  s->fused = fz(d) || fz1(d) || sr1(d) ? 1 : 0;
  if (d->have_matrix && sr1(d)) {  // steps per segment (the longest)
    const Sr1Plan pl = sr1_plan(d);
    const SpmvArgs<double> a =
        d->Ai.args<double>(nullptr, nullptr, nullptr, nullptr, d->Ai.all_items());
    const long long QR = (long long)a.mq * kDiaSliceRows;
    const int L = (int)((a.n + QR - 1) / QR);
    s->march = std::max(1, pl.len > 0 ? pl.len : (L + pl.nseg - 1) / std::max(1, pl.nseg));
  } else {
    s->march = 0;
  }
  s->inplace = d->ai_ok ? 1 : 0;
  {
    const int own = d->fuse == CGX_FUSE_OFF ? CGX_FUSE_STATUS_OFF
                    : !d->have_matrix      ? CGX_FUSE_STATUS_NOT_DIA
                    : d->A.fuse_block()    ? d->A.fuse_block()
                    : (d->fuse == CGX_FUSE_AUTO && !d->A.nt) ? CGX_FUSE_STATUS_CACHED
                                                             : 0;
    s->fuse_status = s->fused ? CGX_FUSE_STATUS_RUNS
                     : own    ? own
                     : (d->alg == CGX_ALG_CG1 && d->fuse != CGX_FUSE_ON) ? CGX_FUSE_STATUS_CG1_AUTO
                     : d->group && d->group->fz_known && !d->fz_all ? CGX_FUSE_STATUS_PEER
                                                                     : CGX_FUSE_STATUS_RUNS;
  }
  s->breakdown = d->h_st ? d->h_st->brk : 0;
  // the layout the SpMV runs on (the one-launch SR step: the in-place one)
  const DevMatrix &M = d->have_matrix && sr1(d) ? d->Ai : d->A;
  s->layout = d->have_matrix ? cgx::public_layout(M) : CGX_LAYOUT_AUTO;
  s->n_dict = M.layout == cgx::L_DC ? M.ndict : M.layout == cgx::L_DIA ? M.dia.ndiag : 0;
  s->graph = d->graph_state;
  s->alg = d->alg;
  return 0;
}

}  // extern "C"
