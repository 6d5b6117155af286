// cgx_dist.cpp -- the multi-GPU CG solver: one rank per GPU, rows
// partitioned into contiguous blocks (cgx_partition.cpp), halo x segments
// exchanged point to point, and the iteration's two dot products fused into
// ONE all-reduce (north star in BASELINE.json).
//
// Recurrence: Chronopoulos-Gear CG (one reduction per iteration; the
// reference's Hestenes-Stiefel form, cg.c:113 and cg.c:129, needs two
// dependent reductions).  Per iteration, on the rank's compute stream A and
// communication stream B:
//
//   A: k_cg1_update   p = r + beta p, s = w + beta s, x += alpha p,
//                     r -= alpha s, gamma partials              -> ev_packed
//   A: k_gather       pack r[send rows] into the send buffer
//   B: halo           ncclSend/ncclRecv with each neighbour (RCCL over xGMI)
//                     straight into r's ghost tail               -> ev_halo
//   A: k_spmv_wave    w = A r over INTERIOR row blocks (no ghost columns),
//                     overlapping the halo on B; delta = w.r partials
//   A: wait ev_halo;  k_spmv_wave over BOUNDARY row blocks
//   A: k_finalize     local (gamma, delta)
//   A: ncclAllReduce  2 doubles, sum
//   A: k_finalize     alpha, beta, stop test on the global sums
//
// Transports: RCCL (one process per GPU, ncclCommInitRank from an id the
// caller distributes), or "local": P partitions driven by one host thread on
// one device (device-to-device copies for the halo, a fixed-order sum kernel
// for the all-reduce) -- the same phase code, used to validate the
// partitioned path on a single GPU.  The host driver runs the iteration as
// phases over all partitions it owns (one in RCCL mode), so every wait is on
// an event that has already been recorded.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cgx_internal.h"

using cgx::CgState;

struct cgx_dist;

namespace {

struct Group {
  std::vector<cgx_dist *> parts;  // RCCL mode: just this rank
  const double **d_srcs = nullptr;  // local mode: every part's d_sums
  bool connected = false;
};

}  // namespace

struct cgx_dist {
  int device = 0, nranks = 1, rank = 0;
  bool local = false;
  Group *group = nullptr;     // owned by part 0 in local mode, by self in RCCL
  bool owns_group = false;
  ncclComm_t comm = nullptr;
  int cus = 256;
  hipStream_t st = nullptr, st_comm = nullptr;
  hipEvent_t ev_packed = nullptr, ev_halo = nullptr, ev_sums = nullptr, ev_sums2 = nullptr;
  cgx_part *part = nullptr;
  long long n_global = 0;
  int row_begin = 0, n_loc = 0, n_ghost = 0, nnz = 0;
  int vec = 4, wpb = 4;
  // SpMV knobs, read from the environment once (CGX_SPMV_TG/DMA/NT/XCD)
  int spmv_tg = 1, spmv_dma = 1, spmv_nt = -1, spmv_xcd = 1;
  // recurrence (cgx_dist_set_alg): CGX_ALG_CG1 (Chronopoulos-Gear, one
  // all-reduce of 2 doubles per iteration) or CGX_ALG_HS (the reference's
  // recurrence, two all-reduces of 1 double, 8 B per row less vector traffic)
  int alg = CGX_ALG_CG1;
  int *d_rp = nullptr, *d_col = nullptr, *d_blk = nullptr, *d_blkk = nullptr;
  int *d_blkrk = nullptr;  // (blk_row, blk_k) pairs for the coded-column kernel
  int *d_list_int = nullptr, *d_list_bnd = nullptr;
  // dictionary-coded columns (k_spmv_dc), as the single-GPU solver: the
  // local numbering keeps them (a slab's ghosts sit at constant offsets)
  unsigned char *d_code = nullptr;
  int *d_dict = nullptr;
  unsigned char *d_rlen = nullptr;  // byte row lengths (rows <= 255 entries)
  int ndict = 0;
  int code_bits = 8;                 // 4: nibble codes (<= 16 offsets)
  void *d_dval = nullptr;            // value-indexed pairs (CGX_DC_VALS): pair values
  bool vi = false;
  int n_int = 0, n_bnd = 0, g_int = 0, g_bnd = 0;
  // interior / boundary row blocks as contiguous runs {first, count} when
  // there are few of them (slab partitions: 1 interior + 2 boundary runs);
  // otherwise the index lists above are used (one launch each)
  std::vector<std::pair<int, int>> runs_int, runs_bnd;
  bool use_runs = false;
  double *d_val = nullptr;
  double *d_b = nullptr, *d_x = nullptr, *d_r = nullptr, *d_p = nullptr,
         *d_s = nullptr, *d_w = nullptr;
  int *d_send_idx = nullptr;
  double *d_sendbuf = nullptr;
  std::vector<int> send_count, send_off, recv_count, recv_off;
  int n_send = 0;
  double *d_pa = nullptr, *d_pb = nullptr, *d_sums = nullptr, *d_gsums = nullptr;
  int vec_grid = 1;
  CgState *d_st = nullptr, *h_st = nullptr;
  double *d_hist = nullptr;
  int hist_alloc = 0;
  size_t dev_bytes = 0;
  bool have_matrix = false, have_rhs = false, bench_ready = false;
  int last_iters = 0;
  // optional SpMV timing: 4 events per iteration (interior start/end,
  // boundary start/end) while rec_spmv is set
  std::vector<hipEvent_t> spmv_ev;
  bool rec_spmv = false;
  size_t ev_i = 0;
  // single rank, no transport: the iteration is [update, SpMV, finalize] on
  // one stream, replayed as hipGraphs of graph_batch iterations
  hipGraphExec_t gexec = nullptr;
  int graph_batch = 16;
};

namespace {

using namespace cgx;

// One rank with no transport: no halo, scalars straight from the partials,
// graph replay.  A 1-rank RCCL communicator (cgx_dist_create with an id at
// nranks 1) keeps the transport phases -- the multi-GPU code path, all-reduce
// included, on one GPU.
bool solo(const cgx_dist *d) { return !d->local && d->comm == nullptr; }

#define CGX_NCCL(call)                                                       \
  do {                                                                       \
    ncclResult_t r_ = (call);                                                \
    if (r_ != ncclSuccess) {                                                 \
      set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,           \
                ncclGetErrorString(r_));                                     \
      return CGX_ECOMM;                                                      \
    }                                                                        \
  } while (0)

template <typename P>
int dalloc(cgx_dist *d, P **p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipErrorUnknown;
  if (env_int("CGX_CONTIG", 1)) {  // physically contiguous, as the solver (fallback: hipMalloc)
    e = hipExtMallocWithFlags((void **)p, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess) e = hipMalloc((void **)p, bytes);
  if (e != hipSuccess) {
    set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    *p = nullptr;
    return CGX_ENOMEM;
  }
  d->dev_bytes += bytes;
  return 0;
}

template <typename P>
void dfree(P **p) {
  if (*p) (void)hipFree((void *)*p);
  *p = nullptr;
}

bool dc_wanted(const cgx_dist *d);

void free_system(cgx_dist *d) {
  if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
  d->gexec = nullptr;
  dfree(&d->d_rp); dfree(&d->d_col); dfree(&d->d_blk); dfree(&d->d_blkk);
  dfree(&d->d_blkrk);
  dfree(&d->d_list_int); dfree(&d->d_list_bnd); dfree(&d->d_val);
  dfree(&d->d_b); dfree(&d->d_x); dfree(&d->d_r); dfree(&d->d_p);
  dfree(&d->d_s); dfree(&d->d_w); dfree(&d->d_send_idx); dfree(&d->d_sendbuf);
  dfree(&d->d_pa); dfree(&d->d_pb); dfree(&d->d_hist);
  dfree(&d->d_code); dfree(&d->d_dict); dfree(&d->d_rlen); dfree(&d->d_dval);
  d->ndict = 0;
  d->vi = false;
  d->hist_alloc = 0;
  if (d->part) cgx_part_destroy(d->part);
  d->part = nullptr;
  d->have_matrix = d->have_rhs = d->bench_ready = false;
  d->dev_bytes = 0;
  if (d->group) d->group->connected = false;
}

int init_common(cgx_dist *d, int device) {
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) {
    set_error("no HIP device available");
    return CGX_ENODEV;
  }
  if (device < 0 || device >= cnt) {
    set_error("device %d out of range", device);
    return CGX_EINVAL;
  }
  hipDeviceProp_t prop;
  CGX_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("device %d is %s; libcgx is built for gfx950 only", device,
              prop.gcnArchName);
    return CGX_ENODEV;
  }
  d->device = device;
  d->cus = prop.multiProcessorCount;
  d->vec = env_int("CGX_SPMV_VEC", 4);
  if (d->vec != 1 && d->vec != 2 && d->vec != 4) d->vec = 4;
  d->wpb = env_int("CGX_SPMV_WPB", 4) == 8 ? 8 : 4;
  d->spmv_tg = env_int("CGX_SPMV_TG", 1);
  d->spmv_dma = d->wpb == 4 && env_int("CGX_SPMV_DMA", 1) == 1 ? 1 : 0;  // as the solver
  d->spmv_nt = env_int("CGX_SPMV_NT", -1);
  d->spmv_xcd = env_int("CGX_SPMV_XCD", 1);
  d->graph_batch = env_int("CGX_GRAPH", 1) ? std::max(1, env_int("CGX_GRAPH_BATCH", 16)) : 0;
  {
    const char *al = getenv("CGX_DIST_ALG");
    d->alg = al && strcmp(al, "hs") == 0 ? CGX_ALG_HS : CGX_ALG_CG1;
  }
  CGX_HIP(hipSetDevice(device));
  CGX_HIP(hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking));
  {
    // halo traffic on a high-priority stream: its RCCL kernel is dispatched
    // ahead of the interior SpMV's remaining workgroups, so the ghosts arrive
    // while the interior rows are still being summed
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    CGX_HIP(hipStreamCreateWithPriority(&d->st_comm, hipStreamNonBlocking,
                                        env_int("CGX_COMM_PRIO", 1) ? greatest : 0));
  }
  CGX_HIP(hipEventCreateWithFlags(&d->ev_packed, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_halo, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_sums, hipEventDisableTiming));
  CGX_HIP(hipEventCreateWithFlags(&d->ev_sums2, hipEventDisableTiming));
  CGX_HIP(hipMalloc((void **)&d->d_st, sizeof(CgState)));
  CGX_HIP(hipMalloc((void **)&d->d_sums, 4 * sizeof(double)));
  CGX_HIP(hipHostMalloc((void **)&d->h_st, sizeof(CgState), hipHostMallocDefault));
  d->d_gsums = d->d_sums + 2;
  return 0;
}

// ------------------------------------------------------------ system setup

int upload_local(cgx_dist *d, long long n_global, int n_loc, int nnz,
                 const int *rp, const int *col_global, const double *val) {
  CGX_HIP(hipSetDevice(d->device));
  free_system(d);
  cgx_part *pt = nullptr;
  int rc = cgx_part_create(n_global, d->nranks, d->rank, n_loc, nnz, rp,
                           col_global, &pt);
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
  for (int q = 1; q < d->nranks; ++q)
    d->recv_off[q] = d->recv_off[q - 1] + d->recv_count[q - 1];

  // wave row blocks of 64 rows, split into interior / boundary lists
  const int cap = spmv_cap(64, true);
  std::vector<int> blk = n_loc > 0 ? plan_rowblocks(n_loc, rp, 64, cap - kPad)
                                   : std::vector<int>{0};
  const int nblk = (int)blk.size() - 1;
  std::vector<int> blkk(blk.size()), lint, lbnd;
  for (size_t i = 0; i < blk.size(); ++i) blkk[i] = n_loc > 0 ? rp[blk[i]] : 0;
  for (int b = 0; b < nblk; ++b) {
    bool ghost = false;
    for (int k = blkk[b]; k < blkk[b + 1] && !ghost; ++k) ghost = col_local[k] >= n_loc;
    (ghost ? lbnd : lint).push_back(b);
  }
  d->n_int = (int)lint.size();
  d->n_bnd = (int)lbnd.size();
  auto runs = [](const std::vector<int> &l) {
    std::vector<std::pair<int, int>> r;
    for (int b : l) {
      if (!r.empty() && r.back().first + r.back().second == b) r.back().second++;
      else r.push_back({b, 1});
    }
    return r;
  };
  d->runs_int = runs(lint);
  d->runs_bnd = runs(lbnd);
  d->use_runs = d->runs_int.size() <= 4 && d->runs_bnd.size() <= 4 &&
                env_int("CGX_DIST_RUNS", 1) != 0;
  if (d->use_runs) {
    d->g_int = d->g_bnd = 0;
    for (auto &r : d->runs_int) d->g_int += spmv_launch_grid(64, d->wpb, 1, r.second, 0);
    for (auto &r : d->runs_bnd) d->g_bnd += spmv_launch_grid(64, d->wpb, 1, r.second, 0);
    // several boundary runs (a middle slab's first and last plane): one launch
    // over the boundary block list instead of one per run
    if (d->runs_bnd.size() > 1) d->g_bnd = spmv_launch_grid(64, d->wpb, 1, d->n_bnd, 0);
  } else {
    d->g_int = spmv_launch_grid(64, d->wpb, 1, d->n_int, 0);
    d->g_bnd = spmv_launch_grid(64, d->wpb, 1, d->n_bnd, 0);
  }
  d->vec_grid = vec_grid_for(n_loc, d->cus);

  const size_t nnz_pad = ((size_t)nnz + kPad - 1) / kPad * kPad + kWindowPad;
  const size_t nv = (size_t)n_loc + kPad;
  if ((rc = dalloc(d, &d->d_rp, ((size_t)n_loc + 1) * 4)) ||
      (rc = dalloc(d, &d->d_col, nnz_pad * 4)) ||
      (rc = dalloc(d, &d->d_val, nnz_pad * 8)) ||
      (rc = dalloc(d, &d->d_blk, blk.size() * 4)) ||
      (rc = dalloc(d, &d->d_blkk, blk.size() * 4)) ||
      (rc = dalloc(d, &d->d_blkrk, blk.size() * 8)) ||
      (rc = dalloc(d, &d->d_list_int, (lint.size() + 1) * 4)) ||
      (rc = dalloc(d, &d->d_list_bnd, (lbnd.size() + 1) * 4)) ||
      (rc = dalloc(d, &d->d_b, nv * 8)) || (rc = dalloc(d, &d->d_x, nv * 8)) ||
      (rc = dalloc(d, &d->d_r, (nv + d->n_ghost) * 8)) ||
      (rc = dalloc(d, &d->d_p, (nv + d->n_ghost) * 8)) || (rc = dalloc(d, &d->d_s, nv * 8)) ||
      (rc = dalloc(d, &d->d_w, nv * 8)) ||
      (rc = dalloc(d, &d->d_pa, ((size_t)d->vec_grid + 8) * 8)) ||
      (rc = dalloc(d, &d->d_pb, ((size_t)d->g_int + d->g_bnd + 1) * 8))) {
    free_system(d);
    return rc;
  }
  hipStream_t st = d->st;
  CGX_HIP(hipMemsetAsync(d->d_col, 0, nnz_pad * 4, st));
  CGX_HIP(hipMemsetAsync(d->d_val, 0, nnz_pad * 8, st));
  CGX_HIP(hipMemsetAsync(d->d_r, 0, (nv + d->n_ghost) * 8, st));
  CGX_HIP(hipMemsetAsync(d->d_p, 0, (nv + d->n_ghost) * 8, st));
  if (n_loc > 0) {
    CGX_HIP(hipMemcpyAsync(d->d_rp, rp, ((size_t)n_loc + 1) * 4, hipMemcpyHostToDevice, st));
    if (nnz > 0) {
      CGX_HIP(hipMemcpyAsync(d->d_col, col_local.data(), (size_t)nnz * 4, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d->d_val, val, (size_t)nnz * 8, hipMemcpyHostToDevice, st));
    }
  }
  CGX_HIP(hipMemcpyAsync(d->d_blk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, st));
  CGX_HIP(hipMemcpyAsync(d->d_blkk, blkk.data(), blkk.size() * 4, hipMemcpyHostToDevice, st));
  std::vector<int> blkrk(2 * blk.size());
  for (size_t i = 0; i < blk.size(); ++i) {
    blkrk[2 * i] = blk[i];
    blkrk[2 * i + 1] = blkk[i];
  }
  CGX_HIP(hipMemcpyAsync(d->d_blkrk, blkrk.data(), blkrk.size() * 4, hipMemcpyHostToDevice, st));
  if (n_loc > 0 && nnz > 0 && dc_wanted(d)) {
    std::vector<unsigned char> code((size_t)nnz);
    std::vector<int> dict;
    int nd = build_col_codes(n_loc, rp, col_local.data(), dict, code.data());
    std::vector<unsigned char> rl;
    if (nd > 0 && env_int("CGX_DC_RLEN", 1)) {
      rl.resize((size_t)n_loc);
      if (!build_row_lengths(n_loc, rp, rl.data())) rl.clear();
    }
    // value-indexed pairs (k_spmv_vi) as the solver: byte row lengths, <= 64
    // (offset, value) pairs, every block's code window inside the kernel's
    std::vector<double> dv;
    if (nd > 0 && !rl.empty() && env_int("CGX_DC_VALS", 1) != 0) {
      const int cb = nd <= 16 && env_int("CGX_DC_BITS", 8) == 4 ? 4 : 8, ka = 128 / cb;
      const long long capc = ((512LL + ka) * cb / 8 + 15) & ~15LL;
      bool fits = true;
      for (size_t b = 0; b + 1 < blkk.size() && fits; ++b)
        fits = ((long long)(blkk[b + 1] - (blkk[b] & ~(ka - 1))) * cb + 7) / 8 <= capc;
      if (fits) {
        const int np = build_val_pairs<double>(nnz, val, code.data(), dict, dv, 64);
        if (np > 0) nd = np;
      }
    }
    if (nd > 0) {
      if ((rc = dalloc(d, &d->d_code, nnz_pad)) || (rc = dalloc(d, &d->d_dict, 256 * 4)) ||
          (!dv.empty() && (rc = dalloc(d, &d->d_dval, 256 * 8)))) {
        free_system(d);
        return rc;
      }
      dict.resize(256, 0);
      if (!dv.empty()) {
        dv.resize(256, 0.0);
        CGX_HIP(hipMemcpyAsync(d->d_dval, dv.data(), 256 * 8, hipMemcpyHostToDevice, st));
        d->vi = true;
      }
      d->code_bits = nd <= 16 && env_int("CGX_DC_BITS", 8) == 4 ? 4 : 8;
      size_t code_bytes = (size_t)nnz;
      if (d->code_bits == 4) {
        pack_nibbles(nnz, code.data(), code.data());
        code_bytes = ((size_t)nnz + 1) / 2;
      }
      CGX_HIP(hipMemsetAsync(d->d_code, 0, nnz_pad, st));
      CGX_HIP(hipMemcpyAsync(d->d_code, code.data(), code_bytes, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d->d_dict, dict.data(), 256 * 4, hipMemcpyHostToDevice, st));
      if (!rl.empty()) {
        if ((rc = dalloc(d, &d->d_rlen, (size_t)n_loc + 64))) {
          free_system(d);
          return rc;
        }
        CGX_HIP(hipMemcpyAsync(d->d_rlen, rl.data(), (size_t)n_loc, hipMemcpyHostToDevice, st));
      }
      CGX_HIP(hipStreamSynchronize(st));  // the host vectors go out of scope
      d->ndict = nd;
    }
  }
  if (!lint.empty())
    CGX_HIP(hipMemcpyAsync(d->d_list_int, lint.data(), lint.size() * 4, hipMemcpyHostToDevice, st));
  if (!lbnd.empty())
    CGX_HIP(hipMemcpyAsync(d->d_list_bnd, lbnd.data(), lbnd.size() * 4, hipMemcpyHostToDevice, st));
  CGX_HIP(hipStreamSynchronize(st));
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
  for (int q = 1; q < d->nranks; ++q)
    d->send_off[q] = d->send_off[q - 1] + d->send_count[q - 1];
  d->n_send = d->send_off[d->nranks - 1] + d->send_count[d->nranks - 1];
  std::vector<int> loc((size_t)d->n_send);
  cgx_part_send_local(d->part, loc.data());
  dfree(&d->d_send_idx);
  dfree(&d->d_sendbuf);
  if ((rc = dalloc(d, &d->d_send_idx, ((size_t)d->n_send + 1) * 4)) ||
      (rc = dalloc(d, &d->d_sendbuf, ((size_t)d->n_send + 1) * 8)))
    return rc;
  if (d->n_send > 0)
    CGX_HIP(hipMemcpy(d->d_send_idx, loc.data(), (size_t)d->n_send * 4,
                      hipMemcpyHostToDevice));
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
      req_global.insert(req_global.end(), ghosts[q].begin() + off,
                        ghosts[q].begin() + off + cnt);
    }
    int rc = install_sends(d, req_counts, req_global);
    if (rc) return rc;
  }
  if (!g->d_srcs) {
    std::vector<const double *> srcs((size_t)P);
    for (int q = 0; q < P; ++q) srcs[q] = g->parts[q]->d_sums;
    CGX_HIP(hipSetDevice(g->parts[0]->device));
    CGX_HIP(hipMalloc((void **)&g->d_srcs, (size_t)P * sizeof(double *)));
    CGX_HIP(hipMemcpy(g->d_srcs, srcs.data(), (size_t)P * sizeof(double *),
                      hipMemcpyHostToDevice));
  }
  g->connected = true;
  return 0;
}

int ensure_connected(Group *g) {
  if (g->connected) return 0;
  for (cgx_dist *d : g->parts)
    if (!d->have_matrix) {
      set_error("dist: every partition needs set_matrix before solving");
      return CGX_EINVAL;
    }
  if (g->parts[0]->local) return connect_local(g);
  int rc = connect_rccl(g->parts[0]);
  if (rc == 0) g->connected = true;
  return rc;
}

// ---------------------------------------------------------- phase helpers

// Coded columns on the default LDS-DMA kernel unless CGX_DC=0 / CGX_LAYOUT=csr.
bool dc_wanted(const cgx_dist *d) {
  const char *l = getenv("CGX_LAYOUT");
  return d->wpb == 4 && d->spmv_dma == 1 && env_int("CGX_DC", 1) != 0 &&
         !(l && strcmp(l, "csr") == 0);
}

SpmvArgs<double> spmv_args(cgx_dist *d, bool boundary) {
  SpmvArgs<double> a;
  memset(&a, 0, sizeof a);
  a.rp = d->d_rp;
  a.col = d->d_col;
  a.val = d->d_val;
  // CG1: w = A r;  HS: s = A p (cg.c:111).  The gathered vector carries the
  // ghost tail the halo exchange fills.
  a.x = d->alg == CGX_ALG_HS ? d->d_p : d->d_r;
  a.y = d->alg == CGX_ALG_HS ? d->d_s : d->d_w;
  a.blk_row = d->d_blk;
  a.blk_k = d->d_blkk;
  a.blk_rk = d->d_blkrk;
  a.blk_list = boundary ? d->d_list_bnd : d->d_list_int;
  a.blk_first = 0;
  a.nblk = boundary ? d->n_bnd : d->n_int;
  a.part = boundary ? d->d_pb + d->g_int : d->d_pb;
  a.done = &d->d_st->done;
  a.bs = 64;
  a.wpb = d->wpb;
  a.rbw = 1;
  a.st = d->d_st;
  a.tg = d->spmv_tg;
  a.dma = d->spmv_dma;  // 1 or 0: the grids assume one block per wave, 4 waves per WG
  a.nt = d->spmv_nt;
  if (a.nt < 0) a.nt = a.dma && (double)d->nnz * 12.0 > kNtStreamBytes ? 2 : 0;
  a.xcd = a.dma ? d->spmv_xcd : 0;  // XCD-contiguous blocks, as the solver
  a.tk = TicketArgs{};
  if (a.dma == 1 && d->ndict > 0) {
    a.code = d->d_code;
    a.dict = d->d_dict;
    a.ndict_cap = dict_cap(d->ndict);
    a.rlen = d->d_rlen;
    a.code_bits = d->code_bits;
    a.dval = d->vi ? (const double *)d->d_dval : nullptr;
    a.bpw = 1;
  }
  return a;
}

// phase A: the vector update (or the prologue) and the halo pack
int phase_update(cgx_dist *d, bool init) {
  CGX_HIP(hipSetDevice(d->device));
  if (init)
    CGX_HIP(launch_init_cg1<double>(d->n_loc, d->d_b, d->d_x, d->d_r, d->d_p,
                                    d->d_s, d->d_pa, d->vec_grid, d->st));
  else
    CGX_HIP(launch_cg1_update<double>(d->n_loc, d->d_x, d->d_p, d->d_r, d->d_s,
                                      d->d_w, d->d_st, d->d_pa, d->vec_grid,
                                      d->st));
  if (solo(d)) return 0;
  CGX_HIP(launch_gather<double>(d->n_send, d->d_send_idx, d->d_r, d->d_sendbuf,
                                d->st));
  CGX_HIP(hipEventRecord(d->ev_packed, d->st));
  return 0;
}

// phase B: halo exchange on the communication stream
int phase_halo(cgx_dist *d) {
  if (solo(d)) return 0;
  CGX_HIP(hipSetDevice(d->device));
  CGX_HIP(hipStreamWaitEvent(d->st_comm, d->ev_packed, 0));
  double *ghost = (d->alg == CGX_ALG_HS ? d->d_p : d->d_r) + d->n_loc;
  if (d->local) {
    for (cgx_dist *o : d->group->parts) {
      if (o == d || d->recv_count[o->rank] == 0) continue;
      CGX_HIP(hipStreamWaitEvent(d->st_comm, o->ev_packed, 0));
      CGX_HIP(hipMemcpyAsync(ghost + d->recv_off[o->rank],
                             o->d_sendbuf + o->send_off[d->rank],
                             (size_t)d->recv_count[o->rank] * 8,
                             hipMemcpyDeviceToDevice, d->st_comm));
    }
  } else if (d->nranks > 1) {
    CGX_NCCL(ncclGroupStart());
    for (int q = 0; q < d->nranks; ++q) {
      if (q == d->rank) continue;
      if (d->recv_count[q])
        CGX_NCCL(ncclRecv(ghost + d->recv_off[q], d->recv_count[q], ncclFloat64,
                          q, d->comm, d->st_comm));
      if (d->send_count[q])
        CGX_NCCL(ncclSend(d->d_sendbuf + d->send_off[q], d->send_count[q],
                          ncclFloat64, q, d->comm, d->st_comm));
    }
    CGX_NCCL(ncclGroupEnd());
  }
  CGX_HIP(hipEventRecord(d->ev_halo, d->st_comm));
  return 0;
}

// phase C: SpMV (interior overlapping the halo, then boundary) + local sums
// SpMV over one set of row blocks (interior or boundary): one launch per
// contiguous run, partials packed after each other from d_pb + part_off.
int spmv_set(cgx_dist *d, bool boundary) {
  SpmvArgs<double> a = spmv_args(d, boundary);
  if (!d->use_runs || (boundary && d->runs_bnd.size() > 1)) {
    CGX_HIP(launch_spmv<double>(a, boundary ? d->g_bnd : d->g_int, d->vec, d->st));
    return 0;
  }
  a.blk_list = nullptr;
  double *part = boundary ? d->d_pb + d->g_int : d->d_pb;
  for (const auto &r : boundary ? d->runs_bnd : d->runs_int) {
    a.blk_first = r.first;
    a.nblk = r.second;
    a.part = part;
    CGX_HIP(launch_spmv<double>(a, 0, d->vec, d->st));
    part += spmv_launch_grid(64, d->wpb, 1, r.second, 0);
  }
  return 0;
}

int phase_spmv(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const bool rec = d->rec_spmv && d->ev_i + 4 <= d->spmv_ev.size();
  int rc;
  if (rec) CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i], d->st));
  if ((rc = spmv_set(d, false))) return rc;
  if (rec) CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i + 1], d->st));
  if (!solo(d)) CGX_HIP(hipStreamWaitEvent(d->st, d->ev_halo, 0));
  if (rec) CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i + 2], d->st));
  if ((rc = spmv_set(d, true))) return rc;
  if (rec) {
    CGX_HIP(hipEventRecord(d->spmv_ev[d->ev_i + 3], d->st));
    d->ev_i += 4;
  }
  if (solo(d)) return 0;  // phase_reduce finalizes straight from the partials
  if (d->alg == CGX_ALG_HS)  // local p.s -> sums[0]
    CGX_HIP(launch_finalize(FIN_SUM, d->d_pb, d->g_int + d->g_bnd, nullptr, 0, d->d_st,
                            d->d_hist, d->d_sums, d->st));
  else
    CGX_HIP(launch_finalize(FIN_SUM2, d->d_pa, d->vec_grid, d->d_pb,
                            d->g_int + d->g_bnd, d->d_st, d->d_hist, d->d_sums,
                            d->st));
  CGX_HIP(hipEventRecord(d->ev_sums, d->st));
  return 0;
}

// phase D: the one all-reduce of the iteration (gamma, delta), then scalars
int phase_reduce(cgx_dist *d, bool init) {
  CGX_HIP(hipSetDevice(d->device));
  if (solo(d)) {
    CGX_HIP(launch_finalize(init ? FIN_INIT_CG1 : FIN_CG1, d->d_pa, d->vec_grid,
                            d->d_pb, d->g_int + d->g_bnd, d->d_st, d->d_hist,
                            nullptr, d->st));
    return 0;
  }
  const double *g = d->d_gsums;
  if (d->local) {
    for (cgx_dist *o : d->group->parts)
      if (o != d) CGX_HIP(hipStreamWaitEvent(d->st, o->ev_sums, 0));
    CGX_HIP(launch_group_sum(d->group->d_srcs, (int)d->group->parts.size(), 2,
                             d->d_gsums, d->st, 0));
  } else if (d->comm) {
    CGX_NCCL(ncclAllReduce(d->d_sums, d->d_gsums, 2, ncclFloat64, ncclSum,
                           d->comm, d->st));
  } else {
    g = d->d_sums;
  }
  CGX_HIP(launch_finalize(init ? FIN_INIT_CG1 : FIN_CG1, g, 1, g + 1, 1,
                          d->d_st, d->d_hist, nullptr, d->st));
  return 0;
}

int run_phases_eager(Group *g, bool init, long long iters);

int run_phases(Group *g, bool init, long long iters) {
  cgx_dist *d = g->parts[0];
  const int B = d->graph_batch;
  if (!init && solo(d) && B > 0 && iters >= B && !d->rec_spmv) {
    if (!d->gexec) {
      hipGraph_t gr = nullptr;
      CGX_HIP(hipSetDevice(d->device));
      CGX_HIP(hipStreamBeginCapture(d->st, hipStreamCaptureModeThreadLocal));
      int rc = run_phases_eager(g, false, B);
      hipError_t e = hipStreamEndCapture(d->st, &gr);
      if (rc) {
        if (gr) (void)hipGraphDestroy(gr);
        return rc;
      }
      CGX_HIP(e);
      e = hipGraphInstantiate(&d->gexec, gr, nullptr, nullptr, 0);
      (void)hipGraphDestroy(gr);
      CGX_HIP(e);
    }
    while (iters >= B) {
      CGX_HIP(hipGraphLaunch(d->gexec, d->st));
      iters -= B;
    }
  }
  return run_phases_eager(g, init, iters);
}

// ---- HS recurrence (CGX_ALG_HS): the single-GPU folded kernels, with the
// two scalar steps fed by all-reduced sums instead of local partials.  Per
// iteration: halo of p (packed at the end of the previous one) || interior
// SpMV s = A p; boundary SpMV; p.s -> all-reduce -> k_update_rf (alpha,
// r -= alpha s, r.r partials) -> r.r -> all-reduce -> k_xpay_xf (beta, stop,
// x += alpha p, p = r + beta p) -> pack p.  Every rank computes alpha, beta
// and the stop test from the same global sums, so they agree bit for bit.

// one scalar of the iteration summed over the ranks: sums[i] -> gsums[i]
int reduce_one(cgx_dist *d, int i, hipEvent_t ev) {
  if (d->local) {
    for (cgx_dist *o : d->group->parts)
      if (o != d) CGX_HIP(hipStreamWaitEvent(d->st, i == 0 ? o->ev_sums : o->ev_sums2, 0));
    CGX_HIP(launch_group_sum(d->group->d_srcs, (int)d->group->parts.size(), 1, d->d_gsums,
                             d->st, i));
  } else {
    CGX_NCCL(ncclAllReduce(d->d_sums + i, d->d_gsums + i, 1, ncclFloat64, ncclSum, d->comm,
                           d->st));
  }
  (void)ev;
  return 0;
}

int hs_pack(cgx_dist *d) {
  if (solo(d)) return 0;
  CGX_HIP(launch_gather<double>(d->n_send, d->d_send_idx, d->d_p, d->d_sendbuf, d->st));
  CGX_HIP(hipEventRecord(d->ev_packed, d->st));
  return 0;
}

// prologue: x = 0, r = p = b, b.b (cg.c:104-107)
int hs_init(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  CGX_HIP(launch_init_hs<double>(d->n_loc, d->d_b, d->d_x, d->d_r, d->d_p, d->d_pa,
                                 d->vec_grid, d->st));
  if (solo(d)) {
    CGX_HIP(launch_finalize(FIN_INIT_HS, d->d_pa, d->vec_grid, nullptr, 0, d->d_st,
                            d->d_hist, nullptr, d->st));
    return 0;
  }
  CGX_HIP(launch_finalize(FIN_SUM, d->d_pa, d->vec_grid, nullptr, 0, d->d_st, d->d_hist,
                          d->d_sums, d->st));
  CGX_HIP(hipEventRecord(d->ev_sums, d->st));
  return 0;
}

int hs_init_reduce(cgx_dist *d) {
  if (solo(d)) return hs_pack(d);
  int rc = reduce_one(d, 0, d->ev_sums);
  if (rc) return rc;
  CGX_HIP(launch_finalize(FIN_INIT_HS, d->d_gsums, 1, nullptr, 0, d->d_st, d->d_hist,
                          nullptr, d->st));
  return hs_pack(d);
}

// alpha step: all-reduced p.s, r -= alpha s, local r.r
int hs_alpha(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const int gf = (d->vec_grid + 3) / 4;  // 1024-thread workgroups, 4 partials each
  const double *ps = d->d_pb;
  int nps = d->g_int + d->g_bnd;
  if (!solo(d)) {
    int rc = reduce_one(d, 0, d->ev_sums);
    if (rc) return rc;
    ps = d->d_gsums;
    nps = 1;
  }
  CGX_HIP(launch_update_rf<double>(d->n_loc, d->d_r, d->d_s, d->d_st, ps, nps, d->d_pa, gf,
                                   d->st, true));              // cg.c:113, 118-123
  if (solo(d)) return 0;
  CGX_HIP(launch_finalize(FIN_SUM, d->d_pa, 4 * gf, nullptr, 0, d->d_st, d->d_hist,
                          d->d_sums + 1, d->st));
  CGX_HIP(hipEventRecord(d->ev_sums2, d->st));
  return 0;
}

// beta step: all-reduced r.r, stop test, x += alpha p, p = r + beta p
int hs_beta(cgx_dist *d) {
  CGX_HIP(hipSetDevice(d->device));
  const int gf = (d->vec_grid + 3) / 4;
  const double *rr = d->d_pa;
  int nrr = 4 * gf;
  if (!solo(d)) {
    int rc = reduce_one(d, 1, d->ev_sums2);
    if (rc) return rc;
    rr = d->d_gsums + 1;
    nrr = 1;
  }
  CGX_HIP(launch_xpay_xf<double>(d->n_loc, d->d_x, d->d_p, d->d_r, d->d_st, rr, nrr,
                                 d->d_hist, gf, d->st, true));  // cg.c:115-116, 125-132
  return hs_pack(d);
}

int run_phases_eager(Group *g, bool init, long long iters) {
  auto &P = g->parts;
  if (P[0]->alg == CGX_ALG_HS) {
    int rc;
    if (init) {
      for (cgx_dist *d : P) if ((rc = hs_init(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_init_reduce(d))) return rc;
      return 0;
    }
    for (long long it = 0; it < iters; ++it) {
      for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
      for (cgx_dist *d : P) if ((rc = phase_spmv(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_alpha(d))) return rc;
      for (cgx_dist *d : P) if ((rc = hs_beta(d))) return rc;
    }
    return 0;
  }
  for (long long it = 0; it < (init ? 1 : iters); ++it) {
    int rc;
    for (cgx_dist *d : P) if ((rc = phase_update(d, init))) return rc;
    for (cgx_dist *d : P) if ((rc = phase_halo(d))) return rc;
    for (cgx_dist *d : P) if ((rc = phase_spmv(d))) return rc;
    for (cgx_dist *d : P) if ((rc = phase_reduce(d, init))) return rc;
  }
  return 0;
}

int prepare_states(Group *g, int maxit, double tol, int hist_cap) {
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipSetDevice(d->device));
    if (hist_cap > d->hist_alloc) {
      if (d->gexec) {  // the captured graph holds the old history pointer
        CGX_HIP(hipStreamSynchronize(d->st));
        (void)hipGraphExecDestroy(d->gexec);
        d->gexec = nullptr;
      }
      dfree(&d->d_hist);
      int rc = dalloc(d, &d->d_hist, (size_t)hist_cap * 8);
      if (rc) return rc;
      d->hist_alloc = hist_cap;
    }
    memset(d->h_st, 0, sizeof(CgState));
    d->h_st->tol = tol;
    d->h_st->use_tol = tol > 0.0 ? 1 : 0;
    d->h_st->max_iter = maxit;
    d->h_st->hist_cap = std::min(hist_cap, d->hist_alloc);
    CGX_HIP(hipMemcpyAsync(d->d_st, d->h_st, sizeof(CgState),
                           hipMemcpyHostToDevice, d->st));
  }
  return 0;
}

int read_states(Group *g) {
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipSetDevice(d->device));
    CGX_HIP(hipMemcpyAsync(d->h_st, d->d_st, sizeof(CgState),
                           hipMemcpyDeviceToHost, d->st));
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
  const long long total = (long long)maxit + 1;
  if (tol <= 0.0) {
    if ((rc = run_phases(g, false, total))) return rc;
    if ((rc = read_states(g))) return rc;
  } else {
    long long done = 0, batch = 8;
    for (;;) {
      const long long b = std::min(batch, total - done);
      if ((rc = run_phases(g, false, b))) return rc;
      done += b;
      if ((rc = read_states(g))) return rc;
      if (g->parts[0]->h_st->done || done >= total) break;
      batch = std::min<long long>(batch * 2, 256);
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
  if ((rc = run_phases(g, false, warmup))) return rc;
  for (cgx_dist *d : g->parts) {
    CGX_HIP(hipStreamSynchronize(d->st));
    d->bench_ready = true;
  }
  return 0;
}

int group_bench_run(Group *g, int iters, int flags, double *ms,
                    double *spmv_ms) {
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
  hipEvent_t e0, e1;
  CGX_HIP(hipSetDevice(d0->device));
  CGX_HIP(hipEventCreate(&e0));
  CGX_HIP(hipEventCreate(&e1));
  CGX_HIP(hipEventRecord(e0, d0->st));
  int rc = run_phases(g, false, iters);
  d0->rec_spmv = false;
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
    double sum = 0.0;
    for (int i = 0; i < iters; ++i) {
      float a = 0.f, b = 0.f;
      CGX_HIP(hipEventElapsedTime(&a, d0->spmv_ev[4 * i], d0->spmv_ev[4 * i + 1]));
      CGX_HIP(hipEventElapsedTime(&b, d0->spmv_ev[4 * i + 2], d0->spmv_ev[4 * i + 3]));
      sum += (double)a + (double)b;
    }
    *spmv_ms = sum / iters;
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
  if (d->ev_packed) (void)hipEventDestroy(d->ev_packed);
  if (d->ev_halo) (void)hipEventDestroy(d->ev_halo);
  if (d->ev_sums) (void)hipEventDestroy(d->ev_sums);
  if (d->ev_sums2) (void)hipEventDestroy(d->ev_sums2);
  for (hipEvent_t e : d->spmv_ev) (void)hipEventDestroy(e);
  if (d->d_st) (void)hipFree(d->d_st);
  if (d->d_sums) (void)hipFree(d->d_sums);
  if (d->h_st) (void)hipHostFree(d->h_st);
  if (d->st) (void)hipStreamDestroy(d->st);
  if (d->st_comm) (void)hipStreamDestroy(d->st_comm);
  delete d;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" {

int cgx_dist_unique_id(unsigned char id[128]) {
  if (!id) return CGX_EINVAL;
  ncclUniqueId u;
  CGX_NCCL(ncclGetUniqueId(&u));
  memcpy(id, u.internal, sizeof u.internal);
  return 0;
}

int cgx_dist_create(int device, int nranks, int rank,
                    const unsigned char id[128], cgx_dist **out) {
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
      set_error("ncclCommInitRank(%d of %d) failed: %s", rank, nranks,
                ncclGetErrorString(r));
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

int cgx_dist_set_matrix(cgx_dist *d, long long n_global, int n_loc, int nnz,
                        const int *row_ptr, const int *col_global,
                        const double *val) {
  if (!d) return CGX_EINVAL;
  return upload_local(d, n_global, n_loc, nnz, row_ptr, col_global, val);
}

int cgx_dist_set_rhs(cgx_dist *d, const double *b_local) {
  if (!d || !d->have_matrix || (d->n_loc > 0 && !b_local)) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(d->device));
  if (d->n_loc)
    CGX_HIP(hipMemcpy(d->d_b, b_local, (size_t)d->n_loc * 8, hipMemcpyHostToDevice));
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
  if (d->n_loc)
    CGX_HIP(hipMemcpy(x_local, d->d_x, (size_t)d->n_loc * 8, hipMemcpyDeviceToHost));
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

int cgx_dist_bench_run(cgx_dist *d, int iters, int flags, double *total_ms,
                       double *spmv_ms) {
  if (!d || iters < 1 || !total_ms || !spmv_ms || (d->local && !d->owns_group))
    return CGX_EINVAL;
  return group_bench_run(d->group, iters, flags, total_ms, spmv_ms);
}

int cgx_dist_set_alg(cgx_dist *d, int alg) {
  if (!d || (alg != CGX_ALG_HS && alg != CGX_ALG_CG1) || (d->local && !d->owns_group))
    return CGX_EINVAL;
  for (cgx_dist *o : d->group->parts) {
    if (o->alg != alg && o->gexec) {  // a captured graph holds the other recurrence
      (void)hipStreamSynchronize(o->st);
      (void)hipGraphExecDestroy(o->gexec);
      o->gexec = nullptr;
    }
    o->alg = alg;
    o->bench_ready = false;
  }
  return 0;
}

int cgx_dist_info(cgx_dist *d, cgx_dist_stats *s) {
  if (!d || !s) return CGX_EINVAL;
  s->n_global = d->n_global;
  s->row_begin = d->row_begin;
  s->n_loc = d->n_loc;
  s->n_ghost = d->n_ghost;
  s->n_send = d->n_send;
  s->nnz = d->nnz;
  s->interior_blocks = d->n_int;
  s->boundary_blocks = d->n_bnd;
  s->spmv_bytes = (double)d->nnz * 12.0 + 4.0 * (d->n_loc + 1) + 16.0 * d->n_loc;
  s->iter_bytes = s->spmv_bytes + 72.0 * d->n_loc;
  s->halo_bytes = 8.0 * (d->n_ghost + d->n_send);
  s->device_bytes = d->dev_bytes;
  s->spmv_iter_bytes = d->ndict > 0 ? (double)d->nnz * (8.0 + d->code_bits / 8.0) +
                                          (d->d_rlen ? 1.0 * d->n_loc : 4.0 * (d->n_loc + 1)) +
                                          16.0 * d->n_loc + 4.0 * d->ndict
                                    : s->spmv_bytes;
  if (d->ndict > 0 && d->vi)  // value-indexed pairs: no val stream
    s->spmv_iter_bytes = (double)d->nnz * (d->code_bits / 8.0) + 1.0 * d->n_loc +
                         16.0 * d->n_loc + 12.0 * d->ndict;
  s->n_dict = d->ndict;
  s->dict_vals = d->ndict > 0 && d->vi;
  return 0;
}

}  // extern "C"
