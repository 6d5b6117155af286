// cgx_kernels.hip -- hand-written gfx950 kernels for the CG hot path.
//
// Replaces the reference's CPU loops (rnelias/Conjugate-Gradient):
//   mv_mult + mat_get_row   mv_ops.c:160-201, :99-113
//       -> k_spmv_csr (CSR), k_spmv_dc (coded columns), k_spmv_vi
//          (value-indexed pair slices), k_stencil (matrix-free Laplacian)
//   dot_product             mv_ops.c:117-132
//       -> SpMV / vector-kernel epilogue partials + fixed-order sums
//          (k_finalize, or folded into k_update_rf / k_xpay_xf);
//          k_dot_seq for the reference's sequential order (exact mode)
//   sv_mult + vec_add/sub   mv_ops.c:134-259, used at cg.c:115-132
//       -> k_update_rf, k_xpay_xf (HS), k_cg1_update (CG1), k_axpby (ops)
//
// Everything is bandwidth bound (about 0.17 flop/byte), so the design goal is
// one coalesced pass over each array per iteration and no fp64 atomics.
// Compiled with -ffp-contract=off: the reference never fuses multiply-add
// (Makefile:2 builds -O0), and x + alpha*p must round twice to stay
// bit-identical.  Every reduction has a fixed order: runs are bit-reproducible.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "cgx_internal.h"

#pragma clang fp contract(off)

// Same-box A/B experiments (tools/ab_build.sh): the product never defines it.
#ifndef CGX_EXP
#define CGX_EXP 0
#endif

namespace cgx {

namespace {

constexpr int kWave = 64;
typedef __attribute__((address_space(3))) void lds_void;

// 16-byte vector of T.
template <typename T> struct Vec16;
template <> struct Vec16<double> {
  typedef double type __attribute__((ext_vector_type(2)));
  static constexpr int W = 2;
};
template <> struct Vec16<float> {
  typedef float type __attribute__((ext_vector_type(4)));
  static constexpr int W = 4;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_down(v, off, kWave);
  return v;  // valid in lane 0
}

// Deterministic block reduction; result valid in thread 0.
template <int BS>
__device__ __forceinline__ double block_sum(double v, double *red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    s = red[0];
#pragma unroll
    for (int i = 1; i < BS / kWave; ++i) s = s + red[i];
  }
  return s;
}

// ---- "last arriver" local sums (FinArgs).  Placement-independent
// protocol (cdna_hip_programming.md Guideline 16): the partial is published
// with an agent-scope store, drained (vmcnt 0) before the agent-scope ticket;
// the last arriver acquires and reads every partial with agent-scope loads
// (the per-XCD L2s are not coherent with each other).  The counter is re-armed
// by the last arriver, so it is zero again when the kernel ends.
__device__ __forceinline__ void publish(double *slot, double v) {
  __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_pub(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool take_ticket1(unsigned *cnt, unsigned n) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != n - 1) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Two levels, so no counter sees more than kTicketGroup (or the group
// count) device-scope atomics per launch: one counter per group of
// kTicketGroup consecutive workgroups (cnt[1 + g]), whose last arriver
// takes the launch's ticket (cnt[0]).  A single counter serialised every
// workgroup's atomic: ~10 ns each, 150 us for a 15,625-slice SpMV.
__device__ __forceinline__ bool take_ticket(unsigned *cnt, unsigned n) {
  const unsigned g = blockIdx.x / kTicketGroup, ng = (n + kTicketGroup - 1) / kTicketGroup;
  const unsigned gs = min((unsigned)kTicketGroup, n - g * kTicketGroup);
  return take_ticket1(cnt + 1 + g, gs) && take_ticket1(cnt, ng);
}

// sum_parts<1024>'s result (below) computed by a BS-thread workgroup
// (BS | 1024): thread t plays virtual threads t + BS j, whose sequential sums
// go through the same 64-lane trees (lane = v mod 64) and the same final
// in-order sum of the 16 virtual wave sums.  Valid in thread 0.
template <int BS, bool PUB>
__device__ double canon_sum(const double *pa, int na, double *red16) {
  constexpr int V = 1024, J = V / BS, U = 16 / J;  // 16 loads in flight per thread
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  double acc[J];
  bool first[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    acc[j] = 0.0;
    first[j] = true;
  }
  for (int base = 0; base < na; base += U * V) {
    double v[J][U];
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * V + j * BS + threadIdx.x;
        v[j][u] = i < na ? (PUB ? ld_pub(pa + i) : pa[i]) : 0.0;
      }
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + u * V + j * BS + (int)threadIdx.x < na) {
          acc[j] = first[j] ? v[j][u] : acc[j] + v[j][u];
          first[j] = false;
        }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const double w = wave_sum(acc[j]);
    if (lane == 0) red16[wid + j * (BS / kWave)] = w;
  }
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    s = red16[0];
#pragma unroll
    for (int i = 1; i < V / kWave; ++i) s = s + red16[i];
  }
  __syncthreads();
  return s;
}

// Thread t adds pa[t], pa[t+BS], pa[t+2BS], ... in index order, then the
// block tree.  All of a thread's loads (up to U) are issued before the first
// add, so a 40K-entry partial array costs one memory round trip, not one per
// 16 entries.  Starts from the first partial, so a single partial passes
// through unchanged.
template <int BS>
__device__ __forceinline__ double sum_parts(const double *pa, int na, double *red) {
  constexpr int U = 48;
  double acc = 0.0;
  bool first = true;
  for (int i = threadIdx.x; i < na; i += U * BS) {
    double v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = i + j * BS < na ? pa[i + j * BS] : 0.0;
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + j * BS < na) {
        acc = first ? v[j] : acc + v[j];
        first = false;
      }
  }
  const double s = block_sum<BS>(acc, red);
  __syncthreads();
  return s;
}

// Two partial arrays summed with all loads of both in flight at once; each
// sum keeps sum_parts' order (thread t: index order, then the block tree).
template <int BS>
__device__ __forceinline__ void sum_parts2(const double *pa, int na, const double *pb, int nb,
                                           double *red, double &sa, double &sb) {
  constexpr int U = 24;
  double acc_a = 0.0, acc_b = 0.0;
  bool fa = true, fb = true;
  const int nmax = na > nb ? na : nb;
  for (int i = threadIdx.x; i < nmax; i += U * BS) {
    double va[U], vb[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      va[j] = i + j * BS < na ? pa[i + j * BS] : 0.0;
      vb[j] = i + j * BS < nb ? pb[i + j * BS] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (i + j * BS < na) {
        acc_a = fa ? va[j] : acc_a + va[j];
        fa = false;
      }
      if (i + j * BS < nb) {
        acc_b = fb ? vb[j] : acc_b + vb[j];
        fb = false;
      }
    }
  }
  sa = block_sum<BS>(acc_a, red);
  __syncthreads();
  sb = block_sum<BS>(acc_b, red);
  __syncthreads();
}

// CGX_ALG_SR's local sums in one pass: (p.s, s.s) pairs pq[0, na) -- one
// 16-byte load each -- and the r.r partials pc[0, nc), all loads of a pass in
// flight together; each sum in sum_parts' order (thread t: index order, then
// the block tree).
template <int BS>
__device__ __forceinline__ void sum_parts_sr(const double *pq, int na, const double *pc, int nc,
                                             double *red, double &sa, double &sb, double &sc) {
  constexpr int U = 16;
  const double2 *q2 = reinterpret_cast<const double2 *>(pq);
  double a = 0.0, b = 0.0, c = 0.0;
  bool fa = true, fc = true;
  const int nmax = na > nc ? na : nc;
  for (int i = threadIdx.x; i < nmax; i += U * BS) {
    double2 v[U];
    double w[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      v[j] = i + j * BS < na ? q2[i + j * BS] : make_double2(0.0, 0.0);
      w[j] = i + j * BS < nc ? pc[i + j * BS] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (i + j * BS < na) {
        a = fa ? v[j].x : a + v[j].x;
        b = fa ? v[j].y : b + v[j].y;
        fa = false;
      }
      if (i + j * BS < nc) {
        c = fc ? w[j] : c + w[j];
        fc = false;
      }
    }
  }
  sa = block_sum<BS>(a, red);
  __syncthreads();
  sb = block_sum<BS>(b, red);
  __syncthreads();
  sc = block_sum<BS>(c, red);
  __syncthreads();
}

// The SpMV epilogue: the workgroup's x[row]*y[row] terms, wave sums added in
// wave order, one partial per workgroup.
template <int WPB>
__device__ __forceinline__ void epi_store(double dot, double *part) {
  __shared__ double red[WPB];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  dot = wave_sum(dot);
  if (lane == 0) red[wid] = dot;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    s = red[0];
#pragma unroll
    for (int w = 1; w < WPB; ++w) s = s + red[w];
    part[blockIdx.x] = s;
  }
}

// The epilogue of a CGX_ALG_SR SpMV (SpmvArgs::pair): the (p.s, s.s) pair
// per workgroup, each reduced as epi_store, stored together at part[2 b]
// (k_finalize FIN_SR1's layout); otherwise epi_store of p.s.
template <int WPB>
__device__ __forceinline__ void epi_store_p(double dot, double dot2, double *part, int pair) {
  if (!pair) {
    epi_store<WPB>(dot, part);
    return;
  }
  __shared__ double red2[2][WPB];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  dot = wave_sum(dot);
  dot2 = wave_sum(dot2);
  if (lane == 0) {
    red2[0][wid] = dot;
    red2[1][wid] = dot2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = red2[0][0], s2 = red2[1][0];
#pragma unroll
    for (int w = 1; w < WPB; ++w) {
      s = s + red2[0][w];
      s2 = s2 + red2[1][w];
    }
    reinterpret_cast<double2 *>(part)[blockIdx.x] = make_double2(s, s2);
  }
}

// The scalar lines of the recurrence (cg.c:113, 125-129; CG1 analogues) on
// the reduced sums sa, sb -- run by ONE thread (k_finalize).
__device__ void apply_fin(int op, double sa, double sb, CgState *st, double *hist,
                          double *out) {
  switch (op) {
    case FIN_SUM:
      out[0] = sa;
      break;
    case FIN_SUM2:
      out[0] = sa;
      out[1] = sb;
      break;
    case FIN_SUM3:  // out[2] written by k_finalize
      out[0] = sa;
      out[1] = sb;
      break;
    case FIN_INIT_HS:
      st->bb = sa;
      st->rr = sa;  // r = b (cg.c:107), so r.r == b.b bit for bit
      st->rr_x = sa;
      st->tol2bb = st->tol * st->tol * sa;
      st->k = 0;
      st->k_x = 0;
      st->k_u = -1;  // fused step: no previous iteration yet
      st->done = 0;
      st->sr_pend = 0;
      break;
    case FIN_HS_ALPHA:
      st->ps = sa;
      st->alpha = st->rr / sa;  // cg.c:113
      if (!(sa > 0.0) && st->brk == 0) st->brk = st->k + 1;
      break;
    case FIN_HS_BETA: {
      const double rr_new = sa;
      const int k = st->k;
      if (k < st->hist_cap) hist[k] = rr_new;
      if (k >= st->max_iter || (st->use_tol && rr_new <= st->tol2bb)) {
        st->done = 1;  // cg.c:125 break position
      } else {
        st->beta = rr_new / st->rr;  // cg.c:129
        st->rr = rr_new;
        st->k = k + 1;
      }
      break;
    }
    case FIN_INIT_CG1:
      st->bb = sa;
      st->rr = sa;
      st->delta = sb;
      st->brk = sb > 0.0 ? 0 : 1;
      st->tol2bb = st->tol * st->tol * sa;
      st->alpha = sa / sb;
      st->beta = 0.0;
      st->k = 0;
      st->done = 0;
      break;
    case FIN_CG1: {
      const double g = sa, d = sb;
      const int k = st->k;
      if (k < st->hist_cap) hist[k] = g;
      if (k >= st->max_iter || (st->use_tol && g <= st->tol2bb)) {
        st->done = 1;
      } else {
        const double beta = g / st->rr;
        const double den = d - beta * g / st->alpha;
        st->delta = d;
        st->alpha = g / den;
        if (!(den > 0.0) && st->brk == 0) st->brk = k + 2;
        st->beta = beta;
        st->rr = g;
        st->k = k + 1;
      }
      break;
    }
  }
}

// CGX_ALG_SR on one GPU (k_sr1_dia_m's sums of launch j = k_u + 1: p_j.s_j,
// s_j.s_j and the EXACT r_j.r_j of the r_j it computed).  First the stop
// test of iteration j - 1 (cg.c:125's position) on the exact r_j.r_j --
// the reference's own rule, one launch late; the estimate never stops a
// solve -- and its history entry.  Otherwise iteration j's
// scalars: alpha = r.r / p.s (cg.c:113), the estimate r_new.r_new = alpha
// (alpha s.s) - r.r clamped at 0 for beta (cg.c:129) only (oracle_solve_sr).
// A stop at an odd j - 1: launch j completed x (done = 2); at an even one
// x += alpha_{j-1} p_{j-1} is pending (done = 1): the next launch applies
// it, and its finalize marks the solve complete (2).
__device__ void fin_sr1(double ps, double ss, double rr, CgState *st, double *hist) {
  if (st->done) {
    st->done = 2;
    return;
  }
  const int j = st->k_u + 1;
  if (j >= 1) {
    const int k = j - 1;
    if (hist && k < st->hist_cap) hist[k] = rr;
    st->rr = rr;
    st->k = k;
    if (k >= st->max_iter || (st->use_tol && rr <= st->tol2bb)) {
      // x is complete after iteration k's launch when k closes a deferral
      // group (depth 2: odd k; 4: k % 4 == 3), else the next launch adds
      // the pending alpha_i p_i (done = 1)
      const int xd = st->xdef >= 4 ? 4 : 2;
      st->done = (k % xd == xd - 1) ? 2 : 1;
      return;
    }
  }
  const double alpha = rr / ps;
  const double as2 = alpha * ss;
  double est = alpha * as2 - rr;
  if (!(est > 0.0)) est = 0.0;
  if (!(ps > 0.0) && st->brk == 0) st->brk = j + 1;
  st->ps = ps;
  st->alpha = alpha;
  st->k_u = j;
  st->beta = est / rr;
}

// The scalars a partitioned one-launch SR kernel runs with: *st, with the
// all-reduced sums g of the last launch pair applied (fin_sr1 on a private
// copy) while FIN_SUM3_SR1 has not applied them to *st yet (sr_pend) -- so
// no kernel writes a state field another kernel of the iteration reads.
struct Sr1Now {
  int k_u, done;
  double alpha, beta;
};

__device__ __forceinline__ Sr1Now sr1_now(const CgState *st, const double *g) {
  if (!g || !st->sr_pend) return Sr1Now{st->k_u, st->done, st->alpha, st->beta};
  CgState c;
  c.done = st->done;
  c.k_u = st->k_u;
  c.max_iter = st->max_iter;
  c.use_tol = st->use_tol;
  c.tol2bb = st->tol2bb;
  c.hist_cap = 0;
  c.brk = 1;  // (not written back)
  c.alpha = st->alpha;
  c.beta = st->beta;
  c.xdef = st->xdef;
  fin_sr1(g[0], g[1], g[2], &c, nullptr);
  return Sr1Now{c.k_u, c.done, c.alpha, c.beta};
}

// XCD-contiguous workgroup order (speed only, never correctness): the
// hardware deals workgroups round-robin over the 8 XCDs, so workgroups b,
// b+8, b+16, ... share one XCD's L2.  Give XCD x the contiguous range of
// logical workgroups [x*q + min(x, rem), ...) (a bijection for any grid), so
// each L2 sees consecutive rows and a stencil's x re-reads (rows +-1, +-nx,
// +-nx*ny) come from its own L2 instead of the Infinity Cache.
__device__ __forceinline__ int xcd_block() {
  const int b = blockIdx.x, G = gridDim.x;
  if (G < 16) return b;
  const int x = b & 7, i = b >> 3, q = G >> 3, rem = G & 7;
  return x * q + min(x, rem) + i;
}

// The workgroup index whose xcd_block() is logical index L (grid G): where a
// one-workgroup-per-item launch writes item L's partial.
__device__ __forceinline__ int xcd_slot(int L, int G) {
  if (G < 16) return L;
  const int q = G >> 3, rem = G & 7;
  const int x = L < rem * (q + 1) ? L / (q + 1) : rem + (L - rem * (q + 1)) / q;
  const int i = L - (x * q + min(x, rem));
  return 8 * i + x;
}

// The fused step's epilogue (SB slices of 256 threads): per slice the p.s
// partial summed over its four waves in order -- epi_store<4> of a
// 256-thread workgroup -- written at xcd_slot(pos + h, G), the unfused
// k_spmv_dia's slot for it.  With ss (CGX_ALG_SR): one (p.s, s.s) pair per
// workgroup at blockIdx (fused_grid(a) pairs per launch).
template <int SB>
__device__ __forceinline__ void epi_store_slices(double dot, double dot2, double *ss, double *part,
                                                 int pos, int cnt, int G) {
  constexpr int NW = 4 * SB;
  __shared__ double red[2][NW];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  dot = wave_sum(dot);
  if (ss) dot2 = wave_sum(dot2);
  if (lane == 0) {
    red[0][wid] = dot;
    red[1][wid] = dot2;
  }
  __syncthreads();
  if (ss) {  // SR (no unfused twin to match): ONE pair per workgroup, at blockIdx
    if (threadIdx.x == 0) {
      double sa = red[0][0], sb = red[1][0];
#pragma unroll
      for (int v = 1; v < NW; ++v) {
        sa = sa + red[0][v];
        sb = sb + red[1][v];
      }
      reinterpret_cast<double2 *>(ss)[blockIdx.x] = make_double2(sa, sb);
    }
    return;
  }
  const int h = threadIdx.x / kWave;  // thread 0 of wave h sums slice h
  if (lane == 0 && h < cnt) {
    double sa = red[0][4 * h];
#pragma unroll
    for (int v = 1; v < 4; ++v) sa = sa + red[0][4 * h + v];
    part[xcd_slot(pos + h, G)] = sa;
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave complete in order; the fences keep the compiler from
  // moving reads of other lanes' slots above the writes.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix sum over the 64 lanes (all lanes active).
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int t = __shfl_up(v, off, kWave);
    v += lane >= off ? t : 0;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void st_y(T *p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Row-block descriptor (CSR / DC), loaded together with the early-exit flag
// in one scalar round trip: the flag is tested only once both are in, and
// every wave of the grid reads the same flag, so the early return is uniform.
struct Blk {
  int r0, nr, k0, k1;
};

template <typename T>
__device__ __forceinline__ bool load_block(const SpmvArgs<T> &a, int wi, Blk &B, bool list) {
  const int *dp = a.done ? a.done : a.blkrk;  // blkrk[0] == 0: "not done"
  const int stop = *dp;
  const int b = list ? a.items.list[wi] : a.items.first + wi;
  const int *d = a.blkrk + 2 * b;
  B.r0 = d[0];
  B.k0 = d[1];
  B.nr = d[2] - d[0];
  B.k1 = d[3];
  // keep the descriptor's loads ahead of the flag's branch
  asm volatile("" ::"s"(B.r0), "s"(B.nr), "s"(B.k0), "s"(B.k1));
  return stop == 0;
}

template <typename T> struct Pair;
template <> struct Pair<double> {
  typedef double type __attribute__((ext_vector_type(2), aligned(8)));
};
template <> struct Pair<float> {
  typedef float type __attribute__((ext_vector_type(2), aligned(4)));
};

// (x[b], x[b+1]) as one load, for -1 <= b <= ncols - 1: a pair reaches
// past x only where one of its two rows holds no entry there, and the
// product of that half is selected away.  x[-1] is the allocation's front
// guard (dev_alloc), x[ncols] the first padding entry (vectors carry kPad).
template <typename T>
__device__ __forceinline__ typename Pair<T>::type ld_pair(const T *x, int b) {
  return *reinterpret_cast<const typename Pair<T>::type *>(x + b);
}

// ------------------------------------------------------------ k_spmv_csr
// Plain CSR (the reference's struct, mv_ops.h:17-23).  One 64-row block per
// wave (<= CAPW nonzeros, planned on the host): the block's val/col window
// goes HBM -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction,
// no VGPR staging, exec-masked to the block's exact extent), then lane t
// sums row t from LDS sequentially in column order from 0.0 -- the
// reference's per-row order (mv_ops.c:190-194), so y is bit-identical to it
// on chained matrices.  8 x-gathers in flight per row chunk (a 7-point row
// is one round trip; two consecutive columns in every row of the wave -- a
// stencil's -1, 0 -- are one 16-byte pair load); padding terms are selected away (never multiplied by
// 0: an inf/NaN x must not leak into a row that does not reference it).
// A row longer than the window gets a block of its own and is streamed in
// window-sized chunks by lane 0.  NT: the once-per-iteration matrix stream
// and the y store bypass the caches (the CG vectors stay resident).
template <typename T, int CAPW, int U, bool EPI, bool NT, bool LIST>
__global__ __launch_bounds__(256) void k_spmv_csr(SpmvArgs<T> a) {
  constexpr int WPB = 4, AUX = NT ? 2 : 0;
  static_assert(CAPW % 4 == 0, "window");
  __shared__ __attribute__((aligned(16))) T lval_all[WPB * CAPW];
  __shared__ __attribute__((aligned(16))) int lcol_all[WPB * CAPW];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  T *lval = lval_all + wid * CAPW;
  int *lcol = lcol_all + wid * CAPW;
  const int wi = __builtin_amdgcn_readfirstlane(xcd_block() * WPB + wid);
  double dot = 0.0, dot2 = 0.0;
  if (wi < a.items.count) {
    Blk B;
    if (!load_block(a, wi, B, LIST)) return;
    const int r0 = B.r0, nr = B.nr, k0 = B.k0, k1 = B.k1;
    const int kb = k0 & ~3;  // 16-B aligned for both val (T) and col (int)
    const bool fits = k1 - kb <= CAPW;
    if (fits) {
      constexpr int EV = 16 / sizeof(T);
      const int m = k1 - kb;
#pragma unroll
      for (int i = 0; i < (int)((CAPW * sizeof(T) + 1023) / 1024); ++i)
        if (i * kWave * EV < m && (i * kWave + lane) * EV < m)
          __builtin_amdgcn_global_load_lds((const void *)(a.val + kb + i * kWave * EV + lane * EV),
                                           (lds_void *)(lval + i * kWave * EV), 16, 0, AUX);
#pragma unroll
      for (int i = 0; i < (CAPW * 4 + 1023) / 1024; ++i)
        if (i * kWave * 4 < m && (i * kWave + lane) * 4 < m)
          __builtin_amdgcn_global_load_lds((const void *)(a.col + kb + i * kWave * 4 + lane * 4),
                                           (lds_void *)(lcol + i * kWave * 4), 16, 0, AUX);
    }
    // row bounds: one row_ptr load per lane, the row end is the next lane's
    // start (the block's last row ends at k1); x[row] for the epilogue is the
    // diagonal entry's own gather when the row has one (-4% at C3 with both,
    // tools/mb/spmv_lab.hip), else a load of its own
    int j0 = 0, j1 = 0;
    T xrow = T(0), acc = T(0);
    bool have_x = false;
    if (lane < nr) {
      j0 = a.rp[r0 + lane];
      if (a.yacc) acc = a.yacc[r0 + lane];  // column panels: continue the row sum
    }
    if (fits) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      j1 = __shfl_down(j0, 1, kWave);
      if (lane == nr - 1) j1 = k1;
      wave_lds_sync();
      if (lane < nr) {
        const int row = r0 + lane;
        for (int j = j0 - kb; j < j1 - kb; j += U) {
          const int cnt = min(U, j1 - kb - j);
          int cc[U];
          T vv[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int idx = u < cnt ? j + u : j;  // clamped: every LDS read is valid
            cc[u] = u < cnt ? lcol[idx] : 0;
            vv[u] = lval[idx];
          }
          // the chunk's gathers with entries (Q, Q + 1) as ONE pair load of
          // (x[c], x[c + 1]) (Q < 0: none), then the row's products in its
          // order -- the same values as single loads
          auto chunk = [&](auto qc) {
            constexpr int Q = decltype(qc)::value;
            T xx[U];
            typename Pair<T>::type xp{};
#pragma unroll
            for (int u = 0; u < U; ++u) {
              if (u == Q) xp = ld_pair(a.x, cc[u]);
              else if (Q < 0 || u != Q + 1) xx[u] = a.x[cc[u]];
            }
            if constexpr (Q >= 0) {
              xx[Q] = xp.x;
              xx[Q + 1] = xp.y;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const T pr = vv[u] * xx[u];
              acc = u < cnt ? acc + pr : acc;
              if (EPI && u < cnt && cc[u] == row) {
                xrow = xx[u];
                have_x = true;
              }
            }
          };
          if constexpr (U == 7 && sizeof(T) == 8) {
            // a run of consecutive columns (a stencil's -1, 0, +1): the lowest
            // q whose entries q, q + 1 are consecutive in every active lane's
            // row that holds entry q + 1 -- wave-uniform (ballot over the
            // active lanes), so the chunk issues one gather instruction less
            // and no lane diverges.  A pair reaches x[c + 1] <= x[ncols], the
            // vectors' padding; a lane past its row's end loads a pair it
            // never uses.  Round 5, same box, alternating
            // (profiles/r05_ab_csr_pairs_c*.log): C3 in the iteration 185.8 ->
            // 184.8 us, C4 1,215.6 -> 1,212.4 (back to back 1,236 -> 1,225).
            int q = -1;
#pragma unroll
            for (int u = U - 2; u >= 0; --u) {
              const bool ok = u + 1 >= cnt || cc[u + 1] == cc[u] + 1;
              if (__ballot(!ok) == 0) q = u;
            }
            switch (q) {
              case 0: chunk(std::integral_constant<int, 0>{}); break;
              case 1: chunk(std::integral_constant<int, 1>{}); break;
              case 2: chunk(std::integral_constant<int, 2>{}); break;
              case 3: chunk(std::integral_constant<int, 3>{}); break;
              case 4: chunk(std::integral_constant<int, 4>{}); break;
              case 5: chunk(std::integral_constant<int, 5>{}); break;
              default: chunk(std::integral_constant<int, -1>{}); break;
            }
          } else {
            chunk(std::integral_constant<int, -1>{});
          }
        }
      }
    } else {
      for (int c0 = k0; c0 < k1; c0 += CAPW) {
        const int m = min(CAPW, k1 - c0);
        for (int t = lane; t < m; t += kWave) lval[t] = a.val[c0 + t] * a.x[a.col[c0 + t]];
        wave_lds_sync();
        if (lane == 0)
          for (int j = 0; j < m; ++j) acc = acc + lval[j];
        wave_lds_sync();
      }
    }
    if (lane < nr) {
      st_y(a.y + r0 + lane, acc, NT);
      if (EPI) {
        if (!have_x) xrow = a.x[r0 + lane];
        dot = (double)xrow * (double)acc;
        dot2 = (double)acc * (double)acc;
      }
    }
  }
  if (EPI) epi_store_p<WPB>(dot, dot2, a.part, a.pair);
}

// ------------------------------------------------------------- k_spmv_dc
// Dictionary-coded columns (CSR-DC): matrices whose nonzeros use at most 256
// distinct column offsets col - row (stencils, banded matrices) store one
// code byte per nonzero instead of a 4-byte column, col = row + dict[code],
// and one byte per row for its length instead of two row_ptr reads (rows of
// <= 255 entries).  Otherwise k_spmv_csr: the val window and the code window
// land in the wave's LDS slice by LDS-DMA, row bounds come from a wave prefix
// sum of the lengths, lane t decodes and sums row t sequentially (bit-
// identical y).  The dictionary is copied into each wave's LDS slice.
template <typename T, int CAPW, int ND, int U, bool EPI, bool NT, bool LIST>
__global__ __launch_bounds__(256) void k_spmv_dc(SpmvArgs<T> a) {
  constexpr int WPB = 4, AUX = NT ? 2 : 0;
  static_assert(CAPW % 4 == 0 && ND % kWave == 0, "window / dictionary");
  // code window: starts at the 16-B granule holding entry k0, so up to 15
  // more entries than the val window in front
  constexpr int CAPC = (CAPW + 16 + 15) & ~15;
  __shared__ __attribute__((aligned(16))) T lval_all[WPB * CAPW];
  __shared__ __attribute__((aligned(16))) unsigned char lcode_all[WPB * CAPC];
  __shared__ int ldict_all[WPB * ND];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  T *lval = lval_all + wid * CAPW;
  unsigned char *lcode = lcode_all + wid * CAPC;
  int *ldict = ldict_all + wid * ND;
  const int wi = __builtin_amdgcn_readfirstlane(xcd_block() * WPB + wid);
  double dot = 0.0, dot2 = 0.0;
  if (wi < a.items.count) {
    Blk B;
    if (!load_block(a, wi, B, LIST)) return;
    const int r0 = B.r0, nr = B.nr, k0 = B.k0, k1 = B.k1;
    const int kb = k0 & ~3;   // val window: 16-B aligned for double and float
    const int kc = k0 & ~15;  // code window: 16-B aligned
    const bool fits = k1 - kb <= CAPW;
    if (fits) {
      constexpr int EV = 16 / sizeof(T);
      const int m = k1 - kb;
#pragma unroll
      for (int i = 0; i < (int)((CAPW * sizeof(T) + 1023) / 1024); ++i)
        if ((i * kWave + lane) * EV < m)
          __builtin_amdgcn_global_load_lds((const void *)(a.val + kb + i * kWave * EV + lane * EV),
                                           (lds_void *)(lval + i * kWave * EV), 16, 0, AUX);
      const int mc = k1 - kc;
#pragma unroll
      for (int i = 0; i < (CAPC + 1023) / 1024; ++i)
        if ((i * kWave + lane) * 16 < mc)
          __builtin_amdgcn_global_load_lds((const void *)(a.code + kc + i * kWave * 16 + lane * 16),
                                           (lds_void *)(lcode + i * kWave * 16), 16, 0, AUX);
    }
    int len = 0;
    T xrow = T(0), acc = T(0);
    bool have_x = false;  // x[row]: the diagonal's gather (offset 0) when present
    if (lane < nr) len = a.rlen[r0 + lane];
    int dv[ND / kWave];
#pragma unroll
    for (int i = 0; i < ND / kWave; ++i) dv[i] = a.dict[i * kWave + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int j1 = k0 + wave_incl_scan(len, lane);
    const int j0 = j1 - len;
#pragma unroll
    for (int i = 0; i < ND / kWave; ++i) ldict[i * kWave + lane] = dv[i];
    wave_lds_sync();
    const int row = r0 + lane;
    if (fits) {
      if (lane < nr) {
        const int co = kb - kc;  // the val window's first entry in the code window
        for (int j = j0 - kb; j < j1 - kb; j += U) {
          const int cnt = min(U, j1 - kb - j);
          int code[U];
          T vv[U], xx[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int idx = u < cnt ? j + u : j;
            code[u] = lcode[idx + co];
            vv[u] = lval[idx];
          }
          int off[U];
#pragma unroll
          for (int u = 0; u < U; ++u) off[u] = u < cnt ? ldict[code[u]] : 0;
#pragma unroll
          for (int u = 0; u < U; ++u) xx[u] = a.x[row + off[u]];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const T pr = vv[u] * xx[u];
            acc = u < cnt ? acc + pr : acc;
            if (EPI && u < cnt && off[u] == 0) {
              xrow = xx[u];
              have_x = true;
            }
          }
        }
      }
    } else {
      // a single row longer than the window (nr == 1): chunked, lane 0 keeps
      // the sequential sum; codes decoded from memory
      for (int c0 = k0; c0 < k1; c0 += CAPW) {
        const int m = min(CAPW, k1 - c0);
        for (int t = lane; t < m; t += kWave)
          lval[t] = a.val[c0 + t] * a.x[r0 + ldict[a.code[c0 + t]]];
        wave_lds_sync();
        if (lane == 0)
          for (int j = 0; j < m; ++j) acc = acc + lval[j];
        wave_lds_sync();
      }
    }
    if (lane < nr) {
      st_y(a.y + row, acc, NT);
      if (EPI) {
        if (!have_x) xrow = a.x[row];
        dot = (double)xrow * (double)acc;
        dot2 = (double)acc * (double)acc;
      }
    }
  }
  if (EPI) epi_store_p<WPB>(dot, dot2, a.part, a.pair);
}

// ------------------------------------------------------------ k_spmv_dia
// Value-indexed diagonal codes (DIA-VI).  A matrix whose nonzeros lie on at
// most 16 diagonals d_0 < ... < d_{K-1} (col - row), with at most 15
// distinct values (bit patterns) per diagonal -- stencils, banded matrices
// with few coefficients -- stores per row one bit field per diagonal: the
// index of the entry's value in that diagonal's value table, all ones = no
// entry; fields 1-4 bits wide by the diagonal's value count (a Laplacian:
// one bit per diagonal, one byte per row), the row's word 1, 2, 4 or 8
// bytes; no column or value stream.  A row's entries ascend in column, i.e. in diagonal (checked by the
// encoder), so summing k = 0..K-1 adds the CSR row's products in its order:
// y is bit-identical to k_spmv_csr.  Two rows per thread, r even: the
// neighbours x[r + d_k], x[r + 1 + d_k] of both rows are ONE 16-byte (fp64)
// load, issued only by lanes whose rows hold diagonal k (a wave skips a
// diagonal none of its rows hold, e.g. a partition's ghost diagonals) -- half
// the vector-memory instructions of a row-per-thread gather, the lesson of
// the lab (tools/mb/spmv_lab.hip: 82 -> 38 us at C3).  The codes of the two
// rows are one load; the only dependent round trip is codes -> x.
template <typename T>
__device__ __forceinline__ void st_pair(T *y, int r, int n, T a0, T a1, bool nt) {
  typedef typename Pair<T>::type P;
  if (r + 1 < n) {
    P o;
    o.x = a0;
    o.y = a1;
    if (nt) __builtin_nontemporal_store(o, reinterpret_cast<P *>(y + r));
    else *reinterpret_cast<P *>(y + r) = o;
  } else if (r < n) {
    st_y(y + r, a0, nt);
  }
}

// LDS pair access at an EVEN index of a window whose base is 16-B aligned:
// one ds_read_b128 / ds_write_b128 (fp64) instead of two 8-B accesses at a
// 16-B lane stride (the plane-march kernels: slot strides even, halos even;
// same-box A/B at C4 / C3 within the noise: 748-750 vs 755-803 / 134-138 vs
// 133 us per SR iteration -- kept for the halved LDS instruction count).
template <typename T>
struct PairA {
  typedef T type __attribute__((ext_vector_type(2), aligned(2 * sizeof(T))));
};
template <typename T>
__device__ __forceinline__ void lds_ld2(const T *w, int i, T &v0, T &v1) {
  const typename PairA<T>::type v = *reinterpret_cast<const typename PairA<T>::type *>(w + i);
  v0 = v.x;
  v1 = v.y;
}
template <typename T>
__device__ __forceinline__ void lds_st2(T *w, int i, T v0, T v1) {
  typename PairA<T>::type v;
  v.x = v0;
  v.y = v1;
  *reinterpret_cast<typename PairA<T>::type *>(w + i) = v;
}

// The code words of rows r, r + 1 (r even): one load of 2 cb bytes (cb is
// uniform: a scalar branch).  C = unsigned holds words of <= 4 bytes.
template <typename C>
__device__ __forceinline__ void ld_codes(const unsigned char *code, int cb, int r, C &c0, C &c1) {
  const unsigned char *p = code + (long long)r * cb;
  if (cb == 1) {
    const unsigned w = *reinterpret_cast<const unsigned short *>(p);
    c0 = w & 0xffu;
    c1 = w >> 8;
  } else if (cb == 2) {
    const unsigned w = *reinterpret_cast<const unsigned *>(p);
    c0 = w & 0xffffu;
    c1 = w >> 16;
  } else if (sizeof(C) == 4 || cb == 4) {
    const uint2 w = *reinterpret_cast<const uint2 *>(p);
    c0 = w.x;
    c1 = w.y;
  } else {
    const uint4 w = *reinterpret_cast<const uint4 *>(p);
    c0 = (C)((unsigned long long)w.x | ((unsigned long long)w.y << 32));
    c1 = (C)((unsigned long long)w.z | ((unsigned long long)w.w << 32));
  }
}

// diagonal k's field of a code word
template <typename T, typename C>
__device__ __forceinline__ unsigned fld(const SpmvArgs<T> &a, C c, int k) {
  return (unsigned)(c >> a.csh[k]) & a.cmask[k];
}

// DV (DIA-V, KW 1): the values from the stream (SpmvArgs::dval), diagonal k
// of rows r, r + 1 as one pair load, instead of the value table.
template <typename T, int KW, bool EPI, bool NT, bool LIST, bool DV>
__global__ __launch_bounds__(256) void k_spmv_dia(SpmvArgs<T> a) {
  constexpr int KM = 8 * KW;  // diagonals unrolled (<= 8: 32-bit words)
  typedef typename std::conditional<KW == 1, unsigned, unsigned long long>::type C;
  __shared__ T lv[KM * 16];
  typedef typename Pair<T>::type P;
  const int t = threadIdx.x;
  const int wi = xcd_block();
  const int stop = a.done ? *a.done : 0;
  const int s = LIST ? a.items.list[wi] : a.items.first + wi;
  if (stop) return;  // uniform: every thread of the grid reads the same flag
  const int r = s * kDiaSliceRows + 2 * t;
  const int rs = r < a.n ? r : 0;  // a row pair past the end (no entries) reloads x[0]
  C c0, c1;  // the code words of row r / r + 1
  ld_codes(a.dcode, a.cb, r, c0, c1);
  const T tv = t < a.ndiag * 16 ? a.vtab[t] : T(0);
  P xv[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    // unconditional (a lane whose rows hold no entry on diagonal k reloads
    // its own x[r]): a conditional load makes the compiler wait on it
    const unsigned n0 = fld(a, c0, k), n1 = fld(a, c1, k);
    xv[k] = ld_pair(a.x, k < a.ndiag && (n0 != a.cmask[k] || n1 != a.cmask[k]) ? r + a.doff[k] : rs);
  }
  // x[r], x[r+1] for the epilogue: a pair load of its own (picking the main
  // diagonal's registers costs the compiler 4x the VGPRs)
  P xr = P{T(0), T(0)};
  if (EPI && r < a.n) xr = ld_pair(a.x, r);
  P dvv[DV ? KM : 1];
  if constexpr (DV) {
#pragma unroll
    for (int k = 0; k < KM; ++k)  // rows < the padded rows: in bounds
      dvv[k] = k < a.ndiag ? ld_pair(a.dval + (size_t)k * a.dvs, r) : P{T(0), T(0)};
  }
  if (t < a.ndiag * 16) lv[t] = tv;
  __syncthreads();
  T a0 = T(0), a1 = T(0);
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < a.ndiag) {
      const unsigned n0 = fld(a, c0, k), n1 = fld(a, c1, k);
      const T w0 = DV ? dvv[DV ? k : 0].x : lv[k * 16 + n0];
      const T w1 = DV ? dvv[DV ? k : 0].y : lv[k * 16 + n1];
      const T p0 = w0 * xv[k].x, p1 = w1 * xv[k].y;
      a0 = n0 != a.cmask[k] ? a0 + p0 : a0;
      a1 = n1 != a.cmask[k] ? a1 + p1 : a1;
    }
  }
  st_pair(a.y, r, a.n, a0, a1, NT);
  double dot = 0.0, dot2 = 0.0;
  if (EPI) {
    if (r < a.n) {
      dot = (double)xr.x * (double)a0;
      dot2 = (double)a0 * (double)a0;
    }
    if (r + 1 < a.n) {
      dot = dot + (double)xr.y * (double)a1;
      dot2 = dot2 + (double)a1 * (double)a1;
    }
  }
  if (EPI) epi_store_p<4>(dot, dot2, a.part, a.pair);
}

// ------------------------------------------------- fused HS step (DIA-VI)
// The scalar step at the top of a fused launch -- the folded k_xpay_xf's
// logic (cg.c:125-129): r.r of the last r-update (*rr_new: k_update_rf's
// canonical last-arriver sum, or its all-reduce over the ranks), the stop
// test, beta; every thread computes it from the same state, workgroup 0 of
// the publishing launch writes it back.  A kernel never writes a state field
// its own workgroups read; the stop flag follows the folded path's protocol
// (1 here, 2 by the next k_update_rf).
struct FuseStep {
  bool first, stop;
  double alpha, beta;
};

// CGX_ALG_SR (sr): *rr_new_p is k_update_rf's estimate alpha^2 s.s - r.r,
// for beta only; the stop test is k_update_rf's, on the exact r.r one
// launch later (oracle_solve_sr), which sets done = 1 when an even
// iteration's deferred x update is pending: stop here means "apply it".
__device__ __forceinline__ FuseStep fuse_step(CgState *st, double *hist, const double *rr_new_p,
                                              bool publish, bool sr = false) {
  FuseStep f;
  const int k = st->k_u;
  f.first = k < 0;
  f.alpha = st->alpha;
  f.beta = 0.0;
  f.stop = false;
  if (sr) {
    f.stop = st->done == 1;
    if (!f.first) f.beta = *rr_new_p / st->rr_u;  // cg.c:129
    if (!f.first && !f.stop && publish && blockIdx.x == 0 && threadIdx.x == 0) {
      st->beta = f.beta;
      st->k = k + 1;
      st->k_x = k + 1;
    }
    return f;
  }
  if (!f.first) {
    const double rr_new = *rr_new_p;
    f.stop = k >= st->max_iter || (st->use_tol && rr_new <= st->tol2bb);
    f.beta = rr_new / st->rr_u;  // cg.c:129
    if (publish && blockIdx.x == 0 && threadIdx.x == 0) {
      if (k < st->hist_cap) hist[k] = rr_new;
      if (f.stop) {
        st->k = k;
        st->done = 1;
      } else {
        st->beta = f.beta;
        st->rr = rr_new;
        st->rr_x = rr_new;
        st->k = k + 1;
        st->k_x = k + 1;
      }
    }
  }
  return f;
}

// p_new = r + beta p_old (cg.c:131-132), two roundings as the reference
template <typename T>
__device__ __forceinline__ typename Pair<T>::type p_next(typename Pair<T>::type r,
                                                         typename Pair<T>::type p, T beta) {
  typename Pair<T>::type o;
  const T b0 = beta * p.x, b1 = beta * p.y;
  o.x = r.x + b0;
  o.y = r.y + b1;
  return o;
}

// k_spmv_dia's shape (two rows per thread, 512-row slice per workgroup)
// with the previous iteration's vector update fused in.  p_new of the slice
// and of its halo rows [s0 - hl, s0 + 512 + hr) is computed ONCE per
// workgroup into an LDS window (NF pair passes per thread): every "near"
// diagonal (|d| <= kHaloMax) reads p_new from there; the far ones (the
// +-nx*ny planes of a 3-D stencil; NFAR >= their count, slots a.fark) gather
// r and p_old and compute p_new themselves.  GH (a partition's boundary
// items): a column >= n is a ghost, whose p_new the halo exchange put in the
// p_new buffer's ghost tail -- read there, element by element, in the window
// and the far slots.  Then p_new for the own rows (and every other
// launch x, below), s = A p_new summed in diagonal order (the CSR row's
// order), the p_new.s partial.  Bytes per row: 1-4 code + 8 r + 8 p_old +
// 8 p_new + 8 s, + 24 (x read and written, p_{k-1} read) every other
// launch.  Every value is the unfused path's (same roundings): x and the
// r.r history are bit-identical to SpMV + k_update_rf + k_xpay_xf.
template <typename T, int SB, int NF, int NFAR, bool NT, bool LIST, bool GH>
__global__ __launch_bounds__(256 * SB) void k_spmv_dia_h(SpmvArgs<T> a, FuseArgs<T> f) {
  constexpr int BS = 256 * SB;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  T *win = reinterpret_cast<T *>(dyn_lds);
  __shared__ T lv[kDiaMax * 16];
  typedef typename Pair<T>::type P;
  const int t = threadIdx.x;
  // this workgroup's super-item: list positions [pos, pos + cnt), cnt <= SB
  // adjacent slices (SB = 2: Items::pairs, or the natural pairing of a
  // contiguous run; SB = 1: one slice, the k_spmv_dia shape)
  const int w = xcd_block();
  int pos, cnt;
  if (SB == 1) {
    pos = w;
    cnt = 1;
  } else if (a.items.pairs) {
    pos = a.items.pairs[2 * w];
    cnt = a.items.pairs[2 * w + 1];
  } else {
    pos = 2 * w;
    cnt = min(2, a.items.count - pos);
  }
  const int s = LIST ? a.items.list[pos] : a.items.first + pos;
  if (f.st->done > 1) return;  // uniform
  const FuseStep fs = fuse_step(f.st, f.hist, f.rr_new, f.publish != 0, f.ss != nullptr);
  const T alpha = (T)fs.alpha, beta = (T)fs.beta;
  const int s0 = s * kDiaSliceRows, r = s0 + 2 * t;
  // act: the row pair lies in the super-item's slices (rows >= n there are
  // padding: no entries); own: it holds a row of the matrix
  const int sx = s0 + kDiaSliceRows * cnt, rend = min(a.n, sx);
  const bool act = r < sx;
  const int ra = act ? r : s0;
  const int rs = r < a.n ? r : 0;
  // x (cg.c:115-116) is updated every other iteration: an even iteration k
  // defers x += alpha_k p_k, the odd k + 1 applies both terms in order (the
  // same two roundings each), reading p_k from the p_new buffer before it is
  // overwritten; a stop applies whatever is pending.
  const int k = f.st->k_u;
  const bool odd = (k & 1) != 0;
  const bool xup = !fs.first && (odd || fs.stop);
  // SR's stop (fuse_step): only the deferred x += alpha_k p_k of the even
  // stop iteration k, p_k in the p_new buffer
  const bool xdef = f.ss != nullptr && fs.stop;
  const T alpha_d = (T)f.st->alpha_def;
  if (f.publish && !fs.first && !odd && !fs.stop && blockIdx.x == 0 && t == 0)
    f.st->alpha_def = fs.alpha;
  P po = P(), xo = P(), pd = P();
  auto load_x = [&]() {
    if (xup) {
      po = ld_pair(f.pold, rs);
      xo = ld_pair(f.x, rs);
      if (odd || xdef) pd = ld_pair((const T *)f.pnew, rs);
    }
  };
  auto x_update = [&]() {
    T x0 = xo.x, x1 = xo.y;
    if (odd || xdef) {
      const T d0 = alpha_d * pd.x, d1 = alpha_d * pd.y;
      x0 = x0 + d0;
      x1 = x1 + d1;
    }
    if (!xdef) {
      const T a0 = alpha * po.x, a1 = alpha * po.y;
      x0 = x0 + a0;
      x1 = x1 + a1;
    }
    st_pair(f.x, r, rend, x0, x1, false);
  };
  if (fs.stop) {  // the pending x updates only (then the cg.c:125 break)
    load_x();
    if (xup && r < rend) x_update();
    return;
  }
  unsigned c0, c1;  // the code words of row ra / ra + 1 (<= 4 bytes: fusable())
  ld_codes(a.dcode, a.cb, ra, c0, c1);
  const T tv = t < a.ndiag * 16 ? a.vtab[t] : T(0);
  // far diagonals: slot q holds diagonal a.fark[q] (-1: an unused slot)
  constexpr int NS = NFAR > 0 ? NFAR : 1;
  P rf[NS], pf[NS], gf[NS];
  int fb[NS];
#pragma unroll
  for (int q = 0; q < NFAR; ++q) {
    const int kq = a.fark[q];
    int b = rs;
    if (kq >= 0 && act) {
      const unsigned n0 = fld(a, c0, kq), n1 = fld(a, c1, kq);
      if (n0 != a.cmask[kq] || n1 != a.cmask[kq]) b = r + a.doff[kq];
    }
    fb[q] = b;
    rf[q] = ld_pair(f.r, b);
    pf[q] = ld_pair(f.pold, b);
    if (GH) gf[q] = ld_pair((const T *)f.pnew, b);
  }
  // the window: p_new of rows w0 + i, i < wn (pairs; rows outside [0, ncols)
  // are loaded from a clamped address and never read)
  const int w0 = s0 - a.hl, wn = kDiaSliceRows * cnt + a.hl + a.hr;
  P wr[NF], wp[NF], wg[NF];
  int wj[NF];
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    const int j = min(max(w0 + 2 * t + q * 2 * BS, -1), a.ncols - 1);
    wj[q] = j;
    wr[q] = ld_pair(f.r, j);
    wp[q] = ld_pair(f.pold, j);
    if (GH) wg[q] = ld_pair((const T *)f.pnew, j);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load above is in flight before the first use
  // p_new of a pair at column j: r + beta p_old, or the received ghost value
  auto pnext_at = [&](P rv, P pv, P gv, int j) {
    P o = fs.first ? rv : p_next<T>(rv, pv, beta);
    if (GH) {
      if (j >= a.n) o.x = gv.x;
      if (j + 1 >= a.n) o.y = gv.y;
    }
    return o;
  };
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    const int i = 2 * t + q * 2 * BS;
    const P pn = pnext_at(wr[q], wp[q], wg[q], wj[q]);
    if (i < wn) win[i] = pn.x;
    if (i + 1 < wn) win[i + 1] = pn.y;
  }
  P pk[NS];
#pragma unroll
  for (int q = 0; q < NFAR; ++q) pk[q] = pnext_at(rf[q], pf[q], gf[q], fb[q]);
  if (t < a.ndiag * 16) lv[t] = tv;
  __syncthreads();
  // the x update's operands are loaded here, where the window's and the far
  // slots' load registers are dead (70 -> fewer VGPRs over the launch)
  load_x();
  // s = A p_new in diagonal order: near diagonals from the window, far ones
  // from their slot (the number of far diagonals before k); an inactive pair
  // reads inside the window's allocation and stores nothing
  const int rw = r - w0;
  T a0 = T(0), a1 = T(0);
#pragma unroll
  for (int kk = 0; kk < kDiaMax; ++kk) {
    if (kk < a.ndiag) {
      T v0, v1;
      if ((a.near >> kk) & 1u) {
        const int i = rw + a.doff[kk];
        v0 = win[i];
        v1 = win[i + 1];
      } else {
        const int slot = __builtin_popcount(~a.near & ((1u << kk) - 1u));
        P v = pk[0];
#pragma unroll
        for (int q = 1; q < NFAR; ++q) v = slot == q ? pk[q] : v;
        v0 = v.x;
        v1 = v.y;
      }
      const unsigned n0 = fld(a, c0, kk), n1 = fld(a, c1, kk);
      const T p0 = lv[kk * 16 + n0] * v0, p1 = lv[kk * 16 + n1] * v1;
      a0 = n0 != a.cmask[kk] ? a0 + p0 : a0;
      a1 = n1 != a.cmask[kk] ? a1 + p1 : a1;
    }
  }
  const T pn0 = win[rw], pn1 = win[rw + 1];
  st_pair(a.y, r, rend, a0, a1, NT);
  double dot = 0.0, dot2 = 0.0;
  if (r < rend) {
    st_pair(f.pnew, r, rend, pn0, pn1, false);
    if (xup) x_update();
    dot = (double)pn0 * (double)a0;
    if (r + 1 < rend) dot = dot + (double)pn1 * (double)a1;
    if (f.ss) {
      dot2 = (double)a0 * (double)a0;
      if (r + 1 < rend) dot2 = dot2 + (double)a1 * (double)a1;
    }
  }
  // one partial per slice, at the slot the unfused launch (one workgroup per
  // slice, k_spmv_dia) writes it: the same four wave sums in the same order
  epi_store_slices<SB>(dot, dot2, f.ss, a.part, pos, cnt, a.items.count);
}

// ------------------------------------- fused HS step, plane march (DIA-VI)
// k_spmv_dia_h's iteration with its far diagonals read from LDS instead of
// gathered.  When every far diagonal is +F or -F and F = Q * 512 + e with
// |e| <= the window's halo (C3: F = 46,656 = 91 * 512 + 64, halo 216; C4:
// 160,000 = 312 * 512 + 256, halo 400), the rows F away from super-item j
// lie inside the WINDOW of super-item j +- Q.  A workgroup therefore walks a
// chain of super-items j0, j0 + Q, j0 + 2Q, ... (a column of the grid for a
// 3-D stencil), keeping three windows of p_new in an LDS ring: step m reads
// its near diagonals from window m and the -F / +F ones from windows m - 1
// and m + 1, so each p_new of the chain is computed once and no r / p_old
// gather is issued for the far diagonals (the unit profile of k_spmv_dia_h,
// profiles/r03_c4_units.md: vector-memory-instruction-bound, the far slots
// ~40 % of its loads).  The loads of window m + 2 are in flight while step m
// computes.  A chain is cut into segments of a.mlen steps (a workgroup each;
// a segment computes its two neighbouring windows as well).  Every value is
// k_spmv_dia_h's -- same roundings, the row's diagonal order -- and each
// slice's p.s partial is the sum of its four waves in order at the slot the
// one-workgroup-per-slice launch writes it (a.mpos: slice -> list position),
// so x and the r.r history stay bit-identical to the unfused path.  Single
// GPU only (no ghosts, no SR pairs): launch_spmv_fused checks.
// The two rows' code words as loaded (CB bytes each), split by code_split
// only where they are used: ALU work on a loaded value before a later load
// would make the wave wait for the value right there (k_spmv_dia_m).
template <int CB>
struct CodeRaw {
  typedef typename std::conditional<CB == 4, uint2, unsigned>::type type;
};

template <int CB>
__device__ __forceinline__ typename CodeRaw<CB>::type ld_code_raw(const unsigned char *code, int r) {
  const unsigned char *p = code + (long long)r * CB;
  if constexpr (CB == 1) return *reinterpret_cast<const unsigned short *>(p);
  else if constexpr (CB == 2) return *reinterpret_cast<const unsigned *>(p);
  else return *reinterpret_cast<const uint2 *>(p);
}

template <int CB>
__device__ __forceinline__ void code_split(typename CodeRaw<CB>::type w, unsigned &c0,
                                           unsigned &c1) {
  if constexpr (CB == 1) {
    c0 = w & 0xffu;
    c1 = w >> 8;
  } else if constexpr (CB == 2) {
    c0 = w & 0xffffu;
    c1 = w >> 16;
  } else {
    c0 = w.x;
    c1 = w.y;
  }
}

template <typename T, int SB, int NF, int CB>
__global__ __launch_bounds__(256 * SB) void k_spmv_dia_m(SpmvArgs<T> a, FuseArgs<T> f) {
  constexpr int BS = 256 * SB, SR = kDiaSliceRows * SB;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  T *ring = reinterpret_cast<T *>(dyn_lds);
  __shared__ T lv[kDiaMax * 16];
  __shared__ double red[4 * SB];
  typedef typename Pair<T>::type P;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int w = xcd_block();
  const int chain = w % a.mchains, seg = w / a.mchains;
  const int j0 = chain * SB;
  const int msteps = (a.mslices - j0 + a.mq - 1) / a.mq;
  const int m0 = seg * f.march, m1 = min(m0 + f.march, msteps);
  if (f.st->done > 1) return;  // uniform
  const FuseStep fs = fuse_step(f.st, f.hist, f.rr_new, f.publish != 0);
  const T alpha = (T)fs.alpha, beta = (T)fs.beta;
  const int k = f.st->k_u;
  const bool odd = (k & 1) != 0;
  const bool xup = !fs.first && (odd || fs.stop);
  const T alpha_d = (T)f.st->alpha_def;
  if (f.publish && !fs.first && !odd && !fs.stop && blockIdx.x == 0 && t == 0)
    f.st->alpha_def = fs.alpha;
  if (m0 >= m1) return;  // uniform (workgroup 0 always has steps: it publishes above)
  const int QR = a.mq * kDiaSliceRows;  // rows between the steps of a chain
  const int padn = a.mslices * kDiaSliceRows;
  const bool nt = a.nt != 0;
  const int wn = SR + a.hl + a.hr, ws = a.mws;
  auto base_of = [&](int m) { return (j0 + m * a.mq) * kDiaSliceRows; };
  auto slot = [&](int m) { return ring + ((m + 3) % 3) * ws; };
  P wr[NF], wp[NF];
  auto load_win = [&](int m) {
    const int w0 = base_of(m) - a.hl;
#pragma unroll
    for (int q = 0; q < NF; ++q) {
      const int j = min(max(w0 + 2 * t + q * 2 * BS, -1), a.ncols - 1);
      wr[q] = ld_pair(f.r, j);
      wp[q] = ld_pair(f.pold, j);
    }
  };
  auto store_win = [&](int m) {
    T *win = slot(m);
#pragma unroll
    for (int q = 0; q < NF; ++q) {
      const int i = 2 * t + q * 2 * BS;
      const P pn = fs.first ? wr[q] : p_next<T>(wr[q], wp[q], beta);
      if (i + 1 < wn) lds_st2(win, i, pn.x, pn.y);  // wn even (march plan)
      else if (i < wn) win[i] = pn.x;
    }
  };
  // the x update's operands of step m's rows (p_old, x, and on odd launches
  // p_{k-1} from the p_new buffer)
  struct XOps {
    P po, xo, pd;
  };
  auto load_x = [&](int m, XOps &o) {
    const int r = base_of(m) + 2 * t, rs = r < a.n ? r : 0;
    o.po = ld_pair(f.pold, rs);
    o.xo = ld_pair(f.x, rs);
    if (odd) o.pd = ld_pair((const T *)f.pnew, rs);
  };
  auto x_update = [&](const XOps &o, int r, int rend) {
    T x0 = o.xo.x, x1 = o.xo.y;
    if (odd) {
      const T d0 = alpha_d * o.pd.x, d1 = alpha_d * o.pd.y;
      x0 = x0 + d0;
      x1 = x1 + d1;
    }
    const T a0 = alpha * o.po.x, a1 = alpha * o.po.y;
    st_pair(f.x, r, rend, x0 + a0, x1 + a1, false);
  };
  XOps xc{}, xn{};
  if (fs.stop) {  // the pending x updates only (then the cg.c:125 break)
    if (xup)
      for (int m = m0; m < m1; ++m) {
        const int r = base_of(m) + 2 * t, rend = min(a.n, base_of(m) + SR);
        load_x(m, xc);
        if (r < rend) x_update(xc, r, rend);
      }
    return;
  }
  // Issue order matters: vector-memory operations retire in order (s_waitcnt
  // vmcnt), so a value is waited for together with everything issued before
  // it.  The codes, slot position and x operands of step m + 1 are therefore
  // issued during step m BEFORE window m + 2's loads, and used in step m + 1,
  // after window m + 1's wait has covered them: no step waits on the window
  // prefetch in flight.
  typedef typename CodeRaw<CB>::type CR;
  auto codes_at = [&](int m, CR &cw, int &ps) {
    const int r = base_of(m) + 2 * t;
    cw = ld_code_raw<CB>(a.dcode, r < padn ? r : base_of(m));  // past the last slice: none
    const int js = min(j0 + m * a.mq + min(wid, SB - 1), a.mslices - 1);
    ps = a.mpos ? a.mpos[js] : js;
  };
  const T tv = t < a.ndiag * 16 ? a.vtab[t] : T(0);
  CR cw, cwn{};
  int ps, psn = 0;
  codes_at(m0, cw, ps);
  if (xup) load_x(m0, xc);
  load_win(m0 - 1);
  store_win(m0 - 1);
  load_win(m0);
  store_win(m0);
  load_win(m0 + 1);
  if (t < a.ndiag * 16) lv[t] = tv;
  const int G = a.items.count;
  // One step; its operands (codes, slot position, x operands) arrive in the
  // "cur" set and the next step's are loaded into the "nxt" set.  The loop
  // below alternates the two register sets (no copies: a copy of a value
  // still in flight would wait for the window prefetch behind it).
  auto step = [&](int m, const CR &ccw, int &cps, XOps &cx, CR &ncw, int &nps, XOps &nx) {
    store_win(m + 1);
    // unconditional (past the segment: a reload of its last step / window,
    // L2 hits): a load under a branch leaves a merge that the compiler
    // resolves right away, i.e. a wait on everything in flight
    codes_at(min(m + 1, m1 - 1), ncw, nps);
    load_win(min(m + 2, m1));  // in flight during step m
    if (xup && m + 1 < m1) load_x(m + 1, nx);
    __syncthreads();
    const int base = base_of(m), r = base + 2 * t;
    const int rend = min(a.n, base + SR);
    const T *cur = slot(m), *prv = slot(m - 1), *nxt = slot(m + 1);
    const int rw = 2 * t + a.hl;
    unsigned cc0, cc1;
    code_split<CB>(ccw, cc0, cc1);
    T a0 = T(0), a1 = T(0);
#pragma unroll
    for (int kk = 0; kk < kDiaMax; ++kk) {
      if (kk < a.ndiag) {
        const int d = a.doff[kk];
        const T *src = (a.near >> kk) & 1u ? cur : d < 0 ? prv : nxt;
        const int i = (a.near >> kk) & 1u ? rw + d : d < 0 ? rw + d + QR : rw + d - QR;
        T v0, v1;
        if ((d & 1) == 0) lds_ld2(src, i, v0, v1);  // rw, QR even: an aligned pair
        else {
          v0 = src[i];
          v1 = src[i + 1];
        }
        const unsigned n0 = fld(a, cc0, kk), n1 = fld(a, cc1, kk);
        const T p0 = lv[kk * 16 + n0] * v0, p1 = lv[kk * 16 + n1] * v1;
        a0 = n0 != a.cmask[kk] ? a0 + p0 : a0;
        a1 = n1 != a.cmask[kk] ? a1 + p1 : a1;
      }
    }
    T pn0, pn1;
    lds_ld2(cur, rw, pn0, pn1);
    double dot = 0.0;
    if (r < rend) {
      st_pair(a.y, r, rend, a0, a1, nt);
      st_pair(f.pnew, r, rend, pn0, pn1, false);
      if (xup) x_update(cx, r, rend);
      dot = (double)pn0 * (double)a0;
      if (r + 1 < rend) dot = dot + (double)pn1 * (double)a1;
    }
    // per slice: its four waves' sums in order, at the slice's slot
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();  // also: every read of window m - 1's slot is done before step m + 1 refills it
    if (lane == 0 && wid < SB && j0 + m * a.mq + wid < a.mslices) {
      double sa = red[4 * wid];
#pragma unroll
      for (int v = 1; v < 4; ++v) sa = sa + red[4 * wid + v];
      a.part[xcd_slot(cps, G)] = sa;
    }
  };
  for (int m = m0; m < m1; m += 2) {
    step(m, cw, ps, xc, cwn, psn, xn);
    if (m + 1 < m1) step(m + 1, cwn, psn, xn, cw, ps, xc);
  }
}

// ------------------------------ single-GPU SR iteration, plane march (DIA-VI)
// CGX_ALG_SR on one GPU in ONE launch per iteration (FOLD: the FIN_SR1
// scalar step of the previous launch runs inside it; until round 6 a
// k_finalize launch followed each):
// the partitioned solver's SR recurrence (oracle_solve_sr: alpha = r.r / p.s
// as cg.c:113, beta from the estimate r_new.r_new = alpha (alpha s.s) - r.r)
// needs only the (p.s, s.s, r.r) of the launch that computes s = A p, so the
// r update of the next iteration moves into the next launch instead of a
// separate pass: per window row r_k = r_{k-1} - alpha s_{k-1} and
// p_k = r_k + beta p_{k-1} (the same two roundings each as the oracle), then
// s_k = A p_k from the three-window ring (k_spmv_dia_m's march), and per own
// row r_k, p_k, s_k stored and x += alpha p_{k-1} (every other launch for
// two iterations, as the HS step).  Bytes per row: code + r, s, p read, r, p,
// s written + x / p_{k-2} every other launch = 61 against the HS step's 69
// (fused launch 45 + r update 24).  r_k of the own rows is kept in an LDS
// buffer (two slots) when the window is built.  One (p.s, s.s) pair and one
// r.r per workgroup: each thread sums its rows in step order, then the wave
// tree and the waves in order -- deterministic.
// Partitioned ranks (in-place ghost rows: columns = global - row_begin, the
// rows of the neighbours' boundary planes at [col_lo, 0) and [n, ncols)):
// the same launch over every step while the halo is in flight; the windows'
// ghost rows hold no p_k yet, so s of the edge rows (Sr1Args::elo / ehi:
// those whose row reaches a ghost column) is provisional and stays out of
// the (p.s, s.s) sums -- k_sr1_edge recomputes it after the halo.
// DV (DIA-V, CB 1): the values of step m's rows stream in beside its codes
// (one pair load per diagonal, issued a step ahead) instead of the table.
template <typename T, int SB, int NF, int CB, bool DV, bool FOLD>
__global__ __launch_bounds__(256 * SB)
void k_sr1_dia_m(SpmvArgs<T> a, Sr1Args<T> f) {
  constexpr int BS = 256 * SB, SR = kDiaSliceRows * SB;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  T *ring = reinterpret_cast<T *>(dyn_lds);
  constexpr int NRING = 3, NRB = 2;
  T *rbuf = ring + NRING * a.mws;  // r_k of the own rows, NRB slots of SR
  __shared__ T lv[kDiaMax * 16];
  __shared__ double red[3][4 * SB];
  typedef typename Pair<T>::type P;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int w = xcd_block();
  // chains of cw rows (f.cw, even, <= SR; 0: SR = SB slices) side by side in
  // each step of QR rows; chain c's step m holds rows [c0 + m QR, + wc)
  const int QR = a.mq * kDiaSliceRows;
  const int CW = f.cw > 0 ? f.cw : SR;
  const int nch = (QR + CW - 1) / CW;
  const int chain = w % nch, seg = w / nch;
  const int c0 = chain * CW, wc = min(CW, QR - c0);
  const int msteps = c0 < a.n ? (a.n - c0 + QR - 1) / QR : 0;
  int m0, m1;
  if (f.nseg > 0) {  // the chain's steps in nseg balanced segments
    m0 = (int)((long long)seg * msteps / f.nseg);
    m1 = (int)((long long)(seg + 1) * msteps / f.nseg);
  } else {  // segments of f.march steps
    m0 = seg * f.march;
    m1 = min(m0 + f.march, msteps);
  }
  // The launch's scalars: without FOLD the state as the last k_finalize (or
  // the ranks' all-reduce, applied privately) left it, resolved here; with
  // FOLD (f.st_out: the single GPU, no k_finalize) resolved below, after the
  // prologue's loads are in flight, so that the folded scalar step overlaps
  // them.  (FOLD is a template parameter so that the ranks' kernels carry
  // none of its code: with it as a runtime branch their launch took 3-4 us
  // longer, profiles/r06_ab_sr1.log.)
  Sr1Now sn{};
  if constexpr (!FOLD) {
    sn = sr1_now(f.st, f.g);
    if (sn.done > 1) return;  // uniform
  }
  int k = 0;  // the last finalized iteration (-1: none)
  bool first = false, stop = false, odd = false, xup = false;
  // x deferral: depth 2 (x += alpha p for two iterations in odd launches)
  // or depth 4 (f.pa: four iterations in every launch with k % 4 == 3,
  // p_{k-3} / p_{k-2} / p_{k-1} from pnew / pa / pb, their alphas from
  // alpha_q) -- the same roundings in the same order as one update per
  // iteration (cg.c:115-116)
  const bool d4 = f.pa != nullptr;
  T alpha = T(0), beta = T(0), alpha_d = T(0), aq0 = T(0), aq1 = T(0), aq2 = T(0);
  const int padn = a.mslices * kDiaSliceRows;
  const bool nt = a.nt != 0;
  const int wn = wc + a.hl + a.hr, ws = a.mws;
  auto base_of = [&](int m) { return c0 + m * QR; };
  auto slot = [&](int m) { return ring + ((m + NRING) % NRING) * ws; };
  auto rslot = [&](int m) { return rbuf + ((m + NRB) % NRB) * SR; };
  struct XOps {
    P po, xo, pd;
  };
  auto load_x = [&](int m, XOps &o) {
    const int r = base_of(m) + 2 * t, rs = r < a.n ? r : 0;
    o.po = ld_pair(f.pold, rs);
    o.xo = ld_pair(f.x, rs);
    if (odd) o.pd = ld_pair((const T *)f.pnew, rs);
  };
  auto x_update = [&](const XOps &o, const P &qa, const P &qb, int r, int rend) {
    T x0 = o.xo.x, x1 = o.xo.y;
    if (d4) {  // k % 4 == 3: alpha_{k-3} p_{k-3}, alpha_{k-2} p_{k-2}, alpha_{k-1} p_{k-1}
      const T d0 = aq0 * o.pd.x, d1 = aq0 * o.pd.y;
      x0 = x0 + d0;
      x1 = x1 + d1;
      const T e0 = aq1 * qa.x, e1 = aq1 * qa.y;
      x0 = x0 + e0;
      x1 = x1 + e1;
      const T g0 = aq2 * qb.x, g1 = aq2 * qb.y;
      x0 = x0 + g0;
      x1 = x1 + g1;
    } else if (odd) {
      const T d0 = alpha_d * o.pd.x, d1 = alpha_d * o.pd.y;
      x0 = x0 + d0;
      x1 = x1 + d1;
    }
    const T a0 = alpha * o.po.x, a1 = alpha * o.po.y;
    st_pair(f.x, r, rend, x0 + a0, x1 + a1, false);
  };
  XOps xc{}, xn{};
  double sps = 0.0, sss = 0.0, srr = 0.0;
  auto publish = [&]() {
    sps = wave_sum(sps);
    sss = wave_sum(sss);
    srr = wave_sum(srr);
    if (lane == 0) {
      red[0][wid] = sps;
      red[1][wid] = sss;
      red[2][wid] = srr;
    }
    __syncthreads();
    if (t == 0) {
      double p0 = red[0][0], p1 = red[1][0], p2 = red[2][0];
#pragma unroll
      for (int v = 1; v < 4 * SB; ++v) {
        p0 = p0 + red[0][v];
        p1 = p1 + red[1][v];
        p2 = p2 + red[2][v];
      }
      reinterpret_cast<double2 *>(f.pq)[blockIdx.x] = make_double2(p0, p1);
      f.pc[blockIdx.x] = p2;
    }
  };
  P wr[NF], wp[NF], wsv[NF];
  // a wave whose pairs of pass q all lie past the window skips that pass
  // (wave-uniform: the wave's first pair; SB = 4 at C4: 9 of 16 waves skip
  // pass 1 -- round 5, with the four-slice steps 812 -> 783 us per C4 launch)
  const int wfirst = 2 * __builtin_amdgcn_readfirstlane(wid * kWave);
  for (int q = 0; q < NF; ++q) wr[q] = wp[q] = wsv[q] = P{T(0), T(0)};
  typedef P WinSet[NF];
  // window m's r, p, s pairs into (vr, vp, vs); `all`: every pass, also
  // those past the window (the prologue's loads, which must not sit under a
  // branch) -- a pair past the window loads the window's first pair
  // (unused; one line per wave instruction, an L1 hit)
  auto load_win_to = [&](int m, WinSet &vr, WinSet &vp, WinSet &vs, bool all) {
    const int w0 = base_of(m) - a.hl;
#pragma unroll
    for (int q = 0; q < NF; ++q) {
      if (!all && q > 0 && wfirst + q * 2 * BS >= wn) continue;
      const int i = 2 * t + q * 2 * BS;
      const int j = min(max(i < wn ? w0 + i : w0, a.xlo), a.ncols - 1);
      vr[q] = ld_pair(f.rold, j);
      vp[q] = ld_pair(f.pold, j);
      vs[q] = ld_pair(f.sold, j);
    }
  };
  auto load_win = [&](int m) { load_win_to(m, wr, wp, wsv, false); };
  auto store_win_from = [&](int m, const WinSet &vr, const WinSet &vp, const WinSet &vs) {
    T *win = slot(m), *rb = rslot(m);
#pragma unroll
    for (int q = 0; q < NF; ++q) {
      const int i = 2 * t + q * 2 * BS;
      P rk = vr[q], pk = vr[q];
      if (!first) {
        const T as0 = alpha * vs[q].x, as1 = alpha * vs[q].y;
        rk.x = vr[q].x - as0;
        rk.y = vr[q].y - as1;
        pk = p_next<T>(rk, vp[q], beta);
      }
      if (i + 1 < wn) lds_st2(win, i, pk.x, pk.y);  // wn even (march plan)
      else if (i < wn) win[i] = pk.x;
      const int o = i - a.hl;  // hl even: a pair is in the own rows or not
      if (o >= 0 && o < SR) lds_st2(rb, o, rk.x, rk.y);
    }
  };
  auto store_win = [&](int m) { store_win_from(m, wr, wp, wsv); };
  typedef typename CodeRaw<CB>::type CR;
  constexpr int KV = DV ? kDiaVMax : 1, KL = DV ? kDiaVMax : kDiaMax;
  // DIA-V: the values load a step ahead into a second register set (181
  // VGPRs, 2 waves per SIMD); loaded at the step instead (one set), C3 ran
  // 243 against 235 us per iteration (profiles/r05_ab_dia_v.log)
  typedef P VS[KV];
  auto codes_at = [&](int m, CR &cw, VS &vs) {
    const int r = base_of(m) + 2 * t, rr = r < padn ? r : base_of(m);
    cw = ld_code_raw<CB>(a.dcode, rr);
    if constexpr (DV) {
#pragma unroll
      for (int kk = 0; kk < KV; ++kk)
        vs[kk] = kk < a.ndiag ? ld_pair(a.dval + (size_t)kk * a.dvs, rr) : P{T(0), T(0)};
    }
  };
  const T tv = t < a.ndiag * 16 ? a.vtab[t] : T(0);
  CR cw, cwn{};
  VS vc, vn;
  const bool has_steps = m0 < m1;
  // a near-only plan (DevMatrix::mfar 0: every diagonal within the halo):
  // no step reads its neighbours' windows, so the segment skips window
  // m0 - 1 and never prefetches window m1 past its end
  const bool nearonly = (a.near & ((1u << a.ndiag) - 1u)) == ((1u << a.ndiag) - 1u);
  // FOLD: the segment's prologue loads windows m0 - 1, m0 and m0 + 1 at
  // once, before the scalar step (one memory round trip under it, not three
  // after it: each store waits only for its own set, vector loads retiring
  // in order; m0 + 1 goes into the loop's set; four-slice steps: m0 + 1
  // after it, P3LATE).  Without FOLD the windows
  // load one after the other, after the scalars (the ranks: the three at
  // once, with no scalar step to hide, measured 2-4 us longer per launch on
  // C4's 8 M-row slab, profiles/r06_ab_sr1.log).
  WinSet r1, p1, s1, r2, p2, s2;
  // the four-slice step loads window m0 + 1 after the scalar step instead:
  // the three sets at once left its 1,024-thread kernel 4 VGPRs of spill
  // (C3 124.2-125.6 -> 121.4-122.8 us per iteration, C4 even; box 8,
  // profiles/r06_ab_p3late.log)
  constexpr bool P3LATE = SB == 4;
  if constexpr (FOLD) {
    if (has_steps) {
      codes_at(m0, cw, vc);
      if (!nearonly) load_win_to(m0 - 1, r1, p1, s1, true);
      load_win_to(m0, r2, p2, s2, true);
      if (!P3LATE) load_win_to(m0 + 1, wr, wp, wsv, true);
    }
    // the scalar step of the last launch (FIN_SR1's), run here on its (p.s,
    // s.s) pairs and r.r partials (wave 0: lane l sums entries l, l + 64,
    // ... in order, then the wave tree; every workgroup the same sums),
    // fin_sr1 on a private copy of *f.st; workgroup 0 hands the state (with
    // this launch's alpha_q / alpha_def) over to the next launch in
    // *f.st_out with the history entry
    __shared__ double fbc[4];
    if (wid == 0) {
      const bool fold = f.st->sr_pend != 0;
      double ps = 0.0, ss = 0.0, rr = 0.0;
      if (fold) {
        constexpr int U = 4;
        const double2 *q2 = reinterpret_cast<const double2 *>(f.pq_in);
        for (int i = lane; i < f.np_in; i += kWave * U) {
          double2 v[U];
          double w[U];
#pragma unroll
          for (int j = 0; j < U; ++j) {
            const int ii = i + j * kWave;
            v[j] = ii < f.np_in ? q2[ii] : make_double2(0.0, 0.0);
            w[j] = ii < f.np_in ? f.pc_in[ii] : 0.0;
          }
#pragma unroll
          for (int j = 0; j < U; ++j) {
            ps = ps + v[j].x;
            ss = ss + v[j].y;
            rr = rr + w[j];
          }
        }
        ps = wave_sum(ps);
        ss = wave_sum(ss);
        rr = wave_sum(rr);
      }
      if (lane == 0) {
        CgState c = *f.st;
        if (fold) fin_sr1(ps, ss, rr, &c, blockIdx.x == 0 ? f.hist : nullptr);
        if (blockIdx.x == 0) {
          CgState o = c;
          const int kk = c.k_u;
          const bool od = d4 ? (kk & 3) == 3 : (kk & 1) != 0;
          if (kk >= 0 && !od && c.done == 0) {
            if (d4) o.alpha_q[kk & 3] = c.alpha;
            else o.alpha_def = c.alpha;
          }
          o.sr_pend = 1;
          *f.st_out = o;
        }
        fbc[0] = c.alpha;
        fbc[1] = c.beta;
        fbc[2] = (double)c.k_u;
        fbc[3] = (double)c.done;
      }
    }
    __syncthreads();
    sn = Sr1Now{(int)fbc[2], (int)fbc[3], fbc[0], fbc[1]};
    if (sn.done > 1) return;  // uniform
  }
  k = sn.k_u;
  first = k < 0;
  stop = sn.done == 1;
  odd = d4 ? (k & 3) == 3 : (k & 1) != 0;  // this launch updates x
  xup = !first && odd;
  alpha = (T)sn.alpha;
  beta = (T)sn.beta;
  alpha_d = (T)f.st->alpha_def;
  if (!FOLD && !first && !odd && !stop && blockIdx.x == 0 && t == 0) {
    if (d4) const_cast<CgState *>(f.st)->alpha_q[k & 3] = sn.alpha;
    else const_cast<CgState *>(f.st)->alpha_def = sn.alpha;
  }
  if (d4) {
    aq0 = (T)f.st->alpha_q[0];
    aq1 = (T)f.st->alpha_q[1];
    aq2 = (T)f.st->alpha_q[2];
  }
  if (stop) {
    // fin_sr1 stopped at iteration k (k_u) with x updates pending.  Depth 2
    // (k even): alpha_k p_k, p_k in the p_new buffer of this launch.  Depth
    // 4 (k % 4 = q < 3): alpha_i p_i for i = k - q .. k in order, p_{k-2} /
    // p_{k-1} / p_k in this launch's pnew / pa / pb, alpha_i in alpha_q
    const int q = k & 3;
    const T b0 = d4 ? (T)f.st->alpha_q[(k - 2) & 3] : T(0),
            b1 = d4 ? (T)f.st->alpha_q[(k - 1) & 3] : T(0),
            b2 = d4 ? (T)f.st->alpha_q[k & 3] : alpha_d;
    for (int m = m0; m < m1; ++m) {
      const int r = base_of(m) + 2 * t, rend = min(a.n, base_of(m) + wc), rs = r < a.n ? r : 0;
      P xo = ld_pair(f.x, rs);
      if (d4 && q >= 2) {
        const P v = ld_pair((const T *)f.pnew, rs);
        const T e0 = b0 * v.x, e1 = b0 * v.y;
        xo.x = xo.x + e0;
        xo.y = xo.y + e1;
      }
      if (d4 && q >= 1) {
        const P v = ld_pair(f.pa, rs);
        const T e0 = b1 * v.x, e1 = b1 * v.y;
        xo.x = xo.x + e0;
        xo.y = xo.y + e1;
      }
      const P v = ld_pair(d4 ? f.pb : (const T *)f.pnew, rs);
      const T e0 = b2 * v.x, e1 = b2 * v.y;
      if (r < rend) st_pair(f.x, r, rend, xo.x + e0, xo.y + e1, false);
    }
    return;
  }
  if (!has_steps) {  // no steps: zero sums (the next scalar step adds every workgroup's)
    publish();
    return;
  }
  if constexpr (!FOLD) codes_at(m0, cw, vc);
  if (xup) load_x(m0, xc);
  if constexpr (FOLD) {
    if (!nearonly) store_win_from(m0 - 1, r1, p1, s1);
    store_win_from(m0, r2, p2, s2);
    if (P3LATE) load_win(m0 + 1);
  } else {
    if (!nearonly) {
      load_win(m0 - 1);
      store_win(m0 - 1);
    }
    load_win(m0);
    store_win(m0);
    load_win(m0 + 1);
  }
  if (t < a.ndiag * 16) lv[t] = tv;
  const int mlast = nearonly ? max(m0, m1 - 1) : m1;  // the last window any step reads
  auto step = [&](int m, const CR &ccw, const VS &cvs, XOps &cx, CR &ncw, VS &nvs, XOps &nx) {
    store_win(m + 1);
    // depth 4's two more p operands of step m's rows: issued before this
    // step's other loads, used after its compute (no wait on the prefetch)
    P qa{}, qb{};
    if (d4 && xup) {
      const int r = base_of(m) + 2 * t, rs = r < a.n ? r : 0;
      qa = ld_pair(f.pa, rs);
      qb = ld_pair(f.pb, rs);
    }
    codes_at(min(m + 1, m1 - 1), ncw, nvs);
    load_win(min(m + 2, mlast));  // in flight during step m
    if (xup && m + 1 < m1) load_x(m + 1, nx);
    __syncthreads();
    const int base = base_of(m), r = base + 2 * t;
    const int rend = min(a.n, base + wc);
    const T *cur = slot(m), *prv = slot(m - 1), *nxt = slot(m + 1);
    const T *rb = rslot(m);
    const int rw = 2 * t + a.hl;
    unsigned cc0, cc1;
    code_split<CB>(ccw, cc0, cc1);
    T a0 = T(0), a1 = T(0);
#pragma unroll
    for (int kk = 0; kk < KL; ++kk) {
      if (kk < a.ndiag) {
        const int d = a.doff[kk];
        const T *src = (a.near >> kk) & 1u ? cur : d < 0 ? prv : nxt;
        const int i = (a.near >> kk) & 1u ? rw + d : d < 0 ? rw + d + QR : rw + d - QR;
        T v0, v1;
        if ((d & 1) == 0) lds_ld2(src, i, v0, v1);  // rw, QR even: an aligned pair
        else {
          v0 = src[i];
          v1 = src[i + 1];
        }
        const unsigned n0 = fld(a, cc0, kk), n1 = fld(a, cc1, kk);
        const T w0 = DV ? cvs[DV ? kk : 0].x : lv[kk * 16 + n0];
        const T w1 = DV ? cvs[DV ? kk : 0].y : lv[kk * 16 + n1];
        const T p0 = w0 * v0, p1 = w1 * v1;
        a0 = n0 != a.cmask[kk] ? a0 + p0 : a0;
        a1 = n1 != a.cmask[kk] ? a1 + p1 : a1;
      }
    }
    T pn0, pn1, rk0, rk1;
    lds_ld2(cur, rw, pn0, pn1);
    lds_ld2(rb, 2 * t, rk0, rk1);
    if (r < rend) {
      st_pair(a.y, r, rend, a0, a1, nt);
      st_pair(f.pnew, r, rend, pn0, pn1, false);
      st_pair(f.rnew, r, rend, rk0, rk1, false);
      if (xup) x_update(cx, qa, qb, r, rend);
      const bool own = r >= f.elo && r < f.ehi;  // edge pairs: k_sr1_edge's (p.s, s.s)
      if (own) {
        sps = sps + (double)pn0 * (double)a0;
        sss = sss + (double)a0 * (double)a0;
      }
      srr = srr + (double)rk0 * (double)rk0;
      if (r + 1 < rend) {
        if (own) {
          sps = sps + (double)pn1 * (double)a1;
          sss = sss + (double)a1 * (double)a1;
        }
        srr = srr + (double)rk1 * (double)rk1;
      }
    }
    __syncthreads();  // every read of window m - 1's slot (and r slot m) is done before step m + 1 refills it
  };
  for (int m = m0; m < m1; m += 2) {
    step(m, cw, vc, xc, cwn, vn, xn);
    if (m + 1 < m1) step(m + 1, cwn, vn, xn, cw, vc, xc);
  }
  publish();
}

// The edge rows of a partitioned rank's one-launch SR step, after the halo:
// rows [0, elo) and [ehi, n) (row pairs; Sr1Args), whose rows reach a ghost
// column.  s = A p_k with p_k from the p_new buffer -- the own rows as
// k_sr1_dia_m stored them, the ghost rows as the halo put them -- in the
// row's diagonal order with k_sr1_dia_m's roundings (so s is what one launch
// with every p_k in place computes), then the (p.s, s.s) pair per workgroup
// (r.r: k_sr1_dia_m has all own rows; 0 here).
template <typename T>
__global__ __launch_bounds__(256) void k_sr1_edge(SpmvArgs<T> a, Sr1Args<T> f) {
  __shared__ T lv[kDiaMax * 16];
  __shared__ double red[2][4];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  // pair i of the edge rows: na below, nb above (no ehi arithmetic unless
  // there are rows above: ehi is INT_MAX then)
  const int na = f.elo / 2, nb = f.ehi < a.n ? (a.n - f.ehi + 1) / 2 : 0;
  const int i = blockIdx.x * 256 + t;
  const bool live = i < na + nb;
  const int r = i < na ? 2 * i : live ? f.ehi + 2 * (i - na) : 0;
  if (t < a.ndiag * 16) lv[t] = a.vtab[t];
  const T *p = f.pnew;
  const int rl = live ? r : 0;
  const bool two = live && r + 1 < a.n;
  unsigned c0, c1;
  ld_codes(a.dcode, a.cb, rl, c0, c1);
  // every load out before the first use, unconditionally and independent of
  // the codes (clamped into the ghosted vector; a missing entry's value is
  // never used): one memory round trip, not a code load then the gathers
  T v0[kDiaMax], v1[kDiaMax];
#pragma unroll
  for (int kk = 0; kk < kDiaMax; ++kk) {
    if (kk < a.ndiag) {
      const int d = a.doff[kk];
      v0[kk] = p[min(max(rl + d, a.xlo), a.ncols - 1)];
      v1[kk] = p[min(max(rl + 1 + d, a.xlo), a.ncols - 1)];
    }
  }
  // DIA-V: the two rows' values on each diagonal (rows < the padded rows)
  T w0[kDiaVMax], w1[kDiaVMax];
  if (a.dval) {
#pragma unroll
    for (int kk = 0; kk < kDiaVMax; ++kk) {
      w0[kk] = kk < a.ndiag ? a.dval[(size_t)kk * a.dvs + rl] : T(0);
      w1[kk] = kk < a.ndiag ? a.dval[(size_t)kk * a.dvs + rl + 1] : T(0);
    }
  }
  const T p0 = p[rl], p1 = p[two ? rl + 1 : rl];
  // the state after the loads are out (its loads would otherwise go first)
  const Sr1Now sn = sr1_now(f.st, f.g);
  if (sn.done) return;  // uniform (a stop: k_sr1_dia_m's x update only)
  __syncthreads();  // lv
  T a0 = T(0), a1 = T(0);
#pragma unroll
  for (int kk = 0; kk < kDiaMax; ++kk) {
    if (kk < a.ndiag) {
      const unsigned n0 = fld(a, c0, kk), n1 = fld(a, c1, kk);
      const bool dv = a.dval && kk < kDiaVMax;
      const T e0 = dv ? w0[kk < kDiaVMax ? kk : 0] : lv[kk * 16 + n0];
      const T e1 = dv ? w1[kk < kDiaVMax ? kk : 0] : lv[kk * 16 + n1];
      const T q0 = e0 * v0[kk], q1 = e1 * v1[kk];
      a0 = n0 != a.cmask[kk] ? a0 + q0 : a0;
      a1 = n1 != a.cmask[kk] ? a1 + q1 : a1;
    }
  }
  double ps = 0.0, ss = 0.0;
  if (live) {
    a.y[r] = a0;
    ps = (double)p0 * (double)a0;
    ss = (double)a0 * (double)a0;
    if (two) {
      a.y[r + 1] = a1;
      ps = ps + (double)p1 * (double)a1;
      ss = ss + (double)a1 * (double)a1;
    }
  }
  ps = wave_sum(ps);
  ss = wave_sum(ss);
  if (lane == 0) {
    red[0][wid] = ps;
    red[1][wid] = ss;
  }
  __syncthreads();
  if (t == 0) {
    const double p0 = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const double p1 = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    reinterpret_cast<double2 *>(f.pq)[blockIdx.x] = make_double2(p0, p1);
    f.pc[blockIdx.x] = 0.0;
  }
}

// ---------------------------------------- fused CG1 step (DIA-VI)
// The Chronopoulos-Gear iteration in ONE launch: k_cg1_update's vector
// recurrences (p = r + beta p; s = w + beta s; x += alpha p; r -= alpha s)
// and the SpMV w = A r of the new r, with both dot products of the single
// all-reduce (gamma = r.r, delta = w.r) as per-workgroup partials.  alpha,
// beta and the stop flag come from CgState (k_finalize FIN_CG1 of the last
// launch's sums, all-reduced across ranks when partitioned).  r, s and w are
// double-buffered (this launch reads r_o, s_o, w_o -- also at its halo
// rows -- and writes r_n, s_n, w_n); p and x are read and written at the own
// rows only.  r_new of the slice and its halo rows is computed ONCE per
// workgroup into an LDS window (NF pair passes per thread): the near
// diagonals read it there, the far ones compute r_new of their column from
// r, w, s gathers (NFAR slots).  GH (a partition's boundary items): a
// column >= n is a ghost whose r_new the halo exchange put in r_n's ghost
// tail.  Every element is computed with k_cg1_update's roundings and summed
// in the row's diagonal (= column) order, so x matches the unfused CG1 to
// the grouping of the two dot products.  Bytes per row: 1-4 code + 24 (r,
// s, w) + 16 (p, x) read, 40 written (p, s, r, w, x).
template <typename T, int NF, int NFAR, bool NT, bool LIST, bool GH>
__global__ __launch_bounds__(256) void k_cg1_dia_h(SpmvArgs<T> a, Cg1Args<T> f) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  T *win = reinterpret_cast<T *>(dyn_lds);
  __shared__ T lv[kDiaMax * 16];
  __shared__ double red[8];
  typedef typename Pair<T>::type P;
  const int t = threadIdx.x;
  const int wi = xcd_block();
  const int sl = LIST ? a.items.list[wi] : a.items.first + wi;
  if (f.st->done) return;  // uniform (FIN_CG1 set it after the last x update)
  const T alpha = (T)f.st->alpha, beta = (T)f.st->beta;
  const int s0 = sl * kDiaSliceRows, r = s0 + 2 * t;
  const int rs = r < a.n ? r : 0;
  unsigned c0, c1;
  ld_codes(a.dcode, a.cb, r, c0, c1);
  const T tv = t < a.ndiag * 16 ? a.vtab[t] : T(0);
  constexpr int NS = NFAR > 0 ? NFAR : 1;
  P fr[NS], fw[NS], fs[NS], fg[NS];
  int fb[NS];
#pragma unroll
  for (int q = 0; q < NFAR; ++q) {
    const int kq = a.fark[q];
    int b = rs;
    if (kq >= 0) {
      const unsigned n0 = fld(a, c0, kq), n1 = fld(a, c1, kq);
      if (n0 != a.cmask[kq] || n1 != a.cmask[kq]) b = r + a.doff[kq];
    }
    fb[q] = b;
    fr[q] = ld_pair(f.r_o, b);
    fw[q] = ld_pair(f.w_o, b);
    fs[q] = ld_pair(f.s_o, b);
    if (GH) fg[q] = ld_pair((const T *)f.r_n, b);
  }
  const int w0 = s0 - a.hl, wn = kDiaSliceRows + a.hl + a.hr;
  P wr[NF], ww[NF], ws[NF], wg[NF];
  int wj[NF];
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    const int j = min(max(w0 + 2 * t + q * 2 * 256, -1), a.ncols - 1);
    wj[q] = j;
    wr[q] = ld_pair(f.r_o, j);
    ww[q] = ld_pair(f.w_o, j);
    ws[q] = ld_pair(f.s_o, j);
    if (GH) wg[q] = ld_pair((const T *)f.r_n, j);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load above is in flight before the first use
  // r_new of a pair: r - alpha (w + beta s), k_cg1_update's roundings; or the
  // received ghost value
  auto rnext = [&](P rv, P wv, P sv, P gv, int j) {
    P o;
    const T b0 = beta * sv.x, b1 = beta * sv.y;
    const T s0v = wv.x + b0, s1v = wv.y + b1;
    const T a0 = alpha * s0v, a1 = alpha * s1v;
    o.x = rv.x - a0;
    o.y = rv.y - a1;
    if (GH) {
      if (j >= a.n) o.x = gv.x;
      if (j + 1 >= a.n) o.y = gv.y;
    }
    return o;
  };
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    const int i = 2 * t + q * 2 * 256;
    const P rn = rnext(wr[q], ww[q], ws[q], wg[q], wj[q]);
    if (i < wn) win[i] = rn.x;
    if (i + 1 < wn) win[i + 1] = rn.y;
  }
  P rk[NS];
#pragma unroll
  for (int q = 0; q < NFAR; ++q) rk[q] = rnext(fr[q], fw[q], fs[q], fg[q], fb[q]);
  if (t < a.ndiag * 16) lv[t] = tv;
  __syncthreads();
  // own rows' operands (after the window's load registers are dead)
  P ro = P(), so = P(), wo = P(), po = P(), xo = P();
  if (r < a.n) {
    ro = ld_pair(f.r_o, r);
    so = ld_pair(f.s_o, r);
    wo = ld_pair(f.w_o, r);
    po = ld_pair((const T *)f.p, r);
    xo = ld_pair((const T *)f.x, r);
  }
  const int rw = r - w0;
  T a0 = T(0), a1 = T(0);
#pragma unroll
  for (int kk = 0; kk < kDiaMax; ++kk) {
    if (kk < a.ndiag) {
      T v0, v1;
      if ((a.near >> kk) & 1u) {
        const int i = rw + a.doff[kk];
        v0 = win[i];
        v1 = win[i + 1];
      } else {
        const int slot = __builtin_popcount(~a.near & ((1u << kk) - 1u));
        P v = rk[0];
#pragma unroll
        for (int q = 1; q < NFAR; ++q) v = slot == q ? rk[q] : v;
        v0 = v.x;
        v1 = v.y;
      }
      const unsigned n0 = fld(a, c0, kk), n1 = fld(a, c1, kk);
      const T p0 = lv[kk * 16 + n0] * v0, p1 = lv[kk * 16 + n1] * v1;
      a0 = n0 != a.cmask[kk] ? a0 + p0 : a0;
      a1 = n1 != a.cmask[kk] ? a1 + p1 : a1;
    }
  }
  double gam = 0.0, del = 0.0;
  if (r < a.n) {
    const T rn0 = win[rw], rn1 = win[rw + 1];
    // k_cg1_update's order: p, s, x, r (r_new == the window's value)
    const T bp0 = beta * po.x, bp1 = beta * po.y;
    const T pn0 = ro.x + bp0, pn1 = ro.y + bp1;
    const T bs0 = beta * so.x, bs1 = beta * so.y;
    const T sn0 = wo.x + bs0, sn1 = wo.y + bs1;
    const T ap0 = alpha * pn0, ap1 = alpha * pn1;
    st_pair(f.p, r, a.n, pn0, pn1, false);
    st_pair(f.s_n, r, a.n, sn0, sn1, false);
    st_pair(f.x, r, a.n, xo.x + ap0, xo.y + ap1, false);
    st_pair(f.r_n, r, a.n, rn0, rn1, false);
    st_pair(a.y, r, a.n, a0, a1, NT);
    gam = (double)rn0 * (double)rn0;
    del = (double)rn0 * (double)a0;
    if (r + 1 < a.n) {
      gam = gam + (double)rn1 * (double)rn1;
      del = del + (double)rn1 * (double)a1;
    }
  }
  // the two partials, each reduced like epi_store<4>
  gam = wave_sum(gam);
  del = wave_sum(del);
  const int lane = t & (kWave - 1), wid = t / kWave;
  if (lane == 0) {
    red[wid] = gam;
    red[4 + wid] = del;
  }
  __syncthreads();
  if (t == 0) {
    double g = red[0], d = red[4];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      g = g + red[q];
      d = d + red[4 + q];
    }
    f.pg[blockIdx.x] = g;
    a.part[blockIdx.x] = d;
  }
}

// The send rows of r_new for the fused partitioned CG1 step: r_new = r -
// alpha (w + beta s) at the rows the neighbours gather (the same roundings
// as k_cg1_dia_h's window).
template <typename T>
__global__ __launch_bounds__(256) void k_pack_rnext(int n_send, const int *__restrict__ idx,
                                                    const T *__restrict__ r,
                                                    const T *__restrict__ w,
                                                    const T *__restrict__ s,
                                                    T *__restrict__ out, const CgState *st) {
  if (st->done) return;
  const T alpha = (T)st->alpha, beta = (T)st->beta;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n_send; i += gridDim.x * 256) {
    const int j = idx[i];
    const T bs = beta * s[j];
    const T sn = w[j] + bs;
    const T as = alpha * sn;
    out[i] = r[j] - as;
  }
}

// The send rows of p_new for the fused partitioned step: p_new = r + beta
// p_old at the rows the neighbours gather (the unfused path packs p after
// k_xpay_xf; the fused step computes p inside the SpMV launch, after the
// halo is needed).  Same roundings as p_next.
template <typename T>
__global__ __launch_bounds__(256) void k_pack_pnext(int n_send, const int *__restrict__ idx,
                                                    const T *__restrict__ r,
                                                    const T *__restrict__ pold,
                                                    T *__restrict__ out, const CgState *st,
                                                    const double *rr_new) {
  const int k = st->k_u;
  const bool first = k < 0;
  const T beta = first ? T(0) : (T)(*rr_new / st->rr_u);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n_send; i += gridDim.x * 256) {
    const int j = idx[i];
    if (first) {
      out[i] = r[j];
    } else {
      const T b = beta * pold[j];
      out[i] = r[j] + b;
    }
  }
}

// The send rows of p_k for the one-launch SR step on partitioned ranks
// (k_sr1_dia_m): r_k = r - alpha s, p_k = r_k + beta p of the last
// iteration's buffers at the rows the neighbours need, the roundings of the
// kernel's window rows; r (= b = p_0) on the first iteration.  alpha, beta
// from k_finalize(FIN_SR1) of the all-reduced sums.
template <typename T>
__global__ __launch_bounds__(256) void k_pack_sr(int n_send, const int *__restrict__ idx,
                                                 const T *__restrict__ rold,
                                                 const T *__restrict__ pold,
                                                 const T *__restrict__ sold, T *__restrict__ out,
                                                 const CgState *st, const double *g) {
  const Sr1Now sn = sr1_now(st, g);
  if (sn.done > 1) return;
  const bool first = sn.k_u < 0;
  const T alpha = (T)sn.alpha, beta = (T)sn.beta;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n_send; i += gridDim.x * 256) {
    const int j = idx[i];
    if (first) {
      out[i] = rold[j];
    } else {
      const T as = alpha * sold[j];
      const T rk = rold[j] - as;
      const T bp = beta * pold[j];
      out[i] = rk + bp;
    }
  }
}

// -------------------------------------------------------------- k_stencil
// Matrix-free SpMV of the same Laplacian: row r sums its products in the CSR
// row's column order from 0 with the same values, so y is bit-identical to
// the CSR SpMV.  Only x (once) and y move: the upper bound SURVEY.md 8f asks
// for beside the stored-matrix runs.  Two rows per thread (r even), as in
// k_spmv_dia: x[r +- nx], x[r +- nx*ny] and x[r], x[r+1] are pair loads,
// x[r-1] / x[r+2] the neighbouring lanes' centre pair (one extra load at the
// wave edges); grid coordinates from exact reciprocal divisions.
__device__ __forceinline__ int fdiv(int a, int d, double inv) {
  int q = (int)((double)a * inv);  // exact floor(a / d) for 0 <= a < 2^31
  q -= q * d > a;
  q += (q + 1) * d <= a;
  return q;
}

struct LapFlags {
  bool ml, mj, mi, pi, pj, pL;  // neighbour present: -pl, -nx, -1, +1, +nx, +pl
};

__device__ __forceinline__ LapFlags lap_flags(int r, const LapSpec &g, double inv_pl,
                                              double inv_nx) {
  const int pl = g.nx * g.ny;
  const int l = g.dim == 3 ? fdiv(r, pl, inv_pl) : 0;
  const int rem = r - l * pl;
  const int j = fdiv(rem, g.nx, inv_nx);
  const int i = rem - j * g.nx;
  return LapFlags{g.dim == 3 && l > 0, j > 0,           i > 0,
                  i < g.nx - 1,        j < g.ny - 1,    g.dim == 3 && l < g.nz - 1};
}

template <typename T, bool EPI, bool NT>
__global__ __launch_bounds__(256) void k_stencil(SpmvArgs<T> a) {
  typedef typename Pair<T>::type P;
  const LapSpec g = a.lap;
  const int nx = g.nx, pl = g.nx * g.ny, n = a.n;
  const int stop = a.done ? *a.done : 0;
  if (stop) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int r = (xcd_block() * 256 + threadIdx.x) * 2;
  const int rr = r < n ? r : 0;
  const double inv_pl = a.inv_pl, inv_nx = a.inv_nx;
  const LapFlags f0 = lap_flags(rr, g, inv_pl, inv_nx);
  const bool v1 = rr + 1 < n;
  const LapFlags f1 = lap_flags(v1 ? rr + 1 : rr, g, inv_pl, inv_nx);
  const T *x = a.x;
  // every load goes out before the first use, unconditionally (a missing
  // neighbour pair reloads x[r]: a conditional load makes the compiler wait)
  const T eL = x[lane == 0 && f0.mi ? rr - 1 : rr];
  const T eR = x[lane == kWave - 1 && v1 && f1.pi ? rr + 2 : rr];
  const P zm = ld_pair(x, f0.ml || (v1 && f1.ml) ? rr - pl : rr);
  const P ym = ld_pair(x, f0.mj || (v1 && f1.mj) ? rr - nx : rr);
  const P c = ld_pair(x, rr);
  const P yp = ld_pair(x, f0.pj || (v1 && f1.pj) ? rr + nx : rr);
  const P zp = ld_pair(x, f0.pL || (v1 && f1.pL) ? rr + pl : rr);
  __builtin_amdgcn_sched_barrier(0);  // no use of a load is scheduled above the last load
  T left = __shfl_up(c.y, 1, kWave), right = __shfl_down(c.x, 1, kWave);
  if (lane == 0) left = eL;
  if (lane == kWave - 1) right = eR;
  const T m1 = T(-1), dg = T(g.dim == 3 ? 6 : 4);
  T a0 = T(0), a1 = T(0);
  a0 = f0.ml ? a0 + m1 * zm.x : a0;
  a0 = f0.mj ? a0 + m1 * ym.x : a0;
  a0 = f0.mi ? a0 + m1 * left : a0;
  a0 = a0 + dg * c.x;
  a0 = f0.pi ? a0 + m1 * c.y : a0;
  a0 = f0.pj ? a0 + m1 * yp.x : a0;
  a0 = f0.pL ? a0 + m1 * zp.x : a0;
  a1 = f1.ml ? a1 + m1 * zm.y : a1;
  a1 = f1.mj ? a1 + m1 * ym.y : a1;
  a1 = f1.mi ? a1 + m1 * c.x : a1;
  a1 = a1 + dg * c.y;
  a1 = f1.pi ? a1 + m1 * right : a1;
  a1 = f1.pj ? a1 + m1 * yp.y : a1;
  a1 = f1.pL ? a1 + m1 * zp.y : a1;
  double dot = 0.0, dot2 = 0.0;
  if (r < n) {
    st_pair(a.y, r, n, a0, a1, NT);
    if (EPI) {
      dot = (double)c.x * (double)a0;
      dot2 = (double)a0 * (double)a0;
      if (v1) {
        dot = dot + (double)c.y * (double)a1;
        dot2 = dot2 + (double)a1 * (double)a1;
      }
    }
  }
  if (EPI) epi_store_p<4>(dot, dot2, a.part, a.pair);
}

// ------------------------------------------------------- vector kernels
// All grid-stride over 16-byte vectors; the scalar tail (n % W) is handled
// by global thread 0.  Reductions: per-thread fixed-order sums, then
// block_sum -> part[blockIdx.x]; consumers add the partials in index order.

// x = 0, r = b, p = b; part = b.b partials (HS prologue, cg.c:104-108).
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_init_hs(int n, const T *__restrict__ b, T *__restrict__ x,
                                                T *__restrict__ r, T *__restrict__ p,
                                                double *__restrict__ part) {
  __shared__ double red[BS / kWave];
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    const V bv = reinterpret_cast<const V *>(b)[i];
    reinterpret_cast<V *>(x)[i] = V(T(0));
    reinterpret_cast<V *>(r)[i] = bv;
    reinterpret_cast<V *>(p)[i] = bv;
#pragma unroll
    for (int j = 0; j < W; ++j) acc = acc + (double)bv[j] * (double)bv[j];
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T bv = b[i];
      x[i] = T(0);
      r[i] = bv;
      p[i] = bv;
      acc = acc + (double)bv * (double)bv;
    }
  const double s = block_sum<BS>(acc, red);
  if (threadIdx.x == 0 && part) part[blockIdx.x] = s;
}

// x = 0, r = b, p = s = 0; part = b.b partials (CG1 prologue)
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_init_cg1(int n, const T *__restrict__ b,
                                                 T *__restrict__ x, T *__restrict__ r,
                                                 T *__restrict__ p, T *__restrict__ s,
                                                 double *__restrict__ part) {
  __shared__ double red[BS / kWave];
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    const V bv = reinterpret_cast<const V *>(b)[i];
    reinterpret_cast<V *>(x)[i] = V(T(0));
    reinterpret_cast<V *>(p)[i] = V(T(0));
    reinterpret_cast<V *>(s)[i] = V(T(0));
    reinterpret_cast<V *>(r)[i] = bv;
#pragma unroll
    for (int j = 0; j < W; ++j) acc = acc + (double)bv[j] * (double)bv[j];
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T bv = b[i];
      x[i] = T(0);
      p[i] = T(0);
      s[i] = T(0);
      r[i] = bv;
      acc = acc + (double)bv * (double)bv;
    }
  const double sum = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// x += alpha*p (cg.c:115-118); r -= alpha*s (cg.c:122-123); part = r.r
// (exact mode: the reference's order of updates, finalize launches between)
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_update_xr(int n, T *__restrict__ x,
                                                  const T *__restrict__ p, T *__restrict__ r,
                                                  const T *__restrict__ s,
                                                  const CgState *__restrict__ st,
                                                  double *__restrict__ part) {
  __shared__ double red[BS / kWave];
  if (st->done) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const T alpha = (T)st->alpha;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    V xv = reinterpret_cast<const V *>(x)[i];
    const V pv = reinterpret_cast<const V *>(p)[i];
    V rv = reinterpret_cast<const V *>(r)[i];
    const V sv = reinterpret_cast<const V *>(s)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T ap = alpha * pv[j];
      xv[j] = xv[j] + ap;
      const T as = alpha * sv[j];
      rv[j] = rv[j] - as;
      acc = acc + (double)rv[j] * (double)rv[j];
    }
    reinterpret_cast<V *>(x)[i] = xv;
    reinterpret_cast<V *>(r)[i] = rv;
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T ap = alpha * p[i];
      x[i] = x[i] + ap;
      const T as = alpha * s[i];
      const T ri = r[i] - as;
      r[i] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  if (part) {
    const double sum = block_sum<BS>(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = sum;
  }
}

// p = r + beta*p (cg.c:131-132)
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_xpay(int n, T *__restrict__ p, const T *__restrict__ r,
                                             const CgState *__restrict__ st) {
  if (st->done) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const T beta = (T)st->beta;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  for (int i = gid; i < nv; i += stride) {
    V pv = reinterpret_cast<const V *>(p)[i];
    const V rv = reinterpret_cast<const V *>(r)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T bp = beta * pv[j];
      pv[j] = rv[j] + bp;
    }
    reinterpret_cast<V *>(p)[i] = pv;
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T bp = beta * p[i];
      p[i] = r[i] + bp;
    }
}

// Folded HS (the default fast path): no finalize kernels.  Every workgroup
// of the vector kernels sums the previous kernel's partials itself -- the
// same sum_parts<1024> order as k_finalize<1024>, so alpha, beta and the
// stop test are bit-identical to the finalize path -- and workgroup 0
// publishes the state for later kernels.  A kernel never writes a field its
// own workgroups read: k_update_rf reads rr_x / k_x and writes rr_u / k_u /
// alpha; k_xpay_xf reads rr_u / k_u / alpha and writes rr_x / k_x / rr / k /
// beta / done.  Deferred x: the x update (cg.c:115-116) runs in the p-update,
// which reads p anyway (one 8n-byte read less per iteration, same roundings).
// The stop flag: k_xpay_xf sets 1 after the stop iteration's x update, the
// next k_update_rf turns it into 2; only 2 stops k_xpay_xf (a 1 seen there
// was written by its own workgroup 0 during this launch).
// The first grid-stride element's loads are issued before the partial sum,
// so the HBM round trip overlaps the L2 round trip of the partials (same
// elements, same order: bit-identical).
template <typename T, bool NT>
__global__ __launch_bounds__(kFoldBS) void k_update_rf(int n, T *__restrict__ r,
                                                       const T *__restrict__ s,
                                                       CgState *__restrict__ st,
                                                       const double *__restrict__ ps_part,
                                                       int nps, double *__restrict__ rr_part,
                                                       FinArgs fin, const double *sr,
                                                       double *hist) {
  __shared__ double red[kFoldBS / kWave];
  __shared__ double bcast;
  const int done = st->done;
  if (done) {
    if (done == 1 && blockIdx.x == 0 && threadIdx.x == 0) st->done = 2;
    return;
  }
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * kFoldBS + threadIdx.x, stride = gridDim.x * kFoldBS;
  V rv0 = V(), sv0 = V();
  if (gid < nv) {
    rv0 = reinterpret_cast<const V *>(r)[gid];
    sv0 = reinterpret_cast<const V *>(s)[gid];
  }
  // CGX_ALG_SR: p.s, s.s and the exact r.r of the current r come reduced
  // together (one all-reduce); r_new.r_new = alpha^2 s.s - r.r (r.s = p.s)
  // for the next beta.  First the stop test of the PREVIOUS iteration
  // (cg.c:125's position) on that exact r.r (oracle_solve_sr): uniform over
  // the grid (every workgroup reads the same values); r stays as it is.  An
  // odd stop iteration's x is complete (done = 2), an even one's deferred x
  // update is applied by the next fused launch (done = 1; fuse_step).
  if (sr) {
    const int kp = st->k_x - 1;
    const bool stop = kp >= 0 && (kp >= st->max_iter || (st->use_tol && sr[2] <= st->tol2bb));
    if (kp >= 0 && blockIdx.x == 0 && threadIdx.x == 0) {
      if (kp < st->hist_cap) hist[kp] = sr[2];
      st->rr = sr[2];
      if (stop) {
        st->k = kp;
        st->done = (kp & 1) ? 2 : 1;
      }
    }
    if (stop) return;
  }
  const double ps = sr ? sr[0] : sum_parts<kFoldBS>(ps_part, nps, red);
  if (threadIdx.x == 0) {
    const double rr = sr ? sr[2] : st->rr_x;
    const double alpha = rr / ps;  // cg.c:113
    bcast = alpha;
    if (blockIdx.x == 0) {
      st->ps = ps;
      st->alpha = alpha;
      st->rr_u = rr;
      st->k_u = st->k_x;
      if (!(ps > 0.0) && st->brk == 0) st->brk = st->k_x + 1;  // p.s <= 0: NaN follows
      if (sr) {
        const double as = alpha * sr[1];
        const double e = alpha * as - rr;
        st->rr_new = e > 0.0 ? e : 0.0;  // cancellation below 0: converged (beta 0)
      }
    }
  }
  __syncthreads();
  const T alpha = (T)bcast;
  double acc = 0.0;
  auto step = [&](int i, V rv, const V sv) {
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T as = alpha * sv[j];
      rv[j] = rv[j] - as;
      acc = acc + (double)rv[j] * (double)rv[j];
    }
    if constexpr (NT) __builtin_nontemporal_store(rv, reinterpret_cast<V *>(r) + i);
    else reinterpret_cast<V *>(r)[i] = rv;
  };
  int i = gid;
  if (i < nv) {
    step(i, rv0, sv0);
    i += stride;
  }
  for (; i < nv; i += stride)
    step(i, reinterpret_cast<const V *>(r)[i], reinterpret_cast<const V *>(s)[i]);
  if (gid == 0)
    for (int k = nv * W; k < n; ++k) {
      const T as = alpha * s[k];
      const T ri = r[k] - as;
      r[k] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  // one partial per 256-thread quarter, reduced exactly as block_sum<256>:
  // the same terms per partial and the same order as k_update_xr<T, 256>
  // (exact-mode grid), so r.r (and beta) match the finalize path bit for bit
  acc = wave_sum(acc);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x < kFoldBS / 256) {
    constexpr int WQ = 256 / kWave;
    double q = red[threadIdx.x * WQ];
#pragma unroll
    for (int w = 1; w < WQ; ++w) q = q + red[threadIdx.x * WQ + w];
    if (fin.cnt) {
      publish(rr_part + blockIdx.x * (kFoldBS / 256) + threadIdx.x, q);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      rr_part[blockIdx.x * (kFoldBS / 256) + threadIdx.x] = q;
    }
  }
  if (fin.cnt) {
    // the four quarter partials are published (and drained) by threads 0-3;
    // the barrier orders them before thread 0's ticket
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) last = take_ticket(fin.cnt, gridDim.x);
    __syncthreads();
    if (!last) return;
    __shared__ double red16[kFoldBS / kWave];
    const double sa = canon_sum<kFoldBS, true>(fin.pa, fin.na, red16);
    if (threadIdx.x == 0) fin.out[0] = sa;
  }
}

// pn != p (double-buffered p, the single-GPU solver): x is updated every
// other iteration, as in the fused step -- an even k defers x += alpha_k p_k
// (alpha to st->alpha_def), the odd k + 1 adds alpha_{k-1} p_{k-1} (read
// from pn before p_new overwrites it) and then alpha_k p_k, the same two
// roundings in order; a stop applies what is pending.  8 B per row less on
// average, and the SpMV after an even iteration finds half the dirty lines.
// pn == p: x every iteration, p in place.
template <typename T, bool NT>
__global__ __launch_bounds__(kFoldBS) void k_xpay_xf(int n, T *__restrict__ x, const T *p, T *pn,
                                                     const T *__restrict__ r,
                                                     CgState *__restrict__ st,
                                                     const double *__restrict__ rr_part, int nrr,
                                                     double *__restrict__ hist) {
  __shared__ double red[kFoldBS / kWave];
  __shared__ double bcast;
  __shared__ int bstop;
  if (st->done > 1) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * kFoldBS + threadIdx.x, stride = gridDim.x * kFoldBS;
  const int kk = st->k_u;
  const bool defer = pn != p, odd = (kk & 1) != 0;
  const bool xpre = !defer || odd;  // x (and p_{k-1}) needed unless a stop says so
  V pv0 = V(), rv0 = V(), xv0 = V(), pd0 = V();
  if (gid < nv) {
    pv0 = reinterpret_cast<const V *>(p)[gid];
    rv0 = reinterpret_cast<const V *>(r)[gid];
    if (xpre) xv0 = reinterpret_cast<const V *>(x)[gid];
    if (xpre && defer) pd0 = reinterpret_cast<const V *>(pn)[gid];
  }
  const double rr_new = sum_parts<kFoldBS>(rr_part, nrr, red);
  if (threadIdx.x == 0) {
    const int k = kk;
    const bool stop = k >= st->max_iter || (st->use_tol && rr_new <= st->tol2bb);
    const double beta = rr_new / st->rr_u;  // cg.c:129
    bcast = beta;
    bstop = stop;
    if (blockIdx.x == 0) {  // cg.c:125-129
      if (k < st->hist_cap) hist[k] = rr_new;
      if (stop) {
        st->k = k;
        st->done = 1;
      } else {
        st->beta = beta;
        st->rr = rr_new;
        st->rr_x = rr_new;
        st->k = k + 1;
        st->k_x = k + 1;
        if (defer && !odd) st->alpha_def = st->alpha;
      }
    }
  }
  __syncthreads();
  const bool stop = bstop != 0;
  const bool xup = !defer || odd || stop, two = defer && odd;
  const T alpha = (T)st->alpha, beta = (T)bcast, alpha_d = (T)st->alpha_def;
  auto step = [&](int i, V pv, const V rv, bool pre) {
    if (xup) {
      V xv = pre && xpre ? xv0 : reinterpret_cast<const V *>(x)[i];
      if (two) {
        const V pd = pre ? pd0 : reinterpret_cast<const V *>(pn)[i];
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const T ap = alpha_d * pd[j];
          xv[j] = xv[j] + ap;
        }
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T ap = alpha * pv[j];
        xv[j] = xv[j] + ap;
      }
      if constexpr (NT) __builtin_nontemporal_store(xv, reinterpret_cast<V *>(x) + i);
      else reinterpret_cast<V *>(x)[i] = xv;
    }
    if (!stop) {
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T bp = beta * pv[j];
        pv[j] = rv[j] + bp;
      }
      if constexpr (NT) __builtin_nontemporal_store(pv, reinterpret_cast<V *>(pn) + i);
      else reinterpret_cast<V *>(pn)[i] = pv;
    }
  };
  int i = gid;
  if (i < nv) {
    step(i, pv0, rv0, true);
    i += stride;
  }
  for (; i < nv; i += stride)
    step(i, reinterpret_cast<const V *>(p)[i], stop ? V() : reinterpret_cast<const V *>(r)[i],
         false);
  if (gid == 0)
    for (int k = nv * W; k < n; ++k) {
      const T pk = p[k];
      if (xup) {
        T xk = x[k];
        if (two) {
          const T ad = alpha_d * pn[k];
          xk = xk + ad;
        }
        const T ap = alpha * pk;
        x[k] = xk + ap;
      }
      if (!stop) {
        const T bp = beta * pk;
        pn[k] = r[k] + bp;
      }
    }
}

// CGX_ALG_SR without the fused step (any layout -- CSR, DC, column panels,
// cache-resident DIA, a partition's ranks): the SpMV stores
// (p.s, s.s) pairs (SpmvArgs::pair), k_finalize FIN_SR1 -- or, on the ranks,
// the all-reduce applied privately (sr1_now; FIN_SUM3_SR1 applies it to the
// state one iteration later) -- gives alpha_j = r_j.r_j / p_j.s_j
// (cg.c:113), beta_j from the estimate alpha (alpha s.s) - r.r (cg.c:129)
// and the stop test of iteration j - 1 on the exact r_j.r_j (cg.c:125's
// rule, one launch late); this launch does the rest of iteration j in ONE
// pass, with oracle_solve_sr's roundings: r_{j+1} = r_j - alpha s_j,
// p_{j+1} = r_{j+1} + beta p_j (into the other p buffer), x += alpha p_j
// deferred pairwise as k_xpay_xf (an odd j adds alpha_{j-1} p_{j-1}, read
// from pn before p_{j+1} overwrites it, then alpha_j p_j), and the exact
// r_{j+1}.r_{j+1} partials (4 per workgroup, k_update_rf's layout) for the
// next reduction.  Reads r, s, p (+ x, p_{j-1} every other launch), writes
// r, p_{j+1} (+ x): 40 B/row + 12 on average, against the HS pair of
// vector launches' 48 + 12.  done == 1 (a stop at an even iteration, its x
// update deferred): x += alpha_def p_{j-1} only -- the next finalize marks
// done = 2.  pn == p (a partition's ranks: p in place, its ghost tail
// refreshed by the halo): x += alpha p every iteration, nothing deferred.
// FOLD (the single-GPU solver, round 5): no k_finalize between the SpMV and
// this launch -- every workgroup sums the SpMV's (p.s, s.s) pairs and the
// previous r.r partials itself (sum_parts_sr, k_finalize<1024>'s order at
// 1,024 threads: the same alpha, beta and stop test) and runs fin_sr1 on a
// private copy of the state; the last workgroup to finish (two-level ticket:
// every workgroup has read the state by then) writes the new state and the
// history entry.  The r.r partials go to a buffer other than the one read
// (pc_out: the solver alternates two).
template <typename T, bool NT, bool FOLD>
__global__ __launch_bounds__(kFoldBS) void k_update_sr(int n, T *__restrict__ x,
                                                       T *__restrict__ r,
                                                       const T *__restrict__ s, const T *p,
                                                       T *pn, CgState *__restrict__ st,
                                                       const double *g,
                                                       double *__restrict__ rr_part,
                                                       SrFold fo) {
  __shared__ double red[kFoldBS / kWave];
  Sr1Now sn;
  CgState c;
  double rr_in = 0.0;
  if constexpr (FOLD) {
    static_assert(kFoldBS == 1024, "k_finalize<1024>'s summation order");
    double ps, ss;
    sum_parts_sr<kFoldBS>(fo.pq, fo.nq, fo.pc, fo.nc, red, ps, ss, rr_in);
    __shared__ double bc[3];  // the sums are valid in thread 0: broadcast
    if (threadIdx.x == 0) {
      bc[0] = ps;
      bc[1] = ss;
      bc[2] = rr_in;
    }
    __syncthreads();
    ps = bc[0];
    ss = bc[1];
    rr_in = bc[2];
    c.done = st->done;
    c.k_u = st->k_u;
    c.k = st->k;
    c.max_iter = st->max_iter;
    c.use_tol = st->use_tol;
    c.tol2bb = st->tol2bb;
    c.hist_cap = 0;
    c.brk = st->brk;
    c.alpha = st->alpha;
    c.beta = st->beta;
    c.rr = st->rr;
    c.ps = st->ps;
    c.xdef = st->xdef;
    fin_sr1(ps, ss, rr_in, &c, nullptr);  // uniform: every workgroup the same
    sn = Sr1Now{c.k_u, c.done, c.alpha, c.beta};
  } else {
    sn = sr1_now(st, g);
  }
  const T alpha_d = (T)st->alpha_def;
  const bool defer = pn != p;
  // the iteration's vector work (returns early on a stop)
  auto body = [&]() {
    if (sn.done > 1) return;  // uniform
    typedef typename Vec16<T>::type V;
    constexpr int W = Vec16<T>::W;
    const int nv = n / W;
    const int gid = blockIdx.x * kFoldBS + threadIdx.x, stride = gridDim.x * kFoldBS;
    if (sn.done == 1) {  // the stop iteration's deferred x update, nothing else
      if (!defer) return;  // x is complete
      for (int i = gid; i < nv; i += stride) {
        V xv = reinterpret_cast<const V *>(x)[i];
        const V pd = reinterpret_cast<const V *>(pn)[i];
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const T ad = alpha_d * pd[j];
          xv[j] = xv[j] + ad;
        }
        reinterpret_cast<V *>(x)[i] = xv;
      }
      if (gid == 0)
        for (int k = nv * W; k < n; ++k) {
          const T ad = alpha_d * pn[k];
          x[k] = x[k] + ad;
        }
      return;
    }
    const int k = sn.k_u;  // this iteration (fin_sr1 made it k_u)
    const bool odd = defer && (k & 1) != 0;       // x += alpha_{k-1} p_{k-1} + alpha_k p_k
    const bool xup = !defer || odd, xone = !defer;  // xone: x += alpha_k p_k alone
    const T alpha = (T)sn.alpha, beta = (T)sn.beta;
    if (defer && !odd && blockIdx.x == 0 && threadIdx.x == 0)
      st->alpha_def = sn.alpha;  // read at k + 1 (only odd launches use it)
    double acc = 0.0;
    for (int i = gid; i < nv; i += stride) {
      V rv = reinterpret_cast<const V *>(r)[i];
      const V sv = reinterpret_cast<const V *>(s)[i];
      V pv = reinterpret_cast<const V *>(p)[i];
      V xv = V(), pd = V();
      if (xup) xv = reinterpret_cast<const V *>(x)[i];
      if (odd) pd = reinterpret_cast<const V *>(pn)[i];
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T as = alpha * sv[j];
        rv[j] = rv[j] - as;
        acc = acc + (double)rv[j] * (double)rv[j];
      }
      if (xup) {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          if (!xone) {
            const T ad = alpha_d * pd[j];
            xv[j] = xv[j] + ad;
          }
          const T ap = alpha * pv[j];
          xv[j] = xv[j] + ap;
        }
        if constexpr (NT) __builtin_nontemporal_store(xv, reinterpret_cast<V *>(x) + i);
        else reinterpret_cast<V *>(x)[i] = xv;
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T bp = beta * pv[j];
        pv[j] = rv[j] + bp;
      }
      if constexpr (NT) {
        __builtin_nontemporal_store(rv, reinterpret_cast<V *>(r) + i);
        __builtin_nontemporal_store(pv, reinterpret_cast<V *>(pn) + i);
      } else {
        reinterpret_cast<V *>(r)[i] = rv;
        reinterpret_cast<V *>(pn)[i] = pv;
      }
    }
    if (gid == 0)
      for (int e = nv * W; e < n; ++e) {
        const T as = alpha * s[e];
        const T re = r[e] - as;
        acc = acc + (double)re * (double)re;
        const T pe = p[e];
        if (xup) {
          T xe = x[e];
          if (!xone) {
            const T ad = alpha_d * pn[e];
            xe = xe + ad;
          }
          const T ap = alpha * pe;
          x[e] = xe + ap;
        }
        const T bp = beta * pe;
        r[e] = re;
        pn[e] = re + bp;
      }
    // one partial per 256-thread quarter (k_update_rf's layout and order)
    acc = wave_sum(acc);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) red[wid] = acc;
    __syncthreads();
    if (threadIdx.x < kFoldBS / 256) {
      constexpr int WQ = 256 / kWave;
      double q = red[threadIdx.x * WQ];
  #pragma unroll
      for (int w = 1; w < WQ; ++w) q = q + red[threadIdx.x * WQ + w];
      rr_part[blockIdx.x * (kFoldBS / 256) + threadIdx.x] = q;
    }
  };
  body();
  if constexpr (FOLD) {
    // the state once every workgroup has read it: the last arriver writes
    // what fin_sr1 changed, and the history entry of iteration j - 1
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) last = take_ticket(fo.tick, gridDim.x);
    __syncthreads();
    if (last && threadIdx.x == 0) {
      const int j = st->k_u + 1;
      if (!st->done && j >= 1 && j - 1 < st->hist_cap) fo.hist[j - 1] = rr_in;
      st->done = c.done;
      st->k_u = c.k_u;
      st->k = c.k;
      st->brk = c.brk;
      st->alpha = c.alpha;
      st->beta = c.beta;
      st->rr = c.rr;
      st->ps = c.ps;
    }
  }
}

// Chronopoulos-Gear update: p = r + beta p; s = w + beta s; x += alpha p;
// r -= alpha s; part = r.r (gamma of the next iteration).
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_cg1_update(int n, T *__restrict__ x, T *__restrict__ p,
                                                   T *__restrict__ r, T *__restrict__ s,
                                                   const T *__restrict__ w,
                                                   const CgState *__restrict__ st,
                                                   double *__restrict__ part) {
  __shared__ double red[BS / kWave];
  if (st->done) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const T alpha = (T)st->alpha, beta = (T)st->beta;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    V xv = reinterpret_cast<const V *>(x)[i];
    V pv = reinterpret_cast<const V *>(p)[i];
    V rv = reinterpret_cast<const V *>(r)[i];
    V sv = reinterpret_cast<const V *>(s)[i];
    const V wv = reinterpret_cast<const V *>(w)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T bp = beta * pv[j];
      pv[j] = rv[j] + bp;
      const T bs = beta * sv[j];
      sv[j] = wv[j] + bs;
      const T ap = alpha * pv[j];
      xv[j] = xv[j] + ap;
      const T as = alpha * sv[j];
      rv[j] = rv[j] - as;
      acc = acc + (double)rv[j] * (double)rv[j];
    }
    reinterpret_cast<V *>(x)[i] = xv;
    reinterpret_cast<V *>(p)[i] = pv;
    reinterpret_cast<V *>(r)[i] = rv;
    reinterpret_cast<V *>(s)[i] = sv;
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T bp = beta * p[i];
      const T pi = r[i] + bp;
      const T bs = beta * s[i];
      const T si = w[i] + bs;
      const T ap = alpha * pi;
      x[i] = x[i] + ap;
      const T as = alpha * si;
      const T ri = r[i] - as;
      p[i] = pi;
      s[i] = si;
      r[i] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  const double sum = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// Exact-order dot (dot_product, mv_ops.c:128-129): products are formed in
// parallel (each rounded, as the reference does), lane 0 adds them strictly
// in index order starting from 0.0.  O(n) serial -- parity mode only.  The
// products of the NEXT chunk are loaded while lane 0 adds the current one.
template <typename T>
__global__ __launch_bounds__(kWave) void k_dot_seq(int n, const T *__restrict__ a,
                                                   const T *__restrict__ b,
                                                   double *__restrict__ out,
                                                   const int *__restrict__ done) {
  constexpr int CH = 8 * kWave;
  __shared__ double buf[CH];
  if (done && *done) return;
  const int lane = threadIdx.x;
  double acc = 0.0;
  T va[8], vb[8];
  auto load = [&](int base) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * kWave + lane;
      va[j] = i < n ? a[i] : T(0);
      vb[j] = i < n ? b[i] : T(0);
    }
  };
  load(0);
  for (int base = 0; base < n; base += CH) {
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[j * kWave + lane] = (double)(va[j] * vb[j]);
    __syncthreads();
    if (base + CH < n) load(base + CH);
    if (lane == 0) {
      const int m = min(CH, n - base);
      for (int t = 0; t < m; ++t) acc = acc + buf[t];
    }
    __syncthreads();
  }
  if (lane == 0) out[0] = acc;
}

template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_dot_part(int n, const T *__restrict__ a,
                                                 const T *__restrict__ b,
                                                 double *__restrict__ part) {
  __shared__ double red[BS / kWave];
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    const V av = reinterpret_cast<const V *>(a)[i];
    const V bv = reinterpret_cast<const V *>(b)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) acc = acc + (double)av[j] * (double)bv[j];
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) acc = acc + (double)a[i] * (double)b[i];
  const double s = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Fixed-order sum of na (and nb) partials by one workgroup, then the scalar
// step.  Partial loads go out before the done-flag round trip.
template <int BS>
__global__ __launch_bounds__(BS) void k_finalize(int op, const double *pa, int na,
                                                 const double *pb, int nb, CgState *st,
                                                 double *hist, double *out, const double *pc,
                                                 int nc) {
  __shared__ double red[BS / kWave];
  double sa, sb = 0.0, sc = 0.0;
  if (op == FIN_SUM3 || op == FIN_SR1 || op == FIN_SUM3_SR1)
    sum_parts_sr<BS>(pa, na, pc, nc, red, sa, sb, sc);  // pa: (p.s, s.s) pairs
  else if (pb) sum_parts2<BS>(pa, na, pb, nb, red, sa, sb);
  else sa = sum_parts<BS>(pa, na, red);
  if (threadIdx.x != 0) return;
  if (op == FIN_SUM3_SR1) {  // pb: the previous all-reduce's (p.s, s.s, r.r)
    if (st->sr_pend) fin_sr1(pb[0], pb[1], pb[2], st, hist);
    st->sr_pend = 1;
    out[0] = sa;
    out[1] = sb;
    out[2] = sc;
    return;
  }
  if (op == FIN_SUM3) out[2] = sc;
  if (op == FIN_SR1) {
    fin_sr1(sa, sb, sc, st, hist);
    return;
  }
  if (op != FIN_SUM && op != FIN_SUM2 && op != FIN_SUM3 && op != FIN_INIT_HS &&
      op != FIN_INIT_CG1 && st->done)
    return;
  apply_fin(op, sa, sb, st, hist, out);
}

template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_axpby(int op, int n, double sc, const T *__restrict__ a,
                                              const T *__restrict__ b, T *__restrict__ r) {
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  const T s = (T)sc;
  for (int i = gid; i < n; i += stride) {
    T v;
    if (op == 0) v = s * a[i];          // sv_mult, mv_ops.c:141-142
    else if (op == 1) v = a[i] + b[i];  // vec_add, mv_ops.c:229
    else v = a[i] - b[i];               // vec_sub, mv_ops.c:258
    r[i] = v;
  }
}

// In-process all-reduce of the multi-partition transport: every partition
// adds the partitions' local sums in the same fixed order (0..P-1).
__global__ void k_group_sum(const double *const *srcs, int P, int count, double *dst, int off) {
  const int c = threadIdx.x + off;
  if ((int)threadIdx.x >= count) return;
  double acc = srcs[0][c];
  for (int q = 1; q < P; ++q) acc = acc + srcs[q][c];
  dst[c] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather(int m, const int *__restrict__ idx,
                                                const T *__restrict__ x, T *__restrict__ buf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m) buf[i] = x[idx[i]];
}

// STREAM triad a = b + s c (fp64, 16 B per lane per array, grid-stride) and
// a read-only stream: the on-box ceilings the kernels are compared with.
__global__ __launch_bounds__(256) void k_triad(long long n2, double2 *__restrict__ a,
                                               const double2 *__restrict__ b,
                                               const double2 *__restrict__ c, double sc) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256) {
    const double2 bv = b[i], cv = c[i];
    a[i] = make_double2(bv.x + sc * cv.x, bv.y + sc * cv.y);
  }
}

__global__ __launch_bounds__(256) void k_stream_read(long long n2, const double2 *__restrict__ b,
                                                     double *__restrict__ sink) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256) {
    const double2 v = b[i];
    acc += v.x + v.y;
  }
  if (acc == 1.2345e300) sink[0] = acc;  // keeps the loads; never true
}

// Tuned read/write streams (the ceiling a read/write mix
// reaches on this box, beside the naive triad above): R arrays read, W
// written, all arrays n2 16-B chunks at a stride of `stride` chunks in one
// buffer; each lane handles U chunks 256 apart per pass (U R loads in flight
// before the first store), grid = the resident workgroup slots, grid-stride;
// NT: non-temporal stores.  Out w = in w + 0.5 in (w + 1) mod R (never
// elided; the values are irrelevant).
template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void k_stream_rw(long long n2, long long stride,
                                                   double *__restrict__ buf) {
  typedef Vec16<double>::type V;
  V *b = reinterpret_cast<V *>(buf);
  const long long step = (long long)gridDim.x * 256 * U;
  for (long long i0 = (long long)blockIdx.x * 256 * U + threadIdx.x; i0 < n2; i0 += step) {
    V v[R][U];
#pragma unroll
    for (int q = 0; q < R; ++q)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = i0 + u * 256;
        v[q][u] = i < n2 ? b[q * stride + i] : V{0.0, 0.0};
      }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = i0 + u * 256;
        const V o = v[w % R][u] + 0.5 * v[(w + 1) % R][u];
        if (i < n2) {
          if (NT) __builtin_nontemporal_store(o, b + (R + w) * stride + i);
          else b[(R + w) * stride + i] = o;
        }
      }
  }
}

// ------------------------------------------- on-device Laplacian
// CSR of the whole grid written straight into HBM: row r's entries at
// lap_rp(r), columns ascending -- cgx_gen_laplacian2d/3d bit for bit.
__global__ __launch_bounds__(256) void k_gen_laplacian(LapSpec g, int n, int *__restrict__ col,
                                                       double *__restrict__ val) {
  const int nx = g.nx, ny = g.ny, pl = g.nx * g.ny;
  for (int r = blockIdx.x * 256 + threadIdx.x; r < n; r += gridDim.x * 256) {
    long long k = lap_rp(r, g);
    const int i = r % nx, j = (r / nx) % ny, l = r / pl;
    auto put = [&](int c, double v) {
      col[k] = c;
      val[k] = v;
      ++k;
    };
    if (g.dim == 3 && l > 0) put(r - pl, -1.0);
    if (j > 0) put(r - nx, -1.0);
    if (i > 0) put(r - 1, -1.0);
    put(r, g.dim == 3 ? 6.0 : 4.0);
    if (i < nx - 1) put(r + 1, -1.0);
    if (j < ny - 1) put(r + nx, -1.0);
    if (g.dim == 3 && l < g.nz - 1) put(r + pl, -1.0);
  }
}

// Offset codes of a device-resident CSR against a sorted dictionary (binary
// search; a miss raises an error flag).
__global__ __launch_bounds__(256) void k_dc_encode(int n, const int *__restrict__ rp,
                                                   const int *__restrict__ col,
                                                   const int *__restrict__ dict, int nd,
                                                   unsigned char *__restrict__ code,
                                                   int *__restrict__ err,
                                                   const double *__restrict__ val,
                                                   const double *__restrict__ dval) {
  for (int r = blockIdx.x * 256 + threadIdx.x; r < n; r += gridDim.x * 256) {
    for (int k = rp[r]; k < rp[r + 1]; ++k) {
      const int off = col[k] - r;
      int lo = 0, hi = nd - 1;
      while (lo < hi) {  // first entry >= off
        const int mid = (lo + hi) >> 1;
        if (dict[mid] < off) lo = mid + 1;
        else hi = mid;
      }
      if (dict[lo] != off) atomicOr(err, 1);
      if (dval && __double_as_longlong(val[k]) != __double_as_longlong(dval[lo]))
        atomicOr(err, 1);
      code[k] = (unsigned char)lo;
    }
  }
}

// DIA-VI codes of a device-resident CSR (a device-generated Laplacian; host
// matrices are encoded on the host, cgx_matrix.cpp dia_encode_host).  Row r's
// field k = the index of its entry's value in diagonal k's table (bit
// patterns, so -0.0, +0.0 and every NaN payload stay distinct), all ones
// where it has no entry; rows [n, npad) are all ones.  err |= 1 when an entry's diagonal or value is
// not among the candidates, or a row's columns do not strictly ascend (the
// diagonal order would then not be the row's order); the host then keeps
// another layout.
template <typename T>
struct Bits;
template <>
struct Bits<double> {
  typedef unsigned long long U;
  __device__ static U of(double v) { return (U)__double_as_longlong(v); }
};
template <>
struct Bits<float> {
  typedef unsigned U;
  __device__ static U of(float v) { return (U)__float_as_int(v); }
};

template <typename T>
__global__ __launch_bounds__(256) void k_dia_encode(int n, int npad, const int *__restrict__ rp,
                                                    const int *__restrict__ col,
                                                    const T *__restrict__ val, DiaCand c,
                                                    const T *__restrict__ vtab,
                                                    unsigned char *__restrict__ code,
                                                    int *__restrict__ err) {
  typedef typename Bits<T>::U U;
  unsigned long long empty = 0;  // every field all ones: no entry
  for (int q = 0; q < c.ndiag; ++q) empty |= ((1ull << c.cbits[q]) - 1ull) << c.csh[q];
  for (int r = blockIdx.x * 256 + threadIdx.x; r < npad; r += gridDim.x * 256) {
    unsigned long long w = empty;
    if (r < n) {
      int prev = -1;
      for (int k = rp[r]; k < rp[r + 1]; ++k) {
        const int off = col[k] - r;
        int q = 0;
        while (q < c.ndiag && c.doff[q] != off) ++q;
        if (q == c.ndiag || q <= prev) {
          atomicOr(err, 1);
          break;
        }
        prev = q;
        const U vb = Bits<T>::of(val[k]);
        int v = 0;
        while (v < c.nval[q] && Bits<T>::of(vtab[q * 16 + v]) != vb) ++v;
        if (v == c.nval[q]) {
          atomicOr(err, 1);
          break;
        }
        w &= ~(((1ull << c.cbits[q]) - 1ull) << c.csh[q]);
        w |= (unsigned long long)v << c.csh[q];
      }
    }
    unsigned char *p = code + (long long)r * c.cbytes;
    switch (c.cbytes) {
      case 1: *p = (unsigned char)w; break;
      case 2: *reinterpret_cast<unsigned short *>(p) = (unsigned short)w; break;
      case 4: *reinterpret_cast<unsigned *>(p) = (unsigned)w; break;
      default: *reinterpret_cast<unsigned long long *>(p) = w; break;
    }
  }
}

}  // namespace

// ------------------------------------------------------------- launchers

template <typename T>
int spmv_grid(const SpmvArgs<T> &a) {
  switch (a.layout) {
    case L_DIA: return a.items.count;
    case L_STENCIL: return (a.n + 511) / 512;
    default: return (a.items.count + 3) / 4;
  }
}

// Every SpMV launch goes through launch_k: with timing events it is
// hipExtLaunchKernel, whose start / stop events are stamped when the
// kernel itself starts and ends (the kernel's duration, as rocprofv3 sees
// it, without the queue's dispatch latency in front of it).
template <typename T>
static void launch_k(const void *k, int g, hipStream_t st, const LaunchEv &ev,
                     const SpmvArgs<T> &a) {
  void *args[] = {(void *)&a};
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256), args, 0, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256), args, 0, st);
}
#define CGX_K(...) reinterpret_cast<const void *>(&__VA_ARGS__)

// U: x gathers issued per row chunk -- 7 when the rows are short (a 7-point
// row is then exactly one chunk: -4% at C3, tools/mb/spmv_lab.hip), else 8
template <typename T, int CAPW, bool EPI, bool NT>
static void launch_csr_w(const SpmvArgs<T> &a, int g, hipStream_t st, const LaunchEv &ev) {
  const bool l = a.items.list != nullptr;
  if (a.gath == 7) {
    if (l) launch_k(CGX_K(k_spmv_csr<T, CAPW, 7, EPI, NT, true>), g, st, ev, a);
    else launch_k(CGX_K(k_spmv_csr<T, CAPW, 7, EPI, NT, false>), g, st, ev, a);
  } else {
    if (l) launch_k(CGX_K(k_spmv_csr<T, CAPW, 8, EPI, NT, true>), g, st, ev, a);
    else launch_k(CGX_K(k_spmv_csr<T, CAPW, 8, EPI, NT, false>), g, st, ev, a);
  }
}

template <typename T, int CAPW, int ND, bool EPI, bool NT>
static void launch_dc_w(const SpmvArgs<T> &a, int g, hipStream_t st, const LaunchEv &ev) {
  const bool l = a.items.list != nullptr;
  if (a.gath == 7) {
    if (l) launch_k(CGX_K(k_spmv_dc<T, CAPW, ND, 7, EPI, NT, true>), g, st, ev, a);
    else launch_k(CGX_K(k_spmv_dc<T, CAPW, ND, 7, EPI, NT, false>), g, st, ev, a);
  } else {
    if (l) launch_k(CGX_K(k_spmv_dc<T, CAPW, ND, 8, EPI, NT, true>), g, st, ev, a);
    else launch_k(CGX_K(k_spmv_dc<T, CAPW, ND, 8, EPI, NT, false>), g, st, ev, a);
  }
}

template <typename T, int KW, bool EPI, bool NT>
static void launch_dia_w(const SpmvArgs<T> &a, int g, hipStream_t st, const LaunchEv &ev) {
  if (a.items.list) launch_k(CGX_K(k_spmv_dia<T, KW, EPI, NT, true, false>), g, st, ev, a);
  else launch_k(CGX_K(k_spmv_dia<T, KW, EPI, NT, false, false>), g, st, ev, a);
}

template <typename T, bool EPI, bool NT>
static void launch_dia_v(const SpmvArgs<T> &a, int g, hipStream_t st, const LaunchEv &ev) {
  if (a.items.list) launch_k(CGX_K(k_spmv_dia<T, 1, EPI, NT, true, true>), g, st, ev, a);
  else launch_k(CGX_K(k_spmv_dia<T, 1, EPI, NT, false, true>), g, st, ev, a);
}

template <typename T, bool EPI, bool NT>
static hipError_t launch_spmv_en(const SpmvArgs<T> &a, int g, hipStream_t st, const LaunchEv &ev) {
  switch (a.layout) {
    case L_CSR:
      if constexpr (sizeof(T) == 4) {
        launch_csr_w<T, 1024, EPI, NT>(a, g, st, ev);
      } else {
        if (a.capw == 328) launch_csr_w<T, 328, EPI, NT>(a, g, st, ev);
        else if (a.capw == 456) launch_csr_w<T, 456, EPI, NT>(a, g, st, ev);
        else if (a.capw == 512) launch_csr_w<T, 512, EPI, NT>(a, g, st, ev);
        else return hipErrorInvalidValue;
      }
      break;
    case L_DC: {
      const bool big = a.ndict_cap > 64;
      if constexpr (sizeof(T) == 4) {
        if (big) launch_dc_w<T, 1024, 256, EPI, NT>(a, g, st, ev);
        else launch_dc_w<T, 1024, 64, EPI, NT>(a, g, st, ev);
      } else if (a.capw == 328) {
        if (big) launch_dc_w<T, 328, 256, EPI, NT>(a, g, st, ev);
        else launch_dc_w<T, 328, 64, EPI, NT>(a, g, st, ev);
      } else if (a.capw == 456) {
        if (big) launch_dc_w<T, 456, 256, EPI, NT>(a, g, st, ev);
        else launch_dc_w<T, 456, 64, EPI, NT>(a, g, st, ev);
      } else if (a.capw == 512) {
        if (big) launch_dc_w<T, 512, 256, EPI, NT>(a, g, st, ev);
        else launch_dc_w<T, 512, 64, EPI, NT>(a, g, st, ev);
      } else {
        return hipErrorInvalidValue;
      }
      break;
    }
    case L_DIA:
      if (a.dval) {
        if (a.ndiag > kDiaVMax || a.cb != 1) return hipErrorInvalidValue;
        launch_dia_v<T, EPI, NT>(a, g, st, ev);
      } else if (a.ndiag <= 8) launch_dia_w<T, 1, EPI, NT>(a, g, st, ev);
      else launch_dia_w<T, 2, EPI, NT>(a, g, st, ev);
      break;
    case L_STENCIL:
      launch_k(CGX_K(k_stencil<T, EPI, NT>), g, st, ev, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_spmv(const SpmvArgs<T> &a, hipStream_t st, const LaunchEv &ev) {
  const int g = spmv_grid(a);
  if (g <= 0) return hipSuccess;
  const bool epi = a.part != nullptr;
  if (epi && a.nt) return launch_spmv_en<T, true, true>(a, g, st, ev);
  if (epi) return launch_spmv_en<T, true, false>(a, g, st, ev);
  if (a.nt) return launch_spmv_en<T, false, true>(a, g, st, ev);
  return launch_spmv_en<T, false, false>(a, g, st, ev);
}

template <typename T, int SB, int NF, int NFAR, bool GH>
static const void *fused_kernel_g(bool nt, bool list) {
  return nt ? (list ? CGX_K(k_spmv_dia_h<T, SB, NF, NFAR, true, true, GH>)
                    : CGX_K(k_spmv_dia_h<T, SB, NF, NFAR, true, false, GH>))
            : (list ? CGX_K(k_spmv_dia_h<T, SB, NF, NFAR, false, true, GH>)
                    : CGX_K(k_spmv_dia_h<T, SB, NF, NFAR, false, false, GH>));
}

template <typename T, int SB, int NF, int NFAR>
static const void *fused_kernel(bool nt, bool list, bool gh) {
  return gh ? fused_kernel_g<T, SB, NF, NFAR, true>(nt, list)
            : fused_kernel_g<T, SB, NF, NFAR, false>(nt, list);
}

// Slices per fused workgroup: two (512 threads, one window for both) when
// the halo rows exceed a slice -- C4 and its slabs (hl + hr = 800): the
// window re-reads 1.78x instead of 2.56x the rows, 672-681 vs 702 us per
// launch; at C3 (432) one slice per workgroup stays faster (106-107 vs
// 109-110 us; tools/ab_probe.sh, same box, alternating).
static int fuse_slices(int hl, int hr) { return hl + hr > kDiaSliceRows ? 2 : 1; }

template <typename T>
int fused_grid(const SpmvArgs<T> &a) {
  if (a.items.count <= 0) return 0;
  if (fuse_slices(a.hl, a.hr) == 1) return a.items.count;
  return a.items.pairs ? a.items.npairs : (a.items.count + 1) / 2;  // super-items
}

// The plane march applies: a planned chain structure (DevMatrix::plan_march),
// the launch covers the matrix's own item order in full, no ghosts, no SR
// pairs, and the caller allows it (FuseArgs::march = steps per segment).
template <typename T>
static bool march_applies(const SpmvArgs<T> &a, const FuseArgs<T> &f) {
  return f.march > 0 && a.mq > 0 && !f.ghost && !f.ss && a.items.first == 0 &&
         a.items.list == a.mlist && a.items.count == a.mslices;
}

template <typename T>
int march_grid(const SpmvArgs<T> &a, int len) {
  const int steps = (a.mslices + a.mq - 1) / a.mq;  // chain 0's, the longest
  return a.mchains * ((steps + len - 1) / len);
}

template <typename T, int SB, int NF>
static const void *march_kernel(int cb) {
  return cb == 1 ? CGX_K(k_spmv_dia_m<T, SB, NF, 1>)
                 : cb == 2 ? CGX_K(k_spmv_dia_m<T, SB, NF, 2>) : CGX_K(k_spmv_dia_m<T, SB, NF, 4>);
}

template <typename T>
static hipError_t launch_march(const SpmvArgs<T> &a, const FuseArgs<T> &f, hipStream_t st,
                               const LaunchEv &ev) {
  const int sb = a.msb;
  const int wn = sb * kDiaSliceRows + a.hl + a.hr;
  const int nf = (wn + 2 * 256 * sb - 1) / (2 * 256 * sb);
  if (a.mws < wn + 2 || (sb != 1 && sb != 2) || nf > (sb == 1 ? 5 : 3))
    return hipErrorInvalidValue;
  const int nfc = nf <= 2 ? 2 : nf <= 3 ? 3 : 5;
  const int cb = a.cb;
  if (cb != 1 && cb != 2 && cb != 4) return hipErrorInvalidValue;
  const void *k = nullptr;
  switch (sb * 10 + nfc) {
    case 12: k = march_kernel<T, 1, 2>(cb); break;
    case 13: k = march_kernel<T, 1, 3>(cb); break;
    case 15: k = march_kernel<T, 1, 5>(cb); break;
    case 22: k = march_kernel<T, 2, 2>(cb); break;
    case 23: k = march_kernel<T, 2, 3>(cb); break;
    default: return hipErrorInvalidValue;
  }
  const int g = march_grid(a, f.march);
  void *args[] = {(void *)&a, (void *)&f};
  const size_t lds = (size_t)3 * a.mws * sizeof(T) + 16;  // the three-window ring
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256 * sb), args, lds, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256 * sb), args, lds, st);
  return hipGetLastError();
}

template <typename T, int SB, int NF, bool FOLD>
static const void *sr1_kernel_f(int cb, bool dv) {
  // DIA-V: no four-slice step (its value registers exceed a 1,024-thread
  // workgroup's 128 VGPRs)
  if (dv) {
    if constexpr (SB == 4) return nullptr;
    else return cb == 1 ? CGX_K((k_sr1_dia_m<T, SB, NF, 1, true, FOLD>)) : nullptr;
  }
  return cb == 1   ? CGX_K((k_sr1_dia_m<T, SB, NF, 1, false, FOLD>))
         : cb == 2 ? CGX_K((k_sr1_dia_m<T, SB, NF, 2, false, FOLD>))
                   : CGX_K((k_sr1_dia_m<T, SB, NF, 4, false, FOLD>));
}

template <typename T, int SB, int NF>
static const void *sr1_kernel(int cb, bool dv, bool fold) {
  return fold ? sr1_kernel_f<T, SB, NF, true>(cb, dv) : sr1_kernel_f<T, SB, NF, false>(cb, dv);
}

// The plan k_sr1_dia_m runs on the matrix's march plan (mq slices between
// the steps of a chain): steps of sb slices of rows (sb = 1, 2, 4: a
// workgroup of 256 sb threads, two rows each), its LDS ring slots sized for
// them.  sb 0: the matrix's own (msb), four where its two-slice chains pair
// up (mq % 4 == 0, C4 and its slabs; round 5, same box: C4 783 against 812
// us per launch).  With chains of any width (Sr1Args::cw) sb no longer has
// to divide mq: sr1_pick_shape picks it (C3: 91 slices per plane).
template <typename T>
static SpmvArgs<T> sr1_args(const SpmvArgs<T> &a0, int sb = 0) {
  SpmvArgs<T> a = a0;
  if (sb <= 0 && !a.dval && a.msb == 2 && a.mq % 4 == 0 &&
      4 * kDiaSliceRows + a.hl + a.hr <= 2 * 2 * 1024)
    sb = 4;
  if (sb > 0) {
    a.msb = sb;
    a.mchains = (a.mq + sb - 1) / sb;
    a.mws = (sb * kDiaSliceRows + a.hl + a.hr + 3) & ~1;
  }
  return a;
}

// chains per step (k_sr1_dia_m: QR = mq slices of rows in chains of cw rows)
// and chain 0's step count (the longest chain)
template <typename T>
static int sr1_chains(const SpmvArgs<T> &a, int cw) {
  const int QR = a.mq * kDiaSliceRows;
  const int w = cw > 0 ? cw : a.msb * kDiaSliceRows;
  return (QR + w - 1) / w;
}

template <typename T>
static int sr1_steps(const SpmvArgs<T> &a) {
  const long long QR = (long long)a.mq * kDiaSliceRows;
  return a.n > 0 ? (int)((a.n + QR - 1) / QR) : 0;
}

template <typename T>
int sr1_grid(const SpmvArgs<T> &a_in, const Sr1Args<T> &f) {
  const SpmvArgs<T> a = sr1_args(a_in, f.sb);
  const int steps = std::max(1, sr1_steps(a));
  const int nch = sr1_chains(a, f.cw);
  if (f.nseg > 0) return nch * std::min(f.nseg, steps);
  if (f.march <= 0) return 0;
  return nch * ((steps + f.march - 1) / f.march);
}

template <typename T>
int sr1_edge_grid(int n, const Sr1Args<T> &f) {
  const long long pairs = f.elo / 2 + (f.ehi < n ? (n - f.ehi + 1) / 2 : 0);
  return (int)((pairs + 255) / 256);
}

// the kernel instance for the matrix's march plan (nullptr: none) and its LDS
template <typename T>
static const void *sr1_pick(const SpmvArgs<T> &a, size_t &lds, bool fold) {
  const int sb = a.msb;
  const int wn = sb * kDiaSliceRows + a.hl + a.hr;
  const int nf = (wn + 2 * 256 * sb - 1) / (2 * 256 * sb);
  if (a.mws < wn + 2 || (sb != 1 && sb != 2 && sb != 4) ||
      nf > (sb == 1 ? 5 : sb == 2 ? 3 : 2))
    return nullptr;
  const int nfc = nf <= 2 ? 2 : nf <= 3 ? 3 : 5;
  const int cb = a.cb;
  if (cb != 1 && cb != 2 && cb != 4) return nullptr;
  // the three-window ring and two slots of own-row r
  lds = ((size_t)3 * a.mws + (size_t)2 * sb * kDiaSliceRows) * sizeof(T) + 16;
  switch (sb * 10 + nfc) {
    case 12: return sr1_kernel<T, 1, 2>(cb, a.dval != nullptr, fold);
    case 13: return sr1_kernel<T, 1, 3>(cb, a.dval != nullptr, fold);
    case 15: return sr1_kernel<T, 1, 5>(cb, a.dval != nullptr, fold);
    case 22: return sr1_kernel<T, 2, 2>(cb, a.dval != nullptr, fold);
    case 23: return sr1_kernel<T, 2, 3>(cb, a.dval != nullptr, fold);
    case 42: return sr1_kernel<T, 4, 2>(cb, a.dval != nullptr, fold);
    default: return nullptr;
  }
}

// The launch shape of k_sr1_dia_m on `cus` CUs: step width sb, chain width
// and segments per chain, from a per-CU work model fitted to round 5's
// same-box sweeps (profiles/r05_sr_width_probe.log) -- a CU runs
// ceil(workgroups / cus) workgroups of (ceil(L / nseg) + 2) windows each (L
// the longest chain), a window costing a quarter step of fixed work (the
// workgroup's idle lanes still issue), its own rows, and a fifth of its
// in-plane halo (those rows come from L2: the neighbouring chains load them
// at the same time); 5 % more per extra round of resident workgroups (a
// later round's neighbours are not in step: its halos miss L2), 10 % less
// with two or more workgroups per CU (one's barriers overlap the other's
// loads), and a CU with fewer than 12 waves pays for the latency it cannot
// hide.  A step narrower than four slices must hold at least twice its halo
// (C4's sb 2: 826 against 744 us).  Chain widths: sb slices and, for a
// chain count c up to 48 above that one's, ceil(QR / c) rounded up to 32
// rows (> sb / 2 slices) -- the width that lets chains x segments fill the
// CUs instead of leaving some idle (C4's 78 chains x 3 segments ran on 234
// of 256 CUs; 85 chains of 1,888 rows: 744 -> 730 us; C3 picks sb 2, 1,024
// rows: 139 -> 133 us).  cw_force > 0: that width (even) on the narrowest
// sb that holds it, only nseg picked.  With an explicit segment length
// (set_march > 0) callers use cw_force's width or the matrix's sb and its
// width: the auto shape assumes the auto segment count.
template <typename T>
Sr1Shape sr1_pick_shape(const SpmvArgs<T> &a_in, int cus, int cw_force, bool fold) {
  Sr1Shape best{1, 0, 0};
  if (a_in.mq <= 0) return best;
  const int QR = a_in.mq * kDiaSliceRows;
  const double halo = 0.2 * (a_in.hl + a_in.hr);
  const int ncu = std::max(1, cus);
  double best_cost = -1.0;
  auto consider_sb = [&](int sb, int cw_only) {
    const SpmvArgs<T> a = sr1_args(a_in, sb);
    size_t lds = 0;
    const void *k = sr1_pick(a, lds, fold);
    if (!k) return;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256 * sb, lds) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    const long long slots = (long long)per_cu * ncu;
    const int SR = sb * kDiaSliceRows;
    const int L = std::max(1, sr1_steps(a));
    auto consider = [&](int cw) {
      const long long nch = sr1_chains(a, cw);
      const int w = cw > 0 ? cw : SR;
      for (int ns = 1; ns <= L; ++ns) {
        const long long g = nch * ns;
        if (g > sr1_max_grid(a.mslices)) break;
        const long long rounds = (g + slots - 1) / slots;
        const long long per = (g + ncu - 1) / ncu;  // workgroups per CU
        const long long conc = std::min<long long>(per, per_cu);
        const double waves = 4.0 * sb * (double)conc;
        double cost = (double)per * ((L + ns - 1) / ns + 2) * (0.25 * SR + w + halo);
        cost *= 1.0 + 0.05 * (double)(rounds - 1);
        if (conc >= 2) cost *= 0.9;
        if (waves < 12.0) cost *= 12.0 / waves;
        if (best_cost < 0 || cost < best_cost * (1.0 - 1e-9)) {
          best_cost = cost;
          best = Sr1Shape{ns, cw, sb};
        }
      }
    };
    if (cw_only > 0) {
      consider(cw_only);
      return;
    }
    consider(0);
    const int c_min = (QR + SR - 1) / SR;
    for (int c = c_min + 1; c <= c_min + 48; ++c) {
      const int cw = std::min(SR, ((QR + c - 1) / c + 31) & ~31);
      if (cw <= SR / 2 || sr1_chains(a, cw) != c) continue;
      consider(cw);
    }
  };
  if (cw_force > 0) {
    const int cw = std::max(kDiaSliceRows / 4, std::min(4 * kDiaSliceRows, cw_force)) & ~1;
    for (int sb : {1, 2, 4})
      if (cw <= sb * kDiaSliceRows) {
        consider_sb(sb, cw);
        if (best_cost >= 0) break;
      }
    // no step that wide has a kernel for this matrix (DIA-V has no four-slice
    // step; a wide halo none of four slices): the widest step that runs,
    // the width clamped to it -- never the silent one-segment fallback
    // 
    for (int sb : {2, 1})
      if (best_cost < 0 && cw > sb * kDiaSliceRows) consider_sb(sb, sb * kDiaSliceRows);
    return best;
  }
  for (int sb : {1, 2, 4})
    if (sb == 4 || 2 * (a_in.hl + a_in.hr) <= sb * kDiaSliceRows) consider_sb(sb, 0);
  if (best_cost < 0)  // no step of four slices (a wide halo): any that runs
    for (int sb : {1, 2}) consider_sb(sb, 0);
  return best;
}

template <typename T>
hipError_t launch_sr1_march(const SpmvArgs<T> &a_in, const Sr1Args<T> &f, hipStream_t st,
                            const LaunchEv &ev) {
  const SpmvArgs<T> a = sr1_args(a_in, f.sb);
  if (a.mq <= 0 || a.items.count != a.mslices || a.layout != L_DIA ||
      (f.march <= 0 && f.nseg <= 0) || f.nseg < 0 || (f.elo & 1) || (f.ehi < a.n && (f.ehi & 1)) ||
      f.cw < 0 || (f.cw & 1) || f.cw > a.msb * kDiaSliceRows ||
      sr1_grid(a, f) > sr1_max_grid(a.mslices))
    return hipErrorInvalidValue;
  size_t lds = 0;
  const void *k = sr1_pick(a, lds, f.st_out != nullptr);
  if (!k) return hipErrorInvalidValue;
  const int g = sr1_grid(a, f);
  void *args[] = {(void *)&a, (void *)&f};
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256 * a.msb), args, lds, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256 * a.msb), args, lds, st);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_sr1_edge(const SpmvArgs<T> &a, const Sr1Args<T> &f, hipStream_t st,
                           const LaunchEv &ev) {
  if (a.layout != L_DIA || (f.elo & 1) || f.elo < 0 || f.elo > a.n + 1 || f.ehi < f.elo ||
      (f.ehi < a.n && (f.ehi & 1)) || a.ndiag > kDiaMax || (a.dval && a.ndiag > kDiaVMax))
    return hipErrorInvalidValue;
  const int g = sr1_edge_grid(a.n, f);
  if (g <= 0) {  // no edge rows: the launch's events still bracket it
    if (ev.start) (void)hipEventRecord(ev.start, st);
    if (ev.stop) (void)hipEventRecord(ev.stop, st);
    return hipGetLastError();
  }
  void *args[] = {(void *)&a, (void *)&f};
  const void *k = CGX_K(k_sr1_edge<T>);
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256), args, 0, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256), args, 0, st);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_spmv_fused(const SpmvArgs<T> &a, const FuseArgs<T> &f, hipStream_t st,
                             const LaunchEv &ev) {
  if (a.items.count <= 0) return hipSuccess;
  if (a.dval) return hipErrorInvalidValue;  // DIA-V: the fused HS kernels read the value table
  if (march_applies(a, f)) return launch_march(a, f, st, ev);
  const int sb = fuse_slices(a.hl, a.hr);
  const int g = fused_grid(a);
  if (a.layout != L_DIA || a.cb > 4 || g <= 0) return hipErrorInvalidValue;
  const int wn = sb * kDiaSliceRows + a.hl + a.hr;  // the widest window
  const int nf = (wn + 2 * 256 * sb - 1) / (2 * 256 * sb);
  int nfar = 0;
  for (int q = 0; q < 4; ++q) nfar += a.fark[q] >= 0;
  if (nf > (sb == 1 ? 5 : 3)) return hipErrorInvalidValue;
  const bool nt = a.nt != 0, l = a.items.list != nullptr, gh = f.ghost != 0;
  const void *k = nullptr;
  const int nfc = nf <= 2 ? 2 : nf <= 3 ? 3 : 5;
  switch (sb * 100 + nfc * 10 + (nfar == 0 ? 0 : nfar <= 2 ? 2 : 4)) {
    case 120: k = fused_kernel<T, 1, 2, 0>(nt, l, gh); break;
    case 122: k = fused_kernel<T, 1, 2, 2>(nt, l, gh); break;
    case 124: k = fused_kernel<T, 1, 2, 4>(nt, l, gh); break;
    case 130: k = fused_kernel<T, 1, 3, 0>(nt, l, gh); break;
    case 132: k = fused_kernel<T, 1, 3, 2>(nt, l, gh); break;
    case 134: k = fused_kernel<T, 1, 3, 4>(nt, l, gh); break;
    case 150: k = fused_kernel<T, 1, 5, 0>(nt, l, gh); break;
    case 152: k = fused_kernel<T, 1, 5, 2>(nt, l, gh); break;
    case 154: k = fused_kernel<T, 1, 5, 4>(nt, l, gh); break;
    case 220: k = fused_kernel<T, 2, 2, 0>(nt, l, gh); break;
    case 222: k = fused_kernel<T, 2, 2, 2>(nt, l, gh); break;
    case 224: k = fused_kernel<T, 2, 2, 4>(nt, l, gh); break;
    case 230: k = fused_kernel<T, 2, 3, 0>(nt, l, gh); break;
    case 232: k = fused_kernel<T, 2, 3, 2>(nt, l, gh); break;
    case 234: k = fused_kernel<T, 2, 3, 4>(nt, l, gh); break;
    default: return hipErrorInvalidValue;
  }
  void *args[] = {(void *)&a, (void *)&f};
  // the window's allocation, plus the pair an inactive thread of a one-slice
  // super-item reads past it
  const size_t lds = (size_t)(wn + 2) * sizeof(T) + 16;
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256 * sb), args, lds, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256 * sb), args, lds, st);
  return hipGetLastError();
}

template <typename T, int NF, int NFAR, bool GH>
static const void *cg1_kernel_g(bool nt, bool list) {
  return nt ? (list ? CGX_K(k_cg1_dia_h<T, NF, NFAR, true, true, GH>)
                    : CGX_K(k_cg1_dia_h<T, NF, NFAR, true, false, GH>))
            : (list ? CGX_K(k_cg1_dia_h<T, NF, NFAR, false, true, GH>)
                    : CGX_K(k_cg1_dia_h<T, NF, NFAR, false, false, GH>));
}

template <typename T, int NF, int NFAR>
static const void *cg1_kernel(bool nt, bool list, bool gh) {
  return gh ? cg1_kernel_g<T, NF, NFAR, true>(nt, list) : cg1_kernel_g<T, NF, NFAR, false>(nt, list);
}

template <typename T>
hipError_t launch_cg1_fused(const SpmvArgs<T> &a, const Cg1Args<T> &f, hipStream_t st,
                            const LaunchEv &ev) {
  const int g = spmv_grid(a);
  if (g <= 0) return hipSuccess;
  if (a.layout != L_DIA || a.cb > 4 || !a.part || !f.pg || a.dval) return hipErrorInvalidValue;
  const int wn = kDiaSliceRows + a.hl + a.hr;
  const int nf = (wn + 511) / 512;
  int nfar = 0;
  for (int q = 0; q < 4; ++q) nfar += a.fark[q] >= 0;
  if (nf > 5) return hipErrorInvalidValue;
  const bool nt = a.nt != 0, l = a.items.list != nullptr, gh = f.ghost != 0;
  const void *k = nullptr;
  switch ((nf <= 2 ? 2 : nf <= 3 ? 3 : 5) * 10 + (nfar == 0 ? 0 : nfar <= 2 ? 2 : 4)) {
    case 20: k = cg1_kernel<T, 2, 0>(nt, l, gh); break;
    case 22: k = cg1_kernel<T, 2, 2>(nt, l, gh); break;
    case 24: k = cg1_kernel<T, 2, 4>(nt, l, gh); break;
    case 30: k = cg1_kernel<T, 3, 0>(nt, l, gh); break;
    case 32: k = cg1_kernel<T, 3, 2>(nt, l, gh); break;
    case 34: k = cg1_kernel<T, 3, 4>(nt, l, gh); break;
    case 50: k = cg1_kernel<T, 5, 0>(nt, l, gh); break;
    case 52: k = cg1_kernel<T, 5, 2>(nt, l, gh); break;
    case 54: k = cg1_kernel<T, 5, 4>(nt, l, gh); break;
    default: return hipErrorInvalidValue;
  }
  void *args[] = {(void *)&a, (void *)&f};
  const size_t lds = (size_t)wn * sizeof(T) + 16;
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernel(k, dim3(g), dim3(256), args, lds, st, ev.start, ev.stop, 0);
  else
    (void)hipLaunchKernel(k, dim3(g), dim3(256), args, lds, st);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_rnext(int n_send, const int *idx, const T *r, const T *w, const T *s,
                             T *out, const CgState *stt, hipStream_t st) {
  if (n_send <= 0) return hipSuccess;
  const int grid = std::min((n_send + 255) / 256, 1024);
  hipLaunchKernelGGL((k_pack_rnext<T>), dim3(grid), dim3(256), 0, st, n_send, idx, r, w, s, out,
                     stt);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_hs(int n, const T *b, T *x, T *r, T *p, double *part, int grid,
                          hipStream_t st) {
  hipLaunchKernelGGL((k_init_hs<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, b, x, r, p,
                     part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_cg1(int n, const T *b, T *x, T *r, T *p, T *s, double *part, int grid,
                           hipStream_t st) {
  hipLaunchKernelGGL((k_init_cg1<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, b, x, r, p, s,
                     part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_xr(int n, T *x, const T *p, T *r, const T *s, const CgState *stt,
                            double *part, int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_update_xr<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, x, p, r, s,
                     stt, part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_xpay(int n, T *p, const T *r, const CgState *stt, int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_xpay<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, p, r, stt);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_pnext(int n_send, const int *idx, const T *r, const T *pold, T *out,
                             const CgState *stt, const double *rr_new, hipStream_t st) {
  if (n_send <= 0) return hipSuccess;
  const int grid = std::min((n_send + 255) / 256, 1024);
  hipLaunchKernelGGL((k_pack_pnext<T>), dim3(grid), dim3(256), 0, st, n_send, idx, r, pold, out,
                     stt, rr_new);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_sr(int n_send, const int *idx, const T *rold, const T *pold,
                          const T *sold, T *out, const CgState *stt, hipStream_t st,
                          const double *g) {
  if (n_send <= 0) return hipSuccess;
  const int grid = std::min((n_send + 255) / 256, 1024);
  hipLaunchKernelGGL((k_pack_sr<T>), dim3(grid), dim3(256), 0, st, n_send, idx, rold, pold, sold,
                     out, stt, g);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_rf(int n, T *r, const T *s, CgState *stt, const double *ps_part,
                            int nps, double *rr_part, int grid, hipStream_t st,
                            const FinArgs *fin, const double *sr, double *hist, bool nt) {
  const FinArgs f = fin ? *fin : FinArgs{};
  if (nt)
    hipLaunchKernelGGL((k_update_rf<T, true>), dim3(grid), dim3(kFoldBS), 0, st, n, r, s, stt,
                       ps_part, nps, rr_part, f, sr, hist);
  else
    hipLaunchKernelGGL((k_update_rf<T, false>), dim3(grid), dim3(kFoldBS), 0, st, n, r, s, stt,
                       ps_part, nps, rr_part, f, sr, hist);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_xpay_xf(int n, T *x, const T *p, T *pn, const T *r, CgState *stt,
                          const double *rr_part, int nrr, double *hist, int grid, hipStream_t st,
                          bool nt) {
  if (nt)
    hipLaunchKernelGGL((k_xpay_xf<T, true>), dim3(grid), dim3(kFoldBS), 0, st, n, x, p, pn, r,
                       stt, rr_part, nrr, hist);
  else
    hipLaunchKernelGGL((k_xpay_xf<T, false>), dim3(grid), dim3(kFoldBS), 0, st, n, x, p, pn, r,
                       stt, rr_part, nrr, hist);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_sr(int n, T *x, T *r, const T *sv, const T *p, T *pn, CgState *stt,
                            const double *g, double *rr_part, int grid, hipStream_t st, bool nt,
                            const SrFold *fo) {
  if (fo && (g || !fo->pq || !fo->pc || !fo->tick || fo->pc == rr_part ||
             grid > (kTickRegion - 1) * kTicketGroup))
    return hipErrorInvalidValue;
  const SrFold f = fo ? *fo : SrFold{};
  if (fo) {
    if (nt)
      hipLaunchKernelGGL((k_update_sr<T, true, true>), dim3(grid), dim3(kFoldBS), 0, st, n, x, r,
                         sv, p, pn, stt, g, rr_part, f);
    else
      hipLaunchKernelGGL((k_update_sr<T, false, true>), dim3(grid), dim3(kFoldBS), 0, st, n, x, r,
                         sv, p, pn, stt, g, rr_part, f);
  } else if (nt) {
    hipLaunchKernelGGL((k_update_sr<T, true, false>), dim3(grid), dim3(kFoldBS), 0, st, n, x, r,
                       sv, p, pn, stt, g, rr_part, f);
  } else {
    hipLaunchKernelGGL((k_update_sr<T, false, false>), dim3(grid), dim3(kFoldBS), 0, st, n, x, r,
                       sv, p, pn, stt, g, rr_part, f);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_cg1_update(int n, T *x, T *p, T *r, T *s, const T *w, const CgState *stt,
                             double *part, int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_cg1_update<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, x, p, r, s,
                     w, stt, part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dot_seq(int n, const T *a, const T *b, double *out, const int *done,
                          hipStream_t st) {
  hipLaunchKernelGGL((k_dot_seq<T>), dim3(1), dim3(kWave), 0, st, n, a, b, out, done);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dot_part(int n, const T *a, const T *b, double *part, int grid,
                           hipStream_t st) {
  hipLaunchKernelGGL((k_dot_part<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, a, b, part);
  return hipGetLastError();
}

hipError_t launch_finalize(int op, const double *pa, int na, const double *pb, int nb,
                           CgState *stt, double *hist, double *out, hipStream_t st,
                           const double *pc, int nc) {
  hipLaunchKernelGGL((k_finalize<kFinBS>), dim3(1), dim3(kFinBS), 0, st, op, pa, na, pb, nb, stt,
                     hist, out, pc, nc);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_axpby(int op, int n, double s, const T *a, const T *b, T *r, int grid,
                        hipStream_t st) {
  hipLaunchKernelGGL((k_axpby<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, op, n, s, a, b, r);
  return hipGetLastError();
}

hipError_t launch_group_sum(const double *const *srcs, int P, int count, double *dst,
                            hipStream_t st, int off) {
  hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, st, srcs, P, count, dst, off);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_gather(int m, const int *idx, const T *x, T *buf, hipStream_t st) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_gather<T>), dim3((m + 255) / 256), dim3(256), 0, st, m, idx, x, buf);
  return hipGetLastError();
}

hipError_t launch_stream_read(long long n2, const double *b, double *sink, int grid,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, st, n2, (const double2 *)b, sink);
  return hipGetLastError();
}

hipError_t launch_triad(long long n2, double *a, const double *b, const double *c, int grid,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_triad, dim3(grid), dim3(256), 0, st, n2, (double2 *)a, (const double2 *)b,
                     (const double2 *)c, 3.0);
  return hipGetLastError();
}

namespace {
template <int R, int W, bool NT>
hipError_t launch_rw(long long n2, long long stride, double *buf, int cus, hipStream_t st) {
  constexpr int U = 4;
  const void *k = CGX_K(k_stream_rw<R, W, U, NT>);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess || per_cu < 1)
    per_cu = 8;
  hipLaunchKernelGGL((k_stream_rw<R, W, U, NT>), dim3(cus * per_cu), dim3(256), 0, st, n2, stride,
                     buf);
  return hipGetLastError();
}
}  // namespace

int stream_rw_arrays(int kind, int *r, int *w) {
  switch (kind) {
    case CGX_STREAM_COPY: case CGX_STREAM_COPY_NT: *r = 1; *w = 1; return 0;
    case CGX_STREAM_TRIAD_TUNED: case CGX_STREAM_TRIAD_NT: *r = 2; *w = 1; return 0;
    case CGX_STREAM_MIX33: case CGX_STREAM_MIX33_NT: *r = 3; *w = 3; return 0;
    default: return -1;
  }
}

hipError_t launch_stream_rw(int kind, long long n2, long long stride, double *buf, int cus,
                            hipStream_t st) {
  switch (kind) {
    case CGX_STREAM_COPY: return launch_rw<1, 1, false>(n2, stride, buf, cus, st);
    case CGX_STREAM_COPY_NT: return launch_rw<1, 1, true>(n2, stride, buf, cus, st);
    case CGX_STREAM_TRIAD_TUNED: return launch_rw<2, 1, false>(n2, stride, buf, cus, st);
    case CGX_STREAM_TRIAD_NT: return launch_rw<2, 1, true>(n2, stride, buf, cus, st);
    case CGX_STREAM_MIX33: return launch_rw<3, 3, false>(n2, stride, buf, cus, st);
    case CGX_STREAM_MIX33_NT: return launch_rw<3, 3, true>(n2, stride, buf, cus, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_gen_laplacian(const LapSpec &g, int n, int *col, double *val, hipStream_t st) {
  const int grid = std::max(1, std::min((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_gen_laplacian, dim3(grid), dim3(256), 0, st, g, n, col, val);
  return hipGetLastError();
}

hipError_t launch_dc_encode(int n, const int *rp, const int *col, const int *dict, int nd,
                            unsigned char *code, int *err, hipStream_t st, const double *val,
                            const double *dval) {
  const int grid = std::max(1, std::min((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_dc_encode, dim3(grid), dim3(256), 0, st, n, rp, col, dict, nd, code, err,
                     val, dval);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dia_encode(int n, int npad, const int *rp, const int *col, const T *val,
                             const DiaCand &c, const T *vtab, unsigned char *code, int *err,
                             hipStream_t st) {
  if (npad <= 0) return hipSuccess;
  const int grid = std::max(1, std::min((npad + 255) / 256, 16384));
  hipLaunchKernelGGL((k_dia_encode<T>), dim3(grid), dim3(256), 0, st, n, npad, rp, col, val, c,
                     vtab, code, err);
  return hipGetLastError();
}

#define CGX_INSTANTIATE(T)                                                                       \
  template int spmv_grid<T>(const SpmvArgs<T> &);                                                \
  template hipError_t launch_spmv<T>(const SpmvArgs<T> &, hipStream_t, const LaunchEv &);      \
  template int fused_grid<T>(const SpmvArgs<T> &);                                               \
  template int march_grid<T>(const SpmvArgs<T> &, int);                                         \
  template int sr1_grid<T>(const SpmvArgs<T> &, const Sr1Args<T> &);                            \
  template Sr1Shape sr1_pick_shape<T>(const SpmvArgs<T> &, int, int, bool);                           \
  template int sr1_edge_grid<T>(int, const Sr1Args<T> &);                                       \
  template hipError_t launch_sr1_edge<T>(const SpmvArgs<T> &, const Sr1Args<T> &, hipStream_t,   \
                                         const LaunchEv &);                                      \
  template hipError_t launch_pack_sr<T>(int, const int *, const T *, const T *, const T *, T *,  \
                                        const CgState *, hipStream_t, const double *);            \
  template hipError_t launch_sr1_march<T>(const SpmvArgs<T> &, const Sr1Args<T> &, hipStream_t,  \
                                          const LaunchEv &);                                     \
  template hipError_t launch_spmv_fused<T>(const SpmvArgs<T> &, const FuseArgs<T> &, hipStream_t, \
                                           const LaunchEv &);                                    \
  template hipError_t launch_init_hs<T>(int, const T *, T *, T *, T *, double *, int,            \
                                        hipStream_t);                                            \
  template hipError_t launch_init_cg1<T>(int, const T *, T *, T *, T *, T *, double *, int,      \
                                         hipStream_t);                                           \
  template hipError_t launch_update_xr<T>(int, T *, const T *, T *, const T *, const CgState *,  \
                                          double *, int, hipStream_t);                           \
  template hipError_t launch_xpay<T>(int, T *, const T *, const CgState *, int, hipStream_t);    \
  template hipError_t launch_pack_pnext<T>(int, const int *, const T *, const T *, T *,          \
                                           const CgState *, const double *, hipStream_t);        \
  template hipError_t launch_cg1_fused<T>(const SpmvArgs<T> &, const Cg1Args<T> &, hipStream_t,  \
                                          const LaunchEv &);                                     \
  template hipError_t launch_pack_rnext<T>(int, const int *, const T *, const T *, const T *,    \
                                           T *, const CgState *, hipStream_t);                   \
  template hipError_t launch_update_rf<T>(int, T *, const T *, CgState *, const double *, int,   \
                                          double *, int, hipStream_t, const FinArgs *,           \
                                          const double *, double *, bool);                       \
  template hipError_t launch_xpay_xf<T>(int, T *, const T *, T *, const T *, CgState *,         \
                                        const double *, int, double *, int, hipStream_t, bool);  \
  template hipError_t launch_update_sr<T>(int, T *, T *, const T *, const T *, T *, CgState *,    \
                                          const double *, double *, int, hipStream_t, bool,       \
                                          const SrFold *);                                        \
  template hipError_t launch_cg1_update<T>(int, T *, T *, T *, T *, const T *, const CgState *,  \
                                           double *, int, hipStream_t);                          \
  template hipError_t launch_dot_seq<T>(int, const T *, const T *, double *, const int *,        \
                                        hipStream_t);                                            \
  template hipError_t launch_dot_part<T>(int, const T *, const T *, double *, int, hipStream_t); \
  template hipError_t launch_axpby<T>(int, int, double, const T *, const T *, T *, int,          \
                                      hipStream_t);                                              \
  template hipError_t launch_gather<T>(int, const int *, const T *, T *, hipStream_t);           \
  template hipError_t launch_dia_encode<T>(int, int, const int *, const int *, const T *,       \
                                           const DiaCand &, const T *, unsigned char *, int *,  \
                                           hipStream_t);

CGX_INSTANTIATE(double)
CGX_INSTANTIATE(float)

}  // namespace cgx
