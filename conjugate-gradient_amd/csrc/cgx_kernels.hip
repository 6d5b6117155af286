// cgx_kernels.hip -- hand-written gfx950 kernels for the CG hot path.
//
// Replaces the reference's CPU loops (rnelias/Conjugate-Gradient):
//   mv_mult + mat_get_row   mv_ops.c:160-201, :99-113  -> k_spmv (CSR-stream,
//                           LDS-staged per-row sums, persistent grid)
//   dot_product             mv_ops.c:117-132  -> fused block partials + k_finalize
//                           (deterministic two-stage), k_dot_seq (exact order)
//   sv_mult + vec_add/sub   mv_ops.c:134-259, used at cg.c:115-132
//                           -> k_update_xr, k_xpay, k_cg1_update (fused)
//
// Everything is bandwidth bound (about 0.17 flop/byte), so the design goal is
// one coalesced pass over each array per iteration at 16 bytes per lane and
// no fp64 atomics.  Compiled with -ffp-contract=off: the reference never
// fuses multiply-add (Makefile:2 builds -O0), and x + alpha*p must round
// twice to stay bit-identical.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <algorithm>
#include <cstring>

#include "cgx_internal.h"

#pragma clang fp contract(off)

namespace cgx {

namespace {

constexpr int kWave = 64;

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

// The scalar lines of the recurrence (cg.c:113, 125-129; CG1 analogues) on
// the reduced sums sa, sb -- run by ONE thread (k_finalize, or the last
// workgroup of a ticket reduction).
__device__ void apply_fin(int op, double sa, double sb, CgState *st,
                          double *hist, double *out) {
  switch (op) {
    case FIN_SUM:
      out[0] = sa;
      break;
    case FIN_SUM2:
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
      st->done = 0;
      break;
    case FIN_HS_ALPHA:
      st->ps = sa;
      st->alpha = st->rr / sa;  // cg.c:113
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
        st->delta = d;
        st->alpha = g / (d - beta * g / st->alpha);
        st->beta = beta;
        st->rr = g;
        st->k = k + 1;
      }
      break;
    }
  }
}

// In-kernel deterministic two-level reduction ("last arriver" tickets),
// replacing a separate k_finalize launch.  Every workgroup publishes its
// partial (agent-scope sc1 store, drained before its ticket), then takes a
// ticket on its group's counter (kTicketGroup consecutive workgroups); the
// group's last arriver (told by the returned ticket) sums the group's
// partials in fixed order and takes a ticket on the global counter; the
// last of those sums the group sums in fixed order and runs the scalar
// step.  The sums never depend on arrival order, so results are
// bit-reproducible.  Counters are reset by their last arriver, so they are
// zero again when the kernel ends (placement-independent protocol of
// cdna_hip_programming.md Guideline 16: sc1 payload + drained vmcnt +
// agent-scope atomic; the consumer adds an agent acquire and sc1 loads).
__device__ __forceinline__ bool take_ticket(unsigned *cnt, unsigned n,
                                            double *slot, double v) {
  __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned t =
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != n - 1) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__device__ __forceinline__ double ld_published(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// v: this workgroup's partial, valid in thread 0.  All threads must call it.
template <int BS>
__device__ void ticket_finish(double v, const TicketArgs &t, double *red) {
  __shared__ int s_last;
  const int b = blockIdx.x, G = gridDim.x;
  const int ng = (G + kTicketGroup - 1) / kTicketGroup, grp = b / kTicketGroup;
  const int gsz = min(kTicketGroup, G - grp * kTicketGroup);
  if (threadIdx.x == 0) s_last = take_ticket(t.cnt1 + grp, gsz, t.part1 + b, v);
  __syncthreads();
  if (!s_last) return;
  double g = 0.0;
  if (threadIdx.x < kWave) {
    const int i = threadIdx.x;
    g = wave_sum(i < gsz ? ld_published(t.part1 + grp * kTicketGroup + i) : 0.0);
  }
  if (ng > 1) {
    __syncthreads();
    if (threadIdx.x == 0) s_last = take_ticket(t.cnt2, ng, t.part2 + grp, g);
    __syncthreads();
    if (!s_last) return;
    double acc = 0.0;
    for (int i = threadIdx.x; i < ng; i += BS)
      acc = (i == (int)threadIdx.x) ? ld_published(t.part2 + i)
                                    : acc + ld_published(t.part2 + i);
    g = block_sum<BS>(acc, red);
  }
  if (threadIdx.x == 0) apply_fin(t.op, g, 0.0, t.st, t.hist, nullptr);
}

// ---------------------------------------------------------------- SpMV
// CSR-stream: each row block (<= BS rows, <= CAP nonzeros) is streamed with
// coalesced VEC-wide loads of val/col; the products val[k]*x[col[k]] land in
// LDS; then lane t sums row t's products sequentially in column order from
// 0.0 -- the reference's per-row order (mv_ops.c:190-194), so y is
// bit-identical to it on chained matrices.
//
// Latency structure (one row block): every val/col load of the block is
// issued before the first wait (NIT x VEC elements per lane in registers),
// then every x gather, then the products -- two memory round trips per row
// block instead of two per element.  The grid is persistent: workgroup g owns
// a contiguous chunk of row blocks and accumulates the fused x.y epilogue
// over its chunk in a fixed order.  With XCD = true the chunk index is
// remapped so the workgroups that share an XCD (blockIdx % 8, the observed
// round-robin dispatch; speed only, never correctness) own one contiguous
// 1/8 of the rows, keeping the +-plane x re-reads inside that XCD's L2.
template <typename T>
__device__ __forceinline__ T ld_stream(const T *p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}

template <typename T, int BS, int CAP, int VEC, bool EPI, bool NT>
__global__ __launch_bounds__(BS) void k_spmv(SpmvArgs<T> a) {
  constexpr int NIT = CAP / (BS * VEC);  // load iterations per row block
  static_assert(NIT * BS * VEC == CAP, "CAP must be a multiple of BS*VEC");
  typedef T tv __attribute__((ext_vector_type(VEC)));
  typedef int iv __attribute__((ext_vector_type(VEC)));
  __shared__ __attribute__((aligned(16))) T prod[CAP];
  __shared__ double red[BS / kWave];
  if (a.done && *a.done) return;

  const int tid = threadIdx.x;
  const int G = gridDim.x;
  int g = blockIdx.x;
  if (a.xcd && (G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  const int lo = (int)(((long long)a.nblk * g) / G);
  const int hi = (int)(((long long)a.nblk * (g + 1)) / G);
  double dot = 0.0;

  for (int i = lo; i < hi; ++i) {
    const int rb = a.blk_list ? a.blk_list[i] : a.blk_first + i;
    // Row-block descriptor: rows [r0, r0+nr), nonzeros [k0, k1) -- wave-
    // uniform scalar loads, so the stream loads below issue without waiting
    // on row_ptr.
    const int r0 = a.blk_row[rb];
    const int nr = a.blk_row[rb + 1] - r0;
    const int k0 = a.blk_k[rb], k1 = a.blk_k[rb + 1];
    const int kb = k0 & ~(VEC - 1);
    // Per-row bounds for the reduce phase and the epilogue operand: issued
    // together with the stream, consumed after the barrier.
    int j0 = 0, j1 = 0;
    T xrow = T(0);
    if (tid < nr) {
      j0 = a.rp[r0 + tid];
      j1 = a.rp[r0 + tid + 1];
      if (EPI) xrow = a.x[r0 + tid];
    }

    if (k1 - kb <= CAP) {  // always true for multi-row blocks (planner cap)
      tv v[NIT];
      iv c[NIT];
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        int kk = kb + (it * BS + tid) * VEC;
        kk = kk < k1 ? kk : kb;  // out-of-block lanes re-read a valid window
        v[it] = ld_stream(reinterpret_cast<const tv *>(a.val + kk), NT);
        c[it] = ld_stream(reinterpret_cast<const iv *>(a.col + kk), NT);
      }
      T xv[NIT][VEC];
#pragma unroll
      for (int it = 0; it < NIT; ++it)
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int k = kb + (it * BS + tid) * VEC + j;
          const bool ok = k >= k0 && k < k1;
          xv[it][j] = a.x[ok ? c[it][j] : 0];
        }
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int kk = kb + (it * BS + tid) * VEC;
        if (kk >= k0 && kk + VEC <= k1) {
          tv pv;
#pragma unroll
          for (int j = 0; j < VEC; ++j) pv[j] = v[it][j] * xv[it][j];
          *reinterpret_cast<tv *>(prod + (kk - k0)) = pv;
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            const int k = kk + j;
            if (k >= k0 && k < k1) prod[k - k0] = v[it][j] * xv[it][j];
          }
        }
      }
      __syncthreads();
      if (tid < nr) {
        int j = j0 - k0;
        const int je = j1 - k0;
        T acc = T(0);
        for (; j + 4 <= je; j += 4) {  // 4 LDS reads in flight, adds in order
          const T p0 = prod[j], p1 = prod[j + 1], p2 = prod[j + 2], p3 = prod[j + 3];
          acc = acc + p0;
          acc = acc + p1;
          acc = acc + p2;
          acc = acc + p3;
        }
        for (; j < je; ++j) acc = acc + prod[j];
        a.y[r0 + tid] = acc;
        if (EPI) dot = dot + (double)xrow * (double)acc;
      }
    } else {
      // One row longer than CAP (planner guarantees nr == 1): stream it in
      // CAP-sized chunks, lane 0 keeps the sequential sum.
      T acc = T(0);
      for (int c0 = k0; c0 < k1; c0 += CAP) {
        const int m = min(CAP, k1 - c0);
        for (int t = tid; t < m; t += BS)
          prod[t] = a.val[c0 + t] * a.x[a.col[c0 + t]];
        __syncthreads();
        if (tid == 0)
          for (int j = 0; j < m; ++j) acc = acc + prod[j];
        __syncthreads();
      }
      if (tid == 0) {
        a.y[r0] = acc;
        if (EPI) dot = dot + (double)xrow * (double)acc;
      }
    }
    if (i + 1 < hi) __syncthreads();  // prod is reused by the next row block
  }
  if (EPI) {
    const double s = block_sum<BS>(dot, red);
    if (tid == 0) a.part[blockIdx.x] = s;
  }
}

// Wave-independent CSR-stream: the same algorithm with 64-row row blocks per
// WAVE (CAPW products in the wave's own LDS slice), so a wave never waits on
// a workgroup barrier in the main path and the 32 waves of a CU stream and
// gather independently.  Each wave walks RBW consecutive row blocks (1 by
// default: a wave per row block measured fastest).  The workgroup meets once,
// at the end, to combine the fused x.y epilogue.  With XPAY the gathered
// operand is p = r + beta*p_old, computed on the fly, and the owned rows' p is
// written out: the separate p-update pass of cg.c:131-132 disappears.
template <typename T, int CAPW, int VEC>
struct WaveBlock {
  static constexpr int NIT = CAPW / (kWave * VEC);
  typedef T tv __attribute__((ext_vector_type(VEC)));
  typedef int iv __attribute__((ext_vector_type(VEC)));
  int r0, nr, k0, k1, kb;
  tv v[NIT];
  iv c[NIT];

  __device__ __forceinline__ void describe(const SpmvArgs<T> &a, int wb) {
    const int rb = __builtin_amdgcn_readfirstlane(a.blk_list ? a.blk_list[wb] : a.blk_first + wb);
    r0 = __builtin_amdgcn_readfirstlane(a.blk_row[rb]);
    nr = __builtin_amdgcn_readfirstlane(a.blk_row[rb + 1]) - r0;
    k0 = __builtin_amdgcn_readfirstlane(a.blk_k[rb]);
    k1 = __builtin_amdgcn_readfirstlane(a.blk_k[rb + 1]);
    kb = k0 & ~(VEC - 1);
  }
  template <bool NT>
  __device__ __forceinline__ void stream(const SpmvArgs<T> &a, int lane) {
    if (k1 - kb > CAPW) return;  // long row: chunked path loads itself
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      int kk = kb + (it * kWave + lane) * VEC;
      kk = kk < k1 ? kk : kb;  // out-of-block lanes re-read a valid window
      v[it] = ld_stream(reinterpret_cast<const tv *>(a.val + kk), NT);
      c[it] = ld_stream(reinterpret_cast<const iv *>(a.col + kk), NT);
    }
  }
};

// XCD-contiguous block order (speed only, never correctness): workgroups are
// dealt round-robin over the 8 XCDs, so blocks b, b+8, b+16, ... share one
// XCD's L2.  Give XCD x the contiguous range of logical blocks
// [x*q + min(x, rem), ...) (bijective for any grid size), so each L2 sees
// consecutive rows and the stencil's x re-reads (rows +-1, +-nx, +-nx*ny)
// come from its own L2 instead of the Infinity Cache.
__device__ __forceinline__ int xcd_block(int on) {
  const int b = blockIdx.x, G = gridDim.x;
  if (!on || G < 16) return b;
  const int x = b & 7, i = b >> 3, q = G >> 3, rem = G & 7;
  return x * q + min(x, rem) + i;
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave complete in order; the fences keep the compiler from
  // moving reads of other lanes' slots above the writes.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Gathered operand: x[c], or with XPAY the fused search direction
// p[c] = r[c] + beta*p_old[c] (cg.c:131-132, two roundings as the reference).
template <typename T, bool XPAY>
__device__ __forceinline__ T operand(const SpmvArgs<T> &a, T beta, int c) {
  if (!XPAY) return a.x[c];
  const T bp = beta * a.x2[c];
  return a.x[c] + bp;
}

template <typename T, int CAPW, int VEC, bool EPI, bool XPAY>
__device__ __forceinline__ double wave_block_finish(const SpmvArgs<T> &a,
                                                    WaveBlock<T, CAPW, VEC> &B,
                                                    T *prod, int lane, T beta) {
  typedef WaveBlock<T, CAPW, VEC> WB;
  const int r0 = B.r0, nr = B.nr, k0 = B.k0, k1 = B.k1, kb = B.kb;
  int j0 = 0, j1 = 0;
  T xrow = T(0);
  if (lane < nr) {
    j0 = a.rp[r0 + lane];
    j1 = a.rp[r0 + lane + 1];
    if (EPI || XPAY) xrow = operand<T, XPAY>(a, beta, r0 + lane);
    if (XPAY) a.xout[r0 + lane] = xrow;  // p_new for the owned row
  }
  T acc = T(0);
  if (k1 - kb <= CAPW) {
    T xv[WB::NIT][VEC];
#pragma unroll
    for (int it = 0; it < WB::NIT; ++it)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int k = kb + (it * kWave + lane) * VEC + j;
        const bool ok = k >= k0 && k < k1;
        xv[it][j] = operand<T, XPAY>(a, beta, ok ? B.c[it][j] : 0);
      }
#pragma unroll
    for (int it = 0; it < WB::NIT; ++it) {
      const int kk = kb + (it * kWave + lane) * VEC;
      if (kk >= k0 && kk + VEC <= k1) {
        typename WB::tv pv;
#pragma unroll
        for (int j = 0; j < VEC; ++j) pv[j] = B.v[it][j] * xv[it][j];
        *reinterpret_cast<typename WB::tv *>(prod + (kk - k0)) = pv;
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int k = kk + j;
          if (k >= k0 && k < k1) prod[k - k0] = B.v[it][j] * xv[it][j];
        }
      }
    }
    wave_lds_sync();
    if (lane < nr) {
      int j = j0 - k0;
      const int je = j1 - k0;
      for (; j + 4 <= je; j += 4) {  // 4 LDS reads in flight, adds in order
        const T p0 = prod[j], p1 = prod[j + 1], p2 = prod[j + 2], p3 = prod[j + 3];
        acc = acc + p0;
        acc = acc + p1;
        acc = acc + p2;
        acc = acc + p3;
      }
      for (; j < je; ++j) acc = acc + prod[j];
    }
    wave_lds_sync();  // the slot is rewritten by the next row block
  } else {
    // a single row longer than the wave's slice (nr == 1): chunked, lane 0
    // keeps the sequential sum
    for (int c0 = k0; c0 < k1; c0 += CAPW) {
      const int m = min(CAPW, k1 - c0);
      for (int t = lane; t < m; t += kWave)
        prod[t] = a.val[c0 + t] * operand<T, XPAY>(a, beta, a.col[c0 + t]);
      wave_lds_sync();
      if (lane == 0)
        for (int j = 0; j < m; ++j) acc = acc + prod[j];
      wave_lds_sync();
    }
  }
  double d = 0.0;
  if (lane < nr) {
    a.y[r0 + lane] = acc;
    if (EPI) d = (double)xrow * (double)acc;
  }
  return d;
}

// Transposed-gather finish (TG): the block's val/col window is staged in the
// wave's LDS slice in element order, then lane t walks ROW t's nonzeros
// itself -- for the j-th nonzero the 64 lanes read x at 64 consecutive rows'
// columns (for banded/stencil matrices: a few contiguous runs instead of ~20
// scattered lines per instruction).  Products are rounded separately and
// added in column order from 0.0: the reference's per-row order.
// One row's sequential sum over its LDS-staged entries [jb, je), U entries
// per chunk.  Branch-free: clamped LDS index (all 2U LDS reads go out
// together), every gather issued before the first add, padding terms
// selected to +0 (acc + 0 == acc, so the row order and bits are unchanged).
template <typename T, int U, bool XPAY>
__device__ __forceinline__ T row_sum_lds(const SpmvArgs<T> &a, T beta, const T *lval,
                                         const int *lcol, int jb, int je, T acc) {
  for (int j = jb; j < je; j += U) {
    const int cnt = min(U, je - j);
    int cc[U];
    T vv[U], xx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = u < cnt ? j + u : j;
      const int c = lcol[idx];
      cc[u] = u < cnt ? c : 0;
      vv[u] = lval[idx];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) xx[u] = operand<T, XPAY>(a, beta, cc[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const T prod = vv[u] * xx[u];
      acc = acc + (u < cnt ? prod : T(0));
    }
  }
  return acc;
}

template <typename T, int CAPW, int VEC, bool EPI, bool XPAY>
__device__ __forceinline__ double wave_block_finish_t(const SpmvArgs<T> &a,
                                                      WaveBlock<T, CAPW, VEC> &B,
                                                      T *lval, int *lcol,
                                                      int lane, T beta) {
  typedef WaveBlock<T, CAPW, VEC> WB;
  const int r0 = B.r0, nr = B.nr, k0 = B.k0, k1 = B.k1, kb = B.kb;
  int j0 = 0, j1 = 0;
  T xrow = T(0);
  if (lane < nr) {
    j0 = a.rp[r0 + lane];
    j1 = a.rp[r0 + lane + 1];
    if (EPI || XPAY) xrow = operand<T, XPAY>(a, beta, r0 + lane);
    if (XPAY) a.xout[r0 + lane] = xrow;
  }
  T acc = T(0);
  if (k1 - kb <= CAPW) {
#pragma unroll
    for (int it = 0; it < WB::NIT; ++it) {
      const int off = (it * kWave + lane) * VEC;  // window-relative slot
      *reinterpret_cast<typename WB::tv *>(lval + off) = B.v[it];
      *reinterpret_cast<typename WB::iv *>(lcol + off) = B.c[it];
    }
    wave_lds_sync();
    if (lane < nr) acc = row_sum_lds<T, 4, XPAY>(a, beta, lval, lcol, j0 - kb, j1 - kb, acc);
    wave_lds_sync();  // the slice is rewritten by the next row block
  } else {
    T *prod = lval;
    for (int c0 = k0; c0 < k1; c0 += CAPW) {
      const int m = min(CAPW, k1 - c0);
      for (int t = lane; t < m; t += kWave)
        prod[t] = a.val[c0 + t] * operand<T, XPAY>(a, beta, a.col[c0 + t]);
      wave_lds_sync();
      if (lane == 0)
        for (int j = 0; j < m; ++j) acc = acc + prod[j];
      wave_lds_sync();
    }
  }
  double d = 0.0;
  if (lane < nr) {
    a.y[r0 + lane] = acc;
    if (EPI) d = (double)xrow * (double)acc;
  }
  return d;
}

template <typename T, int WPB, int CAPW, int VEC, bool EPI, bool NT, bool XPAY,
          bool TG>
__global__ __launch_bounds__(WPB * kWave, TG ? 6 : 8) void k_spmv_wave(SpmvArgs<T> a) {
  __shared__ __attribute__((aligned(16))) T lds[WPB * CAPW];
  __shared__ __attribute__((aligned(16))) int ldsc[TG ? WPB * CAPW : 1];
  __shared__ double red[WPB];
  if (a.done && *a.done) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  T *prod = lds + wid * CAPW;
  const T beta = XPAY ? (T)a.st->beta : T(0);
  const int RBW = a.rbw;
  const int first = (xcd_block(a.xcd) * WPB + wid) * RBW;
  const int last = min(first + RBW, a.nblk);
  double dot = 0.0;
  for (int i = first; i < last; ++i) {
    WaveBlock<T, CAPW, VEC> B;
    B.describe(a, i);
    B.template stream<NT>(a, lane);
    if (TG)
      dot = dot + wave_block_finish_t<T, CAPW, VEC, EPI, XPAY>(
                      a, B, prod, ldsc + wid * CAPW, lane, beta);
    else
      dot = dot + wave_block_finish<T, CAPW, VEC, EPI, XPAY>(a, B, prod, lane, beta);
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
      s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
    }
    if (a.tk.cnt1) {
      __syncthreads();
      ticket_finish<WPB * kWave>(s, a.tk, red);
    } else if (threadIdx.x == 0) {
      a.part[blockIdx.x] = s;
    }
  }
}

// LDS-DMA CSR-stream: the wave's val/col window goes straight from memory
// into its LDS slice with global_load_lds_dwordx4 (1 KiB per wave-instruction,
// no VGPRs), then lane t walks row t from LDS as in the transposed-gather
// finish (sequential per-row sums: bit-exact).  val/col are padded by one
// window past nnz, so the window load never leaves the allocation.
typedef __attribute__((address_space(3))) void lds_void;

template <typename T, int WPB, int CAPW, bool EPI, bool XPAY, bool NT = false, int U = 4,
          bool EXACT = true>
__global__ __launch_bounds__(WPB * kWave) void k_spmv_dma(SpmvArgs<T> a) {
  // NT: the once-per-iteration matrix stream is loaded non-temporal (aux = 2)
  // so it does not displace the CG vectors from the Infinity Cache.
  constexpr int AUX = NT ? 2 : 0;
  // CAPW entries per wave window; need not fill whole 1 KiB DMA rows (the
  // lanes past it are masked), only keep every region 16-B aligned
  static_assert(CAPW % 4 == 0, "window");
  __shared__ __attribute__((aligned(16))) T lval_all[WPB * CAPW];
  __shared__ __attribute__((aligned(16))) int lcol_all[WPB * CAPW];
  __shared__ double red[WPB];
  __shared__ int arrived;
  if (a.done && *a.done) return;
  // epilogue without a closing barrier: the last wave to arrive sums the
  // workgroup's wave partials (fixed order), the others leave at once
  if (EPI && a.epi_last) {
    if (threadIdx.x == 0) arrived = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  T *lval = lval_all + wid * CAPW;
  int *lcol = lcol_all + wid * CAPW;
  const T beta = XPAY ? (T)a.st->beta : T(0);
  // a.xcd: XCD-contiguous row ranges (workgroups are dealt round-robin to the
  // 8 XCDs; remapped so each XCD walks one contiguous eighth of the blocks and
  // the x lines a row block shares with its +-1 / +-nx / +-nx*ny neighbours
  // hit that XCD's L2 instead of being re-fetched over the fabric)
  const int wb = xcd_block(a.xcd) * WPB + wid;
  double dot = 0.0;
  if (wb < a.nblk) {
    const int rb = __builtin_amdgcn_readfirstlane(a.blk_list ? a.blk_list[wb] : a.blk_first + wb);
    const int r0 = __builtin_amdgcn_readfirstlane(a.blk_row[rb]);
    const int nr = __builtin_amdgcn_readfirstlane(a.blk_row[rb + 1]) - r0;
    const int k0 = __builtin_amdgcn_readfirstlane(a.blk_k[rb]);
    const int k1 = __builtin_amdgcn_readfirstlane(a.blk_k[rb + 1]);
    const int kb = k0 & ~3;  // 16-B aligned for both val (T) and col (int)
    const bool fits = k1 - kb <= CAPW;
    if (fits) {
      // only the 16-B pieces this block needs: the window tail belongs to the
      // next block, and with nt loads the Infinity Cache would not absorb
      // the second read
      constexpr int EV = 16 / sizeof(T);  // elements of T per lane per DMA
      const int m = k1 - kb;
      const int mm = EXACT ? m : CAPW;
#pragma unroll
      for (int i = 0; i < (int)((CAPW * sizeof(T) + 1023) / 1024); ++i)
        if (i * kWave * EV < mm && (i * kWave + lane) * EV < mm)
          __builtin_amdgcn_global_load_lds(
              (const void *)(a.val + kb + i * kWave * EV + lane * EV),
              (lds_void *)(lval + i * kWave * EV), 16, 0, AUX);
#pragma unroll
      for (int i = 0; i < (CAPW * 4 + 1023) / 1024; ++i)
        if (i * kWave * 4 < mm && (i * kWave + lane) * 4 < mm)
          __builtin_amdgcn_global_load_lds(
              (const void *)(a.col + kb + i * kWave * 4 + lane * 4),
              (lds_void *)(lcol + i * kWave * 4), 16, 0, AUX);
    }
    int j0 = 0, j1 = 0;
    T xrow = T(0);
    T acc = T(0);
    if (lane < nr) {
      j0 = a.rp[r0 + lane];
      j1 = a.rp[r0 + lane + 1];
      if (EPI || XPAY) xrow = operand<T, XPAY>(a, beta, r0 + lane);
      if (XPAY) a.xout[r0 + lane] = xrow;
      if (a.yacc) acc = a.yacc[r0 + lane];  // column panels: continue the row sum
    }
    if (fits) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_lds_sync();
      if (lane < nr) {
        // U gathers in flight per row chunk (U = 8: a 7-point row is one round trip)
        acc = row_sum_lds<T, U, XPAY>(a, beta, lval, lcol, j0 - kb, j1 - kb, acc);
      }
    } else {
      for (int c0 = k0; c0 < k1; c0 += CAPW) {
        const int m = min(CAPW, k1 - c0);
        for (int t = lane; t < m; t += kWave)
          lval[t] = a.val[c0 + t] * operand<T, XPAY>(a, beta, a.col[c0 + t]);
        wave_lds_sync();
        if (lane == 0)
          for (int j = 0; j < m; ++j) acc = acc + lval[j];
        wave_lds_sync();
      }
    }
    if (lane < nr) {
      a.y[r0 + lane] = acc;
      if (EPI) dot = (double)xrow * (double)acc;
    }
  }
  if (EPI && a.epi_last) {
    dot = wave_sum(dot);
    if (lane == 0) {
      red[wid] = dot;
      // LDS ops of one wave complete in order, so a peer's red[] store is
      // done before its increment; acq_rel orders ours and the reads below
      const int prev = __hip_atomic_fetch_add(&arrived, 1, __ATOMIC_ACQ_REL,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
      if (prev == WPB - 1) {
        double s = red[0];
#pragma unroll
        for (int w = 1; w < WPB; ++w) s = s + red[w];
        a.part[blockIdx.x] = s;
      }
    }
  } else if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

// Pipelined LDS-DMA CSR-stream.  The per-block chain (descriptor -> row_ptr
// -> stream -> gather -> store) is ~70 us of pure latency on C3 when every
// wave does one block (r01 diagnostics: the val/col stream alone is ~135 us
// at 6.2 TB/s and the two ADD instead of overlapping).  Here a persistent
// wave walks RBW consecutive row blocks with a two-slot LDS ring: while block
// i's x gathers and row sums run, block i+1's val/col window (LDS-DMA, no
// VGPRs), row bounds and epilogue operand are already in flight.  Wait
// discipline (vmcnt counts in issue order): gathers(i) are issued BEFORE the
// prefetch of i+1, so waiting on them leaves the prefetch in flight; the
// top-of-iteration vmcnt(0) then only waits for the prefetch issued one
// block of work earlier.  Row sums stay sequential: bit-exact.
// gathers + next window's LDS-DMA as ONE asm block ending in a partial
// vmcnt.  LLVM's waitcnt pass treats an in-flight global_load_lds as a
// different event type and answers any later VGPR-load use with vmcnt(0),
// which would drain the prefetch; inside the block the order is explicit:
// 8 gathers, then the DMA ops, then vmcnt(#DMA) = gathers complete.
// The DMA addresses are per-op register pairs (an instruction offset would
// also move the LDS address); M0 holds the LDS base, s_nop 0 after each write.
__device__ __forceinline__ void gather8_dma(double (&xv)[8], const double *const (&g)[8],
                                            const void *const (&d)[6], unsigned lv,
                                            unsigned lc) {
  asm volatile(
      "global_load_dwordx2 %0, %8, off\n\t"
      "global_load_dwordx2 %1, %9, off\n\t"
      "global_load_dwordx2 %2, %10, off\n\t"
      "global_load_dwordx2 %3, %11, off\n\t"
      "global_load_dwordx2 %4, %12, off\n\t"
      "global_load_dwordx2 %5, %13, off\n\t"
      "global_load_dwordx2 %6, %14, off\n\t"
      "global_load_dwordx2 %7, %15, off\n\t"
      "s_mov_b32 m0, %22\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %16, off\n\t"
      "s_add_u32 m0, %22, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %17, off\n\t"
      "s_add_u32 m0, %22, 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %18, off\n\t"
      "s_add_u32 m0, %22, 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %19, off\n\t"
      "s_mov_b32 m0, %23\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %20, off\n\t"
      "s_add_u32 m0, %23, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %21, off\n\t"
      "s_waitcnt vmcnt(6)"
      : "=&v"(xv[0]), "=&v"(xv[1]), "=&v"(xv[2]), "=&v"(xv[3]), "=&v"(xv[4]),
        "=&v"(xv[5]), "=&v"(xv[6]), "=&v"(xv[7])
      : "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]), "v"(g[6]),
        "v"(g[7]), "v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]), "v"(d[4]), "v"(d[5]),
        "s"(lv), "s"(lc)
      : "memory", "m0", "scc");
}

__device__ __forceinline__ void gather8_dma(float (&xv)[8], const float *const (&g)[8],
                                            const void *const (&d)[8], unsigned lv,
                                            unsigned lc) {
  asm volatile(
      "global_load_dword %0, %8, off\n\t"
      "global_load_dword %1, %9, off\n\t"
      "global_load_dword %2, %10, off\n\t"
      "global_load_dword %3, %11, off\n\t"
      "global_load_dword %4, %12, off\n\t"
      "global_load_dword %5, %13, off\n\t"
      "global_load_dword %6, %14, off\n\t"
      "global_load_dword %7, %15, off\n\t"
      "s_mov_b32 m0, %24\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %16, off\n\t"
      "s_add_u32 m0, %24, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %17, off\n\t"
      "s_add_u32 m0, %24, 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %18, off\n\t"
      "s_add_u32 m0, %24, 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %19, off\n\t"
      "s_mov_b32 m0, %25\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %20, off\n\t"
      "s_add_u32 m0, %25, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %21, off\n\t"
      "s_add_u32 m0, %25, 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %22, off\n\t"
      "s_add_u32 m0, %25, 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %23, off\n\t"
      "s_waitcnt vmcnt(8)"
      : "=&v"(xv[0]), "=&v"(xv[1]), "=&v"(xv[2]), "=&v"(xv[3]), "=&v"(xv[4]),
        "=&v"(xv[5]), "=&v"(xv[6]), "=&v"(xv[7])
      : "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]), "v"(g[6]),
        "v"(g[7]), "v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]), "v"(d[4]), "v"(d[5]),
        "v"(d[6]), "v"(d[7]), "s"(lv), "s"(lc)
      : "memory", "m0", "scc");
}

template <typename T, int WPB, int CAPW, bool EPI>
__global__ __launch_bounds__(WPB * kWave) void k_spmv_pipe(SpmvArgs<T> a) {
  // Branch-free prefetch: descriptors are preloaded into lanes (readlane),
  // row bounds use clamped indices, windows are always DMA'd (nnz is padded
  // by kWindowPad >= CAPW) and the last block of a wave is peeled.
  static_assert(CAPW * sizeof(T) == 4096 && CAPW * 4 == (sizeof(T) == 8 ? 2048 : 4096),
                "window layout is baked into gather8_dma");
  constexpr int EV = 16 / (int)sizeof(T);
  constexpr int NDMA = (int)(CAPW * sizeof(T) / 1024) + CAPW * 4 / 1024;
  constexpr int U = 8;  // entries per row gathered before the prefetch
  __shared__ __attribute__((aligned(16))) T lval_all[WPB * 2 * CAPW];
  __shared__ __attribute__((aligned(16))) int lcol_all[WPB * 2 * CAPW];
  __shared__ double red[WPB];
  if (a.done && *a.done) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  T *lv = lval_all + wid * 2 * CAPW;
  int *lc = lcol_all + wid * 2 * CAPW;
  const int first = (blockIdx.x * WPB + wid) * a.rbw;
  const int last = min(first + a.rbw, a.nblk);  // rbw <= 63 (host clamps)
  double dot = 0.0;

  int drow = 0, dk = 0;  // lane l: descriptor of block first + l
  if (first < last && lane <= last - first) {
    drow = a.blk_row[a.blk_first + first + lane];
    dk = a.blk_k[a.blk_first + first + lane];
  }

  int r0n = 0, nrn = 0, k0n = 0, k1n = 0, j0n = 0, j1n = 0;
  T xrn = T(0);
  auto load_desc = [&](int blk) {  // scalar descriptor + row bounds (tracked)
    const int l = blk - first;
    r0n = __builtin_amdgcn_readlane(drow, l);
    nrn = __builtin_amdgcn_readlane(drow, l + 1) - r0n;
    k0n = __builtin_amdgcn_readlane(dk, l);
    k1n = __builtin_amdgcn_readlane(dk, l + 1);
  };
  auto load_rows = [&]() {
    const int rr = lane < nrn ? r0n + lane : r0n;
    j0n = a.rp[rr];
    j1n = a.rp[rr + 1];
    if (EPI) xrn = a.x[rr];
  };
  auto lds_addr = [](const void *p) {
    return (unsigned)(uintptr_t)(lds_void *)p;
  };

  auto body = [&](int i, auto pf) {
    constexpr bool PF = decltype(pf)::value;
    const int slot = (i - first) & 1;
    // vmcnt(0) as an intrinsic (0x0F70: expcnt/lgkmcnt at max) so the waitcnt
    // pass also knows nothing is pending
    __builtin_amdgcn_s_waitcnt(0x0F70);
    wave_lds_sync();
    const int r0 = r0n, nr = nrn, k0 = k0n, k1 = k1n, kb = k0n & ~3;
    const int j0 = j0n, j1 = j1n;
    const T xrow = xrn;
    const bool fit = k1 - kb <= CAPW;
    const T *cv = lv + slot * CAPW;
    const int *cc = lc + slot * CAPW;
    T acc = T(0);
    if (!fit) {
      // a single long row: chunked through the slot, lane 0 sums in order
      T *pr = lv + slot * CAPW;
      for (int c0 = k0; c0 < k1; c0 += CAPW) {
        const int m = min(CAPW, k1 - c0);
        for (int t = lane; t < m; t += kWave) pr[t] = a.val[c0 + t] * a.x[a.col[c0 + t]];
        wave_lds_sync();
        if (lane == 0)
          for (int j = 0; j < m; ++j) acc = acc + pr[j];
        wave_lds_sync();
      }
    }
    const int cnt = (fit && lane < nr) ? min(U, j1 - j0) : 0;
    const T *gp[U];
    T v[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = u < cnt ? j0 - kb + u : 0;
      const int c = cc[idx];
      gp[u] = a.x + (u < cnt ? c : 0);
      v[u] = cv[idx];
    }
    if constexpr (PF) {
      load_desc(i + 1);
      const int kbn = k0n & ~3;
      const void *d[NDMA];
#pragma unroll
      for (int q = 0; q < (int)(CAPW * sizeof(T) / 1024); ++q)
        d[q] = (const void *)(a.val + kbn + q * kWave * EV + lane * EV);
#pragma unroll
      for (int q = 0; q < CAPW * 4 / 1024; ++q)
        d[(int)(CAPW * sizeof(T) / 1024) + q] = (const void *)(a.col + kbn + q * kWave * 4 + lane * 4);
      gather8_dma(xv, gp, d, lds_addr(lv + (slot ^ 1) * CAPW), lds_addr(lc + (slot ^ 1) * CAPW));
      load_rows();
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = *gp[u];
    }
    // unconditional: acc + (+0) == acc exactly, so padding terms are inert
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const T prod = v[u] * xv[u];
      acc = acc + (u < cnt ? prod : T(0));
    }
    if (fit && lane < nr)
      for (int j = j0 + U; j < j1; ++j) {  // rows longer than U, in order
        const T prod = cv[j - kb] * a.x[cc[j - kb]];
        acc = acc + prod;
      }
    if (lane < nr) {
      a.y[r0 + lane] = acc;
      if (EPI) dot = dot + (double)xrow * (double)acc;
    }
  };

  if (first < last) {
    load_desc(first);
    {
      const int kb = k0n & ~3;
#pragma unroll
      for (int q = 0; q < (int)(CAPW * sizeof(T) / 1024); ++q)
        __builtin_amdgcn_global_load_lds(
            (const void *)(a.val + kb + q * kWave * EV + lane * EV),
            (lds_void *)(lv + q * kWave * EV), 16, 0, 0);
#pragma unroll
      for (int q = 0; q < CAPW * 4 / 1024; ++q)
        __builtin_amdgcn_global_load_lds(
            (const void *)(a.col + kb + q * kWave * 4 + lane * 4),
            (lds_void *)(lc + q * kWave * 4), 16, 0, 0);
    }
    load_rows();
    int i = first;
    for (; i + 1 < last; ++i) body(i, std::true_type{});
    body(i, std::false_type{});
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

// ------------------------------------------------ LDS-DMA engine SpMV (fp64)
// Persistent workgroups of 1 loader wave + NC consumer waves sharing an
// S-slot LDS ring (the guide's loader/consumer engine).  The loader only
// issues LDS-DMA -- val (4 KiB), col (2 KiB) and row_ptr (256 B) windows of
// one 64-row block per slot, a fixed ENG_OPS instructions per block, in one
// asm block so the compiler's waitcnt pass never sees them -- and keeps
// D - 1 blocks in flight: after issuing block i it waits
// vmcnt((D-1) * ENG_OPS), i.e. for block i-D+1, and publishes that
// slot (full[slot] = block).  Consumers take blocks round-robin, poll their
// slot's full flag, do the gathers and the row sums (same order as the CSR
// row: bit-exact), store y, and release the slot (free[slot] = block).  Their
// vmcnt only ever tracks their own gathers.  Progress: the loader reuses a
// slot only after the block S earlier is released, and D <= S, so
// every wait is on a block that is already published or issued.
// Shapes (CGX_ENG_SHAPE selects; workgroups per CU from the ring's LDS):
//   0: NC 3, S 8, D 6 (3/CU)   1: NC 3, S 6, D 3 (4/CU)
//   2: NC 7, S 12, D 5 (2/CU)  3: NC 7, S 12, D 9 (2/CU)
//   4-7 (REG): NC 7/5/7/11, S 12, D 10/10/8/10 (2/CU; 4-6 256-512 threads)
constexpr int ENG_OPS = 7;
constexpr int ENG_RL = 8;  // REG: rows up to this long leave the slot early
constexpr int ENG_CAPW = 512;                            // doubles per window
constexpr int ENG_SLOT = ENG_CAPW * 8 + ENG_CAPW * 4 + 64 * 4;  // 6400 B

#define CGX_ENG_DMA(NTS)                                                          \
  asm volatile(                                                                   \
      "s_mov_b32 m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" NTS "\n\t"       \
      "s_add_u32 m0, %7, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" NTS "\n\t" \
      "s_add_u32 m0, %7, 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off" NTS "\n\t" \
      "s_add_u32 m0, %7, 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, off" NTS "\n\t" \
      "s_add_u32 m0, %7, 0x1000\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, off" NTS "\n\t"\
      "s_add_u32 m0, %7, 0x1400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, off" NTS "\n\t"\
      "s_add_u32 m0, %7, 0x1800\n\ts_nop 0\n\tglobal_load_lds_dword %6, off"            \
      :                                                                           \
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "v"(c0), "v"(c1), "v"(r), "s"(lds)       \
      : "memory", "m0", "scc")

template <bool NT>
__device__ __forceinline__ void eng_dma_block(const void *v0, const void *v1, const void *v2,
                                              const void *v3, const void *c0, const void *c1,
                                              const void *r, unsigned lds) {
  if (NT) CGX_ENG_DMA(" nt");  // the once-read matrix stream, non-temporal
  else CGX_ENG_DMA("");
}

// two consecutive ints by a SCALAR load (a vector load would make the
// compiler wait vmcnt(0) -- draining the loader's in-flight DMA)
__device__ __forceinline__ void eng_sload2(const int *p, int &lo, int &hi) {
  unsigned long long v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  lo = (int)(unsigned)(v & 0xffffffffu);
  hi = (int)(unsigned)(v >> 32);
}

template <bool EPI, bool NT, int NC, int S, int D, bool REG>
__global__ __launch_bounds__((1 + NC) * kWave) void k_spmv_eng(SpmvArgs<double> a) {
  __shared__ __attribute__((aligned(16))) char ring[S * ENG_SLOT];
  __shared__ int desc[S][4];  // r0, nr, kb, k1 of the slot's block
  __shared__ int full[S], freed[S];
  __shared__ double red[NC];
  if (a.done && *a.done) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  // this workgroup's contiguous block range (XCD-contiguous order)
  const int q = xcd_block(1), G = gridDim.x;
  const int b0 = (int)((long long)a.nblk * q / G), b1 = (int)((long long)a.nblk * (q + 1) / G);
  static_assert(D <= S && (D - 1) * ENG_OPS <= 63, "engine ring shape");
  if (threadIdx.x < S) {
    full[threadIdx.x] = -1;
    freed[threadIdx.x] = -1;
  }
  __syncthreads();
  const unsigned ring_lds = (unsigned)(uintptr_t)(lds_void *)ring;
  double dot = 0.0;
  if (wid == 0) {
    // ------------------------------------------------------------- loader
    for (int i = b0; i < b1; ++i) {
      const int slot = (i - b0) % S;
      if (i - S >= b0)
        while (__hip_atomic_load(&freed[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) !=
               i - S)
          __builtin_amdgcn_s_sleep(1);
      const int rb = a.blk_first + i;
      int r0, r1, k0, k1;
      eng_sload2(a.blk_row + rb, r0, r1);
      eng_sload2(a.blk_k + rb, k0, k1);
      const int nr = r1 - r0;
      const int kb = k0 & ~3;
      const double *vb = a.val + kb + lane * 2;
      const int *cb = a.col + kb + lane * 4;
      eng_dma_block<NT>(vb, vb + 128, vb + 256, vb + 384, cb, cb + 256, a.rp + r0 + lane,
                        ring_lds + slot * ENG_SLOT);
      if (lane == 0) {
        desc[slot][0] = r0;
        desc[slot][1] = nr;
        desc[slot][2] = kb;
        desc[slot][3] = k1;
      }
      const int pub = i - (D - 1);
      if (pub >= b0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * ENG_OPS) : "memory");
        if (lane == 0)
          __hip_atomic_store(&full[(pub - b0) % S], pub, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      for (int pub = (b1 - (D - 1) > b0 ? b1 - (D - 1) : b0); pub < b1; ++pub)
        __hip_atomic_store(&full[(pub - b0) % S], pub, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    // ----------------------------------------------------------- consumers
    const int c = wid - 1;
    for (int i = b0 + c; i < b1; i += NC) {
      const int slot = (i - b0) % S;
      while (__hip_atomic_load(&full[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != i)
        __builtin_amdgcn_s_sleep(1);
      const int r0 = desc[slot][0], nr = desc[slot][1], kb = desc[slot][2], k1 = desc[slot][3];
      const char *sb = ring + slot * ENG_SLOT;
      const double *lval = (const double *)sb;
      const int *lcol = (const int *)(sb + ENG_CAPW * 8);
      const int *lrp = (const int *)(sb + ENG_CAPW * 12);
      double acc = 0.0;
      double xrow = 0.0;
      bool held = true;
      if (k1 - kb <= ENG_CAPW) {
        int j0 = kb, len = 0;
        if (lane < nr) {
          j0 = lrp[lane];
          len = (lane + 1 < kWave ? lrp[lane + 1] : k1) - j0;
        }
        if (REG && !__any(len > ENG_RL)) {
          // rows of <= ENG_RL entries: copy them to registers and hand the
          // slot back before the gathers, so the ring stays DMA in flight
          double vv[ENG_RL], xx[ENG_RL];
          int cc[ENG_RL];
#pragma unroll
          for (int u = 0; u < ENG_RL; ++u) {
            const int idx = u < len ? j0 - kb + u : 0;
            vv[u] = lval[idx];
            cc[u] = lcol[idx];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0)
            __hip_atomic_store(&freed[slot], i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          held = false;
#pragma unroll
          for (int u = 0; u < ENG_RL; ++u) xx[u] = a.x[cc[u]];  // a valid column, masked below
#pragma unroll
          for (int u = 0; u < ENG_RL; ++u) {  // the row's order, products rounded
            const double prod = vv[u] * xx[u];
            acc = acc + (u < len ? prod : 0.0);
          }
        } else if (lane < nr) {
          acc = row_sum_lds<double, 4, false>(a, 0.0, lval, lcol, j0 - kb, j0 + len - kb, acc);
        }
      } else if (lane == 0) {  // one long row: straight from global, in order
        for (int j = lrp[0]; j < k1; ++j) {
          const double prod = a.val[j] * a.x[a.col[j]];
          acc = acc + prod;
        }
      }
      if (lane < nr) {
        if (EPI) xrow = a.x[r0 + lane];
        a.y[r0 + lane] = acc;
        if (EPI) dot = dot + xrow * acc;
      }
      // every LDS read of the slot is complete before it is handed back
      if (held) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store(&freed[slot], i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (wid > 0 && lane == 0) red[wid - 1] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < NC; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

template <int NC, int S, int D, bool REG = false>
void launch_eng(const SpmvArgs<double> &b, int g, hipStream_t st) {
  const dim3 blk((1 + NC) * kWave);
  if (b.part && b.nt) hipLaunchKernelGGL((k_spmv_eng<true, true, NC, S, D, REG>), dim3(g), blk, 0, st, b);
  else if (b.part) hipLaunchKernelGGL((k_spmv_eng<true, false, NC, S, D, REG>), dim3(g), blk, 0, st, b);
  else if (b.nt) hipLaunchKernelGGL((k_spmv_eng<false, true, NC, S, D, REG>), dim3(g), blk, 0, st, b);
  else hipLaunchKernelGGL((k_spmv_eng<false, false, NC, S, D, REG>), dim3(g), blk, 0, st, b);
}

// Dictionary-coded columns (CSR-DC).  A matrix whose nonzeros use at most 256
// distinct column offsets col - row (every stencil, every banded matrix of
// half-bandwidth < 128) stores one code byte per nonzero instead of a 4-byte
// column: col[k] = row + dict[code[k]].  The stream per nonzero drops from
// 12 to 9 bytes (fp64); C3: 281 -> 70 MB of the SpMV's 1045.  Everything
// else is k_spmv_dma: one 64-row block per wave, val and code windows land in
// the wave's LDS slice by LDS-DMA, lane t sums row t from LDS sequentially in
// column order (the reference's order, mv_ops.c:190-194), so y is bit-identical
// to the CSR kernels'.  The dictionary is copied into each wave's LDS slice
// (ND/64 L2-resident loads per lane) and decoded with one LDS read per entry.
// The smaller slice (4.9 KiB instead of 6 KiB at CAPW 512) also lets 8
// workgroups (32 waves, the hardware limit) share a CU instead of 6.
// Code of entry i of a code window: a byte (CB 8) or a nibble (CB 4, entry
// i in bits 4*(i&1) of byte i/2; dictionaries of <= 16 offsets).
template <int CB>
__device__ __forceinline__ int dc_code(const unsigned char *c, int i) {
  if (CB == 8) return c[i];
  return (c[i >> 1] >> ((i & 1) << 2)) & 15;
}

// co: position of the val window's first entry in the code window
template <typename T, int U, int CB>
__device__ __forceinline__ T row_sum_dc(const T *__restrict__ x, int row, const T *lval,
                                        const unsigned char *lcode, int co, const int *ldict,
                                        int jb, int je, T acc) {
  for (int j = jb; j < je; j += U) {
    const int cnt = min(U, je - j);
    int code[U];
    T vv[U], xx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = u < cnt ? j + u : j;  // clamped: every LDS read is valid
      code[u] = dc_code<CB>(lcode, idx + co);
      vv[u] = lval[idx];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) xx[u] = x[u < cnt ? row + ldict[code[u]] : 0];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const T prod = vv[u] * xx[u];
      acc = acc + (u < cnt ? prod : T(0));  // +0 never changes the sum
    }
  }
  return acc;
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

// RL: row bounds from one byte per row (a.rlen, rows of <= 255 entries) and a
// wave prefix sum from the block's first nonzero, instead of two int32
// row_ptr reads per row (C3: 40 -> 10 MB per SpMV).
template <typename T, int WPB, int CAPW, int ND, bool EPI, bool NT, int U, bool RL, int CB,
          bool LIST>
__global__ __launch_bounds__(WPB * kWave) void k_spmv_dc(SpmvArgs<T> a) {
  constexpr int AUX = NT ? 2 : 0;
  static_assert(CAPW % 4 == 0 && ND % kWave == 0 && (CB == 8 || CB == 4), "window / dictionary");
  // code window: starts at the 16-B granule holding entry k0 (KA entries per
  // granule), so up to KA - 1 more entries than the val window in front
  constexpr int KA = 16 * 8 / CB;
  constexpr int CAPC = ((CAPW + KA) * CB / 8 + 15) & ~15;
  __shared__ __attribute__((aligned(16))) T lval_all[WPB * CAPW];
  __shared__ __attribute__((aligned(16))) unsigned char lcode_all[WPB * CAPC];
  __shared__ int ldict_all[WPB * ND];
  __shared__ double red[WPB];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  T *lval = lval_all + wid * CAPW;
  unsigned char *lcode = lcode_all + wid * CAPC;
  int *ldict = ldict_all + wid * ND;
  // Prologue in as few dependent round trips as possible: the early-exit
  // flag and the block descriptor are scalar loads issued together (the
  // flag is tested only once both are in), the dictionary is loaded after
  // the window DMA is on its way.  (The naive order -- flag, then
  // dictionary, then descriptor, then DMA -- costs two more memory round
  // trips per wave, and the kernel is latency-bound: its time tracks the
  // resident waves per CU.)
  const int wb = __builtin_amdgcn_readfirstlane(xcd_block(a.xcd) * WPB + wid);
  double dot = 0.0;
  if (wb < a.nblk) {
    // no early-exit flag (op-level SpMV): read blk_k[0], which is 0 -- a
    // select, not a branch, so the load goes out with the descriptor's
    const int *dp = a.done ? a.done : a.blk_k;
    const int stop = *dp;
    const int rb = LIST ? a.blk_list[wb] : a.blk_first + wb;
    const int *d = a.blk_rk + 2 * rb;  // row, k of this block and the next
    const int r0 = d[0];
    const int k0 = d[1];
    const int nr = d[2] - r0;
    const int k1 = d[3];
    // make the descriptor live before the flag's branch, so its loads are
    // issued with the flag's instead of being sunk past it
    asm volatile("" ::"s"(r0), "s"(nr), "s"(k0), "s"(k1));
    if (stop) return;  // every wave of the grid sees the same flag
    const int kb = k0 & ~3;   // val window: 16-B aligned for double and float
    const int kc = k0 & ~(KA - 1);  // code window: 16-B aligned
    const bool fits = k1 - kb <= CAPW;
    if (fits) {
      constexpr int EV = 16 / sizeof(T);
      const int m = k1 - kb;
#pragma unroll
      for (int i = 0; i < (int)((CAPW * sizeof(T) + 1023) / 1024); ++i)
        if ((i * kWave + lane) * EV < m)
          __builtin_amdgcn_global_load_lds(
              (const void *)(a.val + kb + i * kWave * EV + lane * EV),
              (lds_void *)(lval + i * kWave * EV), 16, 0, AUX);
      const int mc = ((k1 - kc) * CB + 7) / 8;  // code bytes
      const unsigned char *cbase = a.code + (size_t)kc * CB / 8;
#pragma unroll
      for (int i = 0; i < (CAPC + 1023) / 1024; ++i)
        if ((i * kWave + lane) * 16 < mc)
          __builtin_amdgcn_global_load_lds(
              (const void *)(cbase + i * kWave * 16 + lane * 16),
              (lds_void *)(lcode + i * kWave * 16), 16, 0, AUX);
    }
    int j0 = 0, j1 = 0, len = 0;
    T xrow = T(0);
    T acc = T(0);
    if (lane < nr) {
      if (RL) {
        len = a.rlen[r0 + lane];
      } else {
        j0 = a.rp[r0 + lane];
        j1 = a.rp[r0 + lane + 1];
      }
      if (EPI) xrow = a.x[r0 + lane];
    }
    int dv[ND / kWave];
#pragma unroll
    for (int i = 0; i < ND / kWave; ++i) dv[i] = a.dict[i * kWave + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (RL) {
      j1 = k0 + wave_incl_scan(len, lane);
      j0 = j1 - len;
    }
#pragma unroll
    for (int i = 0; i < ND / kWave; ++i) ldict[i * kWave + lane] = dv[i];
    wave_lds_sync();
    if (fits) {
      if (lane < nr)
        acc = row_sum_dc<T, U, CB>(a.x, r0 + lane, lval, lcode, kb - kc, ldict, j0 - kb,
                                   j1 - kb, acc);
    } else {
      // a single row longer than the window (nr == 1): chunked, lane 0 keeps
      // the sequential sum; codes decoded from memory
      for (int c0 = k0; c0 < k1; c0 += CAPW) {
        const int mm = min(CAPW, k1 - c0);
        for (int t = lane; t < mm; t += kWave)
          lval[t] = a.val[c0 + t] * a.x[r0 + ldict[dc_code<CB>(a.code, c0 + t)]];
        wave_lds_sync();
        if (lane == 0)
          for (int j = 0; j < mm; ++j) acc = acc + lval[j];
        wave_lds_sync();
      }
    }
    if (lane < nr) {
      a.y[r0 + lane] = acc;
      if (EPI) dot = (double)xrow * (double)acc;
    }
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

template <typename T, int CAPW, int ND, bool EPI, bool NT, bool LIST>
void launch_dc_k(const SpmvArgs<T> &a, int g, hipStream_t st) {
  constexpr int WPB = 4;
  const dim3 blk(WPB * kWave);
  const int lds_pad = a.lds_pad;  // diagnostic: fewer resident workgroups per CU
  if constexpr (EPI && !LIST && ND == 64 && CAPW == 512 && sizeof(T) == 8) {
    if (a.wpb == 8 && a.rlen && a.code_bits == 8) {  // 8 waves: half the partials
      hipLaunchKernelGGL((k_spmv_dc<T, 8, CAPW, ND, EPI, NT, 8, true, 8, LIST>),
                         dim3((a.nblk + 7) / 8), dim3(8 * kWave), lds_pad, st, a);
      return;
    }
  }
  if (a.rlen && a.code_bits == 4 && ND == 64)
    hipLaunchKernelGGL((k_spmv_dc<T, WPB, CAPW, ND, EPI, NT, 8, true, 4, LIST>), dim3(g), blk,
                       lds_pad, st, a);
  else if (a.rlen)
    hipLaunchKernelGGL((k_spmv_dc<T, WPB, CAPW, ND, EPI, NT, 8, true, 8, LIST>), dim3(g), blk,
                       lds_pad, st, a);
  else if (a.code_bits == 4 && ND == 64)
    hipLaunchKernelGGL((k_spmv_dc<T, WPB, CAPW, ND, EPI, NT, 8, false, 4, LIST>), dim3(g), blk,
                       lds_pad, st, a);
  else
    hipLaunchKernelGGL((k_spmv_dc<T, WPB, CAPW, ND, EPI, NT, 8, false, 8, LIST>), dim3(g), blk,
                       lds_pad, st, a);
}

template <typename T, int CAPW, int ND>
void launch_dc_nd(const SpmvArgs<T> &a, hipStream_t st) {
  const int g = (a.nblk + 3) / 4;
  const bool epi = a.part != nullptr, list = a.blk_list != nullptr;
#define CGX_DC(E, N)                                        \
  do {                                                      \
    if (list) launch_dc_k<T, CAPW, ND, E, N, true>(a, g, st); \
    else launch_dc_k<T, CAPW, ND, E, N, false>(a, g, st);     \
  } while (0)
  if (epi && a.nt) CGX_DC(true, true);
  else if (epi) CGX_DC(true, false);
  else if (a.nt) CGX_DC(false, true);
  else CGX_DC(false, false);
#undef CGX_DC
}

template <typename T, int CAPW>
void launch_dc_w(const SpmvArgs<T> &a, hipStream_t st) {
  if (a.ndict_cap <= 64) launch_dc_nd<T, CAPW, 64>(a, st);
  else launch_dc_nd<T, CAPW, 256>(a, st);
}

// Value-indexed pairs (CSR-VI).  When a matrix has <= 64 distinct
// (col - row, value) pairs -- constant-coefficient stencils, small value
// sets -- one code per nonzero names both the offset and the value:
// col[k] = row + dict[code[k]], val[k] = dval[code[k]] (bit for bit), and
// the val stream disappears.  C3's SpMV moves 241 MB instead of 804 MB
// (codes 70, row lengths 10, x 81, y 81).  Without the val window a wave's
// LDS slice is a few hundred bytes, so a wave takes BPW row blocks at once
// (lane t sums row t of each; their gathers are issued together), which
// divides the waves -- and the epilogue partials -- by BPW while each wave
// keeps the same three dependent memory round trips (descriptor; codes, row
// lengths and dictionary; x gathers).  Every row is summed sequentially in
// column order from 0 (mv_ops.c:190-194), as in every other SpMV kernel.
// The host guarantees every row block's code window fits CAPC bytes
// (rows <= 255 entries, blocks <= CAPW entries).
template <typename T, int CAPW, bool EPI, bool NT, int CB, bool LIST, int BPW, int WPB = 4>
__global__ __launch_bounds__(WPB * kWave) void k_spmv_vi(SpmvArgs<T> a) {
  constexpr int ND = 64, U = 8;
  constexpr int AUX = NT ? 2 : 0;
  constexpr int KA = 16 * 8 / CB;  // entries per 16-B code granule
  constexpr int CAPC = ((CAPW + KA) * CB / 8 + 15) & ~15;
  __shared__ __attribute__((aligned(16))) unsigned char lcode_all[WPB * BPW * CAPC];
  __shared__ int ldict_all[WPB * ND];
  __shared__ T ldv_all[WPB * ND];
  __shared__ double red[WPB];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  unsigned char *lcode = lcode_all + wid * BPW * CAPC;
  int *ldict = ldict_all + wid * ND;
  T *ldv = ldv_all + wid * ND;
  const int wb0 = __builtin_amdgcn_readfirstlane(xcd_block(a.xcd) * WPB + wid) * BPW;
  double dot = 0.0;
  if (wb0 < a.nblk) {
    const int *dp = a.done ? a.done : a.blk_k;
    const int stop = *dp;
    int r0[BPW], nr[BPW], k0[BPW];
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
      const int wb = wb0 + b < a.nblk ? wb0 + b : wb0;  // past the end: a copy, no rows
      const int rb = LIST ? a.blk_list[wb] : a.blk_first + wb;
      const int *d = a.blk_rk + 2 * rb;
      r0[b] = d[0];
      k0[b] = d[1];
      nr[b] = wb0 + b < a.nblk ? d[2] - d[0] : 0;
      const int k1 = d[3];
      asm volatile("" ::"s"(r0[b]), "s"(nr[b]), "s"(k0[b]), "s"(k1));
      if (b == BPW - 1 && stop) return;  // every wave of the grid sees the same flag
      const int kc = k0[b] & ~(KA - 1);
      const int mc = nr[b] ? ((k1 - kc) * CB + 7) / 8 : 0;
      const unsigned char *cbase = a.code + (size_t)kc * CB / 8;
#pragma unroll
      for (int i = 0; i < (CAPC + 1023) / 1024; ++i)
        if ((i * kWave + lane) * 16 < mc)
          __builtin_amdgcn_global_load_lds((const void *)(cbase + i * kWave * 16 + lane * 16),
                                           (lds_void *)(lcode + b * CAPC + i * kWave * 16), 16,
                                           0, AUX);
    }
    int len[BPW];
    T xrow[BPW];
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
      len[b] = lane < nr[b] ? a.rlen[r0[b] + lane] : 0;
      xrow[b] = EPI && lane < nr[b] ? a.x[r0[b] + lane] : T(0);
    }
    const int dv = a.dict[lane];
    const T dvv = a.dval[lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ldict[lane] = dv;
    ldv[lane] = dvv;
    int jb[BPW], maxlen = 0;
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
      // entry index of the row's first code inside block b's window
      jb[b] = k0[b] + wave_incl_scan(len[b], lane) - len[b] - (k0[b] & ~(KA - 1));
      maxlen = max(maxlen, len[b]);
    }
    wave_lds_sync();
    T acc[BPW];
#pragma unroll
    for (int b = 0; b < BPW; ++b) acc[b] = T(0);
    for (int j = 0; j < maxlen; j += U) {
      int code[BPW][U];
      T xx[BPW][U];
#pragma unroll
      for (int b = 0; b < BPW; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u)
          code[b][u] = dc_code<CB>(lcode + b * CAPC, j + u < len[b] ? jb[b] + j + u : 0);
#pragma unroll
      for (int b = 0; b < BPW; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u)
          xx[b][u] = a.x[j + u < len[b] ? r0[b] + lane + ldict[code[b][u]] : 0];
#pragma unroll
      for (int b = 0; b < BPW; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const T prod = ldv[code[b][u]] * xx[b][u];
          acc[b] = acc[b] + (j + u < len[b] ? prod : T(0));  // +0 never changes the sum
        }
    }
#pragma unroll
    for (int b = 0; b < BPW; ++b)
      if (lane < nr[b]) {
        if (NT && a.nt == 2)  // y streamed past the caches too (nt=2)
          __builtin_nontemporal_store(acc[b], a.y + r0[b] + lane);
        else
          a.y[r0[b] + lane] = acc[b];
        if (EPI) dot = dot + (double)xrow[b] * (double)acc[b];
      }
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

template <typename T, int CAPW, int CB, int BPW, int WPB = 4>
void launch_vi_b(const SpmvArgs<T> &a, hipStream_t st) {
  const int g = (a.nblk + WPB * BPW - 1) / (WPB * BPW);
  const dim3 blk(WPB * kWave);
  const bool epi = a.part != nullptr, list = a.blk_list != nullptr;
#define CGX_VI(E, N, L) \
  hipLaunchKernelGGL((k_spmv_vi<T, CAPW, E, N, CB, L, BPW, WPB>), dim3(g), blk, 0, st, a)
  if (list) {
    if (epi && a.nt) CGX_VI(true, true, true);
    else if (epi) CGX_VI(true, false, true);
    else if (a.nt) CGX_VI(false, true, true);
    else CGX_VI(false, false, true);
  } else {
    if (epi && a.nt) CGX_VI(true, true, false);
    else if (epi) CGX_VI(true, false, false);
    else if (a.nt) CGX_VI(false, true, false);
    else CGX_VI(false, false, false);
  }
#undef CGX_VI
}

template <typename T, int CAPW>
void launch_vi(const SpmvArgs<T> &a, hipStream_t st) {
  if (a.code_bits == 4) {
    launch_vi_b<T, CAPW, 4, 1>(a, st);
  } else {
    switch (a.bpw) {
      case 2: launch_vi_b<T, CAPW, 8, 2>(a, st); break;
      case 4: launch_vi_b<T, CAPW, 8, 4>(a, st); break;
      default: launch_vi_b<T, CAPW, 8, 1>(a, st); break;
    }
  }
}

// SELL-64 (sliced ELLPACK, one 64-row slice per wave, column-major inside the
// slice): lane t owns row t of its slice and walks the row's nonzeros in
// column order, so every load is a coalesced wave-wide line (val 512 B, col
// 256 B per instruction), the x gathers of step j hit 64 consecutive rows'
// j-th columns, no row_ptr is streamed and nothing is staged in LDS.  Padding
// (val 0, col = the row itself) sits after the row's real entries, so the
// sequential sum is the reference's order (mv_ops.c:190-194): +-0 products
// never change a sum.  Internal layout only; the C ABI still takes CSR.
template <typename T, int WPB, bool EPI, bool XPAY>
__global__ __launch_bounds__(WPB * kWave) void k_spmv_sell(SpmvArgs<T> a) {
  __shared__ double red[WPB];
  if (a.done && *a.done) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int slice = blockIdx.x * WPB + wid;
  const T beta = XPAY ? (T)a.st->beta : T(0);
  double dot = 0.0;
  if (slice < a.nslices) {
    const long long off = (long long)__builtin_amdgcn_readfirstlane(a.s_off[slice]) * kWave;
    const int len = __builtin_amdgcn_readfirstlane(a.s_len[slice]);
    const int row = slice * kWave + lane;
    const T *vs = a.val + off + lane;
    const int *cs = a.col + off + lane;
    T acc = T(0);
    constexpr int U = 8;
    for (int j0 = 0; j0 < len; j0 += U) {
      T v[U];
      int c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j0 + u < len;  // wave-uniform
        v[u] = ok ? vs[(j0 + u) * kWave] : T(0);
        c[u] = ok ? cs[(j0 + u) * kWave] : 0;
      }
      T xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = operand<T, XPAY>(a, beta, c[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j0 + u < len) {
          const T prod = v[u] * xv[u];
          acc = acc + prod;
        }
    }
    if (row < a.n) {
      T xrow = T(0);
      if (EPI || XPAY) xrow = operand<T, XPAY>(a, beta, row);
      if (XPAY) a.xout[row] = xrow;
      a.y[row] = acc;
      if (EPI) dot = (double)xrow * (double)acc;
    }
  }
  if (EPI) {
    dot = wave_sum(dot);
    if (lane == 0) red[wid] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) s = s + red[w];
      a.part[blockIdx.x] = s;
    }
  }
}

// ------------------------------------------------------- vector kernels
// All grid-stride over 16-byte vectors; the scalar tail (n % W) is handled
// by global thread 0.  Reductions: per-thread fixed-order sums, then
// block_sum -> part[blockIdx.x]; finalize adds the partials in index order.

// x = 0, r = b, p = b; part = b.b partials (HS prologue, cg.c:104-108).
// With p_zero the p written is 0 instead: the fused SpMV then forms
// p_0 = r + 0*0 = r on the fly (beta is 0 before the first update).
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_init_hs(int n, const T *__restrict__ b,
                                                T *__restrict__ x,
                                                T *__restrict__ r,
                                                T *__restrict__ p,
                                                double *__restrict__ part,
                                                int p_zero, TicketArgs tk) {
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
    reinterpret_cast<V *>(p)[i] = p_zero ? V(T(0)) : bv;
#pragma unroll
    for (int j = 0; j < W; ++j) acc = acc + (double)bv[j] * (double)bv[j];
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T bv = b[i];
      x[i] = T(0); r[i] = bv; p[i] = p_zero ? T(0) : bv;
      acc = acc + (double)bv * (double)bv;
    }
  const double s = block_sum<BS>(acc, red);
  if (tk.cnt1) {
    __syncthreads();
    ticket_finish<BS>(s, tk, red);
  } else if (threadIdx.x == 0 && part) {
    part[blockIdx.x] = s;
  }
}

// x = 0, r = b, p = s = 0; part = b.b partials (CG1 prologue)
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_init_cg1(int n, const T *__restrict__ b,
                                                 T *__restrict__ x,
                                                 T *__restrict__ r,
                                                 T *__restrict__ p,
                                                 T *__restrict__ s,
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
      x[i] = T(0); p[i] = T(0); s[i] = T(0); r[i] = bv;
      acc = acc + (double)bv * (double)bv;
    }
  const double sum = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// x += alpha*p (cg.c:115-118); r -= alpha*s (cg.c:122-123); part = r.r
template <typename T, int BS, bool XNT = false>
__global__ __launch_bounds__(BS) void k_update_xr(int n, T *__restrict__ x,
                                                  const T *__restrict__ p,
                                                  T *__restrict__ r,
                                                  const T *__restrict__ s,
                                                  const CgState *__restrict__ st,
                                                  double *__restrict__ part,
                                                  TicketArgs tk) {
  __shared__ double red[BS / kWave];
  if (st->done) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const T alpha = (T)st->alpha;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  double acc = 0.0;
  for (int i = gid; i < nv; i += stride) {
    // XNT: x is touched only here -- keep it out of the Infinity Cache so
    // p, r and Ap (read again within the iteration) stay resident
    V xv = XNT ? __builtin_nontemporal_load(reinterpret_cast<const V *>(x) + i)
               : reinterpret_cast<const V *>(x)[i];
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
    if (XNT) __builtin_nontemporal_store(xv, reinterpret_cast<V *>(x) + i);
    else reinterpret_cast<V *>(x)[i] = xv;
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
  if (part || tk.cnt1) {
    const double sum = block_sum<BS>(acc, red);
    if (tk.cnt1) {
      __syncthreads();
      ticket_finish<BS>(sum, tk, red);
    } else if (threadIdx.x == 0) {
      part[blockIdx.x] = sum;
    }
  }
}

// p = r + beta*p (cg.c:131-132)
template <int BS>
__device__ __forceinline__ double sum_parts(const double *pa, int na,
                                            double *red) {
  // Thread t adds pa[t], pa[t+BS], pa[t+2BS], ... in index order.  All of a
  // thread's loads (up to U) are issued before the first add, so a 40K-entry
  // partial array costs one memory round trip, not one per 16 entries.
  constexpr int U = 48;
  double acc = 0.0;
  int i = threadIdx.x;
  bool first = true;
  for (; i < na; i += U * BS) {
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
__device__ __forceinline__ void sum_parts2(const double *pa, int na, const double *pb,
                                           int nb, double *red, double &sa, double &sb) {
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

// Folded HS (CGX_FOLD): no finalize kernels.  Every workgroup of the vector
// kernels sums the previous kernel's partials itself -- the same
// sum_parts<1024> order as k_finalize<1024>, so alpha, beta and the stop test
// are bit-identical to the finalize path -- and workgroup 0 publishes the
// state for later kernels.  A kernel never writes a field its own workgroups
// read: k_update_rf reads rr_x / k_x and writes rr_u / k_u / alpha;
// k_xpay_xf reads rr_u / k_u / alpha and writes rr_x / k_x / rr / k / beta /
// done.  The stop flag: k_xpay_xf sets 1 after the stop iteration's x update,
// the next k_update_rf turns it into 2; only 2 stops k_xpay_xf (a 1 seen
// there was written by its own workgroup 0 during this launch).
constexpr int kFoldBS = 1024;

// PF: the first grid-stride element's loads are issued before the partial
// sum, so the HBM round trip overlaps the L2 round trip of the partials
// (same elements, same order: bit-identical).
template <typename T, bool PF>
__global__ __launch_bounds__(kFoldBS) void k_update_rf(int n, T *__restrict__ r,
                                                       const T *__restrict__ s,
                                                       CgState *__restrict__ st,
                                                       const double *__restrict__ ps_part,
                                                       int nps, double *__restrict__ rr_part) {
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
  if (PF && gid < nv) {
    rv0 = reinterpret_cast<const V *>(r)[gid];
    sv0 = reinterpret_cast<const V *>(s)[gid];
  }
  const double ps = sum_parts<kFoldBS>(ps_part, nps, red);
  if (threadIdx.x == 0) {
    const double rr = st->rr_x;
    const double alpha = rr / ps;  // cg.c:113
    bcast = alpha;
    if (blockIdx.x == 0) {
      st->ps = ps;
      st->alpha = alpha;
      st->rr_u = rr;
      st->k_u = st->k_x;
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
    reinterpret_cast<V *>(r)[i] = rv;
  };
  int i = gid;
  if (PF && i < nv) {
    step(i, rv0, sv0);
    i += stride;
  }
  for (; i < nv; i += stride)
    step(i, reinterpret_cast<const V *>(r)[i], reinterpret_cast<const V *>(s)[i]);
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T as = alpha * s[i];
      const T ri = r[i] - as;
      r[i] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  // one partial per 256-thread quarter, reduced exactly as block_sum<256>:
  // the same terms per partial and the same order as k_update_r<T, 256>, so
  // r.r (and beta) match the finalize path bit for bit
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
}

template <typename T, bool PF>
__global__ __launch_bounds__(kFoldBS) void k_xpay_xf(int n, T *__restrict__ x,
                                                     T *__restrict__ p,
                                                     const T *__restrict__ r,
                                                     CgState *__restrict__ st,
                                                     const double *__restrict__ rr_part,
                                                     int nrr, double *__restrict__ hist) {
  __shared__ double red[kFoldBS / kWave];
  __shared__ double bcast;
  __shared__ int bstop;
  if (st->done > 1) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const int nv = n / W;
  const int gid = blockIdx.x * kFoldBS + threadIdx.x, stride = gridDim.x * kFoldBS;
  V pv0 = V(), xv0 = V(), rv0 = V();
  if (PF && gid < nv) {
    pv0 = reinterpret_cast<const V *>(p)[gid];
    xv0 = reinterpret_cast<const V *>(x)[gid];
    rv0 = reinterpret_cast<const V *>(r)[gid];
  }
  const double rr_new = sum_parts<kFoldBS>(rr_part, nrr, red);
  if (threadIdx.x == 0) {
    const int k = st->k_u;
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
      }
    }
  }
  __syncthreads();
  const bool stop = bstop != 0;
  const T alpha = (T)st->alpha, beta = (T)bcast;
  auto step = [&](int i, V pv, V xv, const V rv) {
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T ap = alpha * pv[j];
      xv[j] = xv[j] + ap;
    }
    reinterpret_cast<V *>(x)[i] = xv;
    if (!stop) {
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T bp = beta * pv[j];
        pv[j] = rv[j] + bp;
      }
      reinterpret_cast<V *>(p)[i] = pv;
    }
  };
  int i = gid;
  if (PF && i < nv) {
    step(i, pv0, xv0, rv0);
    i += stride;
  }
  for (; i < nv; i += stride) {
    const V pv = reinterpret_cast<const V *>(p)[i];
    const V xv = reinterpret_cast<const V *>(x)[i];
    step(i, pv, xv, stop ? V() : reinterpret_cast<const V *>(r)[i]);
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T pi = p[i];
      const T ap = alpha * pi;
      x[i] = x[i] + ap;
      if (!stop) {
        const T bp = beta * pi;
        p[i] = r[i] + bp;
      }
    }
}

// Deferred-x HS (CGX_XDEFER): x += alpha p moves from the r-update into the
// p-update, which reads p_old anyway -- one 8n-byte read of p less per
// iteration.  Same per-element roundings as k_update_xr / k_xpay.
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_update_r(int n, T *__restrict__ r,
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
    V rv = reinterpret_cast<const V *>(r)[i];
    const V sv = reinterpret_cast<const V *>(s)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T as = alpha * sv[j];
      rv[j] = rv[j] - as;
      acc = acc + (double)rv[j] * (double)rv[j];
    }
    reinterpret_cast<V *>(r)[i] = rv;
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T as = alpha * s[i];
      const T ri = r[i] - as;
      r[i] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  const double sum = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// stop flag 0: x += alpha p_old, p = r + beta p_old; 1 (stopped in this
// iteration, cg.c:125 breaks after the x update): x only; 2: nothing.
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_xpay_x(int n, T *__restrict__ x,
                                               T *__restrict__ p,
                                               const T *__restrict__ r,
                                               const CgState *__restrict__ st) {
  const int done = st->done;
  if (done > 1) return;
  typedef typename Vec16<T>::type V;
  constexpr int W = Vec16<T>::W;
  const T alpha = (T)st->alpha, beta = (T)st->beta;
  const int nv = n / W;
  const int gid = blockIdx.x * BS + threadIdx.x, stride = gridDim.x * BS;
  for (int i = gid; i < nv; i += stride) {
    V pv = reinterpret_cast<const V *>(p)[i];
    V xv = reinterpret_cast<const V *>(x)[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const T ap = alpha * pv[j];
      xv[j] = xv[j] + ap;
    }
    reinterpret_cast<V *>(x)[i] = xv;
    if (done == 0) {
      const V rv = reinterpret_cast<const V *>(r)[i];
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const T bp = beta * pv[j];
        pv[j] = rv[j] + bp;
      }
      reinterpret_cast<V *>(p)[i] = pv;
    }
  }
  if (gid == 0)
    for (int i = nv * W; i < n; ++i) {
      const T pi = p[i];
      const T ap = alpha * pi;
      x[i] = x[i] + ap;
      if (done == 0) {
        const T bp = beta * pi;
        p[i] = r[i] + bp;
      }
    }
}

template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_xpay(int n, T *__restrict__ p,
                                             const T *__restrict__ r,
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

// Chronopoulos-Gear update: p = r + beta p; s = w + beta s; x += alpha p;
// r -= alpha s; part = r.r (gamma of the next iteration).
template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_cg1_update(int n, T *__restrict__ x,
                                                   T *__restrict__ p,
                                                   T *__restrict__ r,
                                                   T *__restrict__ s,
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
      p[i] = pi; s[i] = si; r[i] = ri;
      acc = acc + (double)ri * (double)ri;
    }
  const double sum = block_sum<BS>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// Exact-order dot (dot_product, mv_ops.c:128-129): products are formed in
// parallel (each rounded, as the reference does), lane 0 adds them strictly
// in index order starting from 0.0.  O(n) serial -- parity mode only.
template <typename T>
__global__ __launch_bounds__(kWave) void k_dot_seq(int n, const T *__restrict__ a,
                                                   const T *__restrict__ b,
                                                   double *__restrict__ out,
                                                   const int *__restrict__ done) {
  // The sum is one dependent add chain (the reference's order, mv_ops.c:
  // 127-129); the products of the NEXT chunk are loaded while lane 0 adds the
  // current one, so HBM latency hides behind the chain.
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
    if (base + CH < n) load(base + CH);  // in flight during the adds below
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

// Fixed-order sum of na partials by one workgroup (thread t adds
// pa[t], pa[t+BS], ... in order; then the block tree).  Starts from the first
// partial, so a single partial (exact mode) passes through unchanged.

template <int BS>
__global__ __launch_bounds__(BS) void k_finalize(int op, const double *pa, int na,
                                                 const double *pb, int nb,
                                                 CgState *st, double *hist,
                                                 double *out) {
  __shared__ double red[BS / kWave];
  // partial loads go out before the done-flag round trip; with two partial
  // arrays, both arrays' loads are in flight together (one round trip)
  double sa, sb = 0.0;
  if (pb) sum_parts2<BS>(pa, na, pb, nb, red, sa, sb);
  else sa = sum_parts<BS>(pa, na, red);
  if (threadIdx.x != 0) return;
  if (op == FIN_HS_ALPHA_X) {
    // one thread, so the 1 -> 2 step cannot race: k_xpay_x of the stop
    // iteration (flag 1) has applied the last x update, later ones must not
    if (st->done) {
      if (st->done == 1) st->done = 2;
      return;
    }
    op = FIN_HS_ALPHA;
  }
  if (op != FIN_SUM && op != FIN_SUM2 && op != FIN_INIT_HS &&
      op != FIN_INIT_CG1 && st->done)
    return;
  apply_fin(op, sa, sb, st, hist, out);
}

template <typename T, int BS>
__global__ __launch_bounds__(BS) void k_axpby(int op, int n, double sc,
                                              const T *__restrict__ a,
                                              const T *__restrict__ b,
                                              T *__restrict__ r) {
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
__global__ void k_group_sum(const double *const *srcs, int P, int count,
                            double *dst, int off) {
  const int c = threadIdx.x + off;
  if (threadIdx.x >= count) return;
  double acc = srcs[0][c];
  for (int q = 1; q < P; ++q) acc = acc + srcs[q][c];
  dst[c] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather(int m, const int *__restrict__ idx,
                                                const T *__restrict__ x,
                                                T *__restrict__ buf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m) buf[i] = x[idx[i]];
}

}  // namespace

// ------------------------------------------------------------- launchers

template <typename T, int BS>
static void launch_spmv_bs(const SpmvArgs<T> &a, int grid, int vec,
                           hipStream_t st) {
  constexpr int CAP = BS * (sizeof(T) == 8 ? 8 : 16);  // 16 KiB LDS per 256 lanes
  const bool epi = a.part != nullptr;
#define CGX_SPMV(V, E, N)                                                      \
  hipLaunchKernelGGL((k_spmv<T, BS, CAP, V, E, N>), dim3(grid), dim3(BS), 0,  \
                     st, a)
#define CGX_SPMV_V(V)                                                          \
  do {                                                                         \
    if (a.nt) {                                                                \
      if (epi) CGX_SPMV(V, true, true); else CGX_SPMV(V, false, true);        \
    } else {                                                                   \
      if (epi) CGX_SPMV(V, true, false); else CGX_SPMV(V, false, false);      \
    }                                                                          \
  } while (0)
  if (vec == 4) CGX_SPMV_V(4);
  else if (vec == 2) CGX_SPMV_V(2);
  else CGX_SPMV_V(1);
#undef CGX_SPMV_V
#undef CGX_SPMV
}

template <typename T, int WPB>
static void launch_spmv_wave(const SpmvArgs<T> &a, int vec, hipStream_t st) {
  constexpr int CAPW = sizeof(T) == 8 ? 512 : 1024;  // 4 KiB LDS per wave
  const int per = WPB * (a.rbw < 1 ? 1 : a.rbw);
  const int grid = (a.nblk + per - 1) / per;
  const bool epi = a.part != nullptr;
  const bool xpay = a.x2 != nullptr;
#define CGX_SPMVW(V, E, N, X, G)                                               \
  hipLaunchKernelGGL((k_spmv_wave<T, WPB, CAPW, V, E, N, X, G>), dim3(grid),     \
                     dim3(WPB * kWave), 0, st, a)
#define CGX_SPMVW_G(V, N, X)                                                     \
  do {                                                                           \
    if (a.tg) {                                                                  \
      if (epi) CGX_SPMVW(V, true, N, X, true); else CGX_SPMVW(V, false, N, X, true); \
    } else {                                                                     \
      if (epi) CGX_SPMVW(V, true, N, X, false); else CGX_SPMVW(V, false, N, X, false); \
    }                                                                            \
  } while (0)
#define CGX_SPMVW_X(V, N)                                                      \
  do {                                                                         \
    if (xpay) CGX_SPMVW_G(V, N, true); else CGX_SPMVW_G(V, N, false);         \
  } while (0)
#define CGX_SPMVW_V(V)                                                         \
  do {                                                                         \
    if (a.nt) CGX_SPMVW_X(V, true); else CGX_SPMVW_X(V, false);               \
  } while (0)
  if (vec == 4) CGX_SPMVW_V(4);
  else if (vec == 2) CGX_SPMVW_V(2);
  else CGX_SPMVW_V(1);
#undef CGX_SPMVW_V
#undef CGX_SPMVW_X
#undef CGX_SPMVW_G
#undef CGX_SPMVW
}

template <typename T>
hipError_t launch_spmv(const SpmvArgs<T> &a, int grid, int vec, hipStream_t st) {
  if (a.s_off) {  // SELL-64 layout
    if (a.nslices <= 0) return hipSuccess;
    constexpr int WPB = 4;
    const int g = (a.nslices + WPB - 1) / WPB;
    const bool epi = a.part != nullptr, xp = a.x2 != nullptr;
    if (epi && xp) hipLaunchKernelGGL((k_spmv_sell<T, WPB, true, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi) hipLaunchKernelGGL((k_spmv_sell<T, WPB, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (xp) hipLaunchKernelGGL((k_spmv_sell<T, WPB, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else hipLaunchKernelGGL((k_spmv_sell<T, WPB, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    return hipGetLastError();
  }
  if (a.nblk <= 0) return hipSuccess;
  if (a.code) {  // dictionary-coded columns (k_spmv_dc)
    if (a.bs != 64 || a.dma != 1 || a.x2 || a.yacc) return hipErrorInvalidValue;
    if (a.dval) {  // value-indexed pairs (k_spmv_vi)
      if (!a.rlen || a.ndict_cap > 64 || a.wpb != 4) return hipErrorInvalidValue;
      if constexpr (sizeof(T) == 4) {
        launch_vi<T, 1024>(a, st);
      } else {
        if (a.capw == 328) launch_vi<T, 328>(a, st);
        else if (a.capw == 0 || a.capw == 512) launch_vi<T, 512>(a, st);
        else return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    if (sizeof(T) == 4) launch_dc_w<T, 1024>(a, st);
    else if (a.capw == 328) launch_dc_w<T, 328>(a, st);
    else if (a.capw == 0 || a.capw == 512) launch_dc_w<T, 512>(a, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma == 5 && sizeof(T) == 8 && !a.blk_list && !a.x2) {  // DMA engine
    SpmvArgs<double> b;
    memcpy(&b, &a, sizeof b);
    const int g = grid > 0 ? grid : 1;
    switch (a.rbw) {
      case 1: launch_eng<3, 6, 3>(b, g, st); break;
      case 2: launch_eng<7, 12, 5>(b, g, st); break;
      case 3: launch_eng<7, 12, 9>(b, g, st); break;
      case 4: launch_eng<7, 12, 10, true>(b, g, st); break;
      case 5: launch_eng<5, 12, 10, true>(b, g, st); break;
      case 6: launch_eng<7, 12, 8, true>(b, g, st); break;
      case 7: launch_eng<11, 12, 10, true>(b, g, st); break;
      default: launch_eng<3, 8, 6>(b, g, st); break;
    }
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma == 2 && !a.blk_list && !a.x2) {  // pipelined LDS-DMA
    constexpr int WPB = 2;
    constexpr int CAPW = sizeof(T) == 8 ? 512 : 1024;
    const int per = WPB * (a.rbw < 1 ? 1 : a.rbw);
    const int g = (a.nblk + per - 1) / per;
    if (a.part) hipLaunchKernelGGL((k_spmv_pipe<T, WPB, CAPW, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else hipLaunchKernelGGL((k_spmv_pipe<T, WPB, CAPW, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma == 4) {  // 32-row blocks, 3 KiB windows: 2x the waves per CU
    constexpr int WPB = 4;
    constexpr int CAPW = sizeof(T) == 8 ? 256 : 512;
    const int g = (a.nblk + WPB - 1) / WPB;
    const bool epi = a.part != nullptr;
    if (a.x2) return hipErrorInvalidValue;  // no fused p-update in this variant
    if (epi && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma == 1 && a.wpb == 8 && !a.x2) {  // 8 waves: half the partials
    constexpr int WPB = 8;
    constexpr int CAPW = sizeof(T) == 8 ? 512 : 1024;
    const int g = (a.nblk + WPB - 1) / WPB;
    const bool epi = a.part != nullptr;
    if (epi && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma == 1 && (a.capw == 456 || a.capw == 328) && sizeof(T) == 8 &&
      !a.x2) {
    // smaller windows, sized to the matrix's row blocks (456 = a 7-point
    // block's 448 + alignment, 328 = a 5-point block's 320 + alignment):
    // less LDS per wave, more waves per CU
    constexpr int WPB = 4;
    const int g = (a.nblk + WPB - 1) / WPB;
    const bool epi = a.part != nullptr;
    if (a.capw == 456) {
      constexpr int CAPW = 456;
      if (epi && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else if (epi) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else if (a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    } else {
      constexpr int CAPW = 328;
      if (epi && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else if (epi) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else if (a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
      else hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    }
    return hipGetLastError();
  }
  if (a.bs == 64 && a.dma) {
    constexpr int WPB = 4;
    constexpr int CAPW = sizeof(T) == 8 ? 512 : 1024;
    const int g = (a.nblk + WPB - 1) / WPB;
    const bool epi = a.part != nullptr, xp = a.x2 != nullptr;
    if (epi && xp) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi && a.dma == 3 && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true, 4, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi && a.dma == 8 && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true, 8>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi && a.dma == 8) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, false, 8>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (!xp && a.dma == 8 && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true, 8>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (!xp && a.dma == 8) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, false, 8>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (epi) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, true, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (!xp && a.nt) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else if (xp) hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, true>), dim3(g), dim3(WPB * kWave), 0, st, a);
    else hipLaunchKernelGGL((k_spmv_dma<T, WPB, CAPW, false, false>), dim3(g), dim3(WPB * kWave), 0, st, a);
    return hipGetLastError();
  }
  if (a.bs == 64) {
    if (a.wpb == 8) launch_spmv_wave<T, 8>(a, vec, st);
    else launch_spmv_wave<T, 4>(a, vec, st);
    return hipGetLastError();
  }
  if (a.x2) return hipErrorInvalidValue;  // fused xpay: wave kernel only
  grid = grid < 1 ? 1 : (grid > a.nblk ? a.nblk : grid);
  if (a.bs == 512) launch_spmv_bs<T, 512>(a, grid, vec, st);
  else launch_spmv_bs<T, 256>(a, grid, vec, st);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_hs(int n, const T *b, T *x, T *r, T *p, double *part,
                          int grid, hipStream_t st, bool p_zero,
                          const TicketArgs *tk) {
  TicketArgs t = tk ? *tk : TicketArgs{};
  hipLaunchKernelGGL((k_init_hs<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n,
                     b, x, r, p, part, p_zero ? 1 : 0, t);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_cg1(int n, const T *b, T *x, T *r, T *p, T *s,
                           double *part, int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_init_cg1<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st,
                     n, b, x, r, p, s, part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_xr(int n, T *x, const T *p, T *r, const T *s,
                            const CgState *stt, double *part, int grid,
                            hipStream_t st, const TicketArgs *tk) {
  TicketArgs t = tk ? *tk : TicketArgs{};
  static const bool xnt = env_int("CGX_VEC_XNT", 0) != 0;
  if (xnt)
    hipLaunchKernelGGL((k_update_xr<T, kVecBS, true>), dim3(grid), dim3(kVecBS), 0, st,
                       n, x, p, r, s, stt, part, t);
  else
    hipLaunchKernelGGL((k_update_xr<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st,
                       n, x, p, r, s, stt, part, t);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_xpay(int n, T *p, const T *r, const CgState *stt, int grid,
                       hipStream_t st) {
  hipLaunchKernelGGL((k_xpay<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, p,
                     r, stt);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_r(int n, T *r, const T *s, const CgState *stt,
                           double *part, int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_update_r<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, r,
                     s, stt, part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_xpay_x(int n, T *x, T *p, const T *r, const CgState *stt,
                         int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_xpay_x<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, n, x,
                     p, r, stt);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_update_rf(int n, T *r, const T *s, CgState *stt, const double *ps_part,
                            int nps, double *rr_part, int grid, hipStream_t st, bool pf) {
  if (pf)
    hipLaunchKernelGGL((k_update_rf<T, true>), dim3(grid), dim3(kFoldBS), 0, st, n, r, s, stt,
                       ps_part, nps, rr_part);
  else
    hipLaunchKernelGGL((k_update_rf<T, false>), dim3(grid), dim3(kFoldBS), 0, st, n, r, s, stt,
                       ps_part, nps, rr_part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_xpay_xf(int n, T *x, T *p, const T *r, CgState *stt,
                          const double *rr_part, int nrr, double *hist, int grid,
                          hipStream_t st, bool pf) {
  if (pf)
    hipLaunchKernelGGL((k_xpay_xf<T, true>), dim3(grid), dim3(kFoldBS), 0, st, n, x, p, r, stt,
                       rr_part, nrr, hist);
  else
    hipLaunchKernelGGL((k_xpay_xf<T, false>), dim3(grid), dim3(kFoldBS), 0, st, n, x, p, r, stt,
                       rr_part, nrr, hist);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_cg1_update(int n, T *x, T *p, T *r, T *s, const T *w,
                             const CgState *stt, double *part, int grid,
                             hipStream_t st) {
  hipLaunchKernelGGL((k_cg1_update<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st,
                     n, x, p, r, s, w, stt, part);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dot_seq(int n, const T *a, const T *b, double *out,
                          const int *done, hipStream_t st) {
  hipLaunchKernelGGL((k_dot_seq<T>), dim3(1), dim3(kWave), 0, st, n, a, b, out,
                     done);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dot_part(int n, const T *a, const T *b, double *part,
                           int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_dot_part<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st,
                     n, a, b, part);
  return hipGetLastError();
}

hipError_t launch_finalize(int op, const double *pa, int na, const double *pb,
                           int nb, CgState *stt, double *hist, double *out,
                           hipStream_t st) {
  hipLaunchKernelGGL((k_finalize<kFinBS>), dim3(1), dim3(kFinBS), 0, st, op, pa,
                     na, pb, nb, stt, hist, out);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_axpby(int op, int n, double s, const T *a, const T *b, T *r,
                        int grid, hipStream_t st) {
  hipLaunchKernelGGL((k_axpby<T, kVecBS>), dim3(grid), dim3(kVecBS), 0, st, op,
                     n, s, a, b, r);
  return hipGetLastError();
}

hipError_t launch_group_sum(const double *const *srcs, int P, int count,
                            double *dst, hipStream_t st, int off) {
  hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, st, srcs, P, count, dst, off);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_gather(int m, const int *idx, const T *x, T *buf,
                         hipStream_t st) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_gather<T>), dim3((m + 255) / 256), dim3(256), 0, st, m,
                     idx, x, buf);
  return hipGetLastError();
}

// STREAM triad a = b + s c (fp64, 16 B per lane per array, grid-stride):
// the on-box ceiling the SpMV and vector kernels are compared with.
__global__ __launch_bounds__(256) void k_triad(long long n2, double2 *__restrict__ a,
                                               const double2 *__restrict__ b,
                                               const double2 *__restrict__ c, double sc) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256) {
    const double2 bv = b[i], cv = c[i];
    a[i] = make_double2(bv.x + sc * cv.x, bv.y + sc * cv.y);
  }
}

__global__ __launch_bounds__(256) void k_stream_read(long long n2,
                                                     const double2 *__restrict__ b,
                                                     double *__restrict__ sink) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256) {
    const double2 v = b[i];
    acc += v.x + v.y;
  }
  if (acc == 1.2345e300) sink[0] = acc;  // keeps the loads; never true
}

hipError_t launch_stream_read(long long n2, const double *b, double *sink, int grid,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, st, n2,
                     (const double2 *)b, sink);
  return hipGetLastError();
}

hipError_t launch_triad(long long n2, double *a, const double *b, const double *c,
                        int grid, hipStream_t st) {
  hipLaunchKernelGGL(k_triad, dim3(grid), dim3(256), 0, st, n2, (double2 *)a,
                     (const double2 *)b, (const double2 *)c, 3.0);
  return hipGetLastError();
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

hipError_t launch_gen_laplacian(const LapSpec &g, int n, int *col, double *val,
                                hipStream_t st) {
  const int grid = std::max(1, std::min((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_gen_laplacian, dim3(grid), dim3(256), 0, st, g, n, col, val);
  return hipGetLastError();
}

// Coded columns for a matrix already in device memory (the generated
// Laplacian): row r's entries get the position of col - r in the sorted
// dictionary; an offset missing from it raises *err.
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

hipError_t launch_dc_encode(int n, const int *rp, const int *col, const int *dict, int nd,
                            unsigned char *code, int *err, hipStream_t st,
                            const double *val, const double *dval) {
  const int grid = std::max(1, std::min((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_dc_encode, dim3(grid), dim3(256), 0, st, n, rp, col, dict, nd, code, err,
                     val, dval);
  return hipGetLastError();
}

// Matrix-free SpMV of the same operator: row r sums its products in the CSR
// row's column order from 0 with the same values (-1 products are exact), so
// y is bit-identical to the CSR SpMV.  Only x (once, coalesced along rows)
// and y move: the upper bound SURVEY.md 8f asks for beside the CSR runs.
template <typename T, bool EPI>
__global__ __launch_bounds__(256) void k_stencil(LapSpec g, int n, const T *__restrict__ x,
                                                 T *__restrict__ y, double *__restrict__ part,
                                                 const int *done) {
  __shared__ double red[256 / kWave];
  if (done && *done) return;
  const int nx = g.nx, ny = g.ny, pl = g.nx * g.ny;
  const T m1 = T(-1), dg = T(g.dim == 3 ? 6 : 4);
  double dot = 0.0;
  // one row per thread: XCD-contiguous workgroup order, so each XCD sweeps a
  // contiguous slab and the +-plane x lines stay in its L2
  const bool once = (long long)gridDim.x * 256 >= n;
  const int b0 = once ? xcd_block(1) : blockIdx.x;
  for (int r = b0 * 256 + threadIdx.x; r < n; r += gridDim.x * 256) {
    const int i = r % nx, j = (r / nx) % ny, l = r / pl;
    T acc = T(0);
    if (g.dim == 3 && l > 0) acc = acc + m1 * x[r - pl];
    if (j > 0) acc = acc + m1 * x[r - nx];
    if (i > 0) acc = acc + m1 * x[r - 1];
    const T xr = x[r];
    acc = acc + dg * xr;
    if (i < nx - 1) acc = acc + m1 * x[r + 1];
    if (j < ny - 1) acc = acc + m1 * x[r + nx];
    if (g.dim == 3 && l < g.nz - 1) acc = acc + m1 * x[r + pl];
    y[r] = acc;
    if (EPI) dot = dot + (double)xr * (double)acc;
  }
  if (EPI) {
    const double sum = block_sum<256>(dot, red);
    if (threadIdx.x == 0) part[blockIdx.x] = sum;
  }
}

template <typename T>
hipError_t launch_stencil(const LapSpec &g, int n, const T *x, T *y, double *part,
                          const int *done, int grid, hipStream_t st) {
  if (part)
    hipLaunchKernelGGL((k_stencil<T, true>), dim3(grid), dim3(256), 0, st, g, n, x, y, part,
                       done);
  else
    hipLaunchKernelGGL((k_stencil<T, false>), dim3(grid), dim3(256), 0, st, g, n, x, y,
                       part, done);
  return hipGetLastError();
}

#define CGX_INSTANTIATE(T)                                                     \
  template hipError_t launch_spmv<T>(const SpmvArgs<T> &, int, int,           \
                                     hipStream_t);                             \
  template hipError_t launch_init_hs<T>(int, const T *, T *, T *, T *,        \
                                        double *, int, hipStream_t, bool,      \
                                        const TicketArgs *);                   \
  template hipError_t launch_init_cg1<T>(int, const T *, T *, T *, T *, T *,  \
                                         double *, int, hipStream_t);          \
  template hipError_t launch_update_xr<T>(int, T *, const T *, T *,           \
                                          const T *, const CgState *,         \
                                          double *, int, hipStream_t,         \
                                          const TicketArgs *);                 \
  template hipError_t launch_xpay<T>(int, T *, const T *, const CgState *,    \
                                     int, hipStream_t);                        \
  template hipError_t launch_update_r<T>(int, T *, const T *, const CgState *,\
                                         double *, int, hipStream_t);          \
  template hipError_t launch_xpay_x<T>(int, T *, T *, const T *,              \
                                       const CgState *, int, hipStream_t);     \
  template hipError_t launch_stencil<T>(const LapSpec &, int, const T *, T *, \
                                        double *, const int *, int,            \
                                        hipStream_t);                          \
  template hipError_t launch_update_rf<T>(int, T *, const T *, CgState *,     \
                                          const double *, int, double *, int,  \
                                          hipStream_t, bool);                  \
  template hipError_t launch_xpay_xf<T>(int, T *, T *, const T *, CgState *,  \
                                        const double *, int, double *, int,    \
                                        hipStream_t, bool);                    \
  template hipError_t launch_cg1_update<T>(int, T *, T *, T *, T *,           \
                                           const T *, const CgState *,        \
                                           double *, int, hipStream_t);        \
  template hipError_t launch_dot_seq<T>(int, const T *, const T *, double *,  \
                                        const int *, hipStream_t);             \
  template hipError_t launch_dot_part<T>(int, const T *, const T *, double *, \
                                         int, hipStream_t);                    \
  template hipError_t launch_axpby<T>(int, int, double, const T *, const T *, \
                                      T *, int, hipStream_t);                  \
  template hipError_t launch_gather<T>(int, const int *, const T *, T *,      \
                                       hipStream_t);

CGX_INSTANTIATE(double)
CGX_INSTANTIATE(float)

}  // namespace cgx
