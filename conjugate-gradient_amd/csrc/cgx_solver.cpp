// cgx_solver.cpp -- device-resident CG solver: HIP-stream orchestration of the
// iteration that replaces conj_grad's loop (rnelias/Conjugate-Gradient
// cg.c:88-141).  The whole recurrence state (alpha, beta, r.r, k, stop flag)
// lives on the device in a CgState, so an iteration is a fixed sequence of
// kernel launches with no host round trip; batches of iterations are replayed
// as hipGraphs, and the host only polls the stop flag between batches when a
// tolerance is set.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cgx_internal.h"

using cgx::CgState;

namespace cgx {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

std::vector<int> plan_rowblocks(int n, const int *rp, int rows, int cap) {
  std::vector<int> blk;
  blk.reserve((size_t)n / 128 + 2);
  blk.push_back(0);
  int r = 0;
  while (r < n) {
    const int start = r;
    const int k0 = rp[r];
    if (rp[r + 1] - k0 > cap) {  // long row: a block of its own
      blk.push_back(++r);
      continue;
    }
    while (r < n && r - start < rows && rp[r + 1] - k0 <= cap) ++r;
    blk.push_back(r);
  }
  return blk;
}

// Column panels for matrices whose gathers have no locality (SURVEY.md C5:
// random SPD).  x is read through per-XCD L2s of 4 MiB; when x is larger and
// most entries lie far from the diagonal, every gather is a line fetched from
// the Infinity Cache.  Splitting the columns into panels whose x slice fits
// an L2 and running one SpMV pass per panel keeps the gathers L2-resident,
// for P row_ptr reads and P-1 y round trips more.  Auto-selected when x >
// 8 MiB and >= 30 % of (sampled) entries are more than a panel width from the
// diagonal; CGX_LAYOUT=panel forces, CGX_LAYOUT=csr disables;
// CGX_PANEL_KB sets the x bytes per panel (default 2048).
int choose_panels(int n, const int *rp, const int *col, size_t tsize) {
  const char *l = getenv("CGX_LAYOUT");
  if (n <= 0 || (l && strcmp(l, "panel") != 0)) return 1;  // csr / sell
  const long long pcols =
      std::max<long long>(1024, (long long)env_int("CGX_PANEL_KB", 2048) * 1024 / (long long)tsize);
  if (n <= pcols) return 1;
  if (!l) {
    if ((double)n * (double)tsize <= 8.0 * 1024 * 1024) return 1;
    long long far = 0, tot = 0;
    for (int i = 0; i < n; i += 61)
      for (int k = rp[i]; k < rp[i + 1]; ++k) {
        ++tot;
        far += std::llabs((long long)col[k] - i) > pcols;
      }
    if (far * 10 < tot * 3) return 1;
  }
  return (int)std::min<long long>(64, (n + pcols - 1) / pcols);
}

// The adaptive LDS window applies to plain CSR only (column panels plan
// their own blocks).
bool gen_panels_pending(int n, const int *rp, const int *col, const void *gen) {
  return !gen && col && choose_panels(n, rp, col, 8) > 1;
}

// Panel-major CSR: panel q holds, for every row, the row's entries with
// column in [q*pc, (q+1)*pc), in the row's order; prp[q*(n+1) + i] are
// offsets into the concatenated col/val (panel q's block starts at base q).
template <typename T>
void build_panels(int n, const int *rp, const int *col, const T *val, int P,
                  std::vector<int> &prp, std::vector<int> &pcol, std::vector<T> &pval) {
  const int nnz = rp[n];
  const long long pc = ((long long)n + P - 1) / P;
  std::vector<long long> base((size_t)P + 1, 0);
  for (int k = 0; k < nnz; ++k) base[(size_t)(col[k] / pc) + 1]++;
  for (int q = 0; q < P; ++q) base[q + 1] += base[q];
  prp.assign((size_t)P * ((size_t)n + 1), 0);
  std::vector<int> cnt((size_t)P);
  for (int q = 0; q < P; ++q) prp[(size_t)q * (n + 1)] = (int)base[q];
  for (int i = 0; i < n; ++i) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int k = rp[i]; k < rp[i + 1]; ++k) cnt[(size_t)(col[k] / pc)]++;
    for (int q = 0; q < P; ++q) {
      const size_t o = (size_t)q * (n + 1) + i;
      prp[o + 1] = prp[o] + cnt[q];
    }
  }
  pcol.resize((size_t)nnz);
  pval.resize((size_t)nnz);
  std::vector<int> cur((size_t)P);
  for (int i = 0; i < n; ++i) {
    for (int q = 0; q < P; ++q) cur[q] = prp[(size_t)q * (n + 1) + i];
    for (int k = rp[i]; k < rp[i + 1]; ++k) {
      const int q = (int)(col[k] / pc);
      pcol[(size_t)cur[q]] = col[k];
      pval[(size_t)cur[q]++] = val[k];
    }
  }
}

// SELL-64: slice i = rows [64i, 64i+64), width = its longest row, element
// (j, lane) at 64*(s_off[i] + j) + lane.  Padding (val 0, col = the row)
// follows each row's entries.  Returns false (use CSR) when the padded size
// exceeds max_pad * nnz, i.e. for irregular row lengths.
template <typename T>
bool csr_to_sell64(int n, const int *rp, const int *col, const T *val,
                   double max_pad, std::vector<int> &s_off,
                   std::vector<int> &s_len, std::vector<T> &sval,
                   std::vector<int> &scol) {
  const int nsl = (n + 63) / 64;
  s_off.assign((size_t)nsl + 1, 0);
  s_len.assign((size_t)nsl, 0);
  long long tot = 0;  // in units of 64 elements
  for (int i = 0; i < nsl; ++i) {
    int w = 0;
    for (int r = 64 * i; r < std::min(n, 64 * i + 64); ++r)
      w = std::max(w, rp[r + 1] - rp[r]);
    s_len[i] = w;
    s_off[i] = (int)tot;
    tot += w;
    if (tot > INT32_MAX) return false;
  }
  s_off[nsl] = (int)tot;
  const long long nnz = n > 0 ? rp[n] : 0;
  if ((double)tot * 64 > max_pad * (double)std::max<long long>(nnz, 1) + 64.0 * nsl)
    return false;
  sval.assign((size_t)tot * 64, T(0));
  scol.assign((size_t)tot * 64, 0);
  for (int i = 0; i < nsl; ++i)
    for (int lane = 0; lane < 64; ++lane) {
      const int r = 64 * i + lane;
      const int len = r < n ? rp[r + 1] - rp[r] : 0;
      for (int j = 0; j < s_len[i]; ++j) {
        const size_t e = ((size_t)s_off[i] + j) * 64 + lane;
        if (j < len) {
          sval[e] = val[rp[r] + j];
          scol[e] = col[rp[r] + j];
        } else {
          scol[e] = r < n ? r : 0;
        }
      }
    }
  return true;
}

// Dictionary-coded columns (cgx_internal.h).  Two passes over the nonzeros,
// each split over host threads by row ranges: (1) the distinct offsets
// col - row, in small open-addressing sets, giving up past 256; (2) the code
// bytes.  The dictionary is sorted, so it does not depend on the thread count.
namespace {
constexpr int kDcSlots = 1024;  // > 4 x 256: short probe chains
inline unsigned dc_hash(int key) { return ((unsigned)key * 2654435761u) >> 22; }
struct DcSet {
  int key[kDcSlots];
  short val[kDcSlots];
  bool used[kDcSlots];
  int count = 0;
  DcSet() { memset(used, 0, sizeof used); }
  // index of key, inserting it (-1 when full past 256 distinct keys)
  int find_or_add(int k, bool add) {
    unsigned h = dc_hash(k);
    while (used[h]) {
      if (key[h] == k) return val[h];
      h = (h + 1) & (kDcSlots - 1);
    }
    if (!add || count == 256) return -1;
    used[h] = true;
    key[h] = k;
    val[h] = (short)count;
    return count++;
  }
};
}  // namespace

int build_col_codes(int n, const int *rp, const int *col, std::vector<int> &dict,
                    unsigned char *code) {
  dict.clear();
  if (n <= 0 || rp[n] <= 0) return 0;
  const long long nnz = rp[n];
  int nt = (int)std::min<long long>(16, std::max<long long>(1, nnz >> 22));
  nt = std::max(1, std::min(nt, (int)std::thread::hardware_concurrency()));
  auto row_begin = [&](int t) { return (int)((long long)n * t / nt); };
  std::vector<DcSet> sets((size_t)nt);
  std::vector<int> ok((size_t)nt, 1);
  auto pass1 = [&](int t) {
    DcSet &S = sets[(size_t)t];
    for (int r = row_begin(t); r < row_begin(t + 1) && ok[(size_t)t]; ++r)
      for (int k = rp[r]; k < rp[r + 1]; ++k)
        if (S.find_or_add(col[k] - r, true) < 0) {
          ok[(size_t)t] = 0;
          break;
        }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(pass1, t);
  pass1(0);
  for (auto &x : th) x.join();
  th.clear();
  DcSet all;
  for (int t = 0; t < nt; ++t) {
    if (!ok[(size_t)t]) return 0;
    for (int h = 0; h < kDcSlots; ++h)
      if (sets[(size_t)t].used[h] && all.find_or_add(sets[(size_t)t].key[h], true) < 0) return 0;
  }
  for (int h = 0; h < kDcSlots; ++h)
    if (all.used[h]) dict.push_back(all.key[h]);
  std::sort(dict.begin(), dict.end());
  DcSet idx;  // offset -> code (position in the sorted dictionary)
  for (int k : dict) idx.find_or_add(k, true);
  auto pass2 = [&](int t) {
    for (int r = row_begin(t); r < row_begin(t + 1); ++r)
      for (int k = rp[r]; k < rp[r + 1]; ++k)
        code[k] = (unsigned char)idx.find_or_add(col[k] - r, false);
  };
  for (int t = 1; t < nt; ++t) th.emplace_back(pass2, t);
  pass2(0);
  for (auto &x : th) x.join();
  return (int)dict.size();
}

template <typename T>
int build_val_pairs(long long nnz, const T *val, unsigned char *code, std::vector<int> &dict,
                    std::vector<T> &dval, int cap) {
  const int nd = (int)dict.size();
  dval.clear();
  if (nnz <= 0 || nd <= 0) return 0;
  auto bits = [](T v) {
    unsigned long long b = 0;
    memcpy(&b, &v, sizeof v);
    return b;
  };
  int nt = (int)std::min<long long>(16, std::max<long long>(1, nnz >> 22));
  nt = std::max(1, std::min(nt, (int)std::thread::hardware_concurrency()));
  auto beg = [&](int t) { return nnz * t / nt; };
  // per thread: the distinct value bit patterns of each offset code
  std::vector<std::vector<std::vector<unsigned long long>>> seen(
      (size_t)nt, std::vector<std::vector<unsigned long long>>((size_t)nd));
  std::vector<int> ok((size_t)nt, 1);
  auto pass1 = [&](int t) {
    auto &S = seen[(size_t)t];
    int tot = 0;
    unsigned long long last_b = 0;
    int last_c = -1;
    for (long long k = beg(t); k < beg(t + 1); ++k) {
      const int c = code[k];
      const unsigned long long b = bits(val[k]);
      if (c == last_c && b == last_b) continue;
      auto &L = S[(size_t)c];
      if (std::find(L.begin(), L.end(), b) == L.end()) {
        if (++tot > cap) {
          ok[(size_t)t] = 0;
          return;
        }
        L.push_back(b);
      }
      last_c = c;
      last_b = b;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(pass1, t);
  pass1(0);
  for (auto &x : th) x.join();
  th.clear();
  for (int t = 0; t < nt; ++t)
    if (!ok[(size_t)t]) return 0;
  std::vector<std::vector<unsigned long long>> all((size_t)nd);
  std::vector<int> base((size_t)nd + 1, 0);
  for (int c = 0; c < nd; ++c) {
    auto &A = all[(size_t)c];
    for (int t = 0; t < nt; ++t)
      for (unsigned long long b : seen[(size_t)t][(size_t)c])
        if (std::find(A.begin(), A.end(), b) == A.end()) A.push_back(b);
    std::sort(A.begin(), A.end());
    base[(size_t)c + 1] = base[(size_t)c] + (int)A.size();
  }
  const int np = base[(size_t)nd];
  if (np > cap) return 0;
  std::vector<int> pd((size_t)np);
  dval.resize((size_t)np);
  for (int c = 0; c < nd; ++c)
    for (size_t i = 0; i < all[(size_t)c].size(); ++i) {
      pd[(size_t)base[(size_t)c] + i] = dict[(size_t)c];
      T v;
      const unsigned long long b = all[(size_t)c][i];
      memcpy(&v, &b, sizeof v);
      dval[(size_t)base[(size_t)c] + i] = v;
    }
  auto pass2 = [&](int t) {
    for (long long k = beg(t); k < beg(t + 1); ++k) {
      const int c = code[k];
      const auto &A = all[(size_t)c];
      const unsigned long long b = bits(val[k]);
      code[k] = (unsigned char)(base[(size_t)c] + (std::find(A.begin(), A.end(), b) - A.begin()));
    }
  };
  for (int t = 1; t < nt; ++t) th.emplace_back(pass2, t);
  pass2(0);
  for (auto &x : th) x.join();
  dict = pd;
  return np;
}
template int build_val_pairs<double>(long long, const double *, unsigned char *,
                                     std::vector<int> &, std::vector<double> &, int);
template int build_val_pairs<float>(long long, const float *, unsigned char *,
                                    std::vector<int> &, std::vector<float> &, int);

void pack_nibbles(long long nnz, const unsigned char *code, unsigned char *out) {
  for (long long i = 0; i + 1 < nnz; i += 2)
    out[i >> 1] = (unsigned char)(code[i] | (code[i + 1] << 4));
  if (nnz & 1) out[nnz >> 1] = code[nnz - 1];
}

std::vector<int> lap_offsets(const LapSpec &g) {
  std::vector<int> d{0};
  const int pl = g.nx * g.ny;
  if (g.nx > 1) d.insert(d.end(), {-1, 1});
  if (g.ny > 1) d.insert(d.end(), {-g.nx, g.nx});
  if (g.dim == 3 && g.nz > 1) d.insert(d.end(), {-pl, pl});
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  return d;
}

bool build_row_lengths(int n, const int *rp, unsigned char *rlen) {
  for (int r = 0; r < n; ++r)
    if (rp[r + 1] - rp[r] > 255) return false;
  for (int r = 0; r < n; ++r) rlen[r] = (unsigned char)(rp[r + 1] - rp[r]);
  return true;
}

bool env_wants_dc() {
  const char *l = getenv("CGX_LAYOUT");
  return env_int("CGX_DC", 1) != 0 && !(l && (strcmp(l, "csr") == 0 || strcmp(l, "sell") == 0));
}

int vec_grid_for(int n, int cus) {
  const long long vecs = (n + 1) / 2;
  long long g = (vecs + kVecBS - 1) / kVecBS;
  const long long cap = (long long)cus * 4;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

}  // namespace cgx

// ----------------------------------------------------------------- solver

struct cgx_solver {
  int device = 0;
  int cus = 256;
  hipStream_t stream = nullptr;
  int n = 0, nnz = 0, dtype = CGX_F64;
  int mode = CGX_MODE_FAST, alg = CGX_ALG_HS;
  int vec = 2;
  int spmv_xcd = 0, spmv_nt = -1, spmv_bs = 64, spmv_wpb = 4, spmv_rbw = 1,
      spmv_tg = 1, spmv_dma = 0;
  int nblk = 0, spmv_grid = 0, vec_grid = 0;
  bool use_graph = true;
  bool xdefer = false;  // CGX_XDEFER: x update folded into the p-update
  bool fold = false;    // CGX_FOLD: alpha/beta steps inside the vector kernels
  // column panels (irregular matrices): npanel SpMV passes, panel q's rows in
  // d_rp + q (n+1), its row blocks at blk index panel_off[q] (panel_nblk[q])
  int npanel = 1;
  std::vector<int> panel_off, panel_nblk, panel_grid;
  bool panel_win512 = false;  // fp32 panels: 512-entry LDS windows
  int spmv_capw = 0;           // CGX_SPMV_CAPW: fp64 LDS-DMA window (456 or 512)
  int epi_last = 0;            // CGX_SPMV_EPI_LAST: barrier-free SpMV epilogue
  bool vec_pf = false;         // CGX_VEC_PF: folded kernels issue loads before the partial sum
  // matrix-free Laplacian (cgx_solver_set_stencil): no CSR arrays at all
  bool is_stencil = false;
  cgx::LapSpec lap{};
  int graph_batch = 16;
  int *d_rp = nullptr, *d_col = nullptr, *d_blk = nullptr, *d_blkk = nullptr;
  int *d_blkrk = nullptr;  // (blk_row, blk_k) pairs: one scalar load per descriptor
  // dictionary-coded columns (k_spmv_dc; CGX_DC, default on where it applies):
  // d_code[k] = index of col[k] - row in d_dict (ndict entries, 256 allocated)
  bool want_dc = true;
  int ndict = 0;
  unsigned char *d_code = nullptr;
  int *d_dict = nullptr;
  // value-indexed pairs (CGX_DC_VALS, default on where it applies): the
  // dictionary holds (offset, value) pairs and the SpMV does not read val
  bool want_vi = true;
  bool vi = false;
  void *d_dval = nullptr;
  int vi_bpw = 1;                  // CGX_VI_BPW: row blocks per wave of k_spmv_vi
  bool want_rlen = true;           // CGX_DC_RLEN: byte row lengths instead of rp
  bool want_tile = true;           // CGX_DC_TILE: L2-tiled block order for wide stencils
  int tile_kb = 1536;              // CGX_DC_TILE_KB: x budget of a band sweep per XCD
  int tile_bands = 0;
  int *d_blklist = nullptr;        // the tiled block order (nullptr: natural)
  int want_bits = 8;               // CGX_DC_BITS=4: nibble codes when <= 16 offsets
  int code_bits = 8;
  int dc_lds_pad = 0;              // CGX_DC_LDS_PAD (diagnostic: fewer workgroups per CU)
  bool contig = false;             // CGX_CONTIG: physically contiguous device allocations
  unsigned char *d_rlen = nullptr;
  // SELL-64 internal layout (CGX_LAYOUT=sell): d_col/d_val hold the slices
  bool want_sell = false, sell = false;
  int *d_soff = nullptr, *d_slen = nullptr;
  int nslices = 0;
  long long sell_elems = 0;
  void *d_val = nullptr;
  void *d_b = nullptr, *d_x = nullptr, *d_r = nullptr, *d_p = nullptr,
       *d_s = nullptr, *d_w = nullptr, *d_p2 = nullptr;
  // HS with the fused p-update: p alternates between d_p and d_p2; `par`
  // says which one holds the previous direction (the SpMV's p_old)
  bool fuse_xpay = true;
  int par = 0;
  double *d_pa = nullptr, *d_pb = nullptr;
  int part_cap = 0;
  // in-kernel ticket reduction (replaces the k_finalize launches of HS)
  bool ticket = true;
  int ngmax = 0;
  double *d_tpart2 = nullptr;
  unsigned *d_tcnt = nullptr;  // [ngroups_max] level-1 counters + [1] level-2
  CgState *d_st = nullptr, *h_st = nullptr;
  double *d_hist = nullptr;
  int hist_alloc = 0;
  size_t dev_bytes = 0;
  bool have_matrix = false, have_rhs = false, bench_ready = false;
  int last_iters = 0;
  hipGraphExec_t gexec[2] = {nullptr, nullptr};  // by starting parity
  int gexec_key[2] = {-1, -1};
  std::vector<hipEvent_t> events;
};

void cgx::solver_want_dc(cgx_solver *s, bool on) { s->want_dc = on && env_wants_dc(); }

namespace {

using namespace cgx;

size_t tsize(int dtype) { return dtype == CGX_F32 ? 4 : 8; }

int dalloc(cgx_solver *s, void **p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipErrorUnknown;
  if (s->contig) {  // physically contiguous (CGX_CONTIG), falling back to hipMalloc
    e = hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess) e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    *p = nullptr;
    return CGX_ENOMEM;
  }
  s->dev_bytes += bytes;
  return 0;
}

void dfree(void **p) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
}

void drop_graph(cgx_solver *s) {
  for (int i = 0; i < 2; ++i) {
    if (s->gexec[i]) (void)hipGraphExecDestroy(s->gexec[i]);
    s->gexec[i] = nullptr;
    s->gexec_key[i] = -1;
  }
}

void free_matrix(cgx_solver *s) {
  drop_graph(s);
  dfree((void **)&s->d_rp);
  dfree((void **)&s->d_col);
  dfree((void **)&s->d_blk);
  dfree((void **)&s->d_blkk);
  dfree((void **)&s->d_blkrk);
  dfree((void **)&s->d_soff);
  dfree((void **)&s->d_slen);
  dfree((void **)&s->d_code);
  dfree((void **)&s->d_dict);
  dfree(&s->d_dval);
  s->vi = false;
  dfree((void **)&s->d_rlen);
  dfree((void **)&s->d_blklist);
  s->tile_bands = 0;
  s->ndict = 0;
  s->sell = false;
  s->nslices = 0;
  s->sell_elems = 0;
  dfree(&s->d_val);
  dfree(&s->d_b);
  dfree(&s->d_x);
  dfree(&s->d_r);
  dfree(&s->d_p);
  dfree(&s->d_s);
  dfree(&s->d_w);
  dfree(&s->d_p2);
  dfree((void **)&s->d_pa);
  dfree((void **)&s->d_pb);
  dfree((void **)&s->d_tpart2);
  dfree((void **)&s->d_tcnt);
  dfree((void **)&s->d_hist);
  s->hist_alloc = 0;
  s->dev_bytes = 0;
  s->have_matrix = s->have_rhs = s->bench_ready = false;
  s->is_stencil = false;
  s->n = s->nnz = s->nblk = 0;
}

int check_device(int device) {
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
    set_error("device %d is %s; libcgx is built for gfx950 (MI355X) only",
              device, prop.gcnArchName);
    return CGX_ENODEV;
  }
  return 0;
}

template <typename T>
int upload_matrix(cgx_solver *s, int n, int nnz, const int *rp, const int *col,
                  const T *val, const LapSpec *gen = nullptr) {
  // gen: col/val are generated on the device (cgx_solver_gen_laplacian);
  // rp is the host closed form, used for the row-block plan and uploaded
  if (n < 0 || nnz < 0 || (n > 0 && (!rp || (nnz > 0 && !gen && (!col || !val))))) {
    set_error("set_matrix: invalid arguments");
    return CGX_EINVAL;
  }
  if (n > 0 && (rp[0] != 0 || rp[n] != nnz)) {
    set_error("set_matrix: row_ptr[0] must be 0 and row_ptr[n] == nnz");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  free_matrix(s);
  s->dtype = sizeof(T) == 4 ? CGX_F32 : CGX_F64;
  s->n = n;
  s->nnz = nnz;
  const bool half = s->spmv_dma == 4 && s->spmv_bs == 64;  // 32-row blocks
  int cap = half ? spmv_cap(32, sizeof(T) == 8) : spmv_cap(s->spmv_bs, sizeof(T) == 8);
  s->spmv_capw = 0;
  if (sizeof(T) == 8 && s->spmv_dma == 1 && s->spmv_bs == 64 && s->spmv_wpb == 4 && n > 0 &&
      !gen_panels_pending(n, rp, col, gen)) {
    // LDS window sized to the matrix: 328 entries when every 64-row block
    // fits (C2 5-point: -10% SpMV, -5% per iteration from the occupancy it
    // frees, sweeps 28-29), else the 512 default (456 for 7-point blocks
    // measured neutral to -4%); CGX_SPMV_CAPW=328|456|512 overrides
    int w = env_int("CGX_SPMV_CAPW", 0);
    if (w == 0) {
      int m = 0;
      for (int r = 0; r < n; r += 64) m = std::max(m, rp[std::min(r + 64, n)] - rp[r]);
      w = m + kPad <= 328 ? 328 : 512;
    }
    if (w == 456 || w == 328) {
      s->spmv_capw = w;
      cap = w;
    }
  }
  std::vector<int> blk, blkk;
  std::vector<int> prp, pcol;
  std::vector<T> pval;
  s->npanel = gen ? 1 : choose_panels(n, rp, col, sizeof(T));
  s->panel_win512 = sizeof(T) == 4 && env_int("CGX_PANEL_WIN512", 0) != 0;
  s->panel_off.clear();
  s->panel_nblk.clear();
  s->panel_grid.clear();
  if (s->npanel > 1) {
    // k_spmv_dma over each panel's row blocks; the panel arrays replace the CSR
    build_panels<T>(n, rp, col, val, s->npanel, prp, pcol, pval);
    for (int q = 0; q < s->npanel; ++q) {
      const int *rq = prp.data() + (size_t)q * (n + 1);
      // fp32: 512-entry windows (4 KiB of LDS per wave, 2x the waves of the
      // 1024-entry default) when CGX_PANEL_WIN512 (k_spmv_dma, dma == 4 branch)
      std::vector<int> b = plan_rowblocks(
          n, rq, 64, (s->panel_win512 ? 512 : spmv_cap(64, sizeof(T) == 8)) - kPad);
      s->panel_off.push_back((int)blk.size());
      s->panel_nblk.push_back((int)b.size() - 1);
      s->panel_grid.push_back(spmv_launch_grid(64, s->panel_win512 ? 4 : s->spmv_wpb, 1,
                                               (int)b.size() - 1, 0,
                                               s->panel_win512 ? 4 : 1));
      for (int r : b) {
        blk.push_back(r);
        blkk.push_back(rq[r]);
      }
    }
    rp = prp.data();
    col = pcol.data();
    val = pval.data();
  } else {
    if (n > 0) blk = plan_rowblocks(n, rp, half ? 32 : s->spmv_bs, cap - kPad);  // room for VEC alignment
    else blk.push_back(0);
    blkk.resize(blk.size());
    for (size_t i = 0; i < blk.size(); ++i) blkk[i] = n > 0 ? rp[blk[i]] : 0;
  }
  const size_t rp_len = (size_t)s->npanel * ((size_t)n + 1);
  s->nblk = s->npanel > 1 ? (int)blk.size() - s->npanel : (int)blk.size() - 1;
  const size_t nnz_pad = ((size_t)nnz + kPad - 1) / kPad * kPad + kWindowPad;
  const size_t nv = (size_t)n + kPad;
  int rc;
  // + 64 entries: the engine SpMV DMAs row_ptr[r0 .. r0+63] for every block
  if ((rc = dalloc(s, (void **)&s->d_rp, rp_len * 4 + 256)) ||
      (rc = dalloc(s, (void **)&s->d_col, nnz_pad * 4)) ||
      (rc = dalloc(s, &s->d_val, nnz_pad * sizeof(T)))) {
    free_matrix(s);
    return rc;
  }
  if ((rc = dalloc(s, (void **)&s->d_blk, blk.size() * 4)) ||
      (rc = dalloc(s, (void **)&s->d_blkk, blk.size() * 4)) ||
      (rc = dalloc(s, (void **)&s->d_blkrk, blk.size() * 8)) ||
      (rc = dalloc(s, &s->d_b, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_x, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_r, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_p, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_s, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_w, nv * sizeof(T))) ||
      (rc = dalloc(s, &s->d_p2, nv * sizeof(T)))) {
    free_matrix(s);
    return rc;
  }
  s->spmv_grid = std::min(s->nblk, env_int("CGX_SPMV_GRID", INT_MAX));
  if (s->spmv_grid >= 64 && s->spmv_grid < s->nblk)
    s->spmv_grid &= ~7;  // XCD-aware mapping needs G % 8 == 0
  if (s->spmv_grid < 1) s->spmv_grid = 1;
  s->spmv_grid = spmv_launch_grid(s->spmv_bs, s->spmv_wpb, s->spmv_rbw, s->nblk,
                                  s->spmv_grid, s->spmv_dma);
  if (s->npanel > 1)  // the last panel's launch writes the epilogue partials
    s->spmv_grid = s->panel_grid.back();
  else if (s->spmv_dma == 5 && sizeof(T) == 8)  // engine: persistent, as many as fit per CU
    s->spmv_grid = std::max(1, std::min(s->cus * eng_wg_per_cu(s->spmv_rbw), s->nblk));
  s->vec_grid = env_int("CGX_VEC_GRID", vec_grid_for(n, s->cus));
  s->vec_grid = (std::max(s->vec_grid, 1) + 3) / 4 * 4;  // folded kernels: 4 x 256 threads
  s->part_cap = std::max(s->spmv_grid, s->vec_grid) + 1;
  for (int g : s->panel_grid) s->part_cap = std::max(s->part_cap, g + 1);
  const size_t ngmax = (size_t)s->part_cap / kTicketGroup + 2;
  if ((rc = dalloc(s, (void **)&s->d_pa, (size_t)s->part_cap * 8)) ||
      (rc = dalloc(s, (void **)&s->d_pb, (size_t)s->part_cap * 8)) ||
      (rc = dalloc(s, (void **)&s->d_tpart2, ngmax * 8)) ||
      (rc = dalloc(s, (void **)&s->d_tcnt, (ngmax + 1) * 4))) {
    free_matrix(s);
    return rc;
  }
  CGX_HIP(hipMemsetAsync(s->d_tcnt, 0, (ngmax + 1) * 4, s->stream));
  s->ngmax = (int)ngmax;
  if (env_int("CGX_DEBUG_PTRS", 0))
    fprintf(stderr, "cgx ptrs rp %p col %p val %p x(p) %p y(s) %p r %p\n", (void *)s->d_rp,
            (void *)s->d_col, s->d_val, s->d_p, s->d_s, s->d_r);
  CGX_HIP(hipMemsetAsync(s->d_col, 0, nnz_pad * 4, s->stream));
  CGX_HIP(hipMemsetAsync(s->d_val, 0, nnz_pad * sizeof(T), s->stream));
  if (n > 0) {
    CGX_HIP(hipMemcpyAsync(s->d_rp, rp, rp_len * 4, hipMemcpyHostToDevice, s->stream));
    if (nnz > 0 && gen) {
      CGX_HIP(launch_gen_laplacian(*gen, n, s->d_col, (double *)s->d_val, s->stream));
    } else if (nnz > 0) {
      CGX_HIP(hipMemcpyAsync(s->d_col, col, (size_t)nnz * 4,
                             hipMemcpyHostToDevice, s->stream));
      CGX_HIP(hipMemcpyAsync(s->d_val, val, (size_t)nnz * sizeof(T),
                             hipMemcpyHostToDevice, s->stream));
    }
  }
  CGX_HIP(hipMemcpyAsync(s->d_blk, blk.data(), blk.size() * 4,
                         hipMemcpyHostToDevice, s->stream));
  std::vector<int> blkrk(2 * blk.size());
  for (size_t i = 0; i < blk.size(); ++i) {
    blkrk[2 * i] = blk[i];
    blkrk[2 * i + 1] = blkk[i];
  }
  CGX_HIP(hipMemcpyAsync(s->d_blkrk, blkrk.data(), blkrk.size() * 4, hipMemcpyHostToDevice,
                         s->stream));
  CGX_HIP(hipMemcpyAsync(s->d_blkk, blkk.data(), blkk.size() * 4,
                         hipMemcpyHostToDevice, s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  if (s->want_sell && n > 0 && s->npanel == 1 && !gen) {
    std::vector<int> soff, slen, scol;
    std::vector<T> sval;
    if (csr_to_sell64<T>(n, rp, col, val, 1.25, soff, slen, sval, scol)) {
      dfree((void **)&s->d_col);
      dfree(&s->d_val);
      const size_t ne = sval.size() + kPad;
      if ((rc = dalloc(s, (void **)&s->d_col, ne * 4)) ||
          (rc = dalloc(s, &s->d_val, ne * sizeof(T))) ||
          (rc = dalloc(s, (void **)&s->d_soff, soff.size() * 4)) ||
          (rc = dalloc(s, (void **)&s->d_slen, slen.size() * 4 + 4))) {
        free_matrix(s);
        return rc;
      }
      CGX_HIP(hipMemcpy(s->d_col, scol.data(), scol.size() * 4, hipMemcpyHostToDevice));
      CGX_HIP(hipMemcpy(s->d_val, sval.data(), sval.size() * sizeof(T), hipMemcpyHostToDevice));
      CGX_HIP(hipMemcpy(s->d_soff, soff.data(), soff.size() * 4, hipMemcpyHostToDevice));
      CGX_HIP(hipMemcpy(s->d_slen, slen.data(), slen.size() * 4, hipMemcpyHostToDevice));
      s->sell = true;
      s->nslices = (int)slen.size();
      s->sell_elems = (long long)sval.size();
      s->spmv_grid = spmv_sell_grid(s->nslices);
      if (s->spmv_grid + 1 > s->part_cap) {
        set_error("internal: SELL grid exceeds partial buffer");
        free_matrix(s);
        return CGX_ENOMEM;
      }
    }
  }
  if (s->want_dc && n > 0 && nnz > 0 && s->npanel == 1 && !s->sell &&
      s->spmv_dma == 1 && s->spmv_bs == 64 &&
      (s->spmv_wpb == 4 || (s->spmv_wpb == 8 && sizeof(T) == 8)) &&
      (s->spmv_capw == 0 || s->spmv_capw == 328)) {
    std::vector<unsigned char> code;
    std::vector<int> dict;
    int nd;
    if (gen) {  // generated on the device: the stencil's offsets, encoded there
      dict = lap_offsets(*gen);
      nd = (int)dict.size();
    } else {
      code.resize((size_t)nnz);
      nd = build_col_codes(n, rp, col, dict, code.data());
    }
    std::vector<unsigned char> rl;
    if (nd > 0 && s->want_rlen) {
      rl.resize((size_t)n);
      if (!build_row_lengths(n, rp, rl.data())) rl.clear();
    }
    // value-indexed pairs: 4-wave kernel with row lengths, <= 64 pairs
    std::vector<T> dv;
    // (rows <= 255 entries < every window, so each block's code window fits
    // the kernel's; checked anyway)
    bool vi_fits = true;
    {
      const int capw = sizeof(T) == 4 ? 1024 : (s->spmv_capw == 328 ? 328 : 512);
      const int cb = nd <= 16 && s->want_bits == 4 && !gen ? 4 : 8, ka = 128 / cb;
      const long long capc = ((long long)(capw + ka) * cb / 8 + 15) & ~15LL;
      for (int b = 0; b < s->nblk && vi_fits; ++b)
        vi_fits = ((long long)(blkk[(size_t)b + 1] - (blkk[(size_t)b] & ~(ka - 1))) * cb + 7) / 8 <= capc;
    }
    if (nd > 0 && s->want_vi && !rl.empty() && s->spmv_wpb == 4 && vi_fits) {
      if (gen) {  // one value per offset: 2 dim on the diagonal, -1 off it
        dv.resize((size_t)nd);
        for (int c = 0; c < nd; ++c) dv[(size_t)c] = dict[(size_t)c] == 0 ? T(2 * gen->dim) : T(-1);
      } else {
        const int np = build_val_pairs<T>(nnz, val, code.data(), dict, dv, 64);
        if (np > 0) nd = np;
      }
    }
    if (nd > 0) {
      if ((rc = dalloc(s, (void **)&s->d_code, nnz_pad)) ||
          (rc = dalloc(s, (void **)&s->d_dict, 256 * 4)) ||
          (!dv.empty() && (rc = dalloc(s, &s->d_dval, 256 * sizeof(T))))) {
        free_matrix(s);
        return rc;
      }
      dict.resize(256, 0);
      if (!dv.empty()) {
        dv.resize(256, T(0));
        CGX_HIP(hipMemcpyAsync(s->d_dval, dv.data(), 256 * sizeof(T), hipMemcpyHostToDevice,
                               s->stream));
        s->vi = true;
      }
      s->code_bits = nd <= 16 && s->want_bits == 4 && !gen ? 4 : 8;
      size_t code_bytes = (size_t)nnz;
      if (s->code_bits == 4) {  // in place: byte i/2 is written after entry i is read
        pack_nibbles(nnz, code.data(), code.data());
        code_bytes = ((size_t)nnz + 1) / 2;
      }
      CGX_HIP(hipMemsetAsync(s->d_code, 0, nnz_pad, s->stream));
      CGX_HIP(hipMemcpyAsync(s->d_dict, dict.data(), 256 * 4, hipMemcpyHostToDevice,
                             s->stream));
      if (gen) {
        int *d_err = (int *)s->d_pb;  // scratch: partials are rewritten before use
        CGX_HIP(hipMemsetAsync(d_err, 0, 4, s->stream));
        CGX_HIP(launch_dc_encode(n, s->d_rp, s->d_col, s->d_dict, nd, s->d_code, d_err,
                                 s->stream, (const double *)s->d_val,
                                 s->vi ? (const double *)s->d_dval : nullptr));
        int err = 0;
        CGX_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, s->stream));
        CGX_HIP(hipStreamSynchronize(s->stream));
        if (err) {
          set_error("internal: generated Laplacian has an offset outside its dictionary");
          free_matrix(s);
          return CGX_EINVAL;
        }
      } else {
        CGX_HIP(hipMemcpyAsync(s->d_code, code.data(), code_bytes, hipMemcpyHostToDevice,
                               s->stream));
      }
      if (!rl.empty()) {
        if ((rc = dalloc(s, (void **)&s->d_rlen, (size_t)n + 64))) {
          free_matrix(s);
          return rc;
        }
        CGX_HIP(hipMemcpyAsync(s->d_rlen, rl.data(), (size_t)n, hipMemcpyHostToDevice,
                               s->stream));
      }
      CGX_HIP(hipStreamSynchronize(s->stream));
      s->ndict = nd;
      if (s->spmv_wpb == 8 && (!s->d_rlen || s->code_bits != 8 || nd > 64)) {
        // the 8-wave coded kernel covers byte codes + row lengths + <= 64
        // offsets only; otherwise plain CSR at 8 waves (same partial count)
        dfree((void **)&s->d_code);
        dfree((void **)&s->d_dict);
        dfree(&s->d_dval);
        s->vi = false;
        dfree((void **)&s->d_rlen);
  dfree((void **)&s->d_blklist);
  s->tile_bands = 0;
        s->ndict = 0;
      }
      if (s->ndict > 0 && s->vi) {  // k_spmv_vi: bpw row blocks per wave
        s->spmv_grid = vi_grid(s->nblk, s->code_bits, s->vi_bpw);
      }
      if (s->ndict > 0 && s->spmv_wpb == 4 && s->want_tile) {
        // L2 tiling of the block order.  The x lines a row needs sit at its
        // offsets; with P = the largest |offset| (a 3-D stencil's plane), an
        // XCD sweeping rows in order needs ~3 P x-values resident to hit its
        // 4 MiB L2 on every re-read.  When that exceeds the budget, sweep the
        // rows in T bands of the P-periodic position instead (all planes of
        // band 0, then band 1, ...): ~3 P / T values in flight.  Only the
        // order of the row blocks changes -- each row's sum is the same.
        long long P = 0;
        for (int v : dict) P = std::max(P, (long long)std::abs(v));
        const long long budget = (long long)s->tile_kb * 1024;
        const long long need = 3 * P * (long long)sizeof(T);
        if (P > 0 && need > budget && s->nblk > 0) {
          const long long T_ = (need + budget - 1) / budget;
          std::vector<int> order((size_t)s->nblk);
          for (int b = 0; b < s->nblk; ++b) order[(size_t)b] = b;
          auto band = [&](int b) { return (long long)blk[(size_t)b] % P * T_ / P; };
          auto plane = [&](int b) { return (long long)blk[(size_t)b] / P; };
          std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
            const long long bx = band(x), by = band(y);
            return bx != by ? bx < by : plane(x) < plane(y);
          });
          if ((rc = dalloc(s, (void **)&s->d_blklist, (size_t)s->nblk * 4))) {
            free_matrix(s);
            return rc;
          }
          CGX_HIP(hipMemcpy(s->d_blklist, order.data(), (size_t)s->nblk * 4,
                            hipMemcpyHostToDevice));
          s->tile_bands = (int)T_;
        }
      }
    }
  }
  s->have_matrix = true;
  return 0;
}

// Matrix-free Laplacian: vectors and partial buffers only.
int set_stencil(cgx_solver *s, const LapSpec &g) {
  const long long n = (long long)g.nx * g.ny * g.nz;
  if ((g.dim != 2 && g.dim != 3) || g.nx < 1 || g.ny < 1 || g.nz < 1 ||
      (g.dim == 2 && g.nz != 1) || n > INT32_MAX || lap_rp(n, g) > INT32_MAX) {
    set_error("set_stencil: bad grid");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  free_matrix(s);
  s->dtype = CGX_F64;
  s->n = (int)n;
  s->nnz = (int)lap_rp(n, g);
  s->npanel = 1;
  s->panel_off.clear();
  s->panel_nblk.clear();
  s->panel_grid.clear();
  const size_t nv = (size_t)n + kPad;
  // one row per thread: the stencil's 7 loads per row are latency-bound, so
  // every row gets its own lane (grid-stride at cus*16 WGs ran at 2.3 TB/s)
  s->spmv_grid = (int)std::max<long long>(
      1, std::min<long long>((n + 255) / 256, env_int("CGX_STENCIL_GRID", INT_MAX)));
  s->vec_grid = env_int("CGX_VEC_GRID", vec_grid_for((int)n, s->cus));
  s->vec_grid = (std::max(s->vec_grid, 1) + 3) / 4 * 4;
  s->part_cap = std::max(s->spmv_grid, s->vec_grid) + 1;
  const size_t ngmax = (size_t)s->part_cap / kTicketGroup + 2;
  int rc;
  if ((rc = dalloc(s, &s->d_b, nv * 8)) || (rc = dalloc(s, &s->d_x, nv * 8)) ||
      (rc = dalloc(s, &s->d_r, nv * 8)) || (rc = dalloc(s, &s->d_p, nv * 8)) ||
      (rc = dalloc(s, &s->d_s, nv * 8)) || (rc = dalloc(s, &s->d_w, nv * 8)) ||
      (rc = dalloc(s, &s->d_p2, nv * 8)) ||
      (rc = dalloc(s, (void **)&s->d_pa, (size_t)s->part_cap * 8)) ||
      (rc = dalloc(s, (void **)&s->d_pb, (size_t)s->part_cap * 8)) ||
      (rc = dalloc(s, (void **)&s->d_tpart2, ngmax * 8)) ||
      (rc = dalloc(s, (void **)&s->d_tcnt, (ngmax + 1) * 4))) {
    free_matrix(s);
    return rc;
  }
  CGX_HIP(hipMemsetAsync(s->d_tcnt, 0, (ngmax + 1) * 4, s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  s->ngmax = (int)ngmax;
  s->is_stencil = true;
  s->lap = g;
  s->have_matrix = true;
  return 0;
}

template <typename T>
int upload_rhs(cgx_solver *s, const T *b) {
  if (!s->have_matrix || (s->n > 0 && !b)) {
    set_error("set_rhs: no matrix loaded or NULL b");
    return CGX_EINVAL;
  }
  if ((sizeof(T) == 4) != (s->dtype == CGX_F32)) {
    set_error("set_rhs: dtype does not match the matrix");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  if (s->n > 0)
    CGX_HIP(hipMemcpy(s->d_b, b, (size_t)s->n * sizeof(T),
                      hipMemcpyHostToDevice));
  s->have_rhs = true;
  return 0;
}

template <typename T>
SpmvArgs<T> spmv_args(cgx_solver *s, const void *x, void *y, double *part,
                      bool with_done) {
  SpmvArgs<T> a;
  memset(&a, 0, sizeof a);
  a.rp = s->d_rp;
  a.col = s->d_col;
  a.val = (const T *)s->d_val;
  a.x = (const T *)x;
  a.y = (T *)y;
  a.blk_row = s->d_blk;
  a.blk_k = s->d_blkk;
  a.blk_rk = s->d_blkrk;
  a.blk_list = nullptr;
  a.blk_first = 0;
  a.nblk = s->nblk;
  a.part = part;
  a.done = with_done ? &s->d_st->done : nullptr;
  a.xcd = s->spmv_xcd;
  // by size: 2 = code stream AND the CSR-VI y store past the caches (C3 SpMV
  // 95.0 -> 92.5 us, iteration 195.2 -> 192.4 us; tools/gpu_vi_nt.sh)
  a.nt = s->spmv_nt < 0
             ? ((double)s->nnz * (double)(sizeof(T) + 4) > cgx::kNtStreamBytes ? 2 : 0)
             : s->spmv_nt;
  a.bs = s->spmv_bs;
  a.wpb = s->spmv_wpb;
  a.rbw = s->spmv_rbw;
  a.x2 = nullptr;
  a.xout = nullptr;
  a.st = s->d_st;
  a.tg = s->spmv_tg;
  a.tk = TicketArgs{};
  a.s_off = s->sell ? s->d_soff : nullptr;
  a.s_len = s->sell ? s->d_slen : nullptr;
  a.nslices = s->nslices;
  a.n = s->n;
  a.dma = s->spmv_dma;
  a.yacc = nullptr;
  a.capw = s->spmv_capw;
  a.epi_last = s->epi_last;
  if (s->ndict > 0) {
    a.code = s->d_code;
    a.dict = s->d_dict;
    a.ndict_cap = dict_cap(s->ndict);
    a.rlen = s->d_rlen;
    a.code_bits = s->code_bits;
    a.blk_list = s->d_blklist;
    a.lds_pad = s->dc_lds_pad;
    a.dval = s->vi ? (const T *)s->d_dval : nullptr;
    a.bpw = s->code_bits == 8 ? s->vi_bpw : 1;
  }
  return a;
}

// One SpMV of the solver's matrix: a single launch, or one per column panel
// (rows continue their sums from y; the epilogue partials on the last panel).
template <typename T>
hipError_t launch_spmv_s(cgx_solver *s, SpmvArgs<T> a, hipStream_t st) {
  if (s->is_stencil)
    return launch_stencil<T>(s->lap, s->n, a.x, a.y, a.part, a.done, s->spmv_grid, st);
  if (s->npanel <= 1) return launch_spmv<T>(a, s->spmv_grid, s->vec, st);
  double *part = a.part;
  for (int q = 0; q < s->npanel; ++q) {
    SpmvArgs<T> b = a;
    b.rp = s->d_rp + (size_t)q * ((size_t)s->n + 1);
    b.blk_first = s->panel_off[q];
    b.nblk = s->panel_nblk[q];
    b.yacc = q ? a.y : nullptr;
    b.part = q + 1 == s->npanel ? part : nullptr;
    // dma 4: fp32 CAPW 512; dma 8: 8 gathers per row chunk (CGX_PANEL_U8)
    b.dma = s->panel_win512 ? 4 : (env_int("CGX_PANEL_U8", 0) ? 8 : 1);
    b.capw = 0;                       // panel plans use the default windows
    b.bs = 64;
    const hipError_t e = launch_spmv<T>(b, s->panel_grid[q], s->vec, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

TicketArgs ticket_args(cgx_solver *s, int op) {
  TicketArgs t;
  t.part1 = s->d_pa;
  t.part2 = s->d_tpart2;
  t.cnt1 = s->d_tcnt;
  t.cnt2 = s->d_tcnt + s->ngmax;
  t.op = op;
  t.st = s->d_st;
  t.hist = s->d_hist;
  return t;
}

bool use_ticket(const cgx_solver *s) {
  return s->ticket && s->alg == CGX_ALG_HS && s->mode == CGX_MODE_FAST &&
         (s->spmv_bs == 64 || s->sell) && s->npanel == 1 && !s->is_stencil;
}

bool fused(const cgx_solver *s) {
  return s->fuse_xpay && s->alg == CGX_ALG_HS && (s->spmv_bs == 64 || s->sell) &&
         s->spmv_dma != 2 && s->spmv_dma != 4 && s->npanel == 1 &&
         !(s->spmv_dma == 1 && s->spmv_wpb == 8) &&  // no fused variant at 8 waves
         s->spmv_capw == 0 &&
         !s->is_stencil && s->spmv_dma != 5;
}

// Prologue: x = 0, r = b, p = b (HS) / p = s = 0, w = A r (CG1); b.b; state.
template <typename T>
int enqueue_init(cgx_solver *s) {
  hipStream_t st = s->stream;
  T *b = (T *)s->d_b, *x = (T *)s->d_x, *r = (T *)s->d_r, *p = (T *)s->d_p;
  s->par = 0;
  if (s->alg == CGX_ALG_HS) {
    const bool pz = fused(s);
    if (s->mode == CGX_MODE_EXACT) {
      CGX_HIP(launch_init_hs<T>(s->n, b, x, r, p, nullptr, s->vec_grid, st, pz));
      CGX_HIP(launch_dot_seq<T>(s->n, b, b, s->d_pa, nullptr, st));
      CGX_HIP(launch_finalize(FIN_INIT_HS, s->d_pa, 1, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));
    } else if (use_ticket(s)) {
      const TicketArgs tk = ticket_args(s, FIN_INIT_HS);
      CGX_HIP(launch_init_hs<T>(s->n, b, x, r, p, s->d_pa, s->vec_grid, st, pz,
                                &tk));
    } else {
      CGX_HIP(launch_init_hs<T>(s->n, b, x, r, p, s->d_pa, s->vec_grid, st, pz));
      CGX_HIP(launch_finalize(FIN_INIT_HS, s->d_pa, s->vec_grid, nullptr, 0,
                              s->d_st, s->d_hist, nullptr, st));
    }
  } else {
    CGX_HIP(launch_init_cg1<T>(s->n, b, x, r, p, (T *)s->d_s, s->d_pa,
                               s->vec_grid, st));
    CGX_HIP(launch_spmv_s<T>(s, spmv_args<T>(s, r, s->d_w, s->d_pb, false), st));
    CGX_HIP(launch_finalize(FIN_INIT_CG1, s->d_pa, s->vec_grid, s->d_pb,
                            s->spmv_grid, s->d_st, s->d_hist, nullptr, st));
  }
  return 0;
}

// One CG iteration.  ev0/ev1 (optional) bracket the SpMV launch.
template <typename T>
int enqueue_iter(cgx_solver *s, hipEvent_t ev0, hipEvent_t ev1) {
  hipStream_t st = s->stream;
  T *x = (T *)s->d_x, *r = (T *)s->d_r, *p = (T *)s->d_p, *sv = (T *)s->d_s,
    *w = (T *)s->d_w;
  const int sg = s->spmv_grid;
  if (s->alg == CGX_ALG_HS) {
    const bool exact = s->mode == CGX_MODE_EXACT;
    const bool fx = fused(s);
    // with the fused p-update the SpMV reads p_old, writes p = r + beta p_old
    T *pold = fx ? (T *)(s->par ? s->d_p2 : s->d_p) : p;
    if (fx) p = (T *)(s->par ? s->d_p : s->d_p2);
    SpmvArgs<T> sa = spmv_args<T>(s, fx ? (void *)r : (void *)p, sv,
                                  exact ? nullptr : s->d_pa, true);
    if (fx) {
      sa.x2 = pold;
      sa.xout = p;
    }
    // Tickets only where workgroups live long (k_update_xr): a short-lived
    // SpMV workgroup waiting on its ticket's round trip cost 20% (r01 A/B).
    const bool tkt = use_ticket(s);
    if (ev0) CGX_HIP(hipEventRecord(ev0, st));
    CGX_HIP(launch_spmv_s<T>(s, sa, st));                         // cg.c:111 (+131-132)
    if (ev1) CGX_HIP(hipEventRecord(ev1, st));
    if (fx) s->par ^= 1;
    if (exact) {
      CGX_HIP(launch_dot_seq<T>(s->n, p, sv, s->d_pa, &s->d_st->done, st));
      CGX_HIP(launch_finalize(FIN_HS_ALPHA, s->d_pa, 1, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));           // cg.c:113
      CGX_HIP(launch_update_xr<T>(s->n, x, p, r, sv, s->d_st, nullptr,
                                  s->vec_grid, st));              // cg.c:115-123
      CGX_HIP(launch_dot_seq<T>(s->n, r, r, s->d_pa, &s->d_st->done, st));
      CGX_HIP(launch_finalize(FIN_HS_BETA, s->d_pa, 1, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));           // cg.c:125-129
    } else if (tkt) {  // the beta step runs in k_update_xr's last workgroup
      CGX_HIP(launch_finalize(FIN_HS_ALPHA, s->d_pa, sg, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));
      const TicketArgs tk = ticket_args(s, FIN_HS_BETA);
      CGX_HIP(launch_update_xr<T>(s->n, x, p, r, sv, s->d_st, s->d_pa,
                                  s->vec_grid, st, &tk));
    } else if (s->xdefer && s->fold && !fx) {
      // folded: alpha inside k_update_rf, beta + stop test inside k_xpay_xf
      // (no finalize launches; bit-identical scalars, see k_update_rf)
      const int gf = s->vec_grid / 4;  // 1024-thread workgroups, 4 partials each
      CGX_HIP(launch_update_rf<T>(s->n, r, sv, s->d_st, s->d_pa, sg, s->d_pb, gf,
                                  st, s->vec_pf));                // cg.c:113, 118-123
      CGX_HIP(launch_xpay_xf<T>(s->n, x, p, r, s->d_st, s->d_pb, 4 * gf, s->d_hist,
                                gf, st, s->vec_pf));              // cg.c:115-116, 125-132
      return 0;
    } else if (s->xdefer && !fx) {
      // deferred x: r-update alone, x += alpha p_old folded into the p-update
      CGX_HIP(launch_finalize(FIN_HS_ALPHA_X, s->d_pa, sg, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));           // cg.c:113
      CGX_HIP(launch_update_r<T>(s->n, r, sv, s->d_st, s->d_pa, s->vec_grid,
                                 st));                            // cg.c:118-123
      CGX_HIP(launch_finalize(FIN_HS_BETA, s->d_pa, s->vec_grid, nullptr, 0,
                              s->d_st, s->d_hist, nullptr, st));  // cg.c:125-129
      CGX_HIP(launch_xpay_x<T>(s->n, x, p, r, s->d_st, s->vec_grid,
                               st));                              // cg.c:115-116, 131-132
      return 0;
    } else {
      CGX_HIP(launch_finalize(FIN_HS_ALPHA, s->d_pa, sg, nullptr, 0, s->d_st,
                              s->d_hist, nullptr, st));
      CGX_HIP(launch_update_xr<T>(s->n, x, p, r, sv, s->d_st, s->d_pa,
                                  s->vec_grid, st));
      CGX_HIP(launch_finalize(FIN_HS_BETA, s->d_pa, s->vec_grid, nullptr, 0,
                              s->d_st, s->d_hist, nullptr, st));
    }
    if (!fx)
      CGX_HIP(launch_xpay<T>(s->n, p, r, s->d_st, s->vec_grid, st));  // cg.c:131-132
  } else {
    CGX_HIP(launch_cg1_update<T>(s->n, x, p, r, sv, w, s->d_st, s->d_pa,
                                 s->vec_grid, st));
    if (ev0) CGX_HIP(hipEventRecord(ev0, st));
    CGX_HIP(launch_spmv_s<T>(s, spmv_args<T>(s, r, w, s->d_pb, true), st));
    if (ev1) CGX_HIP(hipEventRecord(ev1, st));
    CGX_HIP(launch_finalize(FIN_CG1, s->d_pa, s->vec_grid, s->d_pb, sg,
                            s->d_st, s->d_hist, nullptr, st));
  }
  return 0;
}

template <typename T>
int enqueue_iters(cgx_solver *s, long long count) {
  int B = s->graph_batch;
  if (B & 1) ++B;  // even: the fused p buffers return to the same parity
  const int key = s->alg * 2 + s->mode;
  if (s->use_graph && count >= B) {
    const int par = s->par;
    if (!s->gexec[par] || s->gexec_key[par] != key) {
      if (s->gexec[par]) (void)hipGraphExecDestroy(s->gexec[par]);
      s->gexec[par] = nullptr;
      hipGraph_t g = nullptr;
      CGX_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
      int rc = 0;
      for (int i = 0; i < B && rc == 0; ++i)
        rc = enqueue_iter<T>(s, nullptr, nullptr);
      hipError_t e = hipStreamEndCapture(s->stream, &g);
      s->par = par;  // capture only recorded the iterations
      if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
      CGX_HIP(e);
      e = hipGraphInstantiate(&s->gexec[par], g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      CGX_HIP(e);
      s->gexec_key[par] = key;
    }
    while (count >= B) {
      CGX_HIP(hipGraphLaunch(s->gexec[par], s->stream));
      count -= B;
    }
  }
  for (long long i = 0; i < count; ++i) {
    int rc = enqueue_iter<T>(s, nullptr, nullptr);
    if (rc) return rc;
  }
  return 0;
}

int prepare_state(cgx_solver *s, int maxit, double tol, int hist_cap) {
  if (hist_cap > s->hist_alloc) {
    drop_graph(s);  // captured graphs hold the old history pointer
    CGX_HIP(hipStreamSynchronize(s->stream));
    dfree((void **)&s->d_hist);
    int rc = dalloc(s, (void **)&s->d_hist, (size_t)hist_cap * 8);
    if (rc) return rc;
    s->hist_alloc = hist_cap;
  }
  memset(s->h_st, 0, sizeof(CgState));
  s->h_st->tol = tol;
  s->h_st->use_tol = tol > 0.0 ? 1 : 0;
  s->h_st->max_iter = maxit;
  s->h_st->hist_cap = std::min(hist_cap, s->hist_alloc);
  CGX_HIP(hipMemcpyAsync(s->d_st, s->h_st, sizeof(CgState),
                         hipMemcpyHostToDevice, s->stream));
  return 0;
}

int read_state(cgx_solver *s) {
  CGX_HIP(hipMemcpyAsync(s->h_st, s->d_st, sizeof(CgState),
                         hipMemcpyDeviceToHost, s->stream));
  CGX_HIP(hipStreamSynchronize(s->stream));
  return 0;
}

template <typename T>
int run_t(cgx_solver *s, int maxit, double tol, int *iters) {
  int rc;
  s->bench_ready = false;
  if ((rc = prepare_state(s, maxit, tol, maxit + 1))) return rc;
  if ((rc = enqueue_init<T>(s))) return rc;
  const long long total = (long long)maxit + 1;
  if (tol <= 0.0) {
    if ((rc = enqueue_iters<T>(s, total))) return rc;
    if ((rc = read_state(s))) return rc;
  } else {
    long long done_iters = 0, batch = 8;
    for (;;) {
      const long long b = std::min(batch, total - done_iters);
      if ((rc = enqueue_iters<T>(s, b))) return rc;
      done_iters += b;
      if ((rc = read_state(s))) return rc;
      if (s->h_st->done || done_iters >= total) break;
      batch = std::min<long long>(batch * 2, 256);
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
  if ((rc = prepare_state(s, INT_MAX - 1, 0.0, 0))) return rc;
  if ((rc = enqueue_init<T>(s))) return rc;
  if ((rc = enqueue_iters<T>(s, warmup))) return rc;
  CGX_HIP(hipStreamSynchronize(s->stream));
  s->bench_ready = true;
  return 0;
}

template <typename T>
int bench_run_t(cgx_solver *s, int iters, int flags, double *total_ms,
                double *spmv_ms) {
  const bool per_spmv = (flags & CGX_BENCH_SPMV_EVENTS) != 0;
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
  if (per_spmv) {
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
  if (!s->have_matrix || (s->n > 0 && (!x || !y))) {
    set_error("spmv: no matrix or NULL vector");
    return CGX_EINVAL;
  }
  if ((sizeof(T) == 4) != (s->dtype == CGX_F32)) {
    set_error("spmv: dtype does not match the matrix");
    return CGX_EINVAL;
  }
  if (s->n == 0) return 0;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpyAsync(s->d_p, x, (size_t)s->n * sizeof(T),
                         hipMemcpyHostToDevice, s->stream));
  CGX_HIP(launch_spmv_s<T>(s, spmv_args<T>(s, s->d_p, s->d_s, nullptr, false),
                           s->stream));
  CGX_HIP(hipMemcpyAsync(y, s->d_s, (size_t)s->n * sizeof(T),
                         hipMemcpyDeviceToHost, s->stream));
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

int cgx_stream_bench(int device, int kind, long long n, int reps, double *gbs) {
  if (!gbs || n < 2 || reps < 1 || (kind != CGX_STREAM_TRIAD && kind != CGX_STREAM_READ))
    return CGX_EINVAL;
  int rc = check_device(device);
  if (rc) return rc;
  CGX_HIP(hipSetDevice(device));
  const long long n2 = n / 2;
  double *buf = nullptr;
  if (hipMalloc((void **)&buf, (size_t)n2 * 16 * 3) != hipSuccess) {
    set_error("stream_bench: out of device memory");
    return CGX_ENOMEM;
  }
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
  double *a = buf, *b = buf + 2 * n2, *c = buf + 4 * n2;
  float best = 1e30f;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMemsetAsync(buf, 0, (size_t)n2 * 48, st);
  for (int r = -2; r < reps && e == hipSuccess; ++r) {  // two untimed warm-ups
    e = hipEventRecord(e0, st);
    if (e == hipSuccess)
      e = kind == CGX_STREAM_TRIAD ? launch_triad(n2, a, b, c, cus * 16, st)
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
  *gbs = (kind == CGX_STREAM_TRIAD ? 48.0 : 16.0) * (double)n2 / (best * 1e-3) / 1e9;
  return 0;
}

int cgx_solver_create(int device, cgx_solver **out) {
  if (!out) return CGX_EINVAL;
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  CGX_HIP(hipSetDevice(device));
  cgx_solver *s = new cgx_solver();
  s->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess)
    s->cus = prop.multiProcessorCount;
  s->vec = cgx::env_int("CGX_SPMV_VEC", 4);
  s->spmv_wpb = cgx::env_int("CGX_SPMV_WPB", 4) == 8 ? 8 : 4;
  // LDS-DMA stream + nt: best or tied-best in three order-rotated A/Bs (r01
  // sweeps 14-16: 192-201 us vs 201-210 us for the register-staged kernel)
  s->spmv_dma = cgx::env_int("CGX_SPMV_DMA", 1);
  s->spmv_rbw = std::max(1, cgx::env_int("CGX_SPMV_RBW", s->spmv_dma == 2 ? 8 : 1));
  if (s->spmv_dma == 2) s->spmv_rbw = std::min(s->spmv_rbw, 63);  // descriptors in lanes
  if (s->spmv_dma == 5)  // engine ring shape (k_spmv_eng), carried in rbw
    s->spmv_rbw = std::min(std::max(cgx::env_int("CGX_ENG_SHAPE", 4), 0), 7);
  // XCD-contiguous block order for the LDS-DMA kernel: time-neutral, but the
  // x lines shared by neighbouring row blocks stay in one XCD's L2 (EA reads
  // 1265 -> 976 MB per C3 SpMV = the algorithmic 965 MB; sweep25)
  s->spmv_xcd = cgx::env_int("CGX_SPMV_XCD", s->spmv_dma == 1 ? 1 : 0);
  // nt helps the LDS-DMA stream, hurts the register-staged one (sweep15)
  // -1 = by size at set_matrix (kNtStreamBytes; nt helps the LDS-DMA stream
  // only, it hurts the register-staged one: sweep15)
  s->spmv_nt = cgx::env_int("CGX_SPMV_NT", s->spmv_dma == 1 || s->spmv_dma == 3 ||
                                                   s->spmv_dma == 4 || s->spmv_dma == 5
                                               ? -1
                                               : 0);
  {
    const int bs = cgx::env_int("CGX_SPMV_BS", 64);
    s->spmv_bs = (bs == 512 || bs == 64) ? bs : 256;
  }
  if (s->vec != 1 && s->vec != 2 && s->vec != 4) s->vec = 4;
  s->use_graph = cgx::env_int("CGX_GRAPH", 1) != 0;
  s->graph_batch = std::max(1, cgx::env_int("CGX_GRAPH_BATCH", 16));
  s->fuse_xpay = cgx::env_int("CGX_FUSE_XPAY", 0) != 0;
  s->xdefer = cgx::env_int("CGX_XDEFER", 1) != 0;  // -4.4% per C3 iteration (sweep20), bit-identical
  s->fold = cgx::env_int("CGX_FOLD", 1) != 0;      // C3 -1%, C2 -8% (sweep22), bit-identical
  s->epi_last = cgx::env_int("CGX_SPMV_EPI_LAST", 0);
  s->vec_pf = cgx::env_int("CGX_VEC_PF", 1) != 0;  // C3 -1.7 us, C2 -0.44 us per iteration (sweep36), bit-identical
  s->spmv_tg = cgx::env_int("CGX_SPMV_TG", 1);
  s->want_dc = cgx::env_wants_dc();
  s->want_rlen = cgx::env_int("CGX_DC_RLEN", 1) != 0;
  s->want_vi = cgx::env_int("CGX_DC_VALS", 1) != 0;
  s->vi_bpw = cgx::env_int("CGX_VI_BPW", 1);
  if (s->vi_bpw != 2 && s->vi_bpw != 4) s->vi_bpw = 1;
  // physically contiguous allocations: -1 to -2% per C3 iteration in two
  // order-swapped A/Bs with 4 allocations per variant (tools/gpu_contig1.sh)
  s->contig = cgx::env_int("CGX_CONTIG", 1) != 0;
  s->want_tile = cgx::env_int("CGX_DC_TILE", 1) != 0;
  s->tile_kb = std::max(64, cgx::env_int("CGX_DC_TILE_KB", 1536));
  s->dc_lds_pad = std::max(0, std::min(cgx::env_int("CGX_DC_LDS_PAD", 0), 65536));
  s->want_bits = cgx::env_int("CGX_DC_BITS", 8) == 4 ? 4 : 8;  // nibbles: neutral at C3 (dc3 sweep)
  s->ticket = cgx::env_int("CGX_TICKET", 0) != 0 && s->spmv_dma == 0;  // DMA/pipe: partials only
  {
    const char *l = getenv("CGX_LAYOUT");
    s->want_sell = l && strcmp(l, "sell") == 0;
  }
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&s->d_st, sizeof(CgState)) != hipSuccess ||
      hipHostMalloc((void **)&s->h_st, sizeof(CgState), hipHostMallocDefault) !=
          hipSuccess) {
    cgx::set_error("cgx_solver_create: stream/state allocation failed");
    cgx_solver_destroy(s);
    return CGX_ENODEV;
  }
  *out = s;
  return 0;
}

void cgx_solver_destroy(cgx_solver *s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  free_matrix(s);
  for (hipEvent_t e : s->events) (void)hipEventDestroy(e);
  if (s->d_st) (void)hipFree(s->d_st);
  if (s->h_st) (void)hipHostFree(s->h_st);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

int cgx_solver_set_mode(cgx_solver *s, int mode, int alg) {
  if (!s || (mode != CGX_MODE_FAST && mode != CGX_MODE_EXACT) ||
      (alg != CGX_ALG_HS && alg != CGX_ALG_CG1)) {
    cgx::set_error("set_mode: bad arguments");
    return CGX_EINVAL;
  }
  if (mode == CGX_MODE_EXACT && alg != CGX_ALG_HS) {
    cgx::set_error("exact mode is defined for the HS recurrence only");
    return CGX_EINVAL;
  }
  s->mode = mode;
  s->alg = alg;
  drop_graph(s);
  return 0;
}

int cgx_solver_set_matrix(cgx_solver *s, int n, int nnz, const int *row_ptr,
                          const int *col, const double *val) {
  if (!s) return CGX_EINVAL;
  return upload_matrix<double>(s, n, nnz, row_ptr, col, val);
}

int cgx_solver_set_matrix_f32(cgx_solver *s, int n, int nnz,
                              const int *row_ptr, const int *col,
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
  return set_stencil(s, LapSpec{dim, nx, ny, dim == 3 ? nz : 1});
}

int cgx_solver_get_matrix(cgx_solver *s, int *row_ptr, int *col, double *val) {
  if (!s || !s->have_matrix || s->is_stencil || s->sell || s->npanel > 1 ||
      s->dtype != CGX_F64 || (s->n > 0 && (!row_ptr || (s->nnz > 0 && (!col || !val))))) {
    set_error("get_matrix: needs an fp64 plain-CSR matrix and output arrays");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  if (s->n > 0) {
    CGX_HIP(hipMemcpy(row_ptr, s->d_rp, ((size_t)s->n + 1) * 4, hipMemcpyDeviceToHost));
    if (s->nnz > 0) {
      CGX_HIP(hipMemcpy(col, s->d_col, (size_t)s->nnz * 4, hipMemcpyDeviceToHost));
      CGX_HIP(hipMemcpy(val, s->d_val, (size_t)s->nnz * 8, hipMemcpyDeviceToHost));
    }
  }
  return 0;
}

int cgx_solver_set_rhs(cgx_solver *s, const double *b) {
  return s ? upload_rhs<double>(s, b) : CGX_EINVAL;
}

int cgx_solver_set_rhs_f32(cgx_solver *s, const float *b) {
  return s ? upload_rhs<float>(s, b) : CGX_EINVAL;
}

int cgx_solver_run(cgx_solver *s, int maxit, double tol, int *iters) {
  if (!s || !s->have_matrix || !s->have_rhs || maxit < 0) {
    cgx::set_error("run: need matrix + rhs and maxit >= 0");
    return CGX_EINVAL;
  }
  if (s->dtype == CGX_F32 && s->mode == CGX_MODE_EXACT) {
    cgx::set_error("exact mode is fp64 only");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  if (s->n == 0) {  // empty system: nothing to iterate, x is empty
    s->last_iters = maxit + 1;
    if (iters) *iters = s->last_iters;
    return 0;
  }
  return s->dtype == CGX_F32 ? run_t<float>(s, maxit, tol, iters)
                             : run_t<double>(s, maxit, tol, iters);
}

int cgx_solver_get_x(cgx_solver *s, double *x) {
  if (!s || !s->have_matrix || s->dtype != CGX_F64 || (s->n && !x))
    return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpy(x, s->d_x, (size_t)s->n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int cgx_solver_get_x_f32(cgx_solver *s, float *x) {
  if (!s || !s->have_matrix || s->dtype != CGX_F32 || (s->n && !x))
    return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  CGX_HIP(hipMemcpy(x, s->d_x, (size_t)s->n * 4, hipMemcpyDeviceToHost));
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
  const double sv = (double)tsize(s->dtype);
  info->n = s->n;
  info->nnz = s->nnz;
  info->dtype = s->dtype;
  info->mode = s->mode;
  info->alg = s->alg;
  info->n_rowblocks = s->nblk;
  info->spmv_grid = s->spmv_grid;
  info->vec_grid = s->vec_grid;
  // B_spmv = nnz*(s_v+4) + 4*(n+1) + 2*n*s_v; B_iter = B_spmv + 9*n*s_v
  info->spmv_bytes = (double)s->nnz * (sv + 4) + 4.0 * (s->n + 1) + 2.0 * s->n * sv;
  info->iter_bytes = info->spmv_bytes + 9.0 * s->n * sv;
  if (s->sell)  // the SELL kernel's own algorithmic bytes: padded slices, no row_ptr
    info->spmv_iter_bytes = (double)s->sell_elems * (sv + 4) + 8.0 * s->nslices +
                            2.0 * s->n * sv;
  else
    info->spmv_iter_bytes = info->spmv_bytes;
  if (s->is_stencil)  // matrix-free: x read once, y written once
    info->spmv_iter_bytes = 2.0 * s->n * sv;
  if (s->npanel > 1)  // the panel passes' own bytes: P row_ptrs, y written P x, read P-1 x
    info->spmv_iter_bytes = (double)s->nnz * (sv + 4) + 4.0 * s->npanel * (s->n + 1.0) +
                            (double)s->n * sv * (1.0 + 2.0 * s->npanel - 1.0);
  if (fused(s)) info->spmv_iter_bytes += 2.0 * s->n * sv;
  if (s->ndict > 0)  // coded columns: one byte per nonzero + the dictionary
    info->spmv_iter_bytes = (double)s->nnz * (sv + s->code_bits / 8.0) + (s->d_rlen ? 1.0 * s->n : 4.0 * (s->n + 1)) +
                            2.0 * s->n * sv + 4.0 * s->ndict;
  info->device_bytes = s->dev_bytes;
  info->n_panels = s->npanel;
  if (s->ndict > 0 && s->vi)  // value-indexed pairs: no val stream
    info->spmv_iter_bytes = (double)s->nnz * (s->code_bits / 8.0) + (double)s->n +
                            2.0 * s->n * sv + (4.0 + sv) * s->ndict;
  info->n_dict = s->ndict;
  info->dict_vals = s->ndict > 0 && s->vi;
  info->tile_bands = s->tile_bands;
  return 0;
}

int cgx_solver_bench_prepare(cgx_solver *s, int warmup) {
  if (!s || !s->have_matrix || !s->have_rhs || s->n == 0 || warmup < 0) {
    cgx::set_error("bench_prepare: need a non-empty system and warmup >= 0");
    return CGX_EINVAL;
  }
  if (s->mode == CGX_MODE_EXACT && s->dtype == CGX_F32) return CGX_EINVAL;
  CGX_HIP(hipSetDevice(s->device));
  return s->dtype == CGX_F32 ? bench_prepare_t<float>(s, warmup)
                             : bench_prepare_t<double>(s, warmup);
}

int cgx_solver_bench_run(cgx_solver *s, int iters, int flags, double *total_ms,
                         double *spmv_ms) {
  if (!s || !s->bench_ready || iters < 1 || !total_ms || !spmv_ms) {
    cgx::set_error("bench_run: call cgx_solver_bench_prepare first; iters >= 1");
    return CGX_EINVAL;
  }
  CGX_HIP(hipSetDevice(s->device));
  return s->dtype == CGX_F32
             ? bench_run_t<float>(s, iters, flags, total_ms, spmv_ms)
             : bench_run_t<double>(s, iters, flags, total_ms, spmv_ms);
}

int cgx_solver_bench(cgx_solver *s, int warmup, int iters, int flags,
                     double *total_ms, double *spmv_ms) {
  int rc = cgx_solver_bench_prepare(s, warmup);
  if (rc) return rc;
  return cgx_solver_bench_run(s, iters, flags, total_ms, spmv_ms);
}

}  // extern "C"
