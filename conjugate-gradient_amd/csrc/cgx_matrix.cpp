// cgx_matrix.cpp -- DevMatrix (cgx_matrix.h): layout choice, encoding and
// upload of a CSR matrix, and the SpMV launch over its layout.
#include "cgx_matrix.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace cgx {

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int host_threads(long long work) {
  int nt = (int)std::min<long long>(16, std::max<long long>(1, work >> 21));
  return std::max(1, std::min(nt, (int)std::thread::hardware_concurrency()));
}

// Runs f(t, lo, hi) over [0, n) split into contiguous ranges on up to 16
// host threads.
template <typename F>
void parallel_rows(long long n, long long work, F f) {
  const int nt = host_threads(work);
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(f, t, n * t / nt, n * (t + 1) / nt);
  f(0, 0, n / nt);
  for (auto &x : th) x.join();
}

template <typename T>
unsigned long long bits_of(T v) {
  unsigned long long b = 0;
  memcpy(&b, &v, sizeof v);
  return b;
}

// Small open-addressing set of (offset, value bits) keys; gives up past cap.
struct PairSet {
  static constexpr int kSlots = 1024;
  int off[kSlots];
  unsigned long long vb[kSlots];
  bool used[kSlots];
  int count = 0;
  PairSet() { memset(used, 0, sizeof used); }
  static unsigned hash(int o, unsigned long long b) {
    const unsigned long long h = ((unsigned long long)(unsigned)o * 0x9e3779b97f4a7c15ULL) ^
                                 (b * 0xbf58476d1ce4e5b9ULL);
    return (unsigned)(h >> 54);  // 10 bits
  }
  // false when the set is full (more than cap distinct keys)
  bool add(int o, unsigned long long b, int cap) {
    unsigned h = hash(o, b);
    while (used[h]) {
      if (off[h] == o && vb[h] == b) return true;
      h = (h + 1) & (kSlots - 1);
    }
    if (count >= cap) return false;
    used[h] = true;
    off[h] = o;
    vb[h] = b;
    ++count;
    return true;
  }
};

// Distinct (col - row, value bits) pairs of rows [lo, hi) -- with_vals false:
// offsets only (vb = 0).  Returns false past cap distinct keys.
// Entry j of a row usually repeats entry j of the previous scanned row
// (stencils): those keys skip the hash set.
template <typename T>
bool scan_pairs(const int *rp, const int *col, const T *val, long long lo, long long hi,
                long long step, bool with_vals, int cap, PairSet &S) {
  constexpr int M = 32;
  int po[M];
  unsigned long long pb[M];
  int plen = 0;
  for (long long r = lo; r < hi; r += step) {
    const int k0 = rp[r], len = rp[r + 1] - k0;
    for (int j = 0; j < len; ++j) {
      const int o = col[k0 + j] - (int)r;
      const unsigned long long b = with_vals ? bits_of(val[k0 + j]) : 0ULL;
      if (j < plen && po[j] == o && pb[j] == b) continue;
      if (!S.add(o, b, cap)) return false;
      if (j < M) {
        po[j] = o;
        pb[j] = b;
      }
    }
    plen = std::min(len, M);
  }
  return true;
}

// Candidate keys: sampled rows (sample) or every row, on host threads; the
// merged set sorted by offset, then value bits (as unsigned).  Empty when
// more than cap distinct keys were found.
template <typename T>
bool find_pairs(int n, const int *rp, const int *col, const T *val, bool with_vals, int cap,
                bool sample, std::vector<int> &off, std::vector<T> &pv) {
  off.clear();
  pv.clear();
  std::vector<PairSet> sets;
  std::vector<int> ok;
  if (sample) {
    // ~64 K rows: every step-th row plus the first and last 4096 rows
    sets.resize(1);
    ok.assign(1, 1);
    const long long step = std::max<long long>(1, n / 65536);
    PairSet &S = sets[0];
    ok[0] = scan_pairs(rp, col, val, 0, std::min(n, 4096), 1, with_vals, cap, S) &&
            scan_pairs(rp, col, val, 0, n, step, with_vals, cap, S) &&
            scan_pairs(rp, col, val, std::max(0, n - 4096), n, 1, with_vals, cap, S);
  } else {
    const int nt = host_threads(rp[n]);
    sets.resize(nt);
    ok.assign(nt, 1);
    parallel_rows(n, rp[n], [&](int t, long long lo, long long hi) {
      ok[t] = scan_pairs(rp, col, val, lo, hi, 1, with_vals, cap, sets[t]);
    });
  }
  PairSet all;
  for (size_t t = 0; t < sets.size(); ++t) {
    if (!ok[t]) return false;
    for (int h = 0; h < PairSet::kSlots; ++h)
      if (sets[t].used[h] && !all.add(sets[t].off[h], sets[t].vb[h], cap)) return false;
  }
  std::vector<std::pair<int, unsigned long long>> keys;
  for (int h = 0; h < PairSet::kSlots; ++h)
    if (all.used[h]) keys.push_back({all.off[h], all.vb[h]});
  std::sort(keys.begin(), keys.end());
  for (auto &k : keys) {
    off.push_back(k.first);
    T v{};
    memcpy(&v, &k.second, sizeof v);
    pv.push_back(v);
  }
  return !keys.empty();
}

// Column panels for matrices whose gathers have no locality (SURVEY.md C5:
// random SPD).  x is read through per-XCD L2s of 4 MiB; when x is larger and
// most entries lie far from the diagonal, every gather is a line fetched
// from the Infinity Cache.  Splitting the columns into panels whose x slice
// fits an L2 and running one SpMV pass per panel keeps the gathers
// L2-resident, for P row_ptr reads and P-1 y round trips more.  Auto: x >
// 8 MiB and >= 30 % of (sampled) entries more than a panel width (3.5 MiB of
// x, of the L2's 4: C5's sweep -- 1 / 3 / 5 / 6 / 7 / 8 / 10 / 14 / 20
// panels: 221 / 392 / 560 / 626 / 622 / 604 / 593 / 550 / 489 it/s) from the
// diagonal.
int choose_panels(int n, const int *rp, const int *col, size_t tsize, bool force) {
  const long long pcols = std::max<long long>(1024, 3584LL * 1024 / (long long)tsize);
  if (n <= pcols) return 1;
  if (!force) {
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

// Panel-major CSR: panel q holds, for every row, the row's entries with
// column in [q*pc, (q+1)*pc), in the row's order; prp[q*(n+1) + i] are
// offsets into the concatenated col/val.  The entries of a row ascend in
// column, so summing panel after panel is the reference's sequential order.
template <typename T>
void build_panels(int n, int ncols, const int *rp, const int *col, const T *val, int P,
                  std::vector<int> &prp, std::vector<int> &pcol, std::vector<T> &pval) {
  const int nnz = rp[n];
  const long long pc = ((long long)ncols + P - 1) / P;
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

// DIA-VI codes cover whole 512-row slices (two rows per thread).
int padded_rows_for(int n) {
  return (int)(((long long)n + kDiaSliceRows - 1) / kDiaSliceRows * kDiaSliceRows);
}

// DIA-VI candidates from the sorted (offset, value bits) keys: <= 16
// diagonals, <= 15 values each, in an order every row's entries follow.
// The order is a topological sort (ties by offset) of "offset a comes
// before offset b in some row", from the same rows the keys came from
// (sample: every step-th row plus the first and last 4096; else all): a
// stored row in ascending columns gives ascending offsets, but a partition's
// ghost columns (local n_loc + position, after the owned ones) come first
// in the rows of its first plane -- the diagonal order is then [ghost below,
// -pl, ..., +pl, ghost above] and the sums stay in the rows' order.  The
// device encoder checks every row against it.  vt[16 k + v] = value v of
// diagonal k.
template <typename T>
bool group_dia(int n, const int *rp, const int *col, bool sample, const std::vector<int> &poff,
               const std::vector<T> &pval, DiaCand &c, std::vector<T> &vt) {
  memset(&c, 0, sizeof c);
  vt.assign(kDiaMax * 16, T(0));
  std::vector<int> offs;
  for (size_t i = 0; i < poff.size(); ++i)
    if (i == 0 || poff[i] != poff[i - 1]) offs.push_back(poff[i]);
  const int K = (int)offs.size();
  if (K == 0 || K > kDiaMax) return false;
  auto idx = [&](int o) {  // K when o is not a candidate
    const int i = (int)(std::lower_bound(offs.begin(), offs.end(), o) - offs.begin());
    return i < K && offs[(size_t)i] == o ? i : K;
  };
  // before[a] bit b: offset a precedes offset b in some scanned row
  const int nt = sample ? 1 : host_threads(rp[n]);
  std::vector<std::array<unsigned, kDiaMax>> before((size_t)nt);
  for (auto &b : before) b.fill(0u);
  auto scan = [&](std::array<unsigned, kDiaMax> &b, long long lo, long long hi, long long step) {
    for (long long r = lo; r < hi; r += step)
      for (int k = rp[r] + 1; k < rp[r + 1]; ++k) {
        const int a = idx(col[k - 1] - (int)r), z = idx(col[k] - (int)r);
        if (a < K && z < K) b[(size_t)a] |= 1u << z;
      }
  };
  if (!col) {
    // generated Laplacian: its rows ascend in column, i.e. in offset
  } else if (sample) {
    const long long step = std::max<long long>(1, n / 65536);
    scan(before[0], 0, std::min(n, 4096), 1);
    scan(before[0], 0, n, step);
    scan(before[0], std::max(0, n - 4096), n, 1);
  } else {
    parallel_rows(n, rp[n], [&](int t, long long lo, long long hi) { scan(before[(size_t)t], lo, hi, 1); });
  }
  std::array<unsigned, kDiaMax> pred{};  // pred[b] bit a: a must come before b
  for (auto &b : before)
    for (int a = 0; a < K; ++a)
      for (int z = 0; z < K; ++z)
        if (b[(size_t)a] >> z & 1u) pred[(size_t)z] |= 1u << a;
  std::vector<int> order;
  unsigned placed = 0;
  while ((int)order.size() < K) {
    int pick = -1;
    for (int q = 0; q < K && pick < 0; ++q)  // smallest offset whose predecessors are placed
      if (!(placed >> q & 1u) && (pred[(size_t)q] & ~placed) == 0) pick = q;
    if (pick < 0) return false;  // the rows disagree on the order: no DIA
    order.push_back(pick);
    placed |= 1u << pick;
  }
  std::vector<int> pos((size_t)K);
  for (int k = 0; k < K; ++k) {
    pos[(size_t)order[(size_t)k]] = k;
    c.doff[k] = offs[(size_t)order[(size_t)k]];
  }
  c.ndiag = K;
  for (size_t i = 0; i < poff.size(); ++i) {
    const int k = pos[(size_t)idx(poff[i])];
    if (c.nval[k] == kDiaVals) return false;
    vt[(size_t)k * 16 + c.nval[k]++] = pval[i];
  }
  dia_pack(c);
  return true;
}

// DIA-VI codes of every row on host threads, the device encoder's checks
// (k_dia_encode) plus the column range: 0 = encoded, 1 = a row leaves the
// candidates (diagonal, value or order), 2 = a column outside [0, ncols).
// A row's entries follow the diagonal order, so the search for the next
// entry's diagonal starts after the previous one's.
template <typename T>
int dia_encode_host(int n, int npad, int col_lo, int ncols, const int *rp, const int *col,
                    const T *val, const DiaCand &c, const std::vector<T> &vt,
                    std::vector<unsigned char> &code) {
  const int cb = c.cbytes;
  unsigned long long empty = 0;
  for (int q = 0; q < c.ndiag; ++q) empty |= ((1ull << c.cbits[q]) - 1ull) << c.csh[q];
  code.resize((size_t)npad * cb);
  const int nt = host_threads(rp[n]);
  std::vector<int> res((size_t)nt, 0);
  parallel_rows(n, rp[n], [&](int t, long long lo, long long hi) {
    // thread-local copies: the byte stores below may alias anything the
    // compiler cannot prove private, and would force reloads per entry
    int doff[kDiaMax], nval[kDiaMax], sh[kDiaMax];
    unsigned long long fm[kDiaMax], vb[kDiaMax * 16];
    const int K = c.ndiag;
    for (int q = 0; q < K; ++q) {
      doff[q] = c.doff[q];
      nval[q] = c.nval[q];
      sh[q] = c.csh[q];
      fm[q] = ((1ull << c.cbits[q]) - 1ull) << c.csh[q];
      for (int v = 0; v < nval[q]; ++v) vb[q * 16 + v] = bits_of(vt[(size_t)q * 16 + v]);
    }
    const unsigned nc = (unsigned)(ncols - col_lo);
    const unsigned long long e0 = empty;
    int err = 0;
    for (long long r = lo; r < hi && !err; ++r) {
      unsigned long long w = e0;
      int q = 0;
      const int k1 = rp[r + 1];
      for (int k = rp[r]; k < k1; ++k) {
        const int cl = col[k];
        if ((unsigned)(cl - col_lo) >= nc) {
          err = 2;
          break;
        }
        const int off = cl - (int)r;
        while (q < K && doff[q] != off) ++q;
        if (q == K) {
          err = 1;
          break;
        }
        const unsigned long long b = bits_of(val[k]);
        int v = 0;
        while (v < nval[q] && vb[q * 16 + v] != b) ++v;
        if (v == nval[q]) {
          err = 1;
          break;
        }
        w = (w & ~fm[q]) | ((unsigned long long)v << sh[q]);
        ++q;
      }
      unsigned char *p = code.data() + (size_t)r * cb;
      switch (cb) {  // little-endian low bytes of the word
        case 1: *p = (unsigned char)w; break;
        case 2: memcpy(p, &w, 2); break;
        case 4: memcpy(p, &w, 4); break;
        default: memcpy(p, &w, 8); break;
      }
    }
    res[(size_t)t] = err;
  });
  for (long long r = n; r < npad; ++r) memcpy(code.data() + (size_t)r * cb, &empty, (size_t)cb);
  int e = 0;
  for (int x : res) e = std::max(e, x);
  return e;
}

// DIA-V of every row on host threads: dia_encode_host's diagonal-order and
// column checks, each diagonal's one-bit field 0 where the row has an entry
// (1, all ones: none) and the entry's value at dval[k npad + r] (0 where
// none, and in the padding rows).  Same return codes.
template <typename T>
int dia_v_encode_host(int n, int npad, int col_lo, int ncols, const int *rp, const int *col,
                      const T *val, const DiaCand &c, std::vector<unsigned char> &code,
                      std::vector<T> &dval) {
  if (c.cbytes != 1 || c.ndiag > kDiaVMax) return 1;
  unsigned empty = 0;
  for (int q = 0; q < c.ndiag; ++q) empty |= 1u << c.csh[q];
  code.assign((size_t)npad, (unsigned char)empty);
  dval.assign((size_t)c.ndiag * npad, T(0));
  const int nt = host_threads(rp[n]);
  std::vector<int> res((size_t)nt, 0);
  parallel_rows(n, rp[n], [&](int t, long long lo, long long hi) {
    int doff[kDiaVMax], sh[kDiaVMax];
    const int K = c.ndiag;
    for (int q = 0; q < K; ++q) {
      doff[q] = c.doff[q];
      sh[q] = c.csh[q];
    }
    T *dv = dval.data();
    int err = 0;
    for (long long r = lo; r < hi && !err; ++r) {
      unsigned w = empty;
      int q = 0;
      for (int k = rp[r]; k < rp[r + 1]; ++k) {
        const int cl = col[k];
        if ((unsigned)(cl - col_lo) >= (unsigned)(ncols - col_lo)) {
          err = 2;
          break;
        }
        const int off = cl - (int)r;
        while (q < K && doff[q] != off) ++q;
        if (q == K) {
          err = 1;
          break;
        }
        w &= ~(1u << sh[q]);
        dv[(size_t)q * npad + r] = val[k];
        ++q;
      }
      code[(size_t)r] = (unsigned char)w;
    }
    res[(size_t)t] = err;
  });
  int e = 0;
  for (int x : res) e = std::max(e, x);
  return e;
}

}  // namespace

void dia_pack(DiaCand &c) {
  int sh = 0;
  for (int k = 0; k < kDiaMax; ++k) {
    const int v = k < c.ndiag ? c.nval[k] : 0;
    c.cbits[k] = k < c.ndiag ? (v <= 1 ? 1 : v <= 3 ? 2 : v <= 7 ? 3 : 4) : 0;
    c.csh[k] = sh;
    sh += c.cbits[k];
  }
  c.cbytes = sh <= 8 ? 1 : sh <= 16 ? 2 : sh <= 32 ? 4 : 8;
}

namespace {

// L2 tiling of the item order for a wide stencil: the x lines a row needs sit
// at its offsets; with P = the largest |offset| (a 3-D stencil's plane), an
// XCD sweeping rows in order needs ~3 P x-values resident to hit its 4 MiB
// L2 on every re-read.  When that exceeds the budget, sweep the rows in T
// bands of the P-periodic position instead (all planes of band 0, then band
// 1, ...): ~3 P / T values in flight.  Only the order of the work items
// changes -- each row's sum is the same.
std::vector<int> tile_order(const std::vector<int> &item_row, long long P, size_t tsize,
                            int &bands) {
  bands = 0;
  const long long budget = 1536LL * 1024;
  const long long need = 3 * P * (long long)tsize;
  const int ni = (int)item_row.size() - 1;
  if (P <= 0 || need <= budget || ni <= 0) return {};
  const long long T_ = (need + budget - 1) / budget;
  std::vector<int> order((size_t)ni);
  for (int b = 0; b < ni; ++b) order[(size_t)b] = b;
  auto band = [&](int b) { return (long long)item_row[(size_t)b] % P * T_ / P; };
  auto plane = [&](int b) { return (long long)item_row[(size_t)b] / P; };
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    const long long bx = band(x), by = band(y);
    return bx != by ? bx < by : plane(x) < plane(y);
  });
  bands = (int)T_;
  return order;
}

}  // namespace

std::vector<int> fuse_pairs(const std::vector<int> &slices) {
  std::vector<int> p;
  const int m = (int)slices.size();
  for (int i = 0; i < m;) {
    const int c = i + 1 < m && slices[(size_t)i + 1] == slices[(size_t)i] + 1 ? 2 : 1;
    p.push_back(i);
    p.push_back(c);
    i += c;
  }
  return p;
}

std::vector<int> plan_rowblocks(int n, const int *rp, int rows, int cap) {
  std::vector<int> blk;
  blk.reserve((size_t)n / 48 + 2);
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

void DevMatrix::release() {
  dev_free(&d_rp);
  dev_free(&d_col);
  dev_free(&d_val);
  dev_free(&d_blkrk);
  dev_free(&d_code);
  dev_free(&d_rlen);
  dev_free(&d_dict);
  dev_free(&d_dcode);
  dev_free(&d_vtab);
  dev_free(&d_dval);
  dev_free(&d_order);
  dev_free(&d_fpairs);
  dev_free(&d_mpos);
  n_fpairs = 0;
  mq = mchains = mws = mlen = mfar = 0;
  msb = 1;
  order.clear();
  blk_row.clear();
  panel_first.clear();
  panel_count.clear();
  n = nnz = ncols = nblk = ndict = tile_bands = 0;
  col_lo = 0;
  csr_reach = 0;
  memset(&dia, 0, sizeof dia);
  kdiag = -1;
  gath = 8;
  npanel = 1;
  layout = L_CSR;
  nt = false;
  dev_bytes = 0;
  encode_fallback = 0;
  setup_host_ms = setup_dev_ms = 0;
}

int DevMatrix::set_stencil(const LapSpec &g) {
  release();
  const long long nn = (long long)g.nx * g.ny * g.nz;
  if ((g.dim != 2 && g.dim != 3) || g.nx < 1 || g.ny < 1 || g.nz < 1 ||
      (g.dim == 2 && g.nz != 1) || nn > INT32_MAX || lap_rp(nn, g) > INT32_MAX) {
    set_error("set_stencil: bad grid");
    return CGX_EINVAL;
  }
  dtype = CGX_F64;
  n = ncols = (int)nn;
  nnz = (int)lap_rp(nn, g);
  layout = L_STENCIL;
  lap = g;
  nt = 16.0 * n + 40.0 * n > kMallBytes;
  return 0;
}

template <typename T>
int DevMatrix::upload(int n_, int ncols_, int nnz_, const int *rp, const int *col, const T *val,
                      int want, bool allow_panels, const LapSpec *gen, int col_lo_,
                      bool allow_dv) {
  const double t0 = now_ms();
  if (n_ < 0 || nnz_ < 0 || ncols_ < n_ || col_lo_ > 0 || (col_lo_ < 0 && (gen || !col)) ||
      (n_ > 0 && (!rp || (nnz_ > 0 && !gen && (!col || !val))))) {
    set_error("set_matrix: invalid arguments");
    return CGX_EINVAL;
  }
  if (n_ > 0 && (rp[0] != 0 || rp[n_] != nnz_)) {
    set_error("set_matrix: row_ptr[0] must be 0 and row_ptr[n] == nnz");
    return CGX_EINVAL;
  }
  // row_ptr non-decreasing (and the longest row) on host threads; columns
  // inside x are checked by the DIA host encoder or, for the other layouts,
  // before the upload: a bad index would be an out-of-bounds device gather
  int maxlen = 0;
  {
    const int nt = host_threads(n_);
    std::vector<int> bad((size_t)nt, -1), mx((size_t)nt, 0);
    parallel_rows(n_, n_, [&](int t, long long lo, long long hi) {
      int m = 0;
      for (long long r = lo; r < hi; ++r) {
        const int len = rp[r + 1] - rp[r];
        if (len < 0) {
          bad[(size_t)t] = (int)r;
          return;
        }
        m = std::max(m, len);
      }
      mx[(size_t)t] = m;
    });
    for (int t = 0; t < nt; ++t) {
      if (bad[(size_t)t] >= 0) {
        set_error("set_matrix: row_ptr decreases at row %d", bad[(size_t)t]);
        return CGX_EINVAL;
      }
      maxlen = std::max(maxlen, mx[(size_t)t]);
    }
  }
  auto bad_column = [&]() {
    set_error("set_matrix: a column index is outside [%d, %d)", col_lo_, ncols_);
    return CGX_EINVAL;
  };
  release();
  dtype = sizeof(T) == 4 ? CGX_F32 : CGX_F64;
  n = n_;
  ncols = ncols_;
  col_lo = col_lo_;
  nnz = nnz_;
  const size_t ts = sizeof(T);
  const size_t nnz_pad = ((size_t)nnz + kPad - 1) / kPad * kPad + kWindowPad;
  int rc;

  // ---- which layout: candidates from a sample (or the generator's stencil)
  const bool want_dia = want == CGX_LAYOUT_AUTO || want == CGX_LAYOUT_DIA;
  const bool want_dc = (want_dia || want == CGX_LAYOUT_DC) && col_lo == 0;
  std::vector<int> poff;  // (offset, value) keys, sorted
  std::vector<T> pval, vt;
  bool dia_ok = false, dc_ok = false;
  if (n > 0 && nnz > 0 && want_dia) {
    if (gen) {  // one value per offset: 2 dim on the diagonal, -1 off it
      poff = lap_offsets(*gen);
      for (int o : poff) pval.push_back(o == 0 ? T(2 * gen->dim) : T(-1));
      dia_ok = group_dia<T>(n, rp, nullptr, true, poff, pval, dia, vt);
    } else if (maxlen <= kDiaMax) {
      dia_ok = find_pairs(n, rp, col, val, true, kDiaMax * kDiaVals, true, poff, pval) &&
               group_dia(n, rp, col, true, poff, pval, dia, vt);
    }
  }

  // ---- DIA-VI from a host matrix: encoded on host threads (every row
  // checked), only the codes and value tables go to the device -- no CSR
  // upload (1 code byte per row instead of 12 bytes per nonzero over PCIe)
  const int npad = padded_rows_for(n);
  if (dia_ok && !gen) {
    std::vector<unsigned char> hcode;
    int e = dia_encode_host(n, npad, col_lo, ncols, rp, col, val, dia, vt, hcode);
    if (e == 1) {  // the sample missed a diagonal or a value: exact scan
      encode_fallback = 1;
      dia_ok = find_pairs(n, rp, col, val, true, kDiaMax * kDiaVals, false, poff, pval) &&
               group_dia(n, rp, col, false, poff, pval, dia, vt);
      if (dia_ok) e = dia_encode_host(n, npad, col_lo, ncols, rp, col, val, dia, vt, hcode);
    }
    if (e == 2) {
      release();
      return bad_column();
    }
    dia_ok = dia_ok && e == 0;
    if (dia_ok) {
      if ((rc = dev_alloc(&d_dcode, hcode.size() + 16, &dev_bytes)) ||
          (rc = dev_alloc(&d_vtab, (size_t)kDiaMax * 16 * ts, &dev_bytes))) {
        release();
        return rc;
      }
      CGX_HIP(hipMemcpyAsync(d_dcode, hcode.data(), hcode.size(), hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d_vtab, vt.data(), (size_t)kDiaMax * 16 * ts, hipMemcpyHostToDevice, st));
      CGX_HIP(hipStreamSynchronize(st));  // hcode goes out of scope
      layout = L_DIA;
      for (int k = 0; k < dia.ndiag; ++k)
        if (dia.doff[k] == 0) kdiag = k;
      return finish_upload(t0);
    }
    memset(&dia, 0, sizeof dia);
  }

  // ---- DIA-V (allow_dv): the nonzeros on <= 8 diagonals with values no
  // table indexes (general coefficients): one presence byte per row and the
  // values diagonal-major -- 1 + s_v ndiag bytes per row against CSR-DC's
  // (s_v + 1) per nonzero + 1 -- so the plane march, and with it the
  // one-launch SR step, applies to them (k_sr1_dia_m<..., DV>)
  if (!dia_ok && !gen && allow_dv && want_dia && n > 0 && nnz > 0 && maxlen <= kDiaVMax) {
    std::vector<int> voff;
    std::vector<T> vzero, vt_unused;
    DiaCand c{};
    bool ok = find_pairs(n, rp, col, val, false, kDiaVMax, true, voff, vzero) &&
              group_dia(n, rp, col, true, voff, vzero, c, vt_unused);
    std::vector<unsigned char> hcode;
    std::vector<T> hval;
    int e = ok ? dia_v_encode_host(n, npad, col_lo, ncols, rp, col, val, c, hcode, hval) : 1;
    if (ok && e == 1) {  // the sample missed a diagonal: exact scan
      ok = find_pairs(n, rp, col, val, false, kDiaVMax, false, voff, vzero) &&
           group_dia(n, rp, col, false, voff, vzero, c, vt_unused);
      if (ok) e = dia_v_encode_host(n, npad, col_lo, ncols, rp, col, val, c, hcode, hval);
    }
    if (e == 2) {
      release();
      return bad_column();
    }
    const double dv_row = 1.0 + (double)ts * c.ndiag, dc_row = (ts + 1.0) * nnz / n + 1.0;
    if (ok && e == 0 && dv_row <= dc_row) {
      // a zero value table: the kernels' table loads stay in bounds
      const std::vector<T> zt((size_t)kDiaMax * 16, T(0));
      if ((rc = dev_alloc(&d_dcode, hcode.size() + 16, &dev_bytes)) ||
          (rc = dev_alloc(&d_vtab, zt.size() * ts, &dev_bytes)) ||
          (rc = dev_alloc(&d_dval, hval.size() * ts + 16, &dev_bytes))) {
        release();
        return rc;
      }
      CGX_HIP(hipMemcpyAsync(d_dcode, hcode.data(), hcode.size(), hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d_vtab, zt.data(), zt.size() * ts, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d_dval, hval.data(), hval.size() * ts, hipMemcpyHostToDevice, st));
      CGX_HIP(hipStreamSynchronize(st));  // the host arrays go out of scope
      dia = c;
      dia_ok = true;
      layout = L_DIA;
      for (int k = 0; k < dia.ndiag; ++k)
        if (dia.doff[k] == 0) kdiag = k;
      return finish_upload(t0);
    }
  }
  if (col_lo < 0) {  // the in-place numbering exists for the DIA step only
    release();
    set_error("set_matrix: in-place ghost columns need the DIA-VI layout");
    return CGX_EINVAL;
  }
  if (!gen && nnz > 0) {
    std::vector<int> bad((size_t)host_threads(nnz), 0);
    parallel_rows(nnz, nnz, [&](int t, long long lo, long long hi) {
      for (long long k = lo; k < hi; ++k)
        if ((unsigned)col[k] >= (unsigned)ncols) {
          bad[(size_t)t] = 1;
          return;
        }
    });
    for (int b : bad)
      if (b) {
        release();
        return bad_column();
      }
  }

  std::vector<int> doff;
  if (!dia_ok && n > 0 && nnz > 0 && want_dc && maxlen <= 255) {
    std::vector<T> dummy;
    if (gen) {
      doff = lap_offsets(*gen);
      dc_ok = true;
    } else {
      dc_ok = find_pairs(n, rp, col, val, false, 256, true, doff, dummy);
    }
  }

  // ---- CSR arrays (panels for irregular fp matrices on one GPU)
  std::vector<int> prp, pcol;
  std::vector<T> pval_panel;
  const bool want_panel = want == CGX_LAYOUT_PANEL;
  npanel = 1;
  if (!dia_ok && !dc_ok && !gen && n > 0 && nnz > 0 && allow_panels &&
      (want == CGX_LAYOUT_AUTO || want_panel))
    npanel = choose_panels(n, rp, col, ts, want_panel);
  if (npanel > 1) {
    build_panels<T>(n, ncols, rp, col, val, npanel, prp, pcol, pval_panel);
  }
  const int *urp = npanel > 1 ? prp.data() : rp;
  const int *ucol = npanel > 1 ? pcol.data() : col;
  const T *uval = npanel > 1 ? pval_panel.data() : val;
  const size_t rp_len = (size_t)npanel * ((size_t)n + 1);
  if ((rc = dev_alloc(&d_rp, rp_len * 4 + 256, &dev_bytes)) ||
      (rc = dev_alloc(&d_col, nnz_pad * 4, &dev_bytes)) ||
      (rc = dev_alloc(&d_val, nnz_pad * ts, &dev_bytes))) {
    release();
    return rc;
  }
  CGX_HIP(hipMemsetAsync(d_col + nnz, 0, (nnz_pad - nnz) * 4, st));
  CGX_HIP(hipMemsetAsync((char *)d_val + (size_t)nnz * ts, 0, (nnz_pad - nnz) * ts, st));
  if (n > 0) {
    CGX_HIP(hipMemcpyAsync(d_rp, urp, rp_len * 4, hipMemcpyHostToDevice, st));
    if (nnz > 0 && gen) {
      CGX_HIP(launch_gen_laplacian(*gen, n, d_col, (double *)d_val, st));
    } else if (nnz > 0) {
      CGX_HIP(hipMemcpyAsync(d_col, ucol, (size_t)nnz * 4, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemcpyAsync(d_val, uval, (size_t)nnz * ts, hipMemcpyHostToDevice, st));
    }
  }

  int *d_err = nullptr;
  CGX_HIP(hipMalloc((void **)&d_err, 16));
  auto read_err = [&](int *out) -> int {
    CGX_HIP(hipMemcpyAsync(out, d_err, 4, hipMemcpyDeviceToHost, st));
    CGX_HIP(hipStreamSynchronize(st));
    return 0;
  };
  auto fail = [&](int code) {
    (void)hipFree(d_err);
    release();
    return code;
  };

  // ---- DIA-VI of a device-generated matrix: device encode against the
  // stencil's candidates, then the generated CSR is dropped
  if (dia_ok) {
    for (int attempt = 0; attempt < 2 && dia_ok; ++attempt) {
      dev_free(&d_dcode);
      dev_free(&d_vtab);
      if ((rc = dev_alloc(&d_dcode, (size_t)npad * dia.cbytes + 16, &dev_bytes)) ||
          (rc = dev_alloc(&d_vtab, (size_t)kDiaMax * 16 * ts, &dev_bytes)))
        return fail(rc);
      CGX_HIP(hipMemcpyAsync(d_vtab, vt.data(), (size_t)kDiaMax * 16 * ts, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemsetAsync(d_err, 0, 4, st));
      CGX_HIP(launch_dia_encode<T>(n, npad, d_rp, d_col, (const T *)d_val, dia, (const T *)d_vtab,
                                   d_dcode, d_err, st));
      int err = 0;
      if ((rc = read_err(&err))) return fail(rc);
      if (!err) break;
      dia_ok = false;
    }
    if (dia_ok) {
      layout = L_DIA;
      kdiag = -1;
      for (int k = 0; k < dia.ndiag; ++k)
        if (dia.doff[k] == 0) kdiag = k;
      (void)hipFree(d_err);
      CGX_HIP(hipStreamSynchronize(st));
      dev_free(&d_rp);
      dev_free(&d_col);
      dev_free(&d_val);
      return finish_upload(t0);
    } else {
      dev_free(&d_dcode);
      dev_free(&d_vtab);
      memset(&dia, 0, sizeof dia);
      if (want_dc && maxlen <= 255 && !dc_ok) {
        std::vector<T> dummy;
        if (gen) {
          doff = lap_offsets(*gen);
          dc_ok = true;
        } else {
          dc_ok = find_pairs(n, rp, col, val, false, 256, true, doff, dummy);
        }
      }
    }
  }

  // ---- row blocks (CSR / DC)
  gath = nnz <= 7LL * n ? 7 : 8;
  if (layout != L_DIA) {
    capw = ts == 4 ? 1024 : 512;
    if (ts == 8 && npanel == 1 && n > 0) {
      // LDS window sized to the matrix: 328 entries when every 64-row block
      // fits (5-point stencils, C2: one more workgroup per CU)
      int m = 0;
      for (int r = 0; r < n; r += 64) m = std::max(m, rp[std::min(r + 64, n)] - rp[r]);
      if (m + kPad <= 328) capw = 328;
      else if (m + kPad <= 456) capw = 456;  // 7-point stencils (C3): 7 workgroups per CU, not 6
    }
    std::vector<int> blkrk;
    blk_row.clear();
    panel_first.clear();
    panel_count.clear();
    for (int q = 0; q < npanel; ++q) {
      const int *rq = urp + (size_t)q * (n + 1);
      std::vector<int> b = n > 0 ? plan_rowblocks(n, rq, 64, capw - kPad) : std::vector<int>{0};
      panel_first.push_back((int)(blkrk.size() / 2));
      panel_count.push_back((int)b.size() - 1);
      for (size_t i = 0; i < b.size(); ++i) {
        blkrk.push_back(b[i]);
        blkrk.push_back(rq[b[i]]);
      }
      if (q == 0) blk_row = b;
    }
    nblk = panel_count.empty() ? 0 : panel_count[0];
    if ((rc = dev_alloc(&d_blkrk, blkrk.size() * 4 + 16, &dev_bytes))) return fail(rc);
    CGX_HIP(hipMemcpyAsync(d_blkrk, blkrk.data(), blkrk.size() * 4, hipMemcpyHostToDevice, st));
    CGX_HIP(hipStreamSynchronize(st));  // blkrk goes out of scope
  }

  // ---- CSR-DC
  if (layout != L_DIA && dc_ok && npanel == 1) {
    if ((rc = dev_alloc(&d_code, nnz_pad, &dev_bytes)) ||
        (rc = dev_alloc(&d_dict, 256 * 4, &dev_bytes)) ||
        (rc = dev_alloc(&d_rlen, (size_t)n + 64, &dev_bytes)))
      return fail(rc);
    std::vector<unsigned char> rl((size_t)n);
    for (int r = 0; r < n; ++r) rl[(size_t)r] = (unsigned char)(rp[r + 1] - rp[r]);
    CGX_HIP(hipMemcpyAsync(d_rlen, rl.data(), (size_t)n, hipMemcpyHostToDevice, st));
    CGX_HIP(hipMemsetAsync(d_code, 0, nnz_pad, st));
    for (int attempt = 0; attempt < 2 && dc_ok; ++attempt) {
      std::vector<int> dd = doff;
      dd.resize(256, 0);
      CGX_HIP(hipMemcpyAsync(d_dict, dd.data(), 256 * 4, hipMemcpyHostToDevice, st));
      CGX_HIP(hipMemsetAsync(d_err, 0, 4, st));
      CGX_HIP(launch_dc_encode(n, d_rp, d_col, d_dict, (int)doff.size(), d_code, d_err, st));
      int err = 0;
      if ((rc = read_err(&err))) return fail(rc);
      if (!err) break;
      if (attempt == 0 && !gen) {
        encode_fallback = 1;
        std::vector<T> dummy;
        dc_ok = find_pairs(n, rp, col, val, false, 256, false, doff, dummy);
      } else {
        dc_ok = false;
      }
    }
    CGX_HIP(hipStreamSynchronize(st));  // rl goes out of scope
    if (dc_ok) {
      ndict = (int)doff.size();
      layout = L_DC;
    } else {
      dev_free(&d_code);
      dev_free(&d_dict);
      dev_free(&d_rlen);
    }
  }
  (void)hipFree(d_err);
  // plain CSR of a banded matrix (<= 256 distinct col - row offsets in the
  // sampled rows, or a generated stencil): its reach, for the L2-tiled order
  csr_reach = 0;
  if (layout == L_CSR && npanel == 1 && n > 0 && nnz > 0) {
    std::vector<int> off = doff;
    std::vector<T> dummy;
    if (off.empty()) {
      if (gen) off = lap_offsets(*gen);
      else if (!find_pairs(n, rp, col, val, false, 256, true, off, dummy)) off.clear();
    }
    for (int v : off) csr_reach = std::max(csr_reach, (long long)std::abs(v));
  }
  return finish_upload(t0);
}

template int DevMatrix::upload<double>(int, int, int, const int *, const int *, const double *,
                                       int, bool, const LapSpec *, int, bool);
template int DevMatrix::upload<float>(int, int, int, const int *, const int *, const float *,
                                      int, bool, const LapSpec *, int, bool);

// The item order, the non-temporal choice and the setup times, once the
// layout's arrays are on the device.
int DevMatrix::finish_upload(double t0) {
  const size_t ts = dtype == CGX_F32 ? 4 : 8;
  int rc;
  std::vector<int> doff;
  if (layout == L_DC) {
    std::vector<int> dd((size_t)ndict);
    CGX_HIP(hipMemcpy(dd.data(), d_dict, (size_t)ndict * 4, hipMemcpyDeviceToHost));
    doff = dd;
  }

  // ---- L2-tiled item order for wide stencils (DC / DIA / banded CSR)
  if (layout == L_DC || layout == L_DIA || (layout == L_CSR && csr_reach > 0)) {
    long long P = csr_reach;
    if (layout == L_DIA)
      for (int k = 0; k < dia.ndiag; ++k) P = std::max(P, (long long)std::abs(dia.doff[k]));
    else if (layout == L_DC)
      for (int v : doff) P = std::max(P, (long long)std::abs(v));
    const std::vector<int> ir = item_rows();
    order = tile_order(ir, P, ts, tile_bands);
    if (!order.empty()) {
      // DIA: the fused step's super-items (adjacent slices of the order)
      const std::vector<int> fp = layout == L_DIA ? fuse_pairs(order) : std::vector<int>{};
      if ((rc = dev_alloc(&d_order, order.size() * 4, &dev_bytes)) ||
          (!fp.empty() && (rc = dev_alloc(&d_fpairs, fp.size() * 4, &dev_bytes)))) {
        release();
        return rc;
      }
      CGX_HIP(hipMemcpyAsync(d_order, order.data(), order.size() * 4, hipMemcpyHostToDevice, st));
      if (!fp.empty())
        CGX_HIP(hipMemcpyAsync(d_fpairs, fp.data(), fp.size() * 4, hipMemcpyHostToDevice, st));
      n_fpairs = (int)fp.size() / 2;
      CGX_HIP(hipStreamSynchronize(st));
    }
  }
  if ((rc = plan_march())) {
    release();
    return rc;
  }
  // the matrix stream and y bypass the caches when the iteration's working
  // set (this layout's stream + five vectors) cannot stay in the 256 MiB
  // Infinity Cache anyway: the vectors then keep what residency there is
  nt = layout_bytes() + 5.0 * ts * n > kMallBytes;
  const double t1 = now_ms();
  CGX_HIP(hipStreamSynchronize(st));
  setup_dev_ms = now_ms() - t1;
  setup_host_ms = t1 - t0;
  return 0;
}

int DevMatrix::download_csr(int *row_ptr, int *col, double *val) const {
  if (n == 0) return 0;
  if (layout != L_DIA) {
    CGX_HIP(hipMemcpy(row_ptr, d_rp, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost));
    if (nnz > 0) {
      CGX_HIP(hipMemcpy(col, d_col, (size_t)nnz * 4, hipMemcpyDeviceToHost));
      CGX_HIP(hipMemcpy(val, d_val, (size_t)nnz * 8, hipMemcpyDeviceToHost));
    }
    return 0;
  }
  // DIA: every row's fields in diagonal order are its entries in column order
  const int cb = dia.cbytes;
  std::vector<unsigned char> code((size_t)n * cb);
  std::vector<double> vt((size_t)kDiaMax * 16);
  CGX_HIP(hipMemcpy(code.data(), d_dcode, code.size(), hipMemcpyDeviceToHost));
  CGX_HIP(hipMemcpy(vt.data(), d_vtab, vt.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> dvv;  // DIA-V: the value of (row, diagonal) from the stream
  const int npad = padded_rows();
  if (dv()) {
    dvv.resize((size_t)dia.ndiag * npad);
    CGX_HIP(hipMemcpy(dvv.data(), d_dval, dvv.size() * 8, hipMemcpyDeviceToHost));
  }
  long long k = 0;
  row_ptr[0] = 0;
  for (int r = 0; r < n; ++r) {
    unsigned long long w = 0;
    memcpy(&w, code.data() + (size_t)r * cb, (size_t)cb);
    for (int q = 0; q < dia.ndiag; ++q) {
      const unsigned m = (1u << dia.cbits[q]) - 1u;
      const unsigned f = (unsigned)(w >> dia.csh[q]) & m;
      if (f == m) continue;
      if (k >= nnz) return CGX_EINVAL;
      col[k] = r + dia.doff[q];
      val[k++] = dv() ? dvv[(size_t)q * npad + r] : vt[(size_t)q * 16 + f];
    }
    row_ptr[r + 1] = (int)k;
  }
  return k == nnz ? 0 : CGX_EINVAL;
}

int DevMatrix::items() const {
  switch (layout) {
    case L_DIA:
    case L_STENCIL: return (n + kDiaSliceRows - 1) / kDiaSliceRows;
    default: return nblk;
  }
}

int DevMatrix::padded_rows() const { return padded_rows_for(n); }

// The plane march (k_spmv_dia_m, cgx_kernels.hip): every far diagonal is +F
// or -F, and F = Q * 512 + e with e inside the window's halo on the side the
// neighbour rows fall (+F: -hl <= e <= hr; -F: -hr <= e <= hl), so the rows F
// away from a super-item lie in the window of the super-item Q slices away.
// Two-slice super-items (wide halos, the fused step's rule) need Q even: the
// chains j0 = 2c, c < Q / 2, then cover every slice once.  Segment length:
// about 2,048 workgroups per launch (8 per CU), fewer than 1 in 8 windows
// recomputed at a segment's ends at C3 / C4.
int DevMatrix::plan_march() {
  dev_free(&d_mpos);
  mq = mchains = mws = mlen = mfar = 0;
  msb = 1;
  if (layout != L_DIA || dia.cbytes > 4 || n == 0) return 0;
  int hl = 0, hr = 0, F = 0;
  bool neg = false, pos = false;
  for (int k = 0; k < dia.ndiag; ++k) {
    const int d = dia.doff[k];
    if (near_diag(k)) {
      hl = std::max(hl, -d);
      hr = std::max(hr, d);
    } else {
      if (F != 0 && std::abs(d) != F) return 0;
      F = std::abs(d);
      (d < 0 ? neg : pos) = true;
    }
  }
  hl = (hl + 1) & ~1;  // as args()
  const int sb = hl + hr > kDiaSliceRows ? 2 : 1;
  if (F == 0) {
    // Near-only (round 6): every diagonal within the halo.  The one-launch SR
    // step still runs as a "march" whose steps are Q slices apart and share
    // nothing (no far diagonal reads the ring's other windows): chains of
    // about 16 steps, Q a multiple of 4 (four-slice steps), one window per
    // step plus one per segment.  One launch per iteration instead of the
    // SpMV + k_update_sr pair (C2, 2-D 1000^2: 2,000-row halos, cache-resident)
    const int ns = items();
    const int wn = sb * kDiaSliceRows + hl + hr;
    if ((wn + 2 * 256 * sb - 1) / (2 * 256 * sb) > (sb == 1 ? 5 : 3)) return 0;
    const int Q = std::max(4, ((ns + 15) / 16 + 3) & ~3);
    mq = Q;
    msb = sb;
    mchains = (Q + sb - 1) / sb;
    mws = (wn + 3) & ~1;
    mlen = std::max(1, (ns + Q - 1) / Q);
    if (!order.empty()) {
      std::vector<int> p((size_t)ns);
      for (int i = 0; i < ns; ++i) p[(size_t)order[(size_t)i]] = i;
      int rc;
      if ((rc = dev_alloc(&d_mpos, p.size() * 4, &dev_bytes))) return rc;
      CGX_HIP(hipMemcpy(d_mpos, p.data(), p.size() * 4, hipMemcpyHostToDevice));
    }
    return 0;
  }
  auto fits = [&](long long q) {
    const long long e = F - q * kDiaSliceRows;
    if (q < 1) return false;
    if (pos && (e < -hl || e > hr)) return false;
    if (neg && (e < -hr || e > hl)) return false;
    return true;
  };
  const long long q0 = F / kDiaSliceRows;
  int Q = 0;
  for (long long q : {q0, q0 + 1})
    if (!Q && fits(q) && (sb == 1 || q % 2 == 0)) Q = (int)q;
  if (!Q) return 0;
  const int ns = items();
  const int wn = sb * kDiaSliceRows + hl + hr;
  if ((wn + 2 * 256 * sb - 1) / (2 * 256 * sb) > (sb == 1 ? 5 : 3)) return 0;
  mq = Q;
  msb = sb;
  mchains = Q / sb;
  mws = (wn + 3) & ~1;
  mfar = 1;
  const int steps = (ns + Q - 1) / Q;
  const int nseg = std::max(1, std::min(steps, (2048 + mchains / 2) / mchains));
  mlen = (steps + nseg - 1) / nseg;
  if (!order.empty()) {
    std::vector<int> p((size_t)ns);
    for (int i = 0; i < ns; ++i) p[(size_t)order[(size_t)i]] = i;
    int rc;
    if ((rc = dev_alloc(&d_mpos, p.size() * 4, &dev_bytes))) return rc;
    CGX_HIP(hipMemcpy(d_mpos, p.data(), p.size() * 4, hipMemcpyHostToDevice));
  }
  return 0;
}

bool DevMatrix::near_diag(int k) const { return std::abs(dia.doff[k]) <= kHaloMax; }

bool DevMatrix::fusable(bool sr1) const { return fuse_block(sr1) == 0; }

int DevMatrix::fuse_block(bool sr1) const {
  if (layout != L_DIA) return CGX_FUSE_STATUS_NOT_DIA;
  if (dv() && !sr1) return CGX_FUSE_STATUS_VALUE_STREAM;
  if (dia.cbytes > 4) return CGX_FUSE_STATUS_WIDE_CODES;
  int nfar = 0;
  for (int k = 0; k < dia.ndiag; ++k) nfar += !near_diag(k);
  return nfar <= 4 ? 0 : CGX_FUSE_STATUS_FAR_DIAGS;
}

std::vector<int> DevMatrix::item_rows() const {
  if (layout == L_CSR || layout == L_DC) return blk_row;
  std::vector<int> r;
  for (int i = 0; i < n; i += kDiaSliceRows) r.push_back(i);
  r.push_back(n);
  return r;
}

double DevMatrix::csr_bytes() const {
  const double sv = dtype == CGX_F32 ? 4.0 : 8.0;
  return (double)nnz * (sv + 4) + 4.0 * (n + 1) + 2.0 * n * sv;
}

double DevMatrix::layout_bytes() const {
  const double sv = dtype == CGX_F32 ? 4.0 : 8.0;
  switch (layout) {
    case L_DIA: return (double)dia.cbytes * n + (dv() ? sv * dia.ndiag * n : 0.0) + 2.0 * n * sv;
    case L_DC: return (double)nnz * (sv + 1) + 1.0 * n + 2.0 * n * sv + 4.0 * ndict;
    case L_STENCIL: return 2.0 * n * sv;
    default:
      if (npanel > 1)  // P row_ptrs, y written P times and read P - 1 times
        return (double)nnz * (sv + 4) + 4.0 * npanel * (n + 1.0) + (double)n * sv * 2.0 * npanel;
      return csr_bytes();
  }
}

template <typename T>
SpmvArgs<T> DevMatrix::args(const T *x, T *y, double *part, const int *done, Items it) const {
  SpmvArgs<T> a;
  memset(&a, 0, sizeof a);
  a.layout = layout;
  a.x = x;
  a.y = y;
  a.part = part;
  a.done = done;
  a.nt = nt ? 1 : 0;
  a.items = it;
  a.blkrk = d_blkrk;
  a.capw = capw;
  a.rp = d_rp;
  a.col = d_col;
  a.val = (const T *)d_val;
  a.code = d_code;
  a.rlen = d_rlen;
  a.dict = d_dict;
  a.ndict_cap = ndict <= 64 ? 64 : 256;
  a.gath = gath;
  a.dcode = d_dcode;
  a.cb = dia.cbytes;
  for (int k = 0; k < kDiaMax; ++k) {
    a.csh[k] = dia.csh[k];
    a.cmask[k] = (1u << dia.cbits[k]) - 1u;
  }
  a.vtab = (const T *)d_vtab;
  a.dval = (const T *)d_dval;
  a.dvs = padded_rows();
  a.ndiag = dia.ndiag;
  a.kdiag = kdiag;
  for (int k = 0; k < kDiaMax; ++k) a.doff[k] = dia.doff[k];
  a.ncols = ncols;
  a.xlo = col_lo - 1;
  a.near = 0;
  a.hl = a.hr = 0;
  int nf = 0;
  for (int q = 0; q < 4; ++q) a.fark[q] = -1;
  for (int k = 0; k < dia.ndiag; ++k)
    if (near_diag(k)) {
      a.near |= 1u << k;
      a.hl = std::max(a.hl, -dia.doff[k]);
      a.hr = std::max(a.hr, dia.doff[k]);
    } else if (nf < 4) {
      a.fark[nf++] = k;
    }
  a.hl = (a.hl + 1) & ~1;  // an even window start: aligned pair loads
  a.mq = mq;
  a.msb = msb;
  a.mchains = mchains;
  a.mslices = items();
  a.mws = mws;
  a.mlen = mlen;
  a.mpos = d_mpos;
  a.mlist = d_order;
  a.n = n;
  a.lap = lap;
  if (layout == L_STENCIL) {
    a.inv_nx = 1.0 / lap.nx;
    a.inv_pl = 1.0 / ((double)lap.nx * lap.ny);
  }
  return a;
}

int DevMatrix::partials(Items it) const {
  switch (layout) {
    case L_DIA: return it.count;
    case L_STENCIL: return (n + kDiaSliceRows - 1) / kDiaSliceRows;
    default:
      if (npanel > 1) return (panel_count.back() + 3) / 4;
      return (it.count + 3) / 4;
  }
}

template <typename T>
hipError_t DevMatrix::spmv(const T *x, T *y, double *part, const int *done, Items it,
                           hipStream_t s, int *nparts, LaunchEv ev, bool pair) const {
  if (nparts) *nparts = partials(it);
  if (layout == L_STENCIL) it = Items{nullptr, 0, (n + kDiaSliceRows - 1) / kDiaSliceRows};
  if (npanel <= 1) {
    SpmvArgs<T> a = args<T>(x, y, part, done, it);
    a.pair = pair ? 1 : 0;
    return launch_spmv<T>(a, s, ev);
  }
  for (int q = 0; q < npanel; ++q) {
    SpmvArgs<T> a = args<T>(x, y, q + 1 == npanel ? part : nullptr, done,
                            Items{nullptr, panel_first[q], panel_count[q]});
    a.pair = pair && q + 1 == npanel ? 1 : 0;
    a.rp = d_rp + (size_t)q * ((size_t)n + 1);
    a.yacc = q ? y : nullptr;
    a.capw = capw;
    LaunchEv e1;
    e1.start = q == 0 ? ev.start : nullptr;
    e1.stop = q + 1 == npanel ? ev.stop : nullptr;
    const hipError_t e = launch_spmv<T>(a, s, e1);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template SpmvArgs<double> DevMatrix::args<double>(const double *, double *, double *,
                                                  const int *, Items) const;
template SpmvArgs<float> DevMatrix::args<float>(const float *, float *, double *, const int *,
                                                Items) const;
template hipError_t DevMatrix::spmv<double>(const double *, double *, double *, const int *,
                                            Items, hipStream_t, int *, LaunchEv, bool) const;
template hipError_t DevMatrix::spmv<float>(const float *, float *, double *, const int *, Items,
                                           hipStream_t, int *, LaunchEv, bool) const;

}  // namespace cgx
