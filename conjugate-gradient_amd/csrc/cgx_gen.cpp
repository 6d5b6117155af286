// cgx_gen.cpp -- synthetic SPD CSR generators for the benchmark configs
// (BASELINE.json configs / SURVEY.md 8d): 5-point 2-D and 7-point 3-D
// Laplacians in natural ordering, and a seeded random SPD matrix.  All
// generators work on a row range so each rank of a partitioned solve builds
// only its own rows (global column indices).  Every generated matrix is
// "chained" (SURVEY.md 8a/a3), so the reference's dense-row mv_mult and CSR
// SpMV agree on it.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cgx_internal.h"

namespace {

inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// -U(0,1] for the unordered pair {a, b}: symmetric by construction.
inline double pair_value(uint64_t seed, int a, int b) {
  if (a > b) std::swap(a, b);
  const uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)a << 32) | (uint32_t)b));
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);  // [0,1)
  return -(1.0 - u);
}

inline int partner(uint64_t seed, int i, int t, int n) {
  const uint64_t h = splitmix64(seed + 0x632be59bd9b4e019ULL * ((uint64_t)i * 64 + t + 1));
  return (int)(h % (uint64_t)n);
}

bool bad_range(long long n, int rb, int re) {
  return n <= 0 || n > INT32_MAX || rb < 0 || re < rb || re > n;
}

}  // namespace

extern "C" {

long long cgx_gen_laplacian2d(int nx, int ny, int row_begin, int row_end,
                              int *row_ptr, int *col, double *val) {
  const long long n = (long long)nx * ny;
  if (nx < 1 || ny < 1 || bad_range(n, row_begin, row_end)) return CGX_EINVAL;
  long long k = 0;
  if (row_ptr) row_ptr[0] = 0;
  for (int r = row_begin; r < row_end; ++r) {
    const int i = r % nx, j = r / nx;
    auto put = [&](int c, double v) {
      if (row_ptr) { col[k] = c; val[k] = v; }
      ++k;
    };
    if (j > 0) put(r - nx, -1.0);
    if (i > 0) put(r - 1, -1.0);
    put(r, 4.0);
    if (i < nx - 1) put(r + 1, -1.0);
    if (j < ny - 1) put(r + nx, -1.0);
    if (row_ptr) row_ptr[r - row_begin + 1] = (int)k;
  }
  return k;
}

long long cgx_gen_laplacian3d(int nx, int ny, int nz, int row_begin,
                              int row_end, int *row_ptr, int *col, double *val) {
  const long long n = (long long)nx * ny * nz;
  if (nx < 1 || ny < 1 || nz < 1 || bad_range(n, row_begin, row_end))
    return CGX_EINVAL;
  const int pl = nx * ny;
  long long k = 0;
  if (row_ptr) row_ptr[0] = 0;
  for (int r = row_begin; r < row_end; ++r) {
    const int i = r % nx, j = (r / nx) % ny, l = r / pl;
    auto put = [&](int c, double v) {
      if (row_ptr) { col[k] = c; val[k] = v; }
      ++k;
    };
    if (l > 0) put(r - pl, -1.0);
    if (j > 0) put(r - nx, -1.0);
    if (i > 0) put(r - 1, -1.0);
    put(r, 6.0);
    if (i < nx - 1) put(r + 1, -1.0);
    if (j < ny - 1) put(r + nx, -1.0);
    if (l < nz - 1) put(r + pl, -1.0);
    if (row_ptr) row_ptr[r - row_begin + 1] = (int)k;
  }
  if (k > INT32_MAX) return CGX_EINVAL;
  return k;
}

// The 7-point pattern of cgx_gen_laplacian3d with a random coefficient per
// grid edge: a_ij = a_ji = -(0.5 + U(0,1]) from the unordered pair {i, j}
// (symmetric by construction), diagonal = sum |a_ij| over the row + 0.01
// (strictly diagonally dominant, so SPD).  Every off-diagonal value is its
// own, so no layout can index the values (DIA-VI needs <= 15 per
// diagonal): the general-coefficient CSR case at a BASELINE shape.
long long cgx_gen_varcoef3d(int nx, int ny, int nz, unsigned long long seed, int row_begin,
                            int row_end, int *row_ptr, int *col, double *val) {
  const long long n = (long long)nx * ny * nz;
  if (nx < 1 || ny < 1 || nz < 1 || bad_range(n, row_begin, row_end)) return CGX_EINVAL;
  const int pl = nx * ny;
  long long k = 0;
  if (row_ptr) row_ptr[0] = 0;
  for (int r = row_begin; r < row_end; ++r) {
    const int i = r % nx, j = (r / nx) % ny, l = r / pl;
    int c[7];
    int m = 0;
    if (l > 0) c[m++] = r - pl;
    if (j > 0) c[m++] = r - nx;
    if (i > 0) c[m++] = r - 1;
    c[m++] = r;
    if (i < nx - 1) c[m++] = r + 1;
    if (j < ny - 1) c[m++] = r + nx;
    if (l < nz - 1) c[m++] = r + pl;
    if (row_ptr) {
      double diag = 0.01;
      double v[7];
      for (int q = 0; q < m; ++q) {
        if (c[q] == r) continue;
        v[q] = pair_value(seed, r, c[q]) - 0.5;  // -U(0,1] - 0.5
        diag += -v[q];
      }
      for (int q = 0; q < m; ++q) {
        col[k + q] = c[q];
        val[k + q] = c[q] == r ? diag : v[q];
      }
      row_ptr[r - row_begin + 1] = (int)(k + m);
    }
    k += m;
  }
  if (k > INT32_MAX) return CGX_EINVAL;
  return k;
}

long long cgx_gen_random_spd(int n, int partners, unsigned long long seed,
                             int row_begin, int row_end, int *row_ptr,
                             int *col, double *val, float *val32) {
  if (partners < 0 || partners > 64 || bad_range(n, row_begin, row_end))
    return CGX_EINVAL;
  const int m = row_end - row_begin;
  // 1. count candidates per local row: diag + band + own partners + reverse
  std::vector<long long> start((size_t)m + 1, 0);
  for (int r = row_begin; r < row_end; ++r)
    start[r - row_begin + 1] = 1 + (r > 0) + (r < n - 1) + partners;
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < partners; ++t) {
      const int j = partner(seed, i, t, n);
      if (j >= row_begin && j < row_end) start[j - row_begin + 1]++;
    }
  for (int i = 0; i < m; ++i) start[i + 1] += start[i];
  std::vector<int> cand((size_t)start[m]);
  std::vector<long long> fill(start.begin(), start.end() - 1);
  for (int r = row_begin; r < row_end; ++r) {
    long long &f = fill[r - row_begin];
    cand[f++] = r;
    if (r > 0) cand[f++] = r - 1;
    if (r < n - 1) cand[f++] = r + 1;
    for (int t = 0; t < partners; ++t) cand[f++] = partner(seed, r, t, n);
  }
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < partners; ++t) {
      const int j = partner(seed, i, t, n);
      if (j >= row_begin && j < row_end) cand[fill[j - row_begin]++] = i;
    }
  // 2. sort + unique each row, emit values
  long long k = 0;
  if (row_ptr) row_ptr[0] = 0;
  for (int li = 0; li < m; ++li) {
    const int r = row_begin + li;
    int *b = cand.data() + start[li], *e = cand.data() + start[li + 1];
    std::sort(b, e);
    e = std::unique(b, e);
    if (row_ptr) {
      double diag = 1.0;
      for (int *c = b; c != e; ++c)
        if (*c != r) diag += -pair_value(seed, r, *c);
      for (int *c = b; c != e; ++c) {
        const double v = (*c == r) ? diag : pair_value(seed, r, *c);
        col[k] = *c;
        if (val) val[k] = v;
        if (val32) val32[k] = (float)v;
        ++k;
      }
      row_ptr[li + 1] = (int)k;
    } else {
      k += e - b;
    }
    if (k > INT32_MAX) return CGX_EINVAL;
  }
  return k;
}

int cgx_csr_is_chained(int n, const int *row_ptr, const int *col) {
  if (n < 0 || (n > 0 && (!row_ptr || !col))) return CGX_EINVAL;
  for (int r = 0; r < n; ++r) {
    const int a = row_ptr[r], b = row_ptr[r + 1];
    if (b <= a) return 0;  // empty row
    for (int k = a + 1; k < b; ++k)
      if (col[k] <= col[k - 1]) return 0;  // not strictly ascending
    if (r + 1 < n && row_ptr[r + 2] > b && col[b] > col[b - 1]) return 0;
  }
  return 1;
}

// Closed-form row_ptr of the Laplacian rows [row_begin, row_end): the
// on-device generator and the matrix-free stencil use the same cgx::lap_rp.
long long cgx_laplacian_row_ptr(int dim, int nx, int ny, int nz, int row_begin,
                                int row_end, int *row_ptr) {
  const cgx::LapSpec g{dim, nx, ny, dim == 3 ? nz : 1};
  const long long n = (long long)nx * ny * g.nz;
  if ((dim != 2 && dim != 3) || nx < 1 || ny < 1 || g.nz < 1 || n > INT32_MAX ||
      row_begin < 0 || row_end < row_begin || row_end > n)
    return CGX_EINVAL;
  const long long base = cgx::lap_rp(row_begin, g);
  if (row_ptr)
    for (long long i = row_begin; i <= row_end; ++i)
      row_ptr[i - row_begin] = (int)(cgx::lap_rp(i, g) - base);
  return cgx::lap_rp(row_end, g) - base;
}

}  // extern "C"
