// cgx_partition.cpp -- row-block domain decomposition for the multi-GPU
// solver.  Pure host code, no GPU: every index computed here
// is integer arithmetic and is tested bit-exactly against a Python
// restatement (tests/test_partition.py).
//
//   rows of rank g:   [floor(g*n/G), floor((g+1)*n/G))   (64-bit products)
//   local columns:    owned rows -> [0, n_loc), ghosts -> n_loc + position
//                     in the ghost list (sorted by global index, hence grouped
//                     by owner rank, owners ascending)
//   halo:             rank g receives recv_count[q] ghosts from each q, stored
//                     contiguously at x[n_loc + recv_off[q]]; it sends to q
//                     the entries q requested, as local indices.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cgx_internal.h"

struct cgx_part {
  long long n_global = 0;
  int nranks = 1, rank = 0;
  int row_begin = 0, row_end = 0;
  int nnz = 0;
  std::vector<int> col_local;
  std::vector<int> ghosts;       // global indices, ascending
  std::vector<int> recv_count;   // per rank
  std::vector<int> send_count;   // per rank (after set_requests)
  std::vector<int> send_local;   // concatenated by rank
  bool have_sends = false;
};

namespace cgx {

long long part_begin(long long n, int G, int g) { return (long long)g * n / G; }

int part_owner(long long n, int G, long long c) {
  long long g = (c * G) / n;  // floor(c*G/n) is within one of the owner
  if (g >= G) g = G - 1;
  while (g + 1 < G && part_begin(n, G, g + 1) <= c) ++g;
  while (g > 0 && part_begin(n, G, g) > c) --g;
  return (int)g;
}

}  // namespace cgx

extern "C" {

void cgx_partition_rows(long long n, int nranks, int rank, int *row_begin,
                        int *row_end) {
  if (nranks < 1 || rank < 0 || rank >= nranks || n < 0) {
    if (row_begin) *row_begin = 0;
    if (row_end) *row_end = 0;
    return;
  }
  if (row_begin) *row_begin = (int)cgx::part_begin(n, nranks, rank);
  if (row_end) *row_end = (int)cgx::part_begin(n, nranks, rank + 1);
}

int cgx_partition_owner(long long n, int nranks, long long col) {
  if (nranks < 1 || n <= 0 || col < 0 || col >= n) return CGX_EINVAL;
  return cgx::part_owner(n, nranks, col);
}

int cgx_part_create(long long n_global, int nranks, int rank, int n_loc,
                    int nnz, const int *row_ptr, const int *col_global,
                    cgx_part **out) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || n_global < 0 ||
      n_global > INT32_MAX || n_loc < 0 || nnz < 0 ||
      (n_loc > 0 && !row_ptr) || (nnz > 0 && !col_global)) {
    cgx::set_error("cgx_part_create: bad arguments");
    return CGX_EINVAL;
  }
  int rb, re;
  cgx_partition_rows(n_global, nranks, rank, &rb, &re);
  if (re - rb != n_loc || (n_loc > 0 && (row_ptr[0] != 0 || row_ptr[n_loc] != nnz))) {
    cgx::set_error("cgx_part_create: rank %d must own rows [%d,%d) (got %d rows)",
                   rank, rb, re, n_loc);
    return CGX_EINVAL;
  }
  cgx_part *p = new cgx_part();
  p->n_global = n_global;
  p->nranks = nranks;
  p->rank = rank;
  p->row_begin = rb;
  p->row_end = re;
  p->nnz = nnz;
  // ghost discovery: every referenced column outside [rb, re), unique, sorted
  std::vector<int> g;
  for (int k = 0; k < nnz; ++k) {
    const int c = col_global[k];
    if (c < 0 || c >= n_global) {
      cgx::set_error("cgx_part_create: column %d out of range", c);
      delete p;
      return CGX_EINVAL;
    }
    if (c < rb || c >= re) g.push_back(c);
  }
  std::sort(g.begin(), g.end());
  g.erase(std::unique(g.begin(), g.end()), g.end());
  p->ghosts = std::move(g);
  // local renumbering
  p->col_local.resize((size_t)nnz);
  for (int k = 0; k < nnz; ++k) {
    const int c = col_global[k];
    if (c >= rb && c < re) {
      p->col_local[k] = c - rb;
    } else {
      const auto it = std::lower_bound(p->ghosts.begin(), p->ghosts.end(), c);
      p->col_local[k] = n_loc + (int)(it - p->ghosts.begin());
    }
  }
  // ghosts grouped by owner (sorted global index => owners ascending)
  p->recv_count.assign((size_t)nranks, 0);
  for (int c : p->ghosts) p->recv_count[cgx::part_owner(n_global, nranks, c)]++;
  p->send_count.assign((size_t)nranks, 0);
  *out = p;
  return 0;
}

void cgx_part_destroy(cgx_part *p) { delete p; }

int cgx_part_info(const cgx_part *p, int *n_loc, int *n_ghost, int *row_begin,
                  int *n_send) {
  if (!p) return CGX_EINVAL;
  if (n_loc) *n_loc = p->row_end - p->row_begin;
  if (n_ghost) *n_ghost = (int)p->ghosts.size();
  if (row_begin) *row_begin = p->row_begin;
  if (n_send) *n_send = (int)p->send_local.size();
  return 0;
}

int cgx_part_local_cols(const cgx_part *p, int *col_local) {
  if (!p || (p->nnz > 0 && !col_local)) return CGX_EINVAL;
  if (p->nnz) memcpy(col_local, p->col_local.data(), (size_t)p->nnz * 4);
  return 0;
}

int cgx_part_ghosts(const cgx_part *p, int *ghost_global) {
  if (!p || (!p->ghosts.empty() && !ghost_global)) return CGX_EINVAL;
  if (!p->ghosts.empty())
    memcpy(ghost_global, p->ghosts.data(), p->ghosts.size() * 4);
  return (int)p->ghosts.size();
}

int cgx_part_recv_counts(const cgx_part *p, int *counts) {
  if (!p || !counts) return CGX_EINVAL;
  memcpy(counts, p->recv_count.data(), (size_t)p->nranks * 4);
  return 0;
}

int cgx_part_set_requests(cgx_part *p, const int *req_counts,
                          const int *req_global) {
  if (!p || !req_counts) return CGX_EINVAL;
  long long total = 0;
  for (int q = 0; q < p->nranks; ++q) {
    if (req_counts[q] < 0 || (q == p->rank && req_counts[q] != 0)) {
      cgx::set_error("cgx_part_set_requests: bad count from rank %d", q);
      return CGX_EINVAL;
    }
    total += req_counts[q];
  }
  if (total > 0 && !req_global) return CGX_EINVAL;
  std::vector<int> loc((size_t)total);
  for (long long i = 0; i < total; ++i) {
    const int c = req_global[i];
    if (c < p->row_begin || c >= p->row_end) {
      cgx::set_error("cgx_part_set_requests: rank %d does not own row %d",
                     p->rank, c);
      return CGX_EINVAL;
    }
    loc[(size_t)i] = c - p->row_begin;
  }
  p->send_count.assign(req_counts, req_counts + p->nranks);
  p->send_local = std::move(loc);
  p->have_sends = true;
  return 0;
}

int cgx_part_send_counts(const cgx_part *p, int *counts) {
  if (!p || !counts || !p->have_sends) return CGX_EINVAL;
  memcpy(counts, p->send_count.data(), (size_t)p->nranks * 4);
  return 0;
}

int cgx_part_send_local(const cgx_part *p, int *send_local) {
  if (!p || !p->have_sends || (!p->send_local.empty() && !send_local))
    return CGX_EINVAL;
  if (!p->send_local.empty())
    memcpy(send_local, p->send_local.data(), p->send_local.size() * 4);
  return (int)p->send_local.size();
}

}  // extern "C"
