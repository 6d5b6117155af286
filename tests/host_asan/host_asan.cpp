// Host-code sanitizer driver (TEST INFRASTRUCTURE): the pure-host parts of
// libcgx -- partitioning (cgx_partition.cpp), generators (cgx_gen.cpp) and
// the reader (cgx_io.cpp) -- compiled with -fsanitize=address,undefined and
// driven through edge cases.  Exit 0 = no sanitizer report and all checks
// held.  Built and run by tests/test_host_sanitizers.py.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cgx.h"

namespace cgx {
void set_error(const char *fmt, ...) {  // the solver's error slot, stubbed
  va_list ap;
  va_start(ap, fmt);
  va_end(ap);
}
}  // namespace cgx

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

static void partitions() {
  // every rank of a G-way split of a random chained matrix; requests/sends
  // wired as a transport would
  for (int n : {0, 1, 7, 64, 1000}) {
    for (int G : {1, 2, 3, 8, 13}) {
      std::vector<cgx_part *> parts(G, nullptr);
      std::vector<std::vector<int>> ghosts(G);
      for (int g = 0; g < G; ++g) {
        int rb, re;
        cgx_partition_rows(n, G, g, &rb, &re);
        std::vector<int> rp(1, 0), col;
        for (int r = rb; r < re; ++r) {
          for (int c : {r - 5, r - 1, r, r + 1, (r * 7919) % (n ? n : 1)})
            if (c >= 0 && c < n && (col.size() == (size_t)rp.back() || col.back() < c))
              col.push_back(c);
          rp.push_back((int)col.size());
        }
        const int rc = cgx_part_create(n, G, g, re - rb, (int)col.size(), rp.data(),
                                       col.empty() ? nullptr : col.data(), &parts[g]);
        CHECK(rc == 0);
        if (rc) continue;
        int nl, ng, rbeg, ns;
        CHECK(cgx_part_info(parts[g], &nl, &ng, &rbeg, &ns) == 0);
        ghosts[g].resize(ng);
        CHECK(cgx_part_ghosts(parts[g], ghosts[g].data()) == ng);
        std::vector<int> loc(col.size() + 1);
        CHECK(cgx_part_local_cols(parts[g], loc.data()) == 0);
      }
      for (int g = 0; g < G; ++g) {
        if (!parts[g]) continue;
        std::vector<int> cnt(G, 0), req;
        for (int q = 0; q < G; ++q) {
          if (!parts[q] || q == g) continue;
          std::vector<int> rc(G);
          cgx_part_recv_counts(parts[q], rc.data());
          int off = 0;
          for (int t = 0; t < g; ++t) off += rc[t];
          cnt[q] = rc[g];
          req.insert(req.end(), ghosts[q].begin() + off, ghosts[q].begin() + off + rc[g]);
        }
        CHECK(cgx_part_set_requests(parts[g], cnt.data(), req.empty() ? nullptr : req.data()) == 0);
        std::vector<int> sl(req.size() + 1);
        CHECK(cgx_part_send_local(parts[g], sl.data()) == (int)req.size());
      }
      for (auto *p : parts) cgx_part_destroy(p);
    }
  }
  // bad arguments: out-of-range column, wrong row count
  int rp[3] = {0, 1, 2}, col[2] = {0, 99};
  cgx_part *p = nullptr;
  CHECK(cgx_part_create(4, 2, 0, 2, 2, rp, col, &p) < 0 && !p);
  CHECK(cgx_part_create(4, 2, 0, 3, 2, rp, col, &p) < 0);
  CHECK(cgx_partition_owner(10, 3, 10) < 0);
  CHECK(cgx_partition_owner(2147483647LL, 7, 2147483646LL) == 6);
}

static void generators() {
  for (auto d : std::vector<std::vector<int>>{{1, 1, 1}, {5, 3, 2}, {7, 1, 4}, {1, 9, 1}}) {
    const int n = d[0] * d[1] * d[2];
    for (auto r : std::vector<std::pair<int, int>>{{0, n}, {n / 3, n}, {n, n}}) {
      const long long nnz = cgx_gen_laplacian3d(d[0], d[1], d[2], r.first, r.second,
                                                nullptr, nullptr, nullptr);
      CHECK(nnz >= 0);
      std::vector<int> rp(r.second - r.first + 1), col(nnz + 1);
      std::vector<double> val(nnz + 1);
      CHECK(cgx_gen_laplacian3d(d[0], d[1], d[2], r.first, r.second, rp.data(), col.data(),
                                val.data()) == nnz);
      std::vector<int> rp2(rp.size());
      CHECK(cgx_laplacian_row_ptr(3, d[0], d[1], d[2], r.first, r.second, rp2.data()) == nnz);
      CHECK(rp == rp2);
    }
  }
  CHECK(cgx_gen_laplacian2d(0, 3, 0, 0, nullptr, nullptr, nullptr) < 0);
  CHECK(cgx_gen_laplacian3d(2, 2, 2, 3, 2, nullptr, nullptr, nullptr) < 0);
  const long long nnz = cgx_gen_random_spd(500, 8, 42, 0, 500, nullptr, nullptr, nullptr, nullptr);
  CHECK(nnz > 0);
  std::vector<int> rp(501), col(nnz);
  std::vector<double> val(nnz);
  std::vector<float> v32(nnz);
  CHECK(cgx_gen_random_spd(500, 8, 42, 0, 500, rp.data(), col.data(), val.data(), v32.data()) == nnz);
  CHECK(cgx_csr_is_chained(500, rp.data(), col.data()) == 1);
  CHECK(cgx_gen_random_spd(10, 65, 1, 0, 10, nullptr, nullptr, nullptr, nullptr) < 0);
}

static struct __mv_sparse *mk() {
  return (struct __mv_sparse *)calloc(1, sizeof(struct __mv_sparse));
}
static void rm(struct __mv_sparse *m) {  // the reader's arrays are malloc/calloc'd
  if (!m) return;
  free(m->values);
  free(m->col_indices);
  free(m->row_ptr);
  free(m);
}

static std::string write_tmp(const char *name, const std::string &text) {
  std::string path = std::string(getenv("ASAN_TMP") ? getenv("ASAN_TMP") : "/tmp") + "/" + name;
  FILE *f = fopen(path.c_str(), "wb");
  fwrite(text.data(), 1, text.size(), f);
  fclose(f);
  return path;
}

static void reader() {
  struct Case { const char *name, *text; int rc, n, nnz, bsize; };
  const Case cases[] = {
      {"ok.txt", "0,1\n0,1,2\n1.5,2.5\n1,1\n", 0, 2, 2, 2},
      {"no_final_newline.txt", "0,1\n0,1,2\n1.5,2.5\n1,1", 0, 2, 2, 2},
      {"three_lines.txt", "0,1\n0,1,2\n1.5,2.5\n", 0, 2, 2, 0},
      {"empty.txt", "", -1, 0, 0, 0},
      {"one_line.txt", "0,1,2,3\n", -1, 0, 0, 0},
      {"long_token.txt", "0\n0,1\n1.000000000000000000000000000000000000000000000000000000000000"
                         "000000000000000000000000000000001\n7\n", 0, 1, 1, 1},
      {"empty_tokens.txt", ",\n0,,2\n,\n,\n", 0, 2, 2, 2},
  };
  for (const Case &c : cases) {
    const std::string path = write_tmp(c.name, c.text);
    struct __mv_sparse *A = mk(), *b = mk();
    const int rc = cgx_read_input_file(path.c_str(), A, b);
    CHECK(rc == c.rc);
    if (rc == 0) {
      CHECK(A->size == c.n);
      CHECK(A->nnz == c.nnz);
      CHECK(b->size == c.bsize);
    }
    rm(A);
    rm(b);
  }
  struct __mv_sparse *A = mk(), *b = mk();
  CHECK(cgx_read_input_file("/nonexistent/file", A, b) < 0);
  CHECK(cgx_read_input_file(nullptr, A, b) < 0);
  rm(A);
  rm(b);
}

int main() {
  partitions();
  generators();
  reader();
  if (fails) fprintf(stderr, "%d checks failed\n", fails);
  else printf("host sanitizer driver: all checks passed\n");
  return fails ? 1 : 0;
}
