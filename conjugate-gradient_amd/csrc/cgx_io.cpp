// cgx_io.cpp -- reader for the reference's input format (cg.c:146-218):
// four lines, comma separated: col_indices, row_ptr (n+1 entries), values,
// b.  A->size = #row_ptr - 1 (cg.c:204), A->nnz = #values, b->size =
// b->nnz = #b (cg.c:210-211).  Tokens end at ',' or '\n' exactly as in the
// reference (an empty token parses as 0).  Unlike the reference it is
// re-entrant (no static counters, cg.c:235-236), bounds-safe (no 64-byte
// token stack, cg.c:317-346) and accepts a file that ends before the fourth
// newline.  It is also fast: each line is cut at commas into chunks parsed on
// host threads (a C3-sized input is ~1.5 GB of text), and an optional binary
// cache (cgx_read_input_cached) skips the text entirely on later reads.
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "cgx_hash.h"
#include "cgx_internal.h"

namespace {

// One token [p, q) as the reference converts it (atoi / atof of the
// characters before the separator).
template <typename T>
T parse_tok(const char *p, const char *q) {
  char small[64];
  const size_t len = (size_t)(q - p);
  std::vector<char> big;
  char *s = small;
  if (len >= sizeof small) {
    big.resize(len + 1);
    s = big.data();
  }
  if (len) memcpy(s, p, len);
  s[len] = '\0';
  if (std::is_integral<T>::value) return (T)strtol(s, nullptr, 10);
  return (T)strtod(s, nullptr);
}

// The tokens of one line [p, e) (no '\n' inside) in order, as the reference
// reads them: a line ended by '\n' has one token more than it has commas
// (an empty one parses as 0); the unterminated last line of a file drops
// the empty token after a trailing comma, and has none when empty.  The
// line is cut at token starts into up to 16 chunks parsed on host threads.
template <typename T>
std::vector<T> parse_line(const char *p, const char *e, bool terminated) {
  std::vector<T> out;
  if (!terminated && p == e) return out;
  const long long len = e - p;
  const int want = (int)std::max<long long>(1, std::min<long long>(16, len >> 22));
  std::vector<const char *> cut{p};
  for (int t = 1; t < want; ++t) {
    const char *c = std::max(p + len * t / want, cut.back());
    c = c < e ? (const char *)memchr(c, ',', (size_t)(e - c)) : nullptr;
    if (c && c + 1 < e && c + 1 > cut.back()) cut.push_back(c + 1);
  }
  const int m = (int)cut.size();
  auto chunk_end = [&](int t) { return t + 1 < m ? cut[(size_t)t + 1] - 1 : e; };
  std::vector<long long> cnt((size_t)m), off((size_t)m + 1, 0);
  auto run = [&](auto f) {
    std::vector<std::thread> th;
    for (int t = 1; t < m; ++t) th.emplace_back(f, t);
    f(0);
    for (auto &x : th) x.join();
  };
  run([&](int t) {
    long long c = 1;
    for (const char *x = cut[(size_t)t], *b = chunk_end(t); x < b; ++x) c += *x == ',';
    if (t == m - 1 && !terminated && e > p && e[-1] == ',') --c;
    cnt[(size_t)t] = c;
  });
  for (int t = 0; t < m; ++t) off[(size_t)t + 1] = off[(size_t)t] + cnt[(size_t)t];
  out.resize((size_t)off[(size_t)m]);
  run([&](int t) {
    const char *x = cut[(size_t)t];
    for (long long k = off[(size_t)t]; k < off[(size_t)t + 1]; ++k) {
      const char *q = x < e ? (const char *)memchr(x, ',', (size_t)(e - x)) : nullptr;
      if (!q) q = e;
      out[(size_t)k] = parse_tok<T>(x, q);
      x = q + 1;
    }
  });
  return out;
}

int fill(struct __mv_sparse *A, struct __mv_sparse *b, const std::vector<int> &col,
         const std::vector<int> &rp, const std::vector<double> &val,
         const std::vector<double> &bv) {
  auto dup = [](const void *src, size_t n, size_t es) {
    void *o = calloc(n ? n : 1, es);
    if (o && n) memcpy(o, src, n * es);
    return o;
  };
  A->size = (int)rp.size() - 1;
  A->nnz = (int)val.size();
  A->values = (double *)dup(val.data(), val.size(), 8);
  A->col_indices = (int *)dup(col.data(), col.size(), 4);
  A->row_ptr = (int *)dup(rp.data(), rp.size(), 4);
  b->size = (int)bv.size();
  b->nnz = (int)bv.size();
  b->values = (double *)dup(bv.data(), bv.size(), 8);
  b->col_indices = nullptr;
  b->row_ptr = nullptr;
  return (A->values && A->col_indices && A->row_ptr && b->values) ? 0 : -1;
}

// The whole text file in memory (-1: it cannot be opened).
int load_text(const char *path, std::vector<char> &buf) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "Error: Failed to open input file (%s)\n", path);
    return -1;
  }
  buf.clear();
  if (fseek(f, 0, SEEK_END) == 0) {
    const long sz = ftell(f);
    if (sz > 0) buf.resize((size_t)sz);
    rewind(f);
  }
  size_t got = buf.empty() ? 0 : fread(buf.data(), 1, buf.size(), f);
  buf.resize(got);
  {  // a file whose size ftell could not give (a pipe)
    char chunk[1 << 16];
    size_t m;
    while ((m = fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + m);
  }
  fclose(f);
  return 0;
}

int parse_text(const char *path, const std::vector<char> &buf, std::vector<int> &col,
               std::vector<int> &rp, std::vector<double> &val, std::vector<double> &bv) {
  // lines 0-3 (cg.c:146-218 reads four); text after the fourth '\n' is ignored
  const char *x = buf.data(), *end = buf.data() + buf.size();
  auto next_line = [&](bool *term, const char **e) {
    const char *a = x;
    if (x > end) {
      *term = false;
      *e = a = end;
      return end;
    }
    const char *q = x < end ? (const char *)memchr(x, '\n', (size_t)(end - x)) : nullptr;
    *term = q != nullptr;
    *e = q ? q : end;
    x = q ? q + 1 : end + 1;
    return a;
  };
  bool term;
  const char *a, *e;
  a = next_line(&term, &e);
  col = parse_line<int>(a, e, term);
  a = next_line(&term, &e);
  rp = parse_line<int>(a, e, term);
  a = next_line(&term, &e);
  val = parse_line<double>(a, e, term);
  a = next_line(&term, &e);
  bv = parse_line<double>(a, e, term);
  if (rp.empty()) {
    fprintf(stderr, "Error: input file %s has no row pointer line\n", path);
    return -1;
  }
  return 0;
}

int read_text(const char *path, std::vector<int> &col, std::vector<int> &rp,
              std::vector<double> &val, std::vector<double> &bv) {
  std::vector<char> buf;
  if (load_text(path, buf)) return -1;
  return parse_text(path, buf, col, rp, val, bv);
}

// Binary cache: header + the four arrays, keyed on the text's size and a
// 64-bit content hash of all of it (cgx_hash.h; hashing runs at memory
// bandwidth on host threads, ~10x faster than parsing).  A cache written for
// another input, or for an earlier version of this one, never matches --
// whatever the paths, sizes or timestamps (the size + mtime key
// of round 2 accepted a rewrite with same-width numbers inside one
// timestamp tick).
struct CacheHdr {
  char magic[8];
  long long src_size;
  unsigned long long src_hash;
  long long ncol, nrp, nval, nb;
};
constexpr char kMagic[8] = {'c', 'g', 'x', 'b', 'i', 'n', '0', '2'};

bool read_cache(const char *cache, long long size, unsigned long long hash, std::vector<int> &col,
                std::vector<int> &rp, std::vector<double> &val, std::vector<double> &bv) {
  FILE *f = fopen(cache, "rb");
  if (!f) return false;
  CacheHdr h;
  bool ok = fread(&h, sizeof h, 1, f) == 1 && memcmp(h.magic, kMagic, 8) == 0 &&
            h.src_size == size && h.src_hash == hash && h.ncol >= 0 && h.nrp >= 1 &&
            h.nval >= 0 && h.nb >= 0 && h.nrp <= INT32_MAX && h.ncol <= INT32_MAX &&
            h.nval <= INT32_MAX && h.nb <= INT32_MAX;
  if (ok) {
    col.resize((size_t)h.ncol);
    rp.resize((size_t)h.nrp);
    val.resize((size_t)h.nval);
    bv.resize((size_t)h.nb);
    ok = fread(col.data(), 4, col.size(), f) == col.size() &&
         fread(rp.data(), 4, rp.size(), f) == rp.size() &&
         fread(val.data(), 8, val.size(), f) == val.size() &&
         fread(bv.data(), 8, bv.size(), f) == bv.size();
  }
  fclose(f);
  return ok;
}

void write_cache(const char *cache, long long size, unsigned long long hash,
                 const std::vector<int> &col,
                 const std::vector<int> &rp, const std::vector<double> &val,
                 const std::vector<double> &bv) {
  std::vector<char> tmp(strlen(cache) + 8);
  snprintf(tmp.data(), tmp.size(), "%s.tmp", cache);
  FILE *f = fopen(tmp.data(), "wb");
  if (!f) return;  // best effort: an unwritable cache only costs the next parse
  CacheHdr h;
  memcpy(h.magic, kMagic, 8);
  h.src_size = size;
  h.src_hash = hash;
  h.ncol = (long long)col.size();
  h.nrp = (long long)rp.size();
  h.nval = (long long)val.size();
  h.nb = (long long)bv.size();
  const bool ok = fwrite(&h, sizeof h, 1, f) == 1 &&
                  fwrite(col.data(), 4, col.size(), f) == col.size() &&
                  fwrite(rp.data(), 4, rp.size(), f) == rp.size() &&
                  fwrite(val.data(), 8, val.size(), f) == val.size() &&
                  fwrite(bv.data(), 8, bv.size(), f) == bv.size();
  if (fclose(f) == 0 && ok) {
    if (rename(tmp.data(), cache) == 0) return;
  }
  remove(tmp.data());
}

}  // namespace

extern "C" int cgx_read_input_file(const char *path, struct __mv_sparse *A,
                                   struct __mv_sparse *b) {
  if (!path || !A || !b) {
    fprintf(stderr, "Error: Matrix must be initialized before reading input\n");
    return -1;
  }
  std::vector<int> col, rp;
  std::vector<double> val, bv;
  if (read_text(path, col, rp, val, bv)) return -1;
  return fill(A, b, col, rp, val, bv);
}

extern "C" int cgx_read_input_cached(const char *path, const char *cache_path,
                                     struct __mv_sparse *A, struct __mv_sparse *b,
                                     int *from_cache) {
  if (!path || !cache_path || !A || !b) {
    fprintf(stderr, "Error: Matrix must be initialized before reading input\n");
    return -1;
  }
  if (from_cache) *from_cache = 0;
  std::vector<char> buf;
  if (load_text(path, buf)) return -1;
  const long long size = (long long)buf.size();
  const unsigned long long hash = cgx::hash_bytes(buf.data(), buf.size());
  std::vector<int> col, rp;
  std::vector<double> val, bv;
  if (read_cache(cache_path, size, hash, col, rp, val, bv)) {
    if (from_cache) *from_cache = 1;
    return fill(A, b, col, rp, val, bv);
  }
  if (parse_text(path, buf, col, rp, val, bv)) return -1;
  write_cache(cache_path, size, hash, col, rp, val, bv);
  return fill(A, b, col, rp, val, bv);
}
