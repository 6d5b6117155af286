// cgx_io.cpp -- reader for the reference's input format (cg.c:146-218):
// four lines, comma separated: col_indices, row_ptr (n+1 entries), values,
// b.  A->size = #row_ptr - 1 (cg.c:204), A->nnz = #values, b->size =
// b->nnz = #b (cg.c:210-211).  Tokens end at ',' or '\n' exactly as in the
// reference (an empty token parses as 0).  Unlike the reference it is
// re-entrant (no static counters, cg.c:235-236), bounds-safe (no 64-byte
// token stack, cg.c:317-346) and accepts a file that ends before the fourth
// newline.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cgx_internal.h"

extern "C" int cgx_read_input_file(const char *path, struct __mv_sparse *A,
                                   struct __mv_sparse *b) {
  if (!path || !A || !b) {
    fprintf(stderr, "Error: Matrix must be initialized before reading input\n");
    return -1;
  }
  FILE *f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "Error: Failed to open input file (%s)\n", path);
    return -1;
  }
  std::vector<char> buf;
  {
    char chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof chunk, f)) > 0)
      buf.insert(buf.end(), chunk, chunk + got);
  }
  fclose(f);
  buf.push_back('\0');
  std::vector<int> col, rp;
  std::vector<double> val, bv;
  int line = 0;
  const char *p = buf.data(), *end = buf.data() + buf.size() - 1;
  std::string tok;
  while (line < 4) {
    const char *q = p;
    while (q < end && *q != ',' && *q != '\n') ++q;
    const bool at_eof = q >= end;
    if (at_eof && q == p) break;  // nothing left
    tok.assign(p, q);
    switch (line) {
      case 0: col.push_back((int)strtol(tok.c_str(), nullptr, 10)); break;
      case 1: rp.push_back((int)strtol(tok.c_str(), nullptr, 10)); break;
      case 2: val.push_back(strtod(tok.c_str(), nullptr)); break;
      case 3: bv.push_back(strtod(tok.c_str(), nullptr)); break;
    }
    if (at_eof) break;
    if (*q == '\n') ++line;
    p = q + 1;
  }
  if (rp.empty()) {
    fprintf(stderr, "Error: input file %s has no row pointer line\n", path);
    return -1;
  }
  const int n = (int)rp.size() - 1;
  auto dup_i = [](const std::vector<int> &v) {
    int *o = (int *)calloc(v.empty() ? 1 : v.size(), sizeof(int));
    if (o && !v.empty()) memcpy(o, v.data(), v.size() * sizeof(int));
    return o;
  };
  auto dup_d = [](const std::vector<double> &v) {
    double *o = (double *)calloc(v.empty() ? 1 : v.size(), sizeof(double));
    if (o && !v.empty()) memcpy(o, v.data(), v.size() * sizeof(double));
    return o;
  };
  A->size = n;
  A->nnz = (int)val.size();
  A->values = dup_d(val);
  A->col_indices = dup_i(col);
  A->row_ptr = dup_i(rp);
  b->size = (int)bv.size();
  b->nnz = (int)bv.size();
  b->values = dup_d(bv);
  b->col_indices = nullptr;
  b->row_ptr = nullptr;
  return (A->values && A->col_indices && A->row_ptr && b->values) ? 0 : -1;
}
