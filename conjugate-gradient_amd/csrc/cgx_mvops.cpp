// cgx_mvops.cpp -- the reference-compatible C ABI: mv_ops.h's 11 functions
// (rnelias/Conjugate-Gradient mv_ops.h:25-42, mv_ops.c) plus conj_grad
// (cg.c:88-141) and the north-star solve(A,b,x,tol,maxit).
//
// Structs keep HOST pointers exactly as in the reference; the arithmetic of
// mv_mult / dot_product / sv_mult / vec_add / vec_sub and the whole CG
// iteration runs on the GPU through a process-wide default context (device
// 0 unless cgx_ops_set_device), serialised by a mutex.  There is no CPU fallback:
// without a gfx950 device these calls fail (-2) and cgx_last_error() says why.
//
// Matrix residency: the reference's conj_grad calls mv_mult once per
// iteration on the same A (cg.c:111 -> mv_ops.c:160-201).  The default
// context keeps the last matrix on the device, keyed by the struct's
// pointers and sizes and checked against a 64-bit content hash of row_ptr,
// col_indices and values computed on host threads WHILE the device works
// (with_matrix), so a caller linked at the op level uploads A once, not once
// per iteration, pays ~nothing for the check -- and a caller that edits A in
// place between calls still gets its new A (the call is redone).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "cgx_hash.h"
#include "cgx_internal.h"

namespace {

using namespace cgx;

std::mutex g_mu;
cgx_solver *g_solver = nullptr;  // for mv_mult / conj_grad / solve

struct Resident {
  const void *rp = nullptr, *col = nullptr, *val = nullptr;
  int size = -1, nnz = -1;
  unsigned long long hash = 0;
  bool valid = false;
};
Resident g_res;
long long g_uploads = 0, g_reuses = 0;

struct OpsCtx {
  int device = -1;
  int cus = 256;
  hipStream_t st = nullptr;
  double *a = nullptr, *b = nullptr, *r = nullptr, *part = nullptr;
  size_t cap = 0;
};
OpsCtx g_ops;

// Numerics and device of the entry points above: set through
// cgx_ops_set_mode / cgx_ops_set_device (the library reads no environment;
// the drop-in CLI maps CGX_MODE / CGX_ALG / CGX_DEVICE onto these calls).
int g_device = 0, g_mode = CGX_MODE_FAST, g_alg = CGX_ALG_HS;
cgx_ops_timing g_timing{};

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int default_solver(cgx_solver **out) {
  if (!g_solver) {
    int rc = cgx_solver_create(g_device, &g_solver);
    if (rc) return rc;
  }
  *out = g_solver;
  return 0;
}

unsigned long long matrix_hash(const struct __mv_sparse *A) {
  const int n = A->size, nnz = A->row_ptr[n];
  unsigned long long h = hash_bytes(A->row_ptr, ((size_t)n + 1) * 4);
  if (nnz > 0) {
    h = hmerge(h, hash_bytes(A->col_indices, (size_t)nnz * 4));
    h = hmerge(h, hash_bytes(A->values, (size_t)nnz * 8));
  }
  return avalanche(h);
}

int upload_matrix(cgx_solver *s, const struct __mv_sparse *A, unsigned long long h) {
  const int n = A->size, nnz = A->row_ptr[n];
  g_res.valid = false;
  int rc = cgx_solver_set_matrix(s, n, nnz, A->row_ptr, A->col_indices, A->values);
  if (rc) return rc;
  ++g_uploads;
  g_res.rp = A->row_ptr;
  g_res.col = A->col_indices;
  g_res.val = A->values;
  g_res.size = n;
  g_res.nnz = nnz;
  g_res.hash = h;
  g_res.valid = true;
  return 0;
}

// Runs op() (device work on the default solver's matrix) with A as that
// matrix.  When the struct's arrays and sizes are those of the resident
// matrix, op() starts at once on it while the content hash of A runs on
// host threads beside it (the check costs the caller only what it does not
// overlap: ~0 for a C3 solve, whose hash takes ~5-8 ms); a hash that differs
// (A edited in place since the upload) re-uploads A and runs op() again, so
// the result is always that of the A passed in.  Otherwise A is uploaded and
// op() runs while A is hashed beside it.
struct MatTiming {
  double hash_ms = 0, upload_ms = 0, op_ms = 0;  // hash: time spent waiting for it
  bool uploaded = false;
};

template <typename F>
int with_matrix(cgx_solver *s, const struct __mv_sparse *A, F &&op, MatTiming *tm = nullptr) {
  MatTiming t;
  const int n = A->size, nnz = A->row_ptr[n];
  const bool same_key = g_res.valid && g_res.rp == A->row_ptr && g_res.col == A->col_indices &&
                        g_res.val == A->values && g_res.size == n && g_res.nnz == nnz;
  auto upload = [&](unsigned long long h) {
    const double t0 = now_ms();
    const int rc = upload_matrix(s, A, h);
    t.upload_ms += now_ms() - t0;
    t.uploaded = true;
    return rc;
  };
  auto run = [&] {
    const double t0 = now_ms();
    const int rc = op();
    t.op_ms = now_ms() - t0;
    return rc;
  };
  int rc = 0;
  if (!same_key) {
    // the hash only keys the next call: it runs on host threads beside the
    // device work (A cannot change while this call holds the caller)
    rc = upload(0);
    unsigned long long h = 0;
    std::thread th([&] { h = matrix_hash(A); });
    if (rc == 0) rc = run();
    const double tw = now_ms();
    th.join();
    t.hash_ms = now_ms() - tw;
    if (rc == 0 && g_res.valid) g_res.hash = h;
  } else {
    unsigned long long h = 0;
    std::thread th([&] { h = matrix_hash(A); });
    rc = run();
    const double tw = now_ms();
    th.join();
    t.hash_ms = now_ms() - tw;
    if (rc == 0) {
      if (h == g_res.hash) {
        ++g_reuses;
      } else {  // A changed in place: the result came from the stale device copy
        rc = upload(h);
        if (rc == 0) rc = run();
      }
    }
  }
  if (tm) *tm = t;
  return rc;
}

int ops_ready(size_t n) {
  if (g_ops.device < 0) {
    const int dev = g_device;
    int rc = check_device(dev, &g_ops.cus);
    if (rc) return rc;
    CGX_HIP(hipSetDevice(dev));
    CGX_HIP(hipStreamCreateWithFlags(&g_ops.st, hipStreamNonBlocking));
    CGX_HIP(hipMalloc((void **)&g_ops.part, (size_t)(g_ops.cus * 4 + 1) * 8));
    g_ops.device = dev;
  }
  CGX_HIP(hipSetDevice(g_ops.device));
  if (n > g_ops.cap) {
    (void)hipFree(g_ops.a);
    (void)hipFree(g_ops.b);
    (void)hipFree(g_ops.r);
    g_ops.a = g_ops.b = g_ops.r = nullptr;
    g_ops.cap = 0;
    const size_t bytes = (n + kPad) * 8;
    CGX_HIP(hipMalloc((void **)&g_ops.a, bytes));
    CGX_HIP(hipMalloc((void **)&g_ops.b, bytes));
    CGX_HIP(hipMalloc((void **)&g_ops.r, bytes));
    g_ops.cap = n;
  }
  return 0;
}

// Out-parameter rule shared by sv_mult / mv_mult / vec_add / vec_sub
// (mv_ops.c:141-152, :172-184, :213-224, :242-253): allocate a zeroed vector
// if *r is NULL, else realloc its values to `size` (mv_mult also zeroes).
int prepare_out(struct __mv_sparse **r, int size, int nnz, bool zero) {
  if (*r == nullptr) {
    struct __mv_sparse *v = (struct __mv_sparse *)calloc(1, sizeof *v);
    if (!v) return CGX_ENOMEM;
    v->values = (double *)calloc(size > 0 ? size : 1, sizeof(double));
    if (!v->values) {
      free(v);
      return CGX_ENOMEM;
    }
    v->size = size;
    v->nnz = nnz;
    v->col_indices = nullptr;
    v->row_ptr = nullptr;
    *r = v;
  } else {
    double *nv = (double *)realloc((*r)->values, (size_t)(size > 0 ? size : 1) * sizeof(double));
    if (!nv) return CGX_ENOMEM;
    (*r)->values = nv;
    if (zero) memset(nv, 0, (size_t)size * sizeof(double));
    (*r)->size = size;
    (*r)->nnz = nnz;
  }
  return 0;
}

// r = op(a, b) on the device; op 0: s*a, 1: a+b, 2: a-b.
int device_axpby(int op, double s, const double *a, const double *b, double *r, int n) {
  if (n <= 0) return 0;
  int rc = ops_ready((size_t)n);
  if (rc) return rc;
  CGX_HIP(hipMemcpyAsync(g_ops.a, a, (size_t)n * 8, hipMemcpyHostToDevice, g_ops.st));
  if (b) CGX_HIP(hipMemcpyAsync(g_ops.b, b, (size_t)n * 8, hipMemcpyHostToDevice, g_ops.st));
  CGX_HIP(launch_axpby<double>(op, n, s, g_ops.a, b ? g_ops.b : nullptr, g_ops.r,
                               vec_grid_for(n, g_ops.cus), g_ops.st));
  CGX_HIP(hipMemcpyAsync(r, g_ops.r, (size_t)n * 8, hipMemcpyDeviceToHost, g_ops.st));
  CGX_HIP(hipStreamSynchronize(g_ops.st));
  return 0;
}

int device_dot(const double *a, const double *b, int n, double *out) {
  if (n <= 0) {
    *out = 0.0;
    return 0;
  }
  int rc = ops_ready((size_t)n);
  if (rc) return rc;
  CGX_HIP(hipMemcpyAsync(g_ops.a, a, (size_t)n * 8, hipMemcpyHostToDevice, g_ops.st));
  CGX_HIP(hipMemcpyAsync(g_ops.b, b, (size_t)n * 8, hipMemcpyHostToDevice, g_ops.st));
  if (g_mode == CGX_MODE_EXACT) {
    CGX_HIP(launch_dot_seq<double>(n, g_ops.a, g_ops.b, g_ops.r, nullptr, g_ops.st));
  } else {
    const int g = vec_grid_for(n, g_ops.cus);
    CGX_HIP(launch_dot_part<double>(n, g_ops.a, g_ops.b, g_ops.part, g, g_ops.st));
    CGX_HIP(launch_finalize(FIN_SUM, g_ops.part, g, nullptr, 0, nullptr, nullptr, g_ops.r,
                            g_ops.st));
  }
  CGX_HIP(hipMemcpyAsync(out, g_ops.r, 8, hipMemcpyDeviceToHost, g_ops.st));
  CGX_HIP(hipStreamSynchronize(g_ops.st));
  return 0;
}

bool is_matrix(const struct __mv_sparse *A) {
  return A && A->row_ptr && A->size >= 0 && (A->nnz == 0 || (A->col_indices && A->values));
}

int run_solve(const struct __mv_sparse *A, const struct __mv_sparse *b, struct __mv_sparse **x,
              double tol, int maxit) {
  if (!is_matrix(A) || !b || !x || (b->size > 0 && !b->values) || A->size != b->size ||
      maxit < 0) {
    set_error("conj_grad/solve: NULL argument, size mismatch or max_iter < 0");
    return CGX_EINVAL;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const double t0 = now_ms();
  cgx_ops_timing t{};
  cgx_solver *s = nullptr;
  int rc = default_solver(&s);
  if (rc) return rc;
  int iters = maxit + 1, ran = g_alg;
  MatTiming mt;
  rc = with_matrix(s, A, [&] {
    // CGX_ALG_SR runs on every matrix (round 5): the one-launch plane march
    // where the matrix plans one, the unfused two-launch SR step otherwise;
    // cgx_ops_last_timing().alg reports the recurrence that ran
    ran = g_alg;
    int r = cgx_solver_set_mode(s, g_mode, ran);
    if (r == 0) r = cgx_solver_set_rhs(s, b->values);
    if (r == 0 && A->size > 0) r = cgx_solver_run(s, maxit, tol, &iters);
    return r;
  }, &mt);
  if (rc) return rc;
  t.uploaded = mt.uploaded;
  t.hash_ms = mt.hash_ms;
  t.setup_ms = mt.hash_ms + mt.upload_ms;
  t.solve_ms = mt.op_ms;
  const double t2 = now_ms();
  struct __mv_sparse *xv = new_mv_struct_with_size(b->size);  // cg.c:104
  if (!xv) return CGX_ENOMEM;
  if (A->size > 0 && (rc = cgx_solver_get_x(s, xv->values))) {
    cgx_free_mv_deep(xv);
    return rc;
  }
  t.download_ms = now_ms() - t2;
  t.total_ms = now_ms() - t0;
  t.iters = iters;
  t.alg = ran;
  {
    cgx_info inf;
    if (cgx_solver_info(s, &inf) == 0) t.breakdown = inf.breakdown;
  }
  g_timing = t;
  *x = xv;  // cg.c:138 (any previous *x is not freed, as in the reference)
  return iters;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------- lifecycle (host)

struct __mv_sparse *new_mv_struct() {  // mv_ops.c:14-21
  return (struct __mv_sparse *)calloc(1, sizeof(struct __mv_sparse));
}

struct __mv_sparse *new_mv_struct_with_size(int size) {  // mv_ops.c:23-37
  struct __mv_sparse *m = new_mv_struct();
  if (!m) return nullptr;
  m->size = size;
  m->nnz = size;
  m->values = (double *)calloc(size > 0 ? size : 1, sizeof(double));
  m->col_indices = nullptr;
  m->row_ptr = nullptr;
  return m;
}

void free_mv_struct(struct __mv_sparse *m) { free(m); }  // mv_ops.c:39-42

void cgx_free_mv_deep(struct __mv_sparse *m) {
  if (!m) return;
  free(m->values);
  free(m->col_indices);
  free(m->row_ptr);
  free(m);
}

struct __mv_sparse *mv_deep_copy(struct __mv_sparse *orig) {  // mv_ops.c:44-74
  if (!orig) return nullptr;
  struct __mv_sparse *cp = new_mv_struct();
  if (!cp) return nullptr;
  cp->size = orig->size;
  cp->nnz = orig->nnz;
  const size_t nv = orig->nnz > 0 ? (size_t)orig->nnz : 1;
  cp->values = (double *)calloc(nv, sizeof(double));
  if (orig->nnz > 0) memcpy(cp->values, orig->values, (size_t)orig->nnz * 8);
  if (orig->col_indices) {
    cp->col_indices = (int *)calloc(nv, sizeof(int));
    if (orig->nnz > 0) memcpy(cp->col_indices, orig->col_indices, (size_t)orig->nnz * 4);
  }
  if (orig->row_ptr) {
    cp->row_ptr = (int *)calloc((size_t)orig->size + 1, sizeof(int));
    memcpy(cp->row_ptr, orig->row_ptr, ((size_t)orig->size + 1) * 4);
  }
  return cp;
}

void print_sparse(struct __mv_sparse *o) {  // mv_ops.c:77-95, same format
  printf("Sparse Object:\n");
  if (!o) {
    printf("\tObject is NULL\n");
    return;
  }
  printf("\tSize: %d\n", o->size);
  printf("\tNNZ: %d\n", o->nnz);
  printf("\tValues: %p\n", (void *)o->values);
  for (int i = 0; i < o->nnz; i++) printf("\t%f\n", o->values[i]);
}

// mv_ops.c:99-113.  Expands row [row_ptr[r], row_ptr[r+1]) into a dense
// n-vector.  (The reference scans greedily past the row end; on chained
// matrices both agree, elsewhere this is the correct expansion.)
int mat_get_row(struct __mv_sparse *A, int row, double *p_row) {
  if (!A || !p_row) return -1;
  if (!A->row_ptr || row < 0 || row >= A->size) return -1;
  memset(p_row, 0, (size_t)A->size * sizeof(double));
  for (int k = A->row_ptr[row]; k < A->row_ptr[row + 1]; ++k) {
    const int c = A->col_indices[k];
    if (c >= 0 && c < A->size) p_row[c] = A->values[k];
  }
  return 0;
}

// ------------------------------------------------------- arithmetic (GPU)

double dot_product(struct __mv_sparse *a, struct __mv_sparse *b) {  // mv_ops.c:117-132
  if (!a || !b) return -1.0;
  if (a->size != b->size) return -1.0;
  std::lock_guard<std::mutex> lk(g_mu);
  double out = 0.0;
  if (device_dot(a->values, b->values, a->size, &out) != 0) {
    fprintf(stderr, "libcgx: dot_product: %s\n", cgx_last_error());
    return -1.0;
  }
  return out;
}

int sv_mult(double sca, struct __mv_sparse *a, struct __mv_sparse **r) {  // mv_ops.c:134-158
  if (!a || !r) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = a->size;
  double *tmp = (double *)malloc((size_t)(n > 0 ? n : 1) * 8);
  if (!tmp) return CGX_ENOMEM;
  int rc = device_axpby(0, sca, a->values, nullptr, tmp, n);
  if (rc == 0) rc = prepare_out(r, n, a->nnz, false);
  if (rc == 0 && n > 0) memcpy((*r)->values, tmp, (size_t)n * 8);
  free(tmp);
  return rc;
}

static int vec_binop(int op, struct __mv_sparse *a, struct __mv_sparse *b,
                     struct __mv_sparse **r) {
  if (!a || !b || !r) return -1;
  if (a->size != b->size) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = a->size;
  double *tmp = (double *)malloc((size_t)(n > 0 ? n : 1) * 8);
  if (!tmp) return CGX_ENOMEM;
  int rc = device_axpby(op, 0.0, a->values, b->values, tmp, n);  // reads a, b first:
  if (rc == 0) rc = prepare_out(r, n, a->nnz, false);            // *r may alias them
  if (rc == 0 && n > 0) memcpy((*r)->values, tmp, (size_t)n * 8);
  free(tmp);
  return rc;
}

int vec_add(struct __mv_sparse *a, struct __mv_sparse *b, struct __mv_sparse **r) {
  return vec_binop(1, a, b, r);  // mv_ops.c:203-230
}

int vec_sub(struct __mv_sparse *a, struct __mv_sparse *b, struct __mv_sparse **r) {
  return vec_binop(2, a, b, r);  // mv_ops.c:232-259
}

int mv_mult(struct __mv_sparse *A, struct __mv_sparse *b, struct __mv_sparse **r) {  // mv_ops.c:160-201
  if (!A || !b || !r) return -1;
  if (A->size != b->size) return -1;
  if (!is_matrix(A)) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = A->size;
  double *tmp = (double *)malloc((size_t)(n > 0 ? n : 1) * 8);
  if (!tmp) return CGX_ENOMEM;
  int rc = 0;
  if (n > 0) {
    cgx_solver *s = nullptr;
    rc = default_solver(&s);
    if (rc == 0)  // A resident across calls (with_matrix)
      rc = with_matrix(s, A, [&] { return cgx_solver_spmv(s, b->values, tmp); });
  }
  if (rc == 0) rc = prepare_out(r, n, b->nnz, true);
  if (rc == 0 && n > 0) memcpy((*r)->values, tmp, (size_t)n * 8);
  free(tmp);
  return rc;
}

int cgx_ops_set_mode(int mode, int alg) {
  if ((mode != CGX_MODE_FAST && mode != CGX_MODE_EXACT) ||
      (alg != CGX_ALG_HS && alg != CGX_ALG_CG1 && alg != CGX_ALG_SR) ||
      (mode == CGX_MODE_EXACT && alg != CGX_ALG_HS)) {
    set_error("cgx_ops_set_mode: bad mode/alg (exact mode is HS only)");
    return CGX_EINVAL;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_mode = mode;
  g_alg = alg;
  return 0;
}

int cgx_ops_set_device(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (device == g_device) return 0;
  if (g_solver || g_ops.device >= 0) {
    set_error("cgx_ops_set_device: call before the first mv_ops / conj_grad / solve call");
    return CGX_EINVAL;
  }
  g_device = device;
  return 0;
}

int cgx_ops_last_timing(cgx_ops_timing *t) {
  if (!t) return CGX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  *t = g_timing;
  return 0;
}

int cgx_ops_counters(long long *uploads, long long *reuses) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (uploads) *uploads = g_uploads;
  if (reuses) *reuses = g_reuses;
  return 0;
}

// ------------------------------------------------------------- solvers

int conj_grad(int max_iter, struct __mv_sparse *mat_A, struct __mv_sparse *vec_b,
              struct __mv_sparse **vec_x) {
  const int rc = run_solve(mat_A, vec_b, vec_x, 0.0, max_iter);
  return rc < 0 ? rc : 0;  // the reference always returns 0 (cg.c:140)
}

int solve(const struct __mv_sparse *A, const struct __mv_sparse *b, struct __mv_sparse **x,
          double tol, int maxit) {
  return run_solve(A, b, x, tol, maxit);
}

}  // extern "C"
