"""Shared test helpers: the reference's 4-line input format, fixture matrices,
and ctypes bindings of the CPU oracle (oracle/liboracle.so).

The oracle is test infrastructure; only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes
import gzip
import json
import os
import subprocess
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
ORACLE_DIR = REPO / "oracle"

_i32p = ctypes.POINTER(ctypes.c_int)
_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)


# --------------------------------------------------------------------------
# Reference input format (cg.c:146-218): 4 comma-separated lines
#   line 0: col_indices (nnz ints)      -> storeColumnIndex, cg.c:180
#   line 1: row_ptr (n+1 ints)          -> storeRowPointer,  cg.c:181
#   line 2: values (nnz doubles)        -> storeValue,       cg.c:182
#   line 3: b (n doubles)               -> storeValue,       cg.c:183
# A.size = #row_ptr - 1 (cg.c:204).  Every line ends with '\n' (the reader
# stops at the 4th newline, cg.c:190-194).
# --------------------------------------------------------------------------

def _open(path, mode):
    path = str(path)
    return gzip.open(path, mode) if path.endswith(".gz") else open(path, mode)


def write_ref_format(path, row_ptr, col, val, b):
    def fmt_f(a):
        return ",".join(repr(float(v)) for v in a)

    def fmt_i(a):
        return ",".join(str(int(v)) for v in a)

    with _open(path, "wt") as f:
        f.write(fmt_i(col) + "\n")
        f.write(fmt_i(row_ptr) + "\n")
        f.write(fmt_f(val) + "\n")
        f.write(fmt_f(b) + "\n")


def read_ref_format(path):
    with _open(path, "rt") as f:
        lines = [f.readline().rstrip("\n") for _ in range(4)]
    col = np.array([int(t) for t in lines[0].split(",")], dtype=np.int32)
    row_ptr = np.array([int(t) for t in lines[1].split(",")], dtype=np.int32)
    val = np.array([float(t) for t in lines[2].split(",")], dtype=np.float64)
    b = np.array([float(t) for t in lines[3].split(",")], dtype=np.float64)
    return row_ptr, col, val, b


# --------------------------------------------------------------------------
# Fixture matrices (numpy, seeded).  All are "chained" (SURVEY.md 8a/a3):
# ascending columns, no empty row, first_col(r+1) <= last_col(r), so the
# reference's dense-row mv_mult equals CSR SpMV -- except diag5, which is the
# documented divergence case.
# --------------------------------------------------------------------------

def csr_from_dense(A):
    n = A.shape[0]
    rp = [0]
    cols, vals = [], []
    for i in range(n):
        nz = np.nonzero(A[i])[0]
        cols.extend(nz.tolist())
        vals.extend(A[i, nz].tolist())
        rp.append(len(cols))
    return (np.array(rp, np.int32), np.array(cols, np.int32),
            np.array(vals, np.float64))


def tridiag(n):
    A = 2.0 * np.eye(n) - np.eye(n, k=1) - np.eye(n, k=-1)
    return csr_from_dense(A)


def dense_spd(n, seed):
    rng = np.random.default_rng(seed)
    M = rng.standard_normal((n, n))
    A = (M + M.T) / 2.0
    A += np.diag(np.abs(A).sum(axis=1) + 1.0)
    rp = np.arange(0, n * n + 1, n, dtype=np.int32)
    col = np.tile(np.arange(n, dtype=np.int32), n)
    b = rng.standard_normal(n)
    return rp, col, A.reshape(-1).astype(np.float64), b


def laplacian2d(nx, ny):
    """5-point, diag 4, off-diagonals -1, natural ordering i + nx*j."""
    rp = [0]
    cols, vals = [], []
    for j in range(ny):
        for i in range(nx):
            r = i + nx * j
            ent = []
            if j > 0:
                ent.append((r - nx, -1.0))
            if i > 0:
                ent.append((r - 1, -1.0))
            ent.append((r, 4.0))
            if i < nx - 1:
                ent.append((r + 1, -1.0))
            if j < ny - 1:
                ent.append((r + nx, -1.0))
            for c, v in ent:
                cols.append(c)
                vals.append(v)
            rp.append(len(cols))
    return (np.array(rp, np.int32), np.array(cols, np.int32),
            np.array(vals, np.float64))


def laplacian3d(nx, ny, nz):
    """7-point, diag 6, off-diagonals -1, natural ordering i + nx*(j + ny*k)."""
    rp = [0]
    cols, vals = [], []
    for k in range(nz):
        for j in range(ny):
            for i in range(nx):
                r = i + nx * (j + ny * k)
                ent = []
                if k > 0:
                    ent.append((r - nx * ny, -1.0))
                if j > 0:
                    ent.append((r - nx, -1.0))
                if i > 0:
                    ent.append((r - 1, -1.0))
                ent.append((r, 6.0))
                if i < nx - 1:
                    ent.append((r + 1, -1.0))
                if j < ny - 1:
                    ent.append((r + nx, -1.0))
                if k < nz - 1:
                    ent.append((r + nx * ny, -1.0))
                for c, v in ent:
                    cols.append(c)
                    vals.append(v)
                rp.append(len(cols))
    return (np.array(rp, np.int32), np.array(cols, np.int32),
            np.array(vals, np.float64))


def random_spd(n, partners, seed):
    """Symmetric, strictly diagonally dominant, chained (tridiagonal band
    always present), off-diagonals -U(0,1]."""
    rng = np.random.default_rng(seed)
    ent = {}
    for i in range(n - 1):
        v = -(1.0 - rng.random())
        ent[(i, i + 1)] = v
        ent[(i + 1, i)] = v
    for i in range(n):
        for j in rng.integers(0, n, size=partners):
            j = int(j)
            if j == i or (i, j) in ent:
                continue
            v = -(1.0 - rng.random())
            ent[(i, j)] = v
            ent[(j, i)] = v
    rows = [[] for _ in range(n)]
    for (i, j), v in ent.items():
        rows[i].append((j, v))
    rp = [0]
    cols, vals = [], []
    for i in range(n):
        off = sorted(rows[i])
        d = sum(abs(v) for _, v in off) + 1.0
        merged = sorted(off + [(i, d)])
        for c, v in merged:
            cols.append(c)
            vals.append(v)
        rp.append(len(cols))
    b = rng.standard_normal(n)
    return (np.array(rp, np.int32), np.array(cols, np.int32),
            np.array(vals, np.float64), b)


# --------------------------------------------------------------------------
# Golden fixtures
# --------------------------------------------------------------------------

def golden_names():
    return sorted(p.name[: -len(".json.gz")] for p in GOLDEN.glob("*.json.gz"))


def load_golden(name):
    with gzip.open(GOLDEN / f"{name}.json.gz", "rt") as f:
        g = json.load(f)
    rp, col, val, b = read_ref_format(GOLDEN / f"{name}.txt.gz")
    g["row_ptr"], g["col"], g["val"], g["b"] = rp, col, val, b
    g["iters"] = {int(k): np.array([float.fromhex(h) for h in v])
                  for k, v in g["iters"].items()}
    g["ops"] = {k: np.array([float.fromhex(h) for h in v])
                for k, v in g.get("ops", {}).items()}
    return g


def bits(a):
    """View a float64 array as uint64 for bit-exact comparison (NaNs with the
    same payload compare equal)."""
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def same_bits_or_both_nan(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.shape != b.shape:
        return False
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((bits(a) == bits(b)) | both_nan))


# --------------------------------------------------------------------------
# Oracle (ctypes)
# --------------------------------------------------------------------------

_oracle = None


def oracle():
    global _oracle
    if _oracle is not None:
        return _oracle
    so = ORACLE_DIR / "liboracle.so"
    if not so.exists():
        subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "liboracle.so"],
                       check=True)
    lib = ctypes.CDLL(str(so))
    lib.oracle_spmv_csr.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _f64p, _f64p]
    lib.oracle_spmv_dense_expand.argtypes = [ctypes.c_int, ctypes.c_int, _i32p,
                                             _i32p, _f64p, _f64p, _f64p]
    lib.oracle_dot.argtypes = [ctypes.c_int, _f64p, _f64p]
    lib.oracle_dot.restype = ctypes.c_double
    lib.oracle_scale.argtypes = [ctypes.c_int, ctypes.c_double, _f64p, _f64p]
    lib.oracle_add.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p]
    lib.oracle_sub.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p]
    lib.oracle_conj_grad.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     _i32p, _i32p, _f64p, _f64p, _f64p,
                                     ctypes.c_int, _f64p]
    lib.oracle_solve.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                 _i32p, _i32p, _f64p, _f64p, _f64p, _f64p]
    lib.oracle_solve_cg1.argtypes = lib.oracle_solve.argtypes
    lib.oracle_solve_sr.argtypes = lib.oracle_solve.argtypes
    lib.oracle_spmv_csr_f32.argtypes = [ctypes.c_int, _i32p, _i32p, _f32p,
                                        _f32p, _f32p]
    lib.oracle_solve_f32.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     _i32p, _i32p, _f32p, _f32p, _f32p, _f64p]
    lib.oracle_solve_mt.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                    _i32p, _i32p, _f64p, _f64p, _f64p,
                                    ctypes.c_int]
    _oracle = lib
    return lib


def _p(a, t):
    return a.ctypes.data_as(t)


def o_spmv(rp, col, val, x):
    n = len(rp) - 1
    y = np.empty(n, np.float64)
    oracle().oracle_spmv_csr(n, _p(rp, _i32p), _p(col, _i32p), _p(val, _f64p),
                             _p(np.ascontiguousarray(x, np.float64), _f64p),
                             _p(y, _f64p))
    return y


def o_spmv_f32(rp, col, val, x):
    n = len(rp) - 1
    y = np.empty(n, np.float32)
    oracle().oracle_spmv_csr_f32(n, _p(rp, _i32p), _p(col, _i32p),
                                 _p(np.ascontiguousarray(val, np.float32), _f32p),
                                 _p(np.ascontiguousarray(x, np.float32), _f32p),
                                 _p(y, _f32p))
    return y


def o_spmv_dense(rp, col, val, x):
    n = len(rp) - 1
    y = np.empty(n, np.float64)
    oracle().oracle_spmv_dense_expand(n, len(col), _p(rp, _i32p), _p(col, _i32p),
                                      _p(val, _f64p),
                                      _p(np.ascontiguousarray(x, np.float64), _f64p),
                                      _p(y, _f64p))
    return y


def o_dot(a, b):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return oracle().oracle_dot(len(a), _p(a, _f64p), _p(b, _f64p))


def o_conj_grad(max_iter, rp, col, val, b, dense_expand=False):
    n = len(rp) - 1
    x = np.empty(n, np.float64)
    hist = np.zeros(max(max_iter + 1, 1), np.float64)
    oracle().oracle_conj_grad(max_iter, n, len(col), _p(rp, _i32p), _p(col, _i32p),
                              _p(val, _f64p), _p(b, _f64p), _p(x, _f64p),
                              1 if dense_expand else 0, _p(hist, _f64p))
    return x, hist


def o_solve(maxit, tol, rp, col, val, b, cg1=False, sr=False):
    n = len(rp) - 1
    x = np.empty(n, np.float64)
    hist = np.zeros(maxit + 1, np.float64)
    fn = (oracle().oracle_solve_cg1 if cg1 else oracle().oracle_solve_sr if sr
          else oracle().oracle_solve)
    its = fn(maxit, tol, n, _p(rp, _i32p), _p(col, _i32p), _p(val, _f64p),
             _p(b, _f64p), _p(x, _f64p), _p(hist, _f64p))
    return x, its, hist[:its]


def o_solve_f32(maxit, tol, rp, col, val, b):
    """oracle_solve_f32: C5's fp32 HS-CG (float vectors, exact double dot
    products, alpha / beta rounded to float once)."""
    rp = np.ascontiguousarray(rp, np.int32)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    n = len(rp) - 1
    x = np.empty(n, np.float32)
    hist = np.zeros(maxit + 1, np.float64)
    its = oracle().oracle_solve_f32(maxit, tol, n, _p(rp, _i32p), _p(col, _i32p),
                                    _p(val, _f32p), _p(b, _f32p), _p(x, _f32p),
                                    _p(hist, _f64p))
    return x, its, hist[:its]


def o_solve_mt(maxit, tol, rp, col, val, b, threads):
    n = len(rp) - 1
    x = np.empty(n, np.float64)
    its = oracle().oracle_solve_mt(maxit, tol, n, _p(rp, _i32p), _p(col, _i32p),
                                   _p(val, _f64p), _p(b, _f64p), _p(x, _f64p),
                                   threads)
    return x, its
