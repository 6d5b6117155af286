"""ctypes binding of libcgx.so (include/cgx.h, include/mv_ops.h).

This is the host-side mirror used by the Python tests and bench.py; the
product is the C ABI itself.  The library must be built (``make -C
conjugate-gradient_amd`` or ``__graft_entry__.build()``); there is no CPU
fallback -- a missing library raises, and compute calls without a gfx950
device return CGX_ENODEV, which this module raises as CgxError.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["CGX_LIB"]) if os.environ.get("CGX_LIB") else HERE / "lib" / "libcgx.so"

CGX_EINVAL, CGX_ENODEV, CGX_ENOMEM, CGX_ECOMM = -1, -2, -3, -4
CGX_MODE_FAST, CGX_MODE_EXACT = 0, 1
CGX_ALG_HS, CGX_ALG_CG1, CGX_ALG_SR = 0, 1, 2
CGX_F64, CGX_F32 = 0, 1
CGX_BENCH_GRAPH, CGX_BENCH_SPMV_EVENTS, CGX_BENCH_SPMV_ONLY = 1, 2, 4
(CGX_LAYOUT_AUTO, CGX_LAYOUT_CSR, CGX_LAYOUT_DC, CGX_LAYOUT_DIA, CGX_LAYOUT_PANEL,
 CGX_LAYOUT_STENCIL) = range(6)
LAYOUT_NAMES = {CGX_LAYOUT_AUTO: "auto", CGX_LAYOUT_CSR: "csr", CGX_LAYOUT_DC: "dc",
                CGX_LAYOUT_DIA: "dia", CGX_LAYOUT_PANEL: "panel", CGX_LAYOUT_STENCIL: "stencil"}
LAYOUTS = {v: k for k, v in LAYOUT_NAMES.items()}

_i32p = ctypes.POINTER(ctypes.c_int)
_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p


class CgxError(RuntimeError):
    pass


class MvSparse(ctypes.Structure):
    """struct __mv_sparse (mv_ops.h:17-23)."""
    _fields_ = [("size", ctypes.c_int), ("nnz", ctypes.c_int),
                ("values", _f64p), ("col_indices", _i32p), ("row_ptr", _i32p)]


class CgxInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("nnz", ctypes.c_int), ("dtype", ctypes.c_int),
                ("mode", ctypes.c_int), ("alg", ctypes.c_int), ("layout", ctypes.c_int),
                ("n_items", ctypes.c_int), ("spmv_grid", ctypes.c_int),
                ("vec_grid", ctypes.c_int), ("spmv_bytes", ctypes.c_double),
                ("iter_bytes", ctypes.c_double), ("spmv_iter_bytes", ctypes.c_double),
                ("device_bytes", ctypes.c_size_t), ("n_panels", ctypes.c_int),
                ("n_dict", ctypes.c_int), ("tile_bands", ctypes.c_int), ("nt", ctypes.c_int),
                ("code_bytes_per_row", ctypes.c_int), ("encode_fallback", ctypes.c_int),
                ("setup_host_ms", ctypes.c_double), ("setup_device_ms", ctypes.c_double),
                ("n_values", ctypes.c_int), ("gathers_per_chunk", ctypes.c_int),
                ("fused", ctypes.c_int), ("fuse_status", ctypes.c_int),
                ("breakdown", ctypes.c_int), ("fuse_march", ctypes.c_int),
                ("dia_value_stream", ctypes.c_int)]


class CgxDistStats(ctypes.Structure):
    _fields_ = [("n_global", ctypes.c_longlong), ("row_begin", ctypes.c_int),
                ("n_loc", ctypes.c_int), ("n_ghost", ctypes.c_int), ("n_send", ctypes.c_int),
                ("nnz", ctypes.c_int), ("interior_items", ctypes.c_int),
                ("boundary_items", ctypes.c_int), ("spmv_bytes", ctypes.c_double),
                ("iter_bytes", ctypes.c_double), ("halo_bytes", ctypes.c_double),
                ("device_bytes", ctypes.c_size_t), ("spmv_iter_bytes", ctypes.c_double),
                ("layout", ctypes.c_int), ("n_dict", ctypes.c_int), ("graph", ctypes.c_int),
                ("alg", ctypes.c_int), ("fused", ctypes.c_int),
                ("fuse_status", ctypes.c_int), ("breakdown", ctypes.c_int),
                ("march", ctypes.c_int), ("inplace", ctypes.c_int)]


_MVP = ctypes.POINTER(MvSparse)
_MVPP = ctypes.POINTER(_MVP)

# name -> (restype, argtypes)
_SIGS = {
    # mv_ops.h
    "new_mv_struct": (_MVP, []),
    "new_mv_struct_with_size": (_MVP, [ctypes.c_int]),
    "free_mv_struct": (None, [_MVP]),
    "mv_deep_copy": (_MVP, [_MVP]),
    "print_sparse": (None, [_MVP]),
    "mat_get_row": (ctypes.c_int, [_MVP, ctypes.c_int, _f64p]),
    "dot_product": (ctypes.c_double, [_MVP, _MVP]),
    "sv_mult": (ctypes.c_int, [ctypes.c_double, _MVP, _MVPP]),
    "mv_mult": (ctypes.c_int, [_MVP, _MVP, _MVPP]),
    "vec_add": (ctypes.c_int, [_MVP, _MVP, _MVPP]),
    "vec_sub": (ctypes.c_int, [_MVP, _MVP, _MVPP]),
    # cgx.h
    "conj_grad": (ctypes.c_int, [ctypes.c_int, _MVP, _MVP, _MVPP]),
    "solve": (ctypes.c_int, [_MVP, _MVP, _MVPP, ctypes.c_double, ctypes.c_int]),
    "cgx_free_mv_deep": (None, [_MVP]),
    "cgx_ops_counters": (ctypes.c_int, [ctypes.POINTER(ctypes.c_longlong)] * 2),
    "cgx_ops_set_mode": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "cgx_ops_set_device": (ctypes.c_int, [ctypes.c_int]),
    "cgx_ops_last_timing": (ctypes.c_int, [_vp]),
    "cgx_last_error": (ctypes.c_char_p, []),
    "cgx_device_count": (ctypes.c_int, []),
    "cgx_device_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "cgx_runtime_versions": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)] * 3),
    "cgx_stream_bench": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "cgx_solver_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "cgx_solver_destroy": (None, [_vp]),
    "cgx_solver_set_mode": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "cgx_solver_set_layout": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_solver_set_fused": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_solver_set_march": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_solver_set_sr_chain": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_solver_set_matrix": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                             _i32p, _i32p, _f64p]),
    "cgx_solver_set_matrix_f32": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                                 _i32p, _i32p, _f32p]),
    "cgx_solver_gen_laplacian": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int]),
    "cgx_solver_set_stencil": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int]),
    "cgx_solver_get_matrix": (ctypes.c_int, [_vp, _i32p, _i32p, _f64p]),
    "cgx_laplacian_row_ptr": (ctypes.c_longlong, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  _i32p]),
    "cgx_solver_set_rhs": (ctypes.c_int, [_vp, _f64p]),
    "cgx_solver_set_rhs_f32": (ctypes.c_int, [_vp, _f32p]),
    "cgx_solver_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_int)]),
    "cgx_solver_get_x": (ctypes.c_int, [_vp, _f64p]),
    "cgx_solver_get_x_f32": (ctypes.c_int, [_vp, _f32p]),
    "cgx_solver_get_history": (ctypes.c_int, [_vp, _f64p, ctypes.c_int]),
    "cgx_solver_spmv": (ctypes.c_int, [_vp, _f64p, _f64p]),
    "cgx_solver_spmv_f32": (ctypes.c_int, [_vp, _f32p, _f32p]),
    "cgx_solver_info": (ctypes.c_int, [_vp, ctypes.POINTER(CgxInfo)]),
    "cgx_solver_bench": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        _f64p, _f64p]),
    "cgx_solver_bench_prepare": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_solver_bench_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                            _f64p, _f64p]),
    "cgx_gen_laplacian2d": (ctypes.c_longlong, [ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int,
                                                _i32p, _i32p, _f64p]),
    "cgx_gen_laplacian3d": (ctypes.c_longlong, [ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, _i32p, _i32p, _f64p]),
    "cgx_gen_random_spd": (ctypes.c_longlong, [ctypes.c_int, ctypes.c_int,
                                               ctypes.c_ulonglong, ctypes.c_int,
                                               ctypes.c_int, _i32p, _i32p, _f64p,
                                               _f32p]),
    "cgx_gen_varcoef3d": (ctypes.c_longlong, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int,
                                              _i32p, _i32p, _f64p]),
    "cgx_csr_is_chained": (ctypes.c_int, [ctypes.c_int, _i32p, _i32p]),
    "cgx_read_input_file": (ctypes.c_int, [ctypes.c_char_p, _MVP, _MVP]),
    "cgx_read_input_cached": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, _MVP, _MVP,
                                             ctypes.POINTER(ctypes.c_int)]),
    # partition layer
    "cgx_partition_rows": (None, [ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "cgx_partition_owner": (ctypes.c_int, [ctypes.c_longlong, ctypes.c_int, ctypes.c_longlong]),
    "cgx_part_create": (ctypes.c_int, [ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, _i32p, _i32p,
                                       ctypes.POINTER(_vp)]),
    "cgx_part_destroy": (None, [_vp]),
    "cgx_part_info": (ctypes.c_int, [_vp] + [ctypes.POINTER(ctypes.c_int)] * 4),
    "cgx_part_local_cols": (ctypes.c_int, [_vp, _i32p]),
    "cgx_part_ghosts": (ctypes.c_int, [_vp, _i32p]),
    "cgx_part_recv_counts": (ctypes.c_int, [_vp, _i32p]),
    "cgx_part_set_requests": (ctypes.c_int, [_vp, _i32p, _i32p]),
    "cgx_part_send_counts": (ctypes.c_int, [_vp, _i32p]),
    "cgx_part_send_local": (ctypes.c_int, [_vp, _i32p]),
    # distributed solver
    "cgx_dist_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "cgx_dist_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "cgx_dist_create_local": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "cgx_dist_destroy": (None, [_vp]),
    "cgx_dist_set_matrix": (ctypes.c_int, [_vp, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                           _i32p, _i32p, _f64p]),
    "cgx_dist_set_rhs": (ctypes.c_int, [_vp, _f64p]),
    "cgx_dist_set_alg": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_set_layout": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_set_graph": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_debug_refuse_capture": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_set_march": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_set_sr_chain": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_set_fused": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double,
                                    ctypes.POINTER(ctypes.c_int)]),
    "cgx_dist_get_x": (ctypes.c_int, [_vp, _f64p]),
    "cgx_dist_get_history": (ctypes.c_int, [_vp, _f64p, ctypes.c_int]),
    "cgx_dist_bench_prepare": (ctypes.c_int, [_vp, ctypes.c_int]),
    "cgx_dist_bench_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _f64p, _f64p]),
    "cgx_dist_info": (ctypes.c_int, [_vp, ctypes.POINTER(CgxDistStats)]),
    "cgx_dist_bench_phases": (ctypes.c_int, [_vp, _f64p, ctypes.POINTER(ctypes.c_int)]),
}

_lib = None


CGX_FUSE_OFF, CGX_FUSE_AUTO, CGX_FUSE_ON = 0, 1, 2
# cgx_info.fuse_status / cgx_dist_stats.fuse_status (cgx.h)
(CGX_FUSE_STATUS_RUNS, CGX_FUSE_STATUS_OFF, CGX_FUSE_STATUS_NOT_DIA, CGX_FUSE_STATUS_WIDE_CODES,
 CGX_FUSE_STATUS_FAR_DIAGS, CGX_FUSE_STATUS_CACHED, CGX_FUSE_STATUS_EXACT, CGX_FUSE_STATUS_PEER,
 CGX_FUSE_STATUS_CG1_AUTO, CGX_FUSE_STATUS_NO_MARCH, CGX_FUSE_STATUS_VALUE_STREAM) = range(11)


def fuse_mode(mode):
    """cgx_*_set_fused mode from "auto" / True / False (or the constant)."""
    if isinstance(mode, str):
        return {"auto": CGX_FUSE_AUTO, "on": CGX_FUSE_ON, "off": CGX_FUSE_OFF}[mode]
    if isinstance(mode, bool):
        return CGX_FUSE_ON if mode else CGX_FUSE_OFF
    return int(mode)


def lib():
    """Load libcgx.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise CgxError(f"{LIB_PATH} not built: run `make -C {HERE}` "
                       "(or __graft_entry__.build())")
    L = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    return (lib().cgx_last_error() or b"").decode(errors="replace")


def check(rc, what=""):
    if rc < 0:
        raise CgxError(f"{what} failed ({rc}): {last_error()}")
    return rc


def _p(a, t):
    return a.ctypes.data_as(t)


# --------------------------------------------------------------- generators

def _gen(fn, args, m, want_f32=False):
    L = lib()
    nnz = getattr(L, fn)(*args, None, None, None, *([None] if fn == "cgx_gen_random_spd" else []))
    check(nnz, fn)
    rp = np.empty(m + 1, np.int32)
    col = np.empty(max(nnz, 1), np.int32)
    if fn == "cgx_gen_random_spd":
        val = None if want_f32 else np.empty(max(nnz, 1), np.float64)
        v32 = np.empty(max(nnz, 1), np.float32) if want_f32 else None
        got = L.cgx_gen_random_spd(*args, _p(rp, _i32p), _p(col, _i32p),
                                   _p(val, _f64p) if val is not None else None,
                                   _p(v32, _f32p) if v32 is not None else None)
        check(got, fn)
        return rp, col[:nnz], (v32 if want_f32 else val)[:nnz]
    val = np.empty(max(nnz, 1), np.float64)
    got = getattr(L, fn)(*args, _p(rp, _i32p), _p(col, _i32p), _p(val, _f64p))
    check(got, fn)
    return rp, col[:nnz], val[:nnz]


def laplacian2d(nx, ny, row_begin=0, row_end=None):
    row_end = nx * ny if row_end is None else row_end
    return _gen("cgx_gen_laplacian2d", (nx, ny, row_begin, row_end), row_end - row_begin)


CGX_STREAM_TRIAD, CGX_STREAM_READ = 0, 1
CGX_STREAM_COPY, CGX_STREAM_COPY_NT = 2, 3
CGX_STREAM_TRIAD_TUNED, CGX_STREAM_TRIAD_NT = 4, 5
CGX_STREAM_MIX33, CGX_STREAM_MIX33_NT = 6, 7
STREAM_KINDS = {"triad": CGX_STREAM_TRIAD, "read": CGX_STREAM_READ, "copy": CGX_STREAM_COPY,
                "copy_nt": CGX_STREAM_COPY_NT, "triad_tuned": CGX_STREAM_TRIAD_TUNED,
                "triad_nt": CGX_STREAM_TRIAD_NT, "mix33": CGX_STREAM_MIX33,
                "mix33_nt": CGX_STREAM_MIX33_NT}


def stream_bench(device, n, reps=10, kind=CGX_STREAM_TRIAD):
    """On-box HBM ceiling (cgx_stream_bench): best-of-reps GB/s over fp64
    arrays of n elements; kind CGX_STREAM_TRIAD (a = b + s c, 24 n bytes),
    CGX_STREAM_READ (read-only sum, 8 n bytes), or a tuned read/write mix
    (CGX_STREAM_COPY / TRIAD_TUNED / MIX33, _NT: non-temporal stores;
    include/cgx.h)."""
    g = ctypes.c_double(0.0)
    check(lib().cgx_stream_bench(device, kind, n, reps, ctypes.byref(g)), "stream_bench")
    return g.value


def laplacian_row_ptr(dim, nx, ny, nz=1, row_begin=0, row_end=None):
    """Closed-form row_ptr of Laplacian rows [row_begin, row_end) (host)."""
    n = nx * ny * (nz if dim == 3 else 1)
    row_end = n if row_end is None else row_end
    rp = np.empty(row_end - row_begin + 1, np.int32)
    nnz = lib().cgx_laplacian_row_ptr(dim, nx, ny, nz, row_begin, row_end, _p(rp, _i32p))
    if nnz < 0:
        raise CgxError(f"laplacian_row_ptr failed ({nnz})")
    return rp


def laplacian3d(nx, ny, nz, row_begin=0, row_end=None):
    row_end = nx * ny * nz if row_end is None else row_end
    return _gen("cgx_gen_laplacian3d", (nx, ny, nz, row_begin, row_end),
                row_end - row_begin)


def varcoef3d(nx, ny, nz, seed=7, row_begin=0, row_end=None):
    """7-point pattern, one random SPD coefficient per grid edge
    (cgx_gen_varcoef3d): no layout can index its values."""
    row_end = nx * ny * nz if row_end is None else row_end
    return _gen("cgx_gen_varcoef3d", (nx, ny, nz, seed, row_begin, row_end),
                row_end - row_begin)


def random_spd(n, partners, seed, row_begin=0, row_end=None, f32=False):
    row_end = n if row_end is None else row_end
    return _gen("cgx_gen_random_spd", (n, partners, seed, row_begin, row_end),
                row_end - row_begin, want_f32=f32)


def is_chained(rp, col):
    rp = np.ascontiguousarray(rp, np.int32)
    col = np.ascontiguousarray(col, np.int32)
    return bool(check(lib().cgx_csr_is_chained(len(rp) - 1, _p(rp, _i32p),
                                                _p(col, _i32p)), "is_chained"))


# ------------------------------------------------------------------ solver

class Solver:
    """Device-resident CG solver (cgx_solver_*)."""

    def __init__(self, device=0, mode=CGX_MODE_FAST, alg=CGX_ALG_HS, layout=CGX_LAYOUT_AUTO,
                 fused="auto"):
        self._h = _vp()
        check(lib().cgx_solver_create(device, ctypes.byref(self._h)), "cgx_solver_create")
        self.set_mode(mode, alg)
        self.set_layout(layout)
        self.set_fused(fused)
        self.n = 0
        self.f32 = False

    def close(self):
        if self._h:
            lib().cgx_solver_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_mode(self, mode, alg=CGX_ALG_HS):
        check(lib().cgx_solver_set_mode(self._h, mode, alg), "set_mode")

    def set_fused(self, mode):
        """Fused HS step on DIA layouts (cgx_solver_set_fused): "auto",
        True (wherever the layout takes it) or False."""
        check(lib().cgx_solver_set_fused(self._h, fuse_mode(mode)), "set_fused")

    def set_march(self, steps=-1):
        """Plane march of the fused HS step (cgx_solver_set_march): -1 auto,
        0 off (the per-slice fused kernel), > 0 slices of a chain per workgroup."""
        check(lib().cgx_solver_set_march(self._h, int(steps)), "set_march")

    def set_sr_chain(self, rows=0):
        """Chain width (rows) of CGX_ALG_SR's one-launch plane march
        (cgx_solver_set_sr_chain): 0 auto, > 0 that width."""
        check(lib().cgx_solver_set_sr_chain(self._h, int(rows)), "set_sr_chain")

    def set_layout(self, layout):
        """CGX_LAYOUT_* (or its name) for the next set_matrix / gen_laplacian."""
        if isinstance(layout, str):
            layout = LAYOUTS[layout]
        check(lib().cgx_solver_set_layout(self._h, layout), "set_layout")

    def gen_laplacian(self, dim, nx, ny, nz=1):
        """Laplacian CSR generated in device memory (cgx_solver_gen_laplacian)."""
        check(lib().cgx_solver_gen_laplacian(self._h, dim, nx, ny, nz), "gen_laplacian")
        self.f32 = False
        self.n = nx * ny * (nz if dim == 3 else 1)

    def set_stencil(self, dim, nx, ny, nz=1):
        """Matrix-free Laplacian operator (cgx_solver_set_stencil)."""
        check(lib().cgx_solver_set_stencil(self._h, dim, nx, ny, nz), "set_stencil")
        self.f32 = False
        self.n = nx * ny * (nz if dim == 3 else 1)

    def matrix(self):
        """The device CSR as numpy arrays (row_ptr, col, val); fp64 plain CSR."""
        i = self.info()
        n, nnz = i["n"], i["nnz"]
        rp = np.empty(n + 1, np.int32)
        col = np.empty(max(nnz, 1), np.int32)
        val = np.empty(max(nnz, 1), np.float64)
        check(lib().cgx_solver_get_matrix(self._h, _p(rp, _i32p), _p(col, _i32p),
                                          _p(val, _f64p)), "get_matrix")
        return rp, col[:nnz], val[:nnz]

    def set_matrix(self, rp, col, val):
        rp = np.ascontiguousarray(rp, np.int32)
        col = np.ascontiguousarray(col, np.int32)
        n = len(rp) - 1
        if np.asarray(val).dtype == np.float32:
            val = np.ascontiguousarray(val, np.float32)
            check(lib().cgx_solver_set_matrix_f32(self._h, n, len(col), _p(rp, _i32p),
                                                  _p(col, _i32p), _p(val, _f32p)),
                  "set_matrix_f32")
            self.f32 = True
        else:
            val = np.ascontiguousarray(val, np.float64)
            check(lib().cgx_solver_set_matrix(self._h, n, len(col), _p(rp, _i32p),
                                              _p(col, _i32p), _p(val, _f64p)),
                  "set_matrix")
            self.f32 = False
        self.n = n

    def set_rhs(self, b):
        if self.f32:
            b = np.ascontiguousarray(b, np.float32)
            check(lib().cgx_solver_set_rhs_f32(self._h, _p(b, _f32p)), "set_rhs_f32")
        else:
            b = np.ascontiguousarray(b, np.float64)
            check(lib().cgx_solver_set_rhs(self._h, _p(b, _f64p)), "set_rhs")

    def run(self, maxit, tol=0.0):
        it = ctypes.c_int(0)
        check(lib().cgx_solver_run(self._h, maxit, tol, ctypes.byref(it)), "run")
        return it.value

    def x(self):
        if self.f32:
            out = np.empty(self.n, np.float32)
            check(lib().cgx_solver_get_x_f32(self._h, _p(out, _f32p)), "get_x_f32")
        else:
            out = np.empty(self.n, np.float64)
            check(lib().cgx_solver_get_x(self._h, _p(out, _f64p)), "get_x")
        return out

    def history(self, cap):
        out = np.zeros(cap, np.float64)
        m = check(lib().cgx_solver_get_history(self._h, _p(out, _f64p), cap), "history")
        return out[:m]

    def spmv(self, x):
        if self.f32:
            x = np.ascontiguousarray(x, np.float32)
            y = np.empty(self.n, np.float32)
            check(lib().cgx_solver_spmv_f32(self._h, _p(x, _f32p), _p(y, _f32p)), "spmv")
        else:
            x = np.ascontiguousarray(x, np.float64)
            y = np.empty(self.n, np.float64)
            check(lib().cgx_solver_spmv(self._h, _p(x, _f64p), _p(y, _f64p)), "spmv")
        return y

    def info(self):
        i = CgxInfo()
        check(lib().cgx_solver_info(self._h, ctypes.byref(i)), "info")
        d = {k: getattr(i, k) for k, _ in CgxInfo._fields_}
        d["layout_name"] = LAYOUT_NAMES.get(d["layout"], "?")
        return d

    def bench_prepare(self, warmup):
        check(lib().cgx_solver_bench_prepare(self._h, warmup), "bench_prepare")

    def bench_run(self, iters, graph=True, spmv_events=False, spmv_only=False):
        """Returns (device ms for all iters, average SpMV ms or -1).
        spmv_only: back-to-back SpMVs y = A p instead of CG iterations."""
        tot = ctypes.c_double(0)
        sp = ctypes.c_double(0)
        flags = ((CGX_BENCH_GRAPH if graph else 0) | (CGX_BENCH_SPMV_EVENTS if spmv_events else 0)
                 | (CGX_BENCH_SPMV_ONLY if spmv_only else 0))
        check(lib().cgx_solver_bench_run(self._h, iters, flags, ctypes.byref(tot),
                                         ctypes.byref(sp)), "bench_run")
        return tot.value, sp.value

    def bench(self, warmup, iters, graph=True, spmv_events=False):
        tot = ctypes.c_double(0)
        sp = ctypes.c_double(0)
        flags = (CGX_BENCH_GRAPH if graph else 0) | (CGX_BENCH_SPMV_EVENTS if spmv_events else 0)
        check(lib().cgx_solver_bench(self._h, warmup, iters, flags, ctypes.byref(tot),
                                     ctypes.byref(sp)), "bench")
        return tot.value, sp.value


# ------------------------------------------------- reference struct helpers

class Mv:
    """A struct __mv_sparse whose arrays are owned by numpy (kept alive here)."""

    def __init__(self, values, col=None, row_ptr=None):
        self.values = np.ascontiguousarray(values, np.float64)
        self.col = None if col is None else np.ascontiguousarray(col, np.int32)
        self.row_ptr = None if row_ptr is None else np.ascontiguousarray(row_ptr, np.int32)
        s = MvSparse()
        if self.row_ptr is not None:
            s.size = len(self.row_ptr) - 1
            s.nnz = len(self.values)
            s.col_indices = _p(self.col, _i32p)
            s.row_ptr = _p(self.row_ptr, _i32p)
        else:
            s.size = s.nnz = len(self.values)
        s.values = _p(self.values, _f64p)
        self.struct = s

    @property
    def ptr(self):
        return ctypes.pointer(self.struct)


def mv_values(p):
    """Copy the values of a libcgx-allocated struct __mv_sparse* to numpy."""
    s = p.contents
    return np.ctypeslib.as_array(s.values, shape=(s.size,)).copy() if s.size > 0 else np.empty(0)


def conj_grad(max_iter, A: Mv, b: Mv):
    out = _MVP()
    rc = lib().conj_grad(max_iter, A.ptr, b.ptr, ctypes.byref(out))
    check(rc, "conj_grad")
    x = mv_values(out)
    lib().cgx_free_mv_deep(out)
    return x


def solve(A: Mv, b: Mv, tol, maxit):
    out = _MVP()
    its = check(lib().solve(A.ptr, b.ptr, ctypes.byref(out), tol, maxit), "solve")
    x = mv_values(out)
    lib().cgx_free_mv_deep(out)
    return x, its


def mv_mult(A: Mv, b: Mv):
    """mv_ops.h mv_mult through the C ABI (the op-level drop-in)."""
    out = _MVP()
    check(lib().mv_mult(A.ptr, b.ptr, ctypes.byref(out)), "mv_mult")
    y = mv_values(out)
    lib().cgx_free_mv_deep(out)
    return y


class CgxOpsTiming(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("setup_ms", ctypes.c_double),
                ("hash_ms", ctypes.c_double), ("solve_ms", ctypes.c_double),
                ("download_ms", ctypes.c_double), ("uploaded", ctypes.c_int),
                ("iters", ctypes.c_int), ("breakdown", ctypes.c_int),
                ("alg", ctypes.c_int)]


def ops_set_mode(mode=CGX_MODE_FAST, alg=CGX_ALG_HS):
    """Numerics of conj_grad / solve / the mv_ops.h arithmetic (process-wide)."""
    check(lib().cgx_ops_set_mode(mode, alg), "ops_set_mode")


def ops_last_timing():
    """Wall-clock split of the last conj_grad / solve call (cgx_ops_last_timing)."""
    t = CgxOpsTiming()
    check(lib().cgx_ops_last_timing(ctypes.byref(t)), "ops_last_timing")
    return {k: getattr(t, k) for k, _ in CgxOpsTiming._fields_}


def ops_counters():
    """(uploads, reuses) of the op-level matrix residency (cgx_ops_counters)."""
    u, r = ctypes.c_longlong(0), ctypes.c_longlong(0)
    check(lib().cgx_ops_counters(ctypes.byref(u), ctypes.byref(r)), "ops_counters")
    return u.value, r.value


# ------------------------------------------------------------ partitioning

def partition_rows(n, nranks, rank):
    rb, re_ = ctypes.c_int(0), ctypes.c_int(0)
    lib().cgx_partition_rows(n, nranks, rank, ctypes.byref(rb), ctypes.byref(re_))
    return rb.value, re_.value


class Partition:
    """cgx_part: ghost discovery, local renumbering and halo send lists of
    one rank's rows (host only)."""

    def __init__(self, n_global, nranks, rank, rp, col_global):
        self.rp = np.ascontiguousarray(rp, np.int32)
        self.col = np.ascontiguousarray(col_global, np.int32)
        self.nranks, self.rank = nranks, rank
        self._h = _vp()
        check(lib().cgx_part_create(n_global, nranks, rank, len(self.rp) - 1, len(self.col),
                                    _p(self.rp, _i32p), _p(self.col, _i32p),
                                    ctypes.byref(self._h)), "cgx_part_create")

    def __del__(self):
        try:
            if self._h:
                lib().cgx_part_destroy(self._h)
        except Exception:
            pass

    def info(self):
        v = [ctypes.c_int(0) for _ in range(4)]
        check(lib().cgx_part_info(self._h, *[ctypes.byref(x) for x in v]), "part_info")
        return dict(n_loc=v[0].value, n_ghost=v[1].value, row_begin=v[2].value,
                    n_send=v[3].value)

    def local_cols(self):
        out = np.empty(max(len(self.col), 1), np.int32)
        check(lib().cgx_part_local_cols(self._h, _p(out, _i32p)), "local_cols")
        return out[:len(self.col)]

    def ghosts(self):
        n = self.info()["n_ghost"]
        out = np.empty(max(n, 1), np.int32)
        check(lib().cgx_part_ghosts(self._h, _p(out, _i32p)), "ghosts")
        return out[:n]

    def recv_counts(self):
        out = np.empty(self.nranks, np.int32)
        check(lib().cgx_part_recv_counts(self._h, _p(out, _i32p)), "recv_counts")
        return out

    def set_requests(self, counts, globals_):
        counts = np.ascontiguousarray(counts, np.int32)
        g = np.ascontiguousarray(globals_, np.int32)
        if len(g) == 0:
            g = np.zeros(1, np.int32)
        check(lib().cgx_part_set_requests(self._h, _p(counts, _i32p), _p(g, _i32p)),
              "set_requests")

    def send_counts(self):
        out = np.empty(self.nranks, np.int32)
        check(lib().cgx_part_send_counts(self._h, _p(out, _i32p)), "send_counts")
        return out

    def send_local(self):
        n = self.info()["n_send"]
        out = np.empty(max(n, 1), np.int32)
        check(lib().cgx_part_send_local(self._h, _p(out, _i32p)), "send_local")
        return out[:n]


# ---------------------------------------------------------- multi-GPU solver

def device_synchronize(device=0):
    check(lib().cgx_device_synchronize(device), "device_synchronize")


def runtime_versions():
    """(HIP runtime, HIP compiled against, RCCL) versions libcgx runs with
    (cgx_runtime_versions): `import torch` before libcgx binds it to the
    ROCm copies PyTorch bundles."""
    v = [ctypes.c_int(0) for _ in range(3)]
    check(lib().cgx_runtime_versions(*[ctypes.byref(x) for x in v]), "runtime_versions")
    return dict(hip_runtime=v[0].value, hip_compiled=v[1].value, rccl=v[2].value)


def dist_unique_id():
    buf = ctypes.create_string_buffer(128)
    check(lib().cgx_dist_unique_id(buf), "cgx_dist_unique_id")
    return buf.raw


class DistSolver:
    """One rank of the multi-GPU CG solver (cgx_dist_*)."""

    def __init__(self, device=0, nranks=1, rank=0, uid=None, _handle=None):
        self._keep = []
        if _handle is not None:
            self._h = _handle
            self._owner = False
            return
        self._h = _vp()
        self._owner = True
        check(lib().cgx_dist_create(device, nranks, rank, uid, ctypes.byref(self._h)),
              "cgx_dist_create")

    @staticmethod
    def local_group(device, nparts):
        arr = (_vp * nparts)()
        check(lib().cgx_dist_create_local(device, nparts, arr), "cgx_dist_create_local")
        parts = [DistSolver(_handle=_vp(arr[i])) for i in range(nparts)]
        parts[0]._owner = True
        return parts

    def close(self):
        if self._h and self._owner:
            lib().cgx_dist_destroy(self._h)
        self._h = _vp()

    def set_matrix(self, n_global, rp, col_global, val):
        rp = np.ascontiguousarray(rp, np.int32)
        col = np.ascontiguousarray(col_global, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        check(lib().cgx_dist_set_matrix(self._h, n_global, len(rp) - 1, len(col),
                                        _p(rp, _i32p), _p(col, _i32p), _p(val, _f64p)),
              "dist_set_matrix")
        self.n_loc = len(rp) - 1

    def set_rhs(self, b):
        b = np.ascontiguousarray(b, np.float64)
        check(lib().cgx_dist_set_rhs(self._h, _p(b, _f64p)), "dist_set_rhs")

    def set_alg(self, alg):
        """CGX_ALG_HS (default, two all-reduces), CGX_ALG_CG1 (one) or
        CGX_ALG_SR (HS with one all-reduce; needs the fused DIA step)."""
        check(lib().cgx_dist_set_alg(self._h, alg), "dist_set_alg")

    def set_layout(self, layout):
        if isinstance(layout, str):
            layout = LAYOUTS[layout]
        check(lib().cgx_dist_set_layout(self._h, layout), "dist_set_layout")

    def set_graph(self, on):
        check(lib().cgx_dist_set_graph(self._h, 1 if on else 0), "dist_set_graph")

    def debug_refuse_capture(self, mode):
        """Test hook (cgx_dist_debug_refuse_capture): refuse this rank's
        captures 1 before / 2 after the RCCL calls are recorded (eager when
        every rank is refused at the same point, CGX_ECOMM and an unusable
        communicator on a mix); 3 as 2 with the peers taken to have captured
        (the mix on one rank); 0 off."""
        check(lib().cgx_dist_debug_refuse_capture(self._h, int(mode)), "dist_debug_refuse_capture")

    def set_march(self, steps):
        """CGX_ALG_SR as one k_sr1_dia_m step per iteration on the in-place
        numbering (cgx_dist_set_march): -1 auto, 0 off (two-launch fused SR),
        > 0 interior steps per workgroup."""
        check(lib().cgx_dist_set_march(self._h, int(steps)), "dist_set_march")

    def set_sr_chain(self, rows=0):
        """Chain width (rows) of the ranks' one-launch SR march
        (cgx_dist_set_sr_chain): 0 auto, > 0 that width."""
        check(lib().cgx_dist_set_sr_chain(self._h, int(rows)), "dist_set_sr_chain")

    def set_fused(self, mode):
        """The fused HS step on all ranks or none: "auto", True, False."""
        check(lib().cgx_dist_set_fused(self._h, fuse_mode(mode)), "dist_set_fused")

    def run(self, maxit, tol=0.0):
        it = ctypes.c_int(0)
        check(lib().cgx_dist_run(self._h, maxit, tol, ctypes.byref(it)), "dist_run")
        return it.value

    def x(self):
        out = np.empty(self.n_loc, np.float64)
        check(lib().cgx_dist_get_x(self._h, _p(out, _f64p)), "dist_get_x")
        return out

    def history(self, cap):
        out = np.zeros(cap, np.float64)
        m = check(lib().cgx_dist_get_history(self._h, _p(out, _f64p), cap), "dist_history")
        return out[:m]

    def bench_prepare(self, warmup):
        check(lib().cgx_dist_bench_prepare(self._h, warmup), "dist_bench_prepare")

    def bench_run(self, iters, spmv_events=False, graph=True):
        """Returns (device ms for all iters, average SpMV ms or -1).
        SpMV events run the iterations eagerly."""
        ms, sp = ctypes.c_double(0), ctypes.c_double(0)
        flags = (CGX_BENCH_SPMV_EVENTS if spmv_events else 0) | (CGX_BENCH_GRAPH if graph else 0)
        check(lib().cgx_dist_bench_run(self._h, iters, flags,
                                       ctypes.byref(ms), ctypes.byref(sp)), "dist_bench_run")
        return ms.value, sp.value

    def bench_phases(self):
        """Per-phase ms per iteration of the last bench_run(spmv_events=True)
        (cgx_dist_bench_phases): first launch, halo-wait gap, second launch,
        tail (sums, all-reduce, updates, pack), period; None before one."""
        ms = np.zeros(5, np.float64)
        it = ctypes.c_int(0)
        check(lib().cgx_dist_bench_phases(self._h, _p(ms, _f64p), ctypes.byref(it)),
              "dist_bench_phases")
        if it.value <= 0:
            return None
        keys = ("first_launch", "halo_wait_gap", "second_launch", "tail", "period")
        return dict({k: float(v) for k, v in zip(keys, ms)}, iters=it.value)

    def info(self):
        st = CgxDistStats()
        check(lib().cgx_dist_info(self._h, ctypes.byref(st)), "dist_info")
        d = {k: getattr(st, k) for k, _ in CgxDistStats._fields_}
        d["layout_name"] = LAYOUT_NAMES.get(d["layout"], "?")
        return d
