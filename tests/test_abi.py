"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports
every function include/*.h declares, its host generators are exact, and its
compute entry points fail loudly (no CPU fallback) when no GPU is present."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import cgx
import helpers as H
from conftest import gpu_available

REPO = Path(__file__).resolve().parent.parent


def declared_functions():
    names = set()
    for h in (REPO / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = re.sub(r"(?m)^\s*#.*$", "", text)
        for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", text):
            name = m.group(1)
            if name not in {"if", "while", "for", "sizeof", "return"}:
                names.add(name)
    return sorted(names)


def test_headers_declare_reference_api():
    names = set(declared_functions())
    # mv_ops.h:25-42 -- the 11 reference prototypes -- and cg.c:24 conj_grad
    ref = {"new_mv_struct", "new_mv_struct_with_size", "free_mv_struct",
           "mv_deep_copy", "print_sparse", "mat_get_row", "dot_product",
           "sv_mult", "mv_mult", "vec_add", "vec_sub", "conj_grad", "solve"}
    assert ref <= names


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports(name):
    L = ctypes.CDLL(str(cgx.LIB_PATH))
    assert hasattr(L, name), name


def test_struct_layout():
    # mv_ops.h:17-23, LP64: offsets 0/4/8/16/24, sizeof 32
    assert ctypes.sizeof(cgx.MvSparse) == 32
    assert [getattr(cgx.MvSparse, f).offset for f in
            ("size", "nnz", "values", "col_indices", "row_ptr")] == [0, 4, 8, 16, 24]


def test_host_struct_lifecycle():
    L = cgx.lib()
    v = L.new_mv_struct_with_size(7)
    assert v.contents.size == 7 and v.contents.nnz == 7
    assert not v.contents.col_indices and not v.contents.row_ptr
    assert np.all(cgx.mv_values(v) == 0.0)
    v.contents.values[3] = 2.5
    c = L.mv_deep_copy(v)
    assert cgx.mv_values(c)[3] == 2.5 and c.contents.values[3] == 2.5
    assert ctypes.addressof(c.contents.values.contents) != ctypes.addressof(v.contents.values.contents)
    L.cgx_free_mv_deep(c)
    L.cgx_free_mv_deep(v)
    assert not L.mv_deep_copy(None)


def test_mat_get_row_host():
    g = H.load_golden("lap2d_32")
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    row = np.empty(g["n"])
    for r in (0, 1, 33, g["n"] - 1):
        assert cgx.lib().mat_get_row(A.ptr, r, row.ctypes.data_as(cgx._f64p)) == 0
        dense = np.zeros(g["n"])
        a, b = g["row_ptr"][r], g["row_ptr"][r + 1]
        dense[g["col"][a:b]] = g["val"][a:b]
        assert np.array_equal(row, dense)
    assert cgx.lib().mat_get_row(None, 0, row.ctypes.data_as(cgx._f64p)) == -1


def test_reference_error_convention_without_gpu_work():
    """NULL / size-mismatch checks come before any device work
    (mv_ops.c:122-126, :138-139, :166-170, :207-211, :236-240)."""
    L = cgx.lib()
    a = cgx.Mv(np.ones(4))
    b = cgx.Mv(np.ones(5))
    out = cgx._MVP()
    assert L.dot_product(a.ptr, None) == -1.0
    assert L.dot_product(a.ptr, b.ptr) == -1.0
    assert L.vec_add(a.ptr, b.ptr, ctypes.byref(out)) == -1
    assert L.vec_sub(None, b.ptr, ctypes.byref(out)) == -1
    assert L.sv_mult(2.0, None, ctypes.byref(out)) == -1
    assert L.mv_mult(None, b.ptr, ctypes.byref(out)) == -1
    assert not out


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_no_cpu_fallback():
    """Without a GPU every compute entry point fails loudly (CGX_ENODEV)."""
    L = cgx.lib()
    h = cgx._vp()
    assert L.cgx_solver_create(0, ctypes.byref(h)) == cgx.CGX_ENODEV
    assert "device" in cgx.last_error()
    g = H.load_golden("kat_tridiag10")
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    out = cgx._MVP()
    assert L.conj_grad(3, A.ptr, b.ptr, ctypes.byref(out)) == cgx.CGX_ENODEV
    assert not out
    assert L.dot_product(b.ptr, b.ptr) == -1.0
    gbs = ctypes.c_double(0.0)
    assert L.cgx_stream_bench(0, 0, 1 << 20, 1, ctypes.byref(gbs)) == cgx.CGX_ENODEV


@pytest.mark.parametrize("shape", [(1, 1), (5, 3), (32, 32), (17, 9)])
def test_gen_laplacian2d_matches_fixture_generator(shape):
    rp, col, val = cgx.laplacian2d(*shape)
    rp2, col2, val2 = H.laplacian2d(*shape)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2)
    assert H.same_bits_or_both_nan(val, val2)


@pytest.mark.parametrize("shape", [(1, 1, 1), (4, 3, 2), (12, 12, 12), (7, 5, 9)])
def test_gen_laplacian3d_matches_fixture_generator(shape):
    rp, col, val = cgx.laplacian3d(*shape)
    rp2, col2, val2 = H.laplacian3d(*shape)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2)
    assert H.same_bits_or_both_nan(val, val2)
    assert cgx.is_chained(rp, col)


def test_gen_row_ranges_concatenate():
    """Row-range generation (one slab per rank) is bit-exact with the whole."""
    nx, ny, nz = 9, 7, 8
    full = cgx.laplacian3d(nx, ny, nz)
    n = nx * ny * nz
    for G in (2, 3, 4, 8):
        cols, vals, nnz0 = [], [], 0
        for g in range(G):
            rb, re_ = n * g // G, n * (g + 1) // G
            rp, c, v = cgx.laplacian3d(nx, ny, nz, rb, re_)
            assert rp[0] == 0
            assert np.array_equal(rp + full[0][rb], full[0][rb:re_ + 1])
            cols.append(c)
            vals.append(v)
        assert np.array_equal(np.concatenate(cols), full[1])
        assert np.array_equal(np.concatenate(vals), full[2])


def test_gen_random_spd_properties():
    n = 3000
    rp, col, val = cgx.random_spd(n, 8, 42)
    assert cgx.is_chained(rp, col)
    A = np.zeros((n, n))
    for i in range(n):
        A[i, col[rp[i]:rp[i + 1]]] = val[rp[i]:rp[i + 1]]
    assert np.array_equal(A, A.T)
    off = np.abs(A).sum(axis=1) - np.abs(np.diag(A))
    assert np.all(np.diag(A) >= off + 1.0 - 1e-12)
    assert np.all(A[~np.eye(n, dtype=bool)] <= 0.0)
    # row ranges and the fp32 copy agree with the whole
    rp2, col2, v2 = cgx.random_spd(n, 8, 42, 1000, 2000)
    assert np.array_equal(col2, col[rp[1000]:rp[2000]])
    assert np.array_equal(v2, val[rp[1000]:rp[2000]])
    _, _, v32 = cgx.random_spd(n, 8, 42, f32=True)
    assert np.array_equal(v32, val.astype(np.float32))
    # different seed -> different matrix
    _, col3, _ = cgx.random_spd(n, 8, 43)
    assert len(col3) != len(col) or not np.array_equal(col3, col)


@pytest.mark.parametrize("name", H.golden_names())
def test_chained_flag_matches_fixture(name):
    g = H.load_golden(name)
    assert cgx.is_chained(g["row_ptr"], g["col"]) == g["chained"]


@pytest.mark.parametrize("dim,shape", [(3, (1, 1, 1)), (3, (4, 3, 2)), (3, (12, 12, 12)),
                                       (3, (7, 5, 9)), (3, (1, 6, 4)), (3, (5, 1, 3)),
                                       (2, (1, 1, 1)), (2, (5, 3, 1)), (2, (32, 32, 1)),
                                       (2, (1, 9, 1)), (2, (17, 9, 1))])
def test_laplacian_row_ptr_closed_form(dim, shape):
    """The closed-form row_ptr the on-device generator and the stencil use
    equals the host generator's, for whole grids and for row ranges."""
    nx, ny, nz = shape
    n = nx * ny * nz
    if dim == 3:
        rp, _, _ = cgx.laplacian3d(nx, ny, nz)
    else:
        rp, _, _ = cgx.laplacian2d(nx, ny)
    assert np.array_equal(cgx.laplacian_row_ptr(dim, nx, ny, nz), rp)
    for rb, re_ in [(0, n), (n // 3, n), (n // 5, (4 * n) // 5), (n, n)]:
        sub = cgx.laplacian_row_ptr(dim, nx, ny, nz, rb, re_)
        assert np.array_equal(sub, rp[rb:re_ + 1] - rp[rb])


def test_laplacian_row_ptr_c4_total():
    """C4 (400^3): the closed form's nnz is SURVEY.md's 447,040,000."""
    nnz = cgx.lib().cgx_laplacian_row_ptr(3, 400, 400, 400, 0, 64_000_000, None)
    assert nnz == 447_040_000
    assert cgx.lib().cgx_laplacian_row_ptr(3, 216, 216, 216, 0, 216 ** 3, None) == 70_263_936


def test_null_handles_fail_cleanly():
    """Every handle-taking entry point rejects a NULL handle (and NULL
    out-pointers) with an error code instead of crashing -- the drop-in
    contract for C callers (mv_ops.c's -1 convention, CGX_EINVAL here)."""
    L = cgx.lib()
    vp = ctypes.c_void_p
    i, d = ctypes.c_int(0), ctypes.c_double(0.0)
    null = None
    assert L.cgx_solver_set_mode(null, 0, 0) < 0
    assert L.cgx_solver_set_matrix(null, 1, 1, null, null, null) < 0
    assert L.cgx_solver_set_matrix_f32(null, 1, 1, null, null, null) < 0
    assert L.cgx_solver_set_rhs(null, null) < 0
    assert L.cgx_solver_set_rhs_f32(null, null) < 0
    assert L.cgx_solver_run(null, 5, 0.0, ctypes.byref(i)) < 0
    assert L.cgx_solver_get_x(null, null) < 0
    assert L.cgx_solver_get_x_f32(null, null) < 0
    assert L.cgx_solver_get_history(null, null, 4) < 0
    assert L.cgx_solver_spmv(null, null, null) < 0
    assert L.cgx_solver_spmv_f32(null, null, null) < 0
    assert L.cgx_solver_info(null, null) < 0
    assert L.cgx_solver_bench_prepare(null, 1) < 0
    assert L.cgx_solver_gen_laplacian(null, 3, 4, 4, 4) < 0
    assert L.cgx_solver_set_stencil(null, 3, 4, 4, 4) < 0
    assert L.cgx_solver_get_matrix(null, null, null, null) < 0
    assert L.cgx_dist_set_rhs(null, null) < 0
    assert L.cgx_dist_run(null, 5, 0.0, ctypes.byref(i)) < 0
    assert L.cgx_dist_get_x(null, null) < 0
    assert L.cgx_dist_get_history(null, null, 4) < 0
    assert L.cgx_dist_bench_prepare(null, 1) < 0
    assert L.cgx_dist_info(null, null) < 0
    assert L.cgx_dist_set_matrix(null, 4, 1, 1, null, null, null) < 0
    assert L.cgx_solver_bench_run(null, 1, 0, ctypes.byref(d), ctypes.byref(d)) < 0
    assert L.cgx_dist_bench_run(null, 1, 0, ctypes.byref(d), ctypes.byref(d)) < 0
    assert L.cgx_part_info(null, null, null, null, null) < 0
    assert L.cgx_part_ghosts(null, null) < 0
    assert L.cgx_part_recv_counts(null, null) < 0
    assert L.cgx_part_send_counts(null, null) < 0
    assert L.cgx_part_send_local(null, null) < 0
    assert L.cgx_part_local_cols(null, null) < 0
    assert L.cgx_solver_create(0, null) < 0
    assert L.cgx_dist_create(0, 1, 0, null, null) < 0
    assert L.cgx_dist_create_local(0, 1, null) < 0
    assert L.cgx_stream_bench(0, 0, 1 << 20, 1, null) < 0
    # destroy functions accept NULL like free()
    L.cgx_solver_destroy(null)
    L.cgx_dist_destroy(null)
    L.cgx_part_destroy(null)
    L.cgx_free_mv_deep(null)
    assert d.value == 0.0 and vp is not None


def test_headers_match_the_library():
    """The public headers are the drop-in contract: no
    configuration by environment variable (the library reads none) and no
    layout name the library does not have ("VI" was renamed DIA)."""
    for h in (REPO / "include").glob("*.h"):
        text = h.read_text()
        assert "environment" not in text.lower(), h.name
        assert not re.search(r"(?<!DIA-)\bVI\b", text), h.name


def test_gen_varcoef3d_properties():
    """cgx_gen_varcoef3d: the 7-point Laplacian's pattern, symmetric values,
    strictly diagonally dominant (SPD), all off-diagonal values distinct,
    row ranges concatenate to the whole."""
    nx, ny, nz = 7, 6, 5
    rp, col, val = cgx.varcoef3d(nx, ny, nz, seed=3)
    rpl, coll, _ = cgx.laplacian3d(nx, ny, nz)
    assert np.array_equal(rp, rpl) and np.array_equal(col, coll)
    n = nx * ny * nz
    A = np.zeros((n, n))
    for i in range(n):
        A[i, col[rp[i]:rp[i + 1]]] = val[rp[i]:rp[i + 1]]
    assert np.array_equal(A, A.T)
    off = np.abs(A).sum(axis=1) - np.abs(np.diag(A))
    assert np.all(np.diag(A) > off)
    offv = A[np.triu(np.ones((n, n), bool), 1) & (A != 0)]
    assert np.all((offv < -0.5) & (offv >= -1.5)) and len(np.unique(offv)) == len(offv)
    parts = [cgx.varcoef3d(nx, ny, nz, 3, n * g // 3, n * (g + 1) // 3) for g in range(3)]
    assert np.array_equal(np.concatenate([p[2] for p in parts]), val)
