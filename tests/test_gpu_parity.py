"""GPU parity: the HIP path (called through the C ABI of libcgx.so) against
the golden vectors of the compiled reference and against the pinned oracle.

Bars (stated here, checked below):
  * SpMV (mv_mult), sv_mult, vec_add, vec_sub: bit-exact.
  * conj_grad / solve in CGX_MODE_EXACT: bit-exact x at every golden max_iter
    (including the all-NaN breakdown of the n = 10 KAT at max_iter 5).
  * default (parallel-reduction) mode: ||x - x_ref||_2 <= FAST_RTOL ||x_ref||_2
    with FAST_RTOL = 1e-12 (the only difference is dot-product summation
    order; simulated worst case on the fixtures is ~1e-14).
  * full-size configs: size-independent properties (bit-exact SpMV against the
    oracle, true relative residual ||b - A x|| / ||b|| <= tol after solve).
"""
import ctypes
import os

import numpy as np
import pytest

import cgx
import helpers as H

pytestmark = pytest.mark.gpu

FAST_RTOL = 1e-12
NAMES = H.golden_names()
CHAINED = [n for n in NAMES if H.load_golden(n)["chained"]]


@pytest.fixture(scope="module")
def solver():
    s = cgx.Solver(0)
    yield s
    s.close()


@pytest.fixture
def exact_env():
    old = os.environ.get("CGX_MODE")
    os.environ["CGX_MODE"] = "exact"
    yield
    if old is None:
        os.environ.pop("CGX_MODE", None)
    else:
        os.environ["CGX_MODE"] = old


def rel(x, ref):
    d = np.linalg.norm(ref)
    return np.linalg.norm(x - ref) / (d if d > 0 else 1.0)


def test_device_visible():
    assert cgx.lib().cgx_device_count() > 0


# ------------------------------------------------------------------ SpMV

@pytest.mark.parametrize("name", CHAINED)
def test_spmv_bit_exact_vs_reference(solver, name):
    g = H.load_golden(name)
    solver.set_mode(cgx.CGX_MODE_FAST)
    solver.set_matrix(g["row_ptr"], g["col"], g["val"])
    y = solver.spmv(g["b"])
    assert H.same_bits_or_both_nan(y, g["ops"]["mv_mult"])


@pytest.mark.parametrize("bs", ["64", "256", "512", "dma", "dma8", "dma32", "dmaw8", "dmaxcd", "dma456", "dma328", "dma512", "dmalast", "eng", "eng0", "eng1", "eng3", "eng4", "eng5", "eng6", "eng7", "notg", "pipe", "pipe1", "pipe63"])
@pytest.mark.parametrize("vec", ["1", "2", "4"])
def test_spmv_variants_bit_exact(vec, bs, monkeypatch):
    """Every SpMV variant (wave / workgroup row blocks, load widths, LDS-DMA,
    pipelined persistent waves with 1/8/63 blocks each) keeps the sequential
    per-row order, fp64 and fp32, including long rows."""
    monkeypatch.setenv("CGX_SPMV_VEC", vec)
    monkeypatch.setenv("CGX_SPMV_DMA", "0")  # register-staged kernels unless named
    if bs in ("dma", "dma8", "dma32", "dmaw8", "dmaxcd", "dma456", "dma328", "dma512",
              "dmalast"):
        monkeypatch.setenv("CGX_SPMV_DMA", {"dma": "1", "dma8": "8", "dma32": "4", "dmaw8": "1",
                                            "dmaxcd": "1", "dma456": "1", "dma328": "1",
                                            "dma512": "1", "dmalast": "1"}[bs])
        if bs == "dmalast":
            monkeypatch.setenv("CGX_SPMV_EPI_LAST", "1")
        if bs in ("dma456", "dma328", "dma512"):
            monkeypatch.setenv("CGX_SPMV_CAPW", bs[3:])
        if bs == "dmaw8":
            monkeypatch.setenv("CGX_SPMV_WPB", "8")
        if bs == "dmaxcd":
            monkeypatch.setenv("CGX_SPMV_XCD", "1")
    elif bs.startswith("pipe"):
        monkeypatch.setenv("CGX_SPMV_DMA", "2")
        if bs != "pipe":
            monkeypatch.setenv("CGX_SPMV_RBW", bs[4:])
    elif bs.startswith("eng"):
        monkeypatch.setenv("CGX_SPMV_DMA", "5")
        if bs != "eng":
            monkeypatch.setenv("CGX_ENG_SHAPE", bs[3:])
    elif bs == "notg":
        monkeypatch.setenv("CGX_SPMV_TG", "0")
    else:
        monkeypatch.setenv("CGX_SPMV_BS", bs)
    rp, col, val, b = H.random_spd(4000, 9, seed=3)
    g = H.load_golden("dense128")
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert H.same_bits_or_both_nan(s.spmv(b), H.o_spmv(rp, col, val, b))
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        assert H.same_bits_or_both_nan(s.spmv(g["b"]), g["ops"]["mv_mult"])
        rp32, col32, v32 = cgx.random_spd(5000, 40, 9, f32=True)
        x32 = np.random.default_rng(2).standard_normal(5000).astype(np.float32)
        s.set_matrix(rp32, col32, v32)
        assert np.array_equal(s.spmv(x32).view(np.uint32),
                              H.o_spmv_f32(rp32, col32, v32, x32).view(np.uint32))
        # a CG run through the fused-epilogue path
        g = H.load_golden("lap3d_12")
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        s.run(20)
        x_ref, _ = H.o_conj_grad(20, g["row_ptr"], g["col"], g["val"], g["b"])
        assert rel(s.x(), x_ref) <= FAST_RTOL


@pytest.mark.parametrize("bs", ["64", "256", "dma", "dma8", "dma32", "pipe", "eng", "eng4"])
def test_spmv_long_rows_variants(bs, monkeypatch):
    monkeypatch.setenv("CGX_SPMV_DMA", "0")
    if bs in ("dma", "dma8", "dma32"):
        monkeypatch.setenv("CGX_SPMV_DMA", {"dma": "1", "dma8": "8", "dma32": "4"}[bs])
    elif bs == "pipe":
        monkeypatch.setenv("CGX_SPMV_DMA", "2")
    elif bs.startswith("eng"):
        monkeypatch.setenv("CGX_SPMV_DMA", "5")
        if bs != "eng":
            monkeypatch.setenv("CGX_ENG_SHAPE", bs[3:])
    else:
        monkeypatch.setenv("CGX_SPMV_BS", bs)
    n = 3000
    rng = np.random.default_rng(8)
    rows = [np.arange(n) if i in (0, 7, n - 1) else
            np.unique(np.concatenate([[max(i - 1, 0), i, min(i + 1, n - 1)], rng.integers(0, n, 3)]))
            for i in range(n)]
    rp = np.zeros(n + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.standard_normal(len(col))
    x = rng.standard_normal(n)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


def test_spmv_long_rows_bit_exact(solver):
    """Rows longer than one LDS row block (2048 products) take the chunked
    path; row sums must still be sequential."""
    n = 6000
    rows = []
    rng = np.random.default_rng(5)
    for i in range(n):
        if i in (0, 1, 2500, n - 1):
            cols = np.arange(n)  # dense rows
        else:
            cols = np.unique(np.concatenate([[max(i - 1, 0), i, min(i + 1, n - 1)],
                                             rng.integers(0, n, 4)]))
        rows.append(cols)
    rp = np.zeros(n + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.standard_normal(len(col))
    x = rng.standard_normal(n)
    solver.set_matrix(rp, col, val)
    assert H.same_bits_or_both_nan(solver.spmv(x), H.o_spmv(rp, col, val, x))


def test_spmv_empty_rows_and_tiny(solver):
    rp = np.array([0, 0, 2, 2, 3], np.int32)
    col = np.array([0, 3, 1], np.int32)
    val = np.array([2.0, -1.0, 5.0])
    x = np.array([1.0, 2.0, 3.0, 4.0])
    solver.set_matrix(rp, col, val)
    assert H.same_bits_or_both_nan(solver.spmv(x), H.o_spmv(rp, col, val, x))


def test_spmv_f32_bit_exact(solver):
    rp, col, val = cgx.random_spd(20000, 16, 11, f32=True)
    x = np.random.default_rng(1).standard_normal(20000).astype(np.float32)
    solver.set_matrix(rp, col, val)
    y = solver.spmv(x)
    assert np.array_equal(y.view(np.uint32), H.o_spmv_f32(rp, col, val, x).view(np.uint32))


@pytest.mark.parametrize("dma", ["0", "1", "2", "4", "5", "8", "1x", "1w", "1c", "1r0", "1b4", "1w8", "1v0", "1v2", "1v4"])
def test_spmv_c3_full_size_bit_exact(dma, monkeypatch):
    """BASELINE config C3 (3-D 7-pt 216^3, 10,077,696 rows): one SpMV,
    bit-exact against the oracle at full size (default and pipelined kernels)."""
    monkeypatch.setenv("CGX_SPMV_DMA", dma[0])
    if dma.endswith("c"):
        monkeypatch.setenv("CGX_LAYOUT", "csr")
    if dma.endswith("r0"):
        monkeypatch.setenv("CGX_DC_RLEN", "0")
    if dma.endswith("b4"):
        monkeypatch.setenv("CGX_DC_BITS", "4")
    if dma.endswith("v0"):
        monkeypatch.setenv("CGX_DC_VALS", "0")
    if dma.endswith("v2") or dma.endswith("v4"):
        monkeypatch.setenv("CGX_VI_BPW", dma[-1])
    if dma.endswith("w8"):
        monkeypatch.setenv("CGX_SPMV_WPB", "8")
    if dma.endswith("x"):
        monkeypatch.setenv("CGX_SPMV_XCD", "1")
    if dma.endswith("w"):
        monkeypatch.setenv("CGX_SPMV_CAPW", "456")
    rp, col, val = cgx.laplacian3d(216, 216, 216)
    x = np.random.default_rng(2).standard_normal(len(rp) - 1)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        # dictionary-coded columns on the default kernel (7 offsets), CSR otherwise
        assert s.info()["n_dict"] == (7 if dma in ("1", "1x", "1r0", "1b4", "1w8", "1v0", "1v2", "1v4") else 0)
        assert s.info()["dict_vals"] == (1 if dma in ("1", "1x", "1b4", "1v2", "1v4") else 0)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


def banded_spd(n, offsets, seed, f32=False):
    """Symmetric banded SPD matrix with the given positive column offsets (and
    their negatives), random values, diagonally dominant; CSR, rows ascending."""
    rng = np.random.default_rng(seed)
    offs = sorted(set([-o for o in offsets] + [0] + list(offsets)))
    rows, cols = [], []
    for o in offs:
        r = np.arange(max(0, -o), min(n, n - o))
        rows.append(r)
        cols.append(r + o)
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    v = -rng.random(len(r))
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    upper = c > r
    vu = dict(zip(zip(r[upper].tolist(), c[upper].tolist()), v[upper].tolist()))
    for i in range(len(r)):
        if c[i] < r[i]:
            v[i] = vu[(int(c[i]), int(r[i]))]
    diag = np.zeros(n)
    np.add.at(diag, r[c != r], np.abs(v[c != r]))
    v[c == r] = diag[r[c == r]] + 1.0
    rp = np.zeros(n + 1, dtype=np.int32)
    np.add.at(rp, r + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    if f32:
        return rp, c.astype(np.int32), v.astype(np.float32)
    return rp, c.astype(np.int32), v


def expect_dict(rp, col, val, vi_ok=True):
    """(n_dict, dict_vals) the solver should pick for a CSR matrix: coded
    columns for <= 256 distinct col - row offsets; value-indexed pairs when
    also <= 64 distinct (offset, value bit pattern) pairs and every row has
    <= 255 entries (the byte row lengths the pair kernel needs)."""
    rp, col = np.asarray(rp), np.asarray(col)
    n = len(rp) - 1
    if len(col) == 0:
        return 0, 0
    off = col.astype(np.int64) - np.repeat(np.arange(n), np.diff(rp))
    noff = len(np.unique(off))
    if noff > 256:
        return 0, 0
    bits = np.asarray(val).view(np.uint64 if np.asarray(val).dtype == np.float64 else np.uint32)
    npair = np.unique(np.stack([off, bits.astype(np.int64)]), axis=1).shape[1]
    if vi_ok and npair <= 64 and np.diff(rp).max() <= 255:
        return npair, 1
    return noff, 0


@pytest.mark.parametrize("bits", ["4", "8"])
@pytest.mark.parametrize("rlen", ["1", "0"])
@pytest.mark.parametrize("capw", ["", "328", "456"])
def test_dictionary_coded_columns_bit_exact(capw, rlen, bits, monkeypatch):
    """CSR-DC (k_spmv_dc): selected exactly when the matrix has <= 256
    distinct column offsets col - row, and bit-identical to the oracle's
    sequential row sums (fp64 and fp32, 64- and 256-entry dictionaries,
    adaptive 328/512 windows; 456 keeps plain CSR; row bounds from byte row
    lengths or from row_ptr; nibble codes for <= 16 offsets or bytes)."""
    monkeypatch.setenv("CGX_DC_BITS", bits)
    monkeypatch.setenv("CGX_DC_RLEN", rlen)
    if capw:
        monkeypatch.setenv("CGX_SPMV_CAPW", capw)
    rng = np.random.default_rng(5)
    cases = [("lap3d_12", None), ("lap2d_32", None), ("dense128", None)]
    with cgx.Solver(0) as s:
        for name, _ in cases:
            g = H.load_golden(name)
            s.set_matrix(g["row_ptr"], g["col"], g["val"])
            nd, vi = s.info()["n_dict"], s.info()["dict_vals"]
            want, want_vi = expect_dict(g["row_ptr"], g["col"], g["val"],
                                        vi_ok=rlen == "1")
            assert (nd, vi) == ((0, 0) if capw == "456" else (want, want_vi)), name
            x = rng.standard_normal(len(g["row_ptr"]) - 1)
            assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(g["row_ptr"], g["col"], g["val"], x))
            assert H.same_bits_or_both_nan(s.spmv(g["b"]), g["ops"]["mv_mult"])
        # 127 positive offsets -> 255 distinct: the 256-entry dictionary
        offs = sorted(rng.choice(np.arange(1, 3000), 127, replace=False).tolist())
        rp, col, val = banded_spd(5000, offs, 7)
        s.set_matrix(rp, col, val)
        assert s.info()["n_dict"] == (0 if capw == "456" else 255)
        x = rng.standard_normal(5000)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        # 257 distinct offsets: stays plain CSR, still bit-exact
        rp, col, val = banded_spd(3000, list(range(1, 129)), 8)
        s.set_matrix(rp, col, val)
        assert s.info()["n_dict"] == 0
        x = rng.standard_normal(3000)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        # 256 distinct offsets, one row of 256 entries (> 255: row_ptr bounds),
        # empty rows, non-symmetric
        n = 700
        rows = [list(range(0, 256))] + [[] if r % 5 == 0 else [r] for r in range(1, n)]
        rp = np.zeros(n + 1, dtype=np.int32)
        rp[1:] = np.cumsum([len(c) for c in rows])
        col = np.array([c for cs in rows for c in cs], dtype=np.int32)
        val = rng.standard_normal(len(col))
        s.set_matrix(rp, col, val)
        assert s.info()["n_dict"] == (0 if capw == "456" else 256)
        x = rng.standard_normal(n)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        # fp32 banded
        rp, col, v32 = banded_spd(6000, [1, 77, 500], 9, f32=True)
        s.set_matrix(rp, col, v32)
        assert s.info()["n_dict"] == 7  # fp32 windows are not resized: CGX_SPMV_CAPW is fp64-only
        x32 = rng.standard_normal(6000).astype(np.float32)
        assert np.array_equal(s.spmv(x32).view(np.uint32),
                              H.o_spmv_f32(rp, col, v32, x32).view(np.uint32))


@pytest.mark.parametrize("seed", range(8))
def test_dictionary_coded_random_patterns(seed):
    """Randomised sparsity patterns for the coded-column encoder and kernel:
    n not a multiple of 64, empty and ragged rows (0-40 entries), 1-256
    distinct offsets drawn from a random band, unsorted offset draws (the
    CSR columns are sorted per row); the SpMV is bit-identical to the oracle,
    and a pattern with 257 offsets stays plain CSR."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(1, 9000))
    nd = int(rng.integers(1, 258))
    offs = rng.choice(np.arange(-4000, 4001), size=nd, replace=False)
    rows = []
    for r in range(n):
        k = int(rng.integers(0, 41)) if rng.random() > 0.1 else 0
        cand = r + offs
        cand = cand[(cand >= 0) & (cand < n)]
        rows.append(np.sort(rng.choice(cand, size=min(k, len(cand)), replace=False)))
    rp = np.zeros(n + 1, dtype=np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32) if rp[-1] else np.zeros(0, np.int32)
    # odd seeds: values from a small set (value-indexed pairs when <= 64
    # (offset, value) pairs), even seeds: all distinct
    if seed % 2:
        val = rng.choice(np.array([-1.0, 2.5, -0.0, 0.0, 1e-300, -3.25]), size=len(col))
    else:
        val = rng.standard_normal(len(col))
    x = rng.standard_normal(n)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert (s.info()["n_dict"], s.info()["dict_vals"]) == expect_dict(rp, col, val)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


@pytest.mark.parametrize("bits,bpw", [("8", "1"), ("8", "2"), ("8", "4"), ("4", "1")])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_value_indexed_pairs_bit_exact(bits, bpw, dtype, monkeypatch):
    """CSR-VI: (offset, value) pair codes -- the SpMV reads no val stream.
    Selected for constant-coefficient stencils and small value sets, off with
    CGX_DC_VALS=0 or > 64 pairs; y bit-identical to the oracle in every case
    (signed zeros and a denormal-range value keep their bit patterns; nibble
    codes for <= 16 pairs)."""
    monkeypatch.setenv("CGX_DC_BITS", bits)
    monkeypatch.setenv("CGX_VI_BPW", bpw)
    rng = np.random.default_rng(77)
    with cgx.Solver(0) as s:
        for name in ("lap3d_12", "lap2d_32"):
            g = H.load_golden(name)
            v = g["val"].astype(np.float32) if dtype == "f32" else g["val"]
            s.set_matrix(g["row_ptr"], g["col"], v)
            assert (s.info()["n_dict"], s.info()["dict_vals"]) == expect_dict(g["row_ptr"], g["col"], v)
            assert s.info()["dict_vals"] == 1
            x = rng.standard_normal(len(g["row_ptr"]) - 1)
            if dtype == "f32":
                x = x.astype(np.float32)
                assert np.array_equal(s.spmv(x).view(np.uint32),
                                      H.o_spmv_f32(g["row_ptr"], g["col"], v, x).view(np.uint32))
            else:
                assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(g["row_ptr"], g["col"], v, x))
        # a banded matrix whose values per offset take a few values: 5 offsets
        # x 12 values = 60 pairs (VI), then 65 pairs (offset codes only)
        for nv, want_vi in ((12, 1), (13, 0)):
            n = 5000
            rp, col, _ = banded_spd(n, [1, 300], 3)
            vals = np.linspace(-2, 2, nv)
            off = col - np.repeat(np.arange(n), np.diff(rp))
            val = vals[(np.arange(len(col)) * 7 + off) % nv]
            if dtype == "f32":
                val = val.astype(np.float32)
            s.set_matrix(rp, col, val)
            nd, vi = s.info()["n_dict"], s.info()["dict_vals"]
            assert (nd, vi) == expect_dict(rp, col, val)
            assert vi == want_vi
            x = rng.standard_normal(n)
            if dtype == "f32":
                x = x.astype(np.float32)
                assert np.array_equal(s.spmv(x).view(np.uint32),
                                      H.o_spmv_f32(rp, col, val, x).view(np.uint32))
            else:
                assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
    monkeypatch.setenv("CGX_DC_VALS", "0")
    g = H.load_golden("lap3d_12")
    with cgx.Solver(0) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        assert (s.info()["n_dict"], s.info()["dict_vals"]) == (7, 0)


def test_dictionary_coded_cg_identical_to_csr(monkeypatch):
    """The coded layout changes only how columns are stored: a CG run is
    bit-identical to the plain-CSR run (x and the r.r history)."""
    g = H.load_golden("lap3d_12")
    out = {}
    for layout in ("csr", "auto"):
        if layout == "csr":
            monkeypatch.setenv("CGX_LAYOUT", "csr")
        else:
            monkeypatch.delenv("CGX_LAYOUT", raising=False)
        with cgx.Solver(0) as s:
            s.set_matrix(g["row_ptr"], g["col"], g["val"])
            assert (s.info()["n_dict"] > 0) == (layout == "auto")
            s.set_rhs(g["b"])
            s.run(40)
            out[layout] = (s.x(), s.history(41))
    assert H.same_bits_or_both_nan(out["csr"][0], out["auto"][0])
    assert H.same_bits_or_both_nan(out["csr"][1], out["auto"][1])


# -------------------------------------------------------- mv_ops.h op list

@pytest.mark.parametrize("name", NAMES)
def test_mv_ops_reference_op_list(name, exact_env):
    """test_mv_ops (cg.c:368-384) through the drop-in mv_ops.h ABI."""
    g = H.load_golden(name)
    L = cgx.lib()
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    out = cgx._MVP()
    assert L.mv_mult(A.ptr, b.ptr, ctypes.byref(out)) == 0
    y = cgx.mv_values(out)
    if g["chained"]:
        assert H.same_bits_or_both_nan(y, g["ops"]["mv_mult"])
    else:  # documented divergence: libcgx computes the correct CSR product
        assert H.same_bits_or_both_nan(y, H.o_spmv(g["row_ptr"], g["col"], g["val"], g["b"]))
    # out-parameter reuse: realloc + overwrite (mv_ops.c:148-152)
    assert L.sv_mult(4.0, b.ptr, ctypes.byref(out)) == 0
    assert H.same_bits_or_both_nan(cgx.mv_values(out), g["ops"]["sv_mult"])
    d = L.dot_product(b.ptr, b.ptr)
    assert H.same_bits_or_both_nan([d], g["ops"]["dot_product"])
    assert L.vec_add(b.ptr, b.ptr, ctypes.byref(out)) == 0
    assert H.same_bits_or_both_nan(cgx.mv_values(out), g["ops"]["vec_add"])
    assert L.vec_sub(b.ptr, b.ptr, ctypes.byref(out)) == 0
    assert H.same_bits_or_both_nan(cgx.mv_values(out), g["ops"]["vec_sub"])
    assert out.contents.size == g["n"] and out.contents.nnz == g["n"]
    L.cgx_free_mv_deep(out)


def test_vec_sub_in_place_alias():
    """cg.c:123 calls vec_sub(r, t, &r): the output aliases the input."""
    L = cgx.lib()
    r = L.new_mv_struct_with_size(1000)
    t = L.new_mv_struct_with_size(1000)
    rv = np.random.default_rng(0).standard_normal(1000)
    tv = np.random.default_rng(1).standard_normal(1000)
    for i in range(1000):
        r.contents.values[i] = rv[i]
        t.contents.values[i] = tv[i]
    rr = ctypes.pointer(r.contents)
    assert L.vec_sub(r, t, ctypes.byref(rr)) == 0
    assert H.same_bits_or_both_nan(cgx.mv_values(rr), rv - tv)
    L.cgx_free_mv_deep(rr)
    L.cgx_free_mv_deep(t)


def test_dot_product_fast_mode_close():
    os.environ.pop("CGX_MODE", None)
    a = cgx.Mv(np.random.default_rng(0).standard_normal(100003))
    b = cgx.Mv(np.random.default_rng(1).standard_normal(100003))
    d = cgx.lib().dot_product(a.ptr, b.ptr)
    ref = H.o_dot(a.values, b.values)
    assert abs(d - ref) <= 1e-12 * np.dot(np.abs(a.values), np.abs(b.values))


# -------------------------------------------------------------- conj_grad

@pytest.mark.parametrize("name", CHAINED)
def test_conj_grad_exact_mode_bit_exact(name, exact_env):
    g = H.load_golden(name)
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    for it, want in g["iters"].items():
        x = cgx.conj_grad(it, A, b)
        assert H.same_bits_or_both_nan(x, want), (name, it)


@pytest.mark.parametrize("name", CHAINED)
def test_conj_grad_fast_mode_within_tolerance(name):
    os.environ.pop("CGX_MODE", None)
    g = H.load_golden(name)
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    for it, want in g["iters"].items():
        x = cgx.conj_grad(it, A, b)
        if np.any(np.isnan(want)):
            assert np.all(np.isnan(x))  # breakdown 0/0 (cg.c:129) in any order
        else:
            assert rel(x, want) <= FAST_RTOL, (name, it, rel(x, want))


def test_kat_values_on_gpu():
    g = H.load_golden("kat_tridiag10")
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    assert list(cgx.conj_grad(4, A, b)) == [5, 9, 12, 14, 15, 15, 14, 12, 9, 5]
    assert np.all(np.isnan(cgx.conj_grad(5, A, b)))


def test_conj_grad_argument_errors():
    L = cgx.lib()
    g = H.load_golden("kat_tridiag10")
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(np.ones(9))
    out = cgx._MVP()
    assert L.conj_grad(3, A.ptr, b.ptr, ctypes.byref(out)) == cgx.CGX_EINVAL
    assert L.conj_grad(-1, A.ptr, cgx.Mv(g["b"]).ptr, ctypes.byref(out)) == cgx.CGX_EINVAL
    assert not out


@pytest.mark.parametrize("name", ["lap2d_32", "lap3d_12", "dense128", "rand_spd_2000"])
def test_solve_tolerance_matches_oracle(name, exact_env):
    """solve(tol) stops at the oracle's iteration and returns conj_grad(k)."""
    g = H.load_golden(name)
    A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
    b = cgx.Mv(g["b"])
    for tol in (1e-3, 1e-8, 1e-12):
        x_o, its_o, _ = H.o_solve(1000, tol, g["row_ptr"], g["col"], g["val"], g["b"])
        x, its = cgx.solve(A, b, tol, 1000)
        assert its == its_o
        assert H.same_bits_or_both_nan(x, x_o)


def test_solver_history_exact(solver):
    g = H.load_golden("lap3d_12")
    solver.set_mode(cgx.CGX_MODE_EXACT)
    solver.set_matrix(g["row_ptr"], g["col"], g["val"])
    solver.set_rhs(g["b"])
    its = solver.run(40)
    assert its == 41
    _, hist = H.o_conj_grad(40, g["row_ptr"], g["col"], g["val"], g["b"])
    assert H.same_bits_or_both_nan(solver.history(41), hist)
    solver.set_mode(cgx.CGX_MODE_FAST)


@pytest.mark.parametrize("graph", ["0", "1"])
def test_graph_and_eager_agree(graph, monkeypatch):
    monkeypatch.setenv("CGX_GRAPH", graph)
    g = H.load_golden("lap2d_32")
    with cgx.Solver(0) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        assert s.run(50) == 51
        x = s.x()
    x_ref, _ = H.o_conj_grad(50, g["row_ptr"], g["col"], g["val"], g["b"])
    assert rel(x, x_ref) <= FAST_RTOL


@pytest.mark.parametrize("name", ["lap2d_32", "lap3d_12", "rand_spd_2000", "dense128"])
def test_cg1_within_tolerance(name):
    g = H.load_golden(name)
    with cgx.Solver(0, alg=cgx.CGX_ALG_CG1) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        its = s.run(500, 1e-10)
        x = s.x()
    x_o, its_o, _ = H.o_solve(500, 1e-10, g["row_ptr"], g["col"], g["val"], g["b"], cg1=True)
    assert abs(its - its_o) <= 1
    assert rel(x, x_o) <= 1e-9


def test_fp32_solve_converges():
    rp, col, val = cgx.random_spd(50000, 16, 5, f32=True)
    b = np.random.default_rng(4).standard_normal(50000).astype(np.float32)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        its = s.run(200, 1e-5)
        x = s.x()
    r = b.astype(np.float64) - H.o_spmv(rp, col, val.astype(np.float64), x.astype(np.float64))
    assert its < 200
    assert np.linalg.norm(r) <= 2e-5 * np.linalg.norm(b)


def test_c3_solve_residual():
    """C3 at full size through the device-resident solver: the true relative
    residual after solve(tol = 1e-8) is below tol (size-independent check)."""
    rp, col, val = cgx.laplacian3d(216, 216, 216)
    n = len(rp) - 1
    b = np.ones(n)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        its = s.run(2000, 1e-8)
        x = s.x()
        hist = s.history(its)
    r = b - H.o_spmv(rp, col, val, x)
    assert np.linalg.norm(r) <= 1.5e-8 * np.linalg.norm(b)
    assert hist[-1] <= 1e-16 * n
    assert its < 2000


def test_empty_system():
    L = cgx.lib()
    A = cgx.Mv(np.zeros(0), np.zeros(0, np.int32), np.zeros(1, np.int32))
    b = cgx.Mv(np.zeros(0))
    out = cgx._MVP()
    assert L.conj_grad(3, A.ptr, b.ptr, ctypes.byref(out)) == 0
    assert out.contents.size == 0
    L.cgx_free_mv_deep(out)


@pytest.mark.parametrize("ticket", ["0", "1"])
@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("dma", ["0", "1"])
def test_reduction_paths_match_oracle_and_reproduce(ticket, fuse, dma, monkeypatch):
    """Finalize kernels vs the in-kernel ticket reduction (register-staged
    SpMV only), with and without the fused p-update, on both SpMV kernels:
    all within FAST_RTOL of the reference order, and each bit-reproducible
    run to run (deterministic reductions, no fp64 atomics)."""
    if ticket == "1" and dma == "1":
        pytest.skip("the LDS-DMA SpMV has no ticket epilogue (solver ignores CGX_TICKET)")
    monkeypatch.setenv("CGX_TICKET", ticket)
    monkeypatch.setenv("CGX_FUSE_XPAY", fuse)
    monkeypatch.setenv("CGX_SPMV_DMA", dma)
    rp, col, val, b = H.random_spd(30000, 9, seed=12)
    x_ref, _ = H.o_conj_grad(60, rp, col, val, b)
    xs, hs = [], []
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        for _ in range(2):
            s.set_rhs(b)
            assert s.run(60) == 61
            xs.append(s.x())
            hs.append(s.history(61))
        its = s.run(1000, 1e-9)
        x_tol = s.x()
    assert rel(xs[0], x_ref) <= FAST_RTOL
    assert H.same_bits_or_both_nan(xs[0], xs[1]) and H.same_bits_or_both_nan(hs[0], hs[1])
    _, its_o, _ = H.o_solve(1000, 1e-9, rp, col, val, b)
    assert abs(its - its_o) <= 1
    r = b - H.o_spmv(rp, col, val, x_tol)
    assert np.linalg.norm(r) <= 1.01e-9 * np.linalg.norm(b)


def test_ticket_large_grid_and_tiny(monkeypatch):
    """Ticket reduction across > kTicketGroup^2 workgroups (two full levels)
    and with a single workgroup."""
    monkeypatch.setenv("CGX_TICKET", "1")
    monkeypatch.setenv("CGX_SPMV_DMA", "0")
    rp, col, val = cgx.laplacian3d(160, 160, 160)   # 4.1 M rows, 64 K SpMV workgroups
    b = np.random.default_rng(3).standard_normal(len(rp) - 1)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        s.run(5)
        x = s.x()
    x_ref, _ = H.o_conj_grad(5, rp, col, val, b)
    assert rel(x, x_ref) <= FAST_RTOL
    g = H.load_golden("kat_tridiag10")
    with cgx.Solver(0) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        s.run(3)
        assert rel(s.x(), g["iters"][3]) <= FAST_RTOL


@pytest.mark.parametrize("fuse", ["0", "1"])
def test_sell_layout_bit_exact(fuse, monkeypatch):
    """SELL-64 internal layout: SpMV bit-exact (padding after each row's
    entries), CG within tolerance; irregular matrices fall back to CSR."""
    monkeypatch.setenv("CGX_LAYOUT", "sell")
    monkeypatch.setenv("CGX_FUSE_XPAY", fuse)
    with cgx.Solver(0) as s:
        for name in ["lap3d_12", "lap2d_32", "dense128", "rand_spd_2000", "kat_tridiag10"]:
            g = H.load_golden(name)
            s.set_matrix(g["row_ptr"], g["col"], g["val"])
            assert H.same_bits_or_both_nan(s.spmv(g["b"]), g["ops"]["mv_mult"]), name
            s.set_rhs(g["b"])
            it = max(k for k in g["iters"] if not np.any(np.isnan(g["iters"][k])))
            s.run(it)
            assert rel(s.x(), g["iters"][it]) <= FAST_RTOL, name
        rp, col, val = cgx.laplacian3d(70, 60, 50)
        x = np.random.default_rng(6).standard_normal(len(rp) - 1)
        s.set_matrix(rp, col, val)
        assert s.info()["spmv_iter_bytes"] < s.info()["spmv_bytes"] + 4 * len(x) * 8
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        rp32, col32, v32 = cgx.random_spd(5000, 40, 9, f32=True)
        x32 = np.random.default_rng(2).standard_normal(5000).astype(np.float32)
        s.set_matrix(rp32, col32, v32)
        assert np.array_equal(s.spmv(x32).view(np.uint32),
                              H.o_spmv_f32(rp32, col32, v32, x32).view(np.uint32))


@pytest.mark.parametrize("dma", ["0", "1"])
def test_deferred_x_bit_identical(dma, monkeypatch):
    """CGX_XDEFER folds x += alpha p into the p-update (one read of p less per
    iteration).  Same per-element roundings and reductions, so x, the r.r
    history and the stop iteration are bit-identical to the standard HS path,
    for fixed iteration counts (max_iter stop) and for tolerance stops that
    land inside a replayed batch (the stop iteration's x update must still
    happen, later ones must not)."""
    monkeypatch.setenv("CGX_SPMV_DMA", dma)
    cases = [H.random_spd(30000, 9, seed=21), None]
    g = H.load_golden("lap3d_12")
    cases[1] = (g["row_ptr"], g["col"], g["val"], g["b"])
    for rp, col, val, b in cases:
        out = {}
        for xd in ("0", "1", "fold", "foldpf"):
            # "fold": CGX_FOLD, the alpha/beta/stop steps inside the vector
            # kernels (no finalize launches) -- same scalars bit for bit;
            # "foldpf": the same with the first loads issued before the
            # partial sums (CGX_VEC_PF)
            monkeypatch.setenv("CGX_XDEFER", "0" if xd == "0" else "1")
            monkeypatch.setenv("CGX_FOLD", "1" if xd.startswith("fold") else "0")
            monkeypatch.setenv("CGX_VEC_PF", "1" if xd == "foldpf" else "0")
            with cgx.Solver(0) as s:
                s.set_matrix(rp, col, val)
                res = []
                for maxit, tol in [(0, 0.0), (1, 0.0), (37, 0.0), (2000, 1e-9), (2000, 1e-6)]:
                    s.set_rhs(b)
                    its = s.run(maxit, tol)
                    res.append((its, s.x(), s.history(its)))
                out[xd] = res
        for other in ("1", "fold", "foldpf"):
            for (i0, x0, h0), (i1, x1, h1) in zip(out["0"], out[other]):
                assert i0 == i1, other
                assert H.same_bits_or_both_nan(x0, x1), other
                assert H.same_bits_or_both_nan(h0, h1), other
    x_ref, _ = H.o_conj_grad(37, g["row_ptr"], g["col"], g["val"], g["b"])
    assert rel(out["1"][2][1], x_ref) <= FAST_RTOL


@pytest.mark.parametrize("xd", ["0", "1", "fold"])
def test_history_after_buffer_growth(xd, monkeypatch):
    """Cached hipGraphs are dropped when a longer run reallocates the r.r
    history buffer (regression: r01, the graph kept the freed pointer)."""
    monkeypatch.setenv("CGX_XDEFER", "0" if xd == "0" else "1")
    monkeypatch.setenv("CGX_FOLD", "1" if xd == "fold" else "0")
    rp, col, val, b = H.random_spd(30000, 9, seed=21)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        s.run(37)
        s.set_rhs(b)
        its = s.run(2000, 1e-9)
        h = s.history(its)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        its2 = s.run(2000, 1e-9)
        h2 = s.history(its2)
    assert its == its2
    assert H.same_bits_or_both_nan(h, h2)


def test_stream_ceilings():
    """The on-box ceilings bench.py reports beside the SpMV roofline: sane
    fractions of the 8 TB/s spec, reads faster than the triad's mix."""
    t = cgx.stream_bench(0, 16 * 2**20, 3, cgx.CGX_STREAM_TRIAD)
    r = cgx.stream_bench(0, 16 * 2**20, 3, cgx.CGX_STREAM_READ)
    assert 2000.0 < t < 8000.0 and 2000.0 < r < 8000.0


@pytest.mark.parametrize("kb", ["8", "64", "64w"])
def test_column_panels_bit_exact(kb, monkeypatch):
    """Column-panel layout (CGX_LAYOUT=panel): rows continue their sequential
    sums panel after panel, so SpMV stays bit-exact in fp64 and fp32, rows
    longer than a window (dense rows crossing every panel) and rows with no
    entry in a panel included; CG matches the oracle."""
    monkeypatch.setenv("CGX_LAYOUT", "panel")
    monkeypatch.setenv("CGX_PANEL_KB", kb.rstrip("w"))
    if kb.endswith("w"):
        monkeypatch.setenv("CGX_PANEL_WIN512", "1")
    rp, col, val, b = H.random_spd(30000, 9, seed=31)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["n_panels"] > 1
        assert H.same_bits_or_both_nan(s.spmv(b), H.o_spmv(rp, col, val, b))
        s.set_rhs(b)
        s.run(40)
        x_ref, _ = H.o_conj_grad(40, rp, col, val, b)
        assert rel(s.x(), x_ref) <= FAST_RTOL
        s.set_rhs(b)
        its = s.run(2000, 1e-9)
        _, its_o, _ = H.o_solve(2000, 1e-9, rp, col, val, b)
        assert abs(its - its_o) <= 1
        # dense rows (long-row path) crossing all panels
        n = 6000
        rng = np.random.default_rng(9)
        rows = [np.arange(n) if i in (0, 17, n - 1) else
                np.unique(np.concatenate([[max(i - 1, 0), i, min(i + 1, n - 1)],
                                          rng.integers(0, n, 4)])) for i in range(n)]
        rp2 = np.zeros(n + 1, np.int32)
        rp2[1:] = np.cumsum([len(c) for c in rows])
        col2 = np.concatenate(rows).astype(np.int32)
        val2 = rng.standard_normal(len(col2))
        x2 = rng.standard_normal(n)
        s.set_matrix(rp2, col2, val2)
        assert H.same_bits_or_both_nan(s.spmv(x2), H.o_spmv(rp2, col2, val2, x2))
        rp32, col32, v32 = cgx.random_spd(20000, 40, 9, f32=True)
        x32 = np.random.default_rng(2).standard_normal(20000).astype(np.float32)
        s.set_matrix(rp32, col32, v32)
        assert s.info()["n_panels"] > 1
        assert np.array_equal(s.spmv(x32).view(np.uint32),
                              H.o_spmv_f32(rp32, col32, v32, x32).view(np.uint32))


def test_column_panels_auto_c5():
    """C5 (random SPD, 5 M rows, fp32) selects column panels by itself and is
    bit-exact at full size; a large Laplacian keeps plain CSR."""
    rp, col, val = cgx.random_spd(5_000_000, 32, 42, f32=True)
    x = np.random.default_rng(3).standard_normal(len(rp) - 1).astype(np.float32)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["n_panels"] == 10
        assert np.array_equal(s.spmv(x).view(np.uint32),
                              H.o_spmv_f32(rp, col, val, x).view(np.uint32))
    del rp, col, val
    rp, col, val = cgx.laplacian3d(128, 128, 128)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["n_panels"] == 1


def lap_dict(dim, nx, ny, nz):
    d = {0}
    if nx > 1:
        d |= {-1, 1}
    if ny > 1:
        d |= {-nx, nx}
    if dim == 3 and nz > 1:
        d |= {-nx * ny, nx * ny}
    return sorted(d)


@pytest.mark.parametrize("dim,shape", [(3, (12, 12, 12)), (3, (7, 5, 9)), (3, (1, 6, 4)),
                                       (2, (32, 32, 1)), (2, (17, 9, 1)), (3, (216, 216, 216))])
def test_device_generated_laplacian_bit_exact(dim, shape):
    """the Laplacian generated in device memory is the host
    generator's CSR bit for bit (C3 at full size included), and solves alike."""
    nx, ny, nz = shape
    host = cgx.laplacian3d(nx, ny, nz) if dim == 3 else cgx.laplacian2d(nx, ny)
    with cgx.Solver(0) as s:
        s.gen_laplacian(dim, nx, ny, nz)
        rp, col, val = s.matrix()
        assert np.array_equal(rp, host[0]) and np.array_equal(col, host[1])
        assert H.same_bits_or_both_nan(val, host[2])
        # coded columns encoded on the device against the stencil's offsets
        n = len(rp) - 1
        offs = np.unique(col - np.repeat(np.arange(n), np.diff(rp)))
        assert s.info()["n_dict"] == len(lap_dict(dim, nx, ny, nz))
        assert set(offs.tolist()) <= set(lap_dict(dim, nx, ny, nz))
        x = np.random.default_rng(6).standard_normal(n)
        if n <= 200_000:
            assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(*host, x))
        if len(rp) - 1 <= 2000:
            b = np.random.default_rng(4).standard_normal(len(rp) - 1)
            s.set_rhs(b)
            s.run(25)
            x_ref, _ = H.o_conj_grad(25, *host, b)
            assert rel(s.x(), x_ref) <= FAST_RTOL


@pytest.mark.parametrize("dim,shape", [(3, (12, 12, 12)), (3, (7, 5, 9)), (3, (1, 6, 4)),
                                       (2, (32, 32, 1)), (2, (17, 9, 1)), (3, (216, 216, 216))])
def test_matrix_free_stencil_bit_exact(dim, shape):
    """the matrix-free stencil SpMV is bit-identical to the CSR
    SpMV of the same Laplacian (same column order, same products), and its
    CG matches the oracle within FAST_RTOL and stops at the same iteration."""
    nx, ny, nz = shape
    rp, col, val = cgx.laplacian3d(nx, ny, nz) if dim == 3 else cgx.laplacian2d(nx, ny)
    n = len(rp) - 1
    x = np.random.default_rng(5).standard_normal(n)
    with cgx.Solver(0) as s:
        s.set_stencil(dim, nx, ny, nz)
        assert s.info()["nnz"] == len(col)
        y = s.spmv(x)
    assert H.same_bits_or_both_nan(y, H.o_spmv(rp, col, val, x))
    if n <= 2000:
        b = np.random.default_rng(6).standard_normal(n)
        with cgx.Solver(0) as s:
            s.set_stencil(dim, nx, ny, nz)
            s.set_rhs(b)
            s.run(25)
            x_ref, _ = H.o_conj_grad(25, rp, col, val, b)
            assert rel(s.x(), x_ref) <= FAST_RTOL
            s.set_rhs(b)
            its = s.run(3000, 1e-10)
        _, its_o, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
        assert abs(its - its_o) <= 1


@pytest.mark.parametrize("bpw", ["1", "2", "4"])
def test_value_indexed_cg(bpw, monkeypatch):
    """CG on value-indexed pairs: with one row block per wave the SpMV
    partials group exactly as the offset-coded kernel's, so the run is
    bit-identical to CGX_DC_VALS=0; 2 and 4 blocks per wave regroup p.s
    (fast-mode tolerance against the oracle, reproducible)."""
    monkeypatch.setenv("CGX_VI_BPW", bpw)
    rp, col, val = cgx.laplacian3d(60, 50, 40)
    b = np.random.default_rng(13).standard_normal(len(rp) - 1)
    out = {}
    for vals in ("1", "0", "1"):
        monkeypatch.setenv("CGX_DC_VALS", vals)
        with cgx.Solver(0) as s:
            s.set_matrix(rp, col, val)
            assert s.info()["dict_vals"] == int(vals)
            s.set_rhs(b)
            s.run(30)
            out.setdefault(vals, []).append((s.x(), s.history(31)))
    x_ref, _ = H.o_conj_grad(30, rp, col, val, b)
    assert rel(out["1"][0][0], x_ref) <= FAST_RTOL
    assert H.same_bits_or_both_nan(out["1"][0][0], out["1"][1][0])
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        want = -(-s.info()["n_rowblocks"] // (int(bpw) * 4))
        assert s.info()["spmv_grid"] == want
        y = s.spmv(b)
        assert H.same_bits_or_both_nan(y, H.o_spmv(rp, col, val, b))
    if bpw == "1":
        assert H.same_bits_or_both_nan(out["1"][0][0], out["0"][0][0])
        assert H.same_bits_or_both_nan(out["1"][0][1], out["0"][0][1])


@pytest.mark.parametrize("wpb", ["8"])
def test_coded_wide_workgroups_cg(wpb, monkeypatch):
    """The 8-wave coded-column kernel (half the epilogue partials) inside
    the HS iteration: x within the fast-mode tolerance, runs reproducible."""
    monkeypatch.setenv("CGX_SPMV_WPB", wpb)
    rp, col, val = cgx.laplacian3d(60, 50, 40)
    b = np.random.default_rng(12).standard_normal(len(rp) - 1)
    xs = []
    for _ in range(2):
        with cgx.Solver(0) as s:
            s.set_matrix(rp, col, val)
            assert s.info()["n_dict"] == 7
            assert s.info()["spmv_grid"] == -(-s.info()["n_rowblocks"] // int(wpb))
            s.set_rhs(b)
            s.run(30)
            xs.append(s.x())
    x_ref, _ = H.o_conj_grad(30, rp, col, val, b)
    assert rel(xs[0], x_ref) <= FAST_RTOL
    assert H.same_bits_or_both_nan(xs[0], xs[1])


@pytest.mark.parametrize("kb", ["", "64", "0"])
def test_tiled_block_order_bit_exact(kb, monkeypatch):
    """L2-tiled row-block order (CGX_DC_TILE_KB budget; 0 = off): the SpMV
    is bit-identical to the oracle whatever the order, and a CG run stays
    within the fast-mode tolerance."""
    if kb == "0":
        monkeypatch.setenv("CGX_DC_TILE", "0")
    elif kb:
        monkeypatch.setenv("CGX_DC_TILE_KB", kb)
    rp, col, val = cgx.laplacian3d(120, 100, 20)  # plane 12000 rows: 288 KB of x per 3 planes
    n = len(rp) - 1
    x = np.random.default_rng(8).standard_normal(n)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["n_dict"] == 7
        assert s.info()["tile_bands"] == {"": 0, "64": 5, "0": 0}[kb]
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        s.set_rhs(x)
        s.run(30)
        x_ref, _ = H.o_conj_grad(30, rp, col, val, x)
        assert rel(s.x(), x_ref) <= FAST_RTOL


def test_c4_full_size_spmv_device_generated():
    """C4 at full size (400^3: 64,000,000 rows, 447,040,000 nnz -- the largest
    BASELINE config, int32 offsets up to 2^28.7): the device-generated CSR
    SpMV equals the matrix-free stencil bit for bit (the stencil is pinned to
    the oracle's CSR SpMV at small sizes by test_matrix_free_stencil_bit_exact)."""
    x = np.random.default_rng(11).standard_normal(400 ** 3)
    with cgx.Solver(0) as s:
        s.gen_laplacian(3, 400, 400, 400)
        assert s.info()["nnz"] == 447_040_000
        assert s.info()["n_dict"] == 7  # coded columns, encoded on the device
        y = s.spmv(x)
    with cgx.Solver(0) as s:
        s.set_stencil(3, 400, 400, 400)
        y2 = s.spmv(x)
    assert H.same_bits_or_both_nan(y, y2)
