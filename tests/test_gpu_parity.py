"""GPU parity: the HIP path (called through the C ABI of libcgx.so) against
the golden vectors of the compiled reference and against the pinned oracle.

Bars (stated here, checked below):
  * SpMV (mv_mult), sv_mult, vec_add, vec_sub: bit-exact, in every device
    layout (CSR, CSR-DC, DIA-VI, column panels, matrix-free stencil).
  * conj_grad / solve in CGX_MODE_EXACT: bit-exact x at every golden max_iter
    (including the all-NaN breakdown of the n = 10 KAT at max_iter 5).
  * default (parallel-reduction) mode: ||x - x_ref||_2 <= FAST_RTOL ||x_ref||_2
    with FAST_RTOL = 1e-12 (the only difference is dot-product summation
    order; simulated worst case on the fixtures is ~1e-14), bit-reproducible
    run to run.
  * full-size configs (C2, C3, C4, C5): size-independent properties
    (bit-exact SpMV against the oracle or the stencil, true relative residual
    ||b - A x|| / ||b|| <= tol after solve).
"""
import ctypes

import numpy as np
import pytest

import cgx
import helpers as H

pytestmark = pytest.mark.gpu

FAST_RTOL = 1e-12
NAMES = H.golden_names()
CHAINED = [n for n in NAMES if H.load_golden(n)["chained"]]
LAYOUTS = ["auto", "csr", "dc", "dia", "panel"]


@pytest.fixture(scope="module")
def solver():
    s = cgx.Solver(0)
    yield s
    s.close()


@pytest.fixture
def exact_env():
    """The op-level entry points in the reference's summation order
    (cgx_ops_set_mode; the library reads no environment)."""
    cgx.ops_set_mode(cgx.CGX_MODE_EXACT)
    yield
    cgx.ops_set_mode(cgx.CGX_MODE_FAST)


def rel(x, ref):
    d = np.linalg.norm(ref)
    return np.linalg.norm(x - ref) / (d if d > 0 else 1.0)


def same32(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32),
                          np.asarray(b, np.float32).view(np.uint32))


def expect_layout(rp, col, val, want="auto"):
    """The layout libcgx must pick on one GPU (cgx_matrix.h): DIA when the
    nonzeros lie on <= 16 diagonals (col - row) with <= 15 distinct values
    (bit patterns) each and one order of the diagonals is followed by every
    row; else DIA-V (layout "dia", dia_value_stream) on <= 8 such diagonals
    with any values when 1 + s_v ndiag bytes per row do not exceed DC's
    (s_v + 1) nnz / n + 1; else DC when <= 256 distinct offsets and rows <=
    255 entries; else CSR.  A forced layout falls back DIA -> DC -> CSR."""
    rp, col = np.asarray(rp), np.asarray(col)
    n = len(rp) - 1
    if want == "panel":  # column panels need x wider than one 3.5 MiB panel
        pcols = max(1024, 3584 * 1024 // np.asarray(val).itemsize)
        return "panel" if len(col) and n > pcols else "csr"
    if want == "csr" or len(col) == 0:
        return "csr"
    lens = np.diff(rp)
    rows = np.repeat(np.arange(n), lens)
    off = col.astype(np.int64) - rows
    v = np.asarray(val)
    bits = v.view(np.uint64 if v.dtype == np.float64 else np.uint32).astype(np.uint64)
    doffs = np.unique(off)
    order_ok = len(doffs) <= 16
    if order_ok:  # the diagonals need one order that every row's entries follow
        same = np.diff(rows) == 0
        edges = set(zip(off[:-1][same].tolist(), off[1:][same].tolist()))
        pred = {d: {a for a, b in edges if b == d} for d in doffs.tolist()}
        placed = set()
        while len(placed) < len(doffs) and order_ok:
            ready = [d for d in doffs.tolist() if d not in placed and pred[d] <= placed]
            order_ok = bool(ready)
            placed |= set(ready[:1])
    dia_ok = order_ok and all(len(np.unique(bits[off == d])) <= 15 for d in doffs)
    ts = v.itemsize
    dv_ok = (order_ok and len(doffs) <= 8 and lens.max() <= 8 and
             1.0 + ts * len(doffs) <= (ts + 1.0) * len(col) / n + 1.0)
    dc_ok = len(doffs) <= 256 and lens.max() <= 255
    if want in ("auto", "dia") and (dia_ok or dv_ok):
        return "dia"
    if want in ("auto", "dia", "dc") and dc_ok:
        return "dc"
    return "csr"


def test_device_visible():
    assert cgx.lib().cgx_device_count() > 0


# ------------------------------------------------------------------ SpMV

@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("name", CHAINED)
def test_spmv_bit_exact_vs_reference(name, layout):
    """mv_mult's golden output (the compiled reference, mv_ops.c:160-201) in
    every layout; the layout picked is the documented one."""
    g = H.load_golden(name)
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        got = s.info()["layout_name"]
        want = expect_layout(g["row_ptr"], g["col"], g["val"], layout)
        if layout == "panel":
            assert got in ("panel", "csr")  # tiny matrices need no panels
        else:
            assert got == want, (got, want)
        assert H.same_bits_or_both_nan(s.spmv(g["b"]), g["ops"]["mv_mult"])


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


def random_pattern(seed, small_values, max_offsets=257):
    """n not a multiple of 64 or 512, empty and ragged rows (0-40 entries),
    1..max_offsets distinct offsets from a random band, columns sorted per
    row."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(1, 9000))
    nd = int(rng.integers(1, max_offsets + 1))
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
    if small_values:  # value-indexed codes when <= 15 values per diagonal
        val = rng.choice(np.array([-1.0, 2.5, -0.0, 0.0, 1e-300, -3.25]), size=len(col))
    else:
        val = rng.standard_normal(len(col))
    return rp, col, val, rng.standard_normal(n)


@pytest.mark.parametrize("layout", ["auto", "csr", "dc", "dia"])
@pytest.mark.parametrize("seed", range(8))
def test_spmv_random_patterns(seed, layout):
    """Randomised patterns through each layout's encoder and kernel: the
    documented layout is picked and y is bit-identical to the oracle (signed
    zeros and a denormal-range value keep their bit patterns).  Odd seeds use
    <= 16 diagonals and a small value set (DIA), even seeds up to 257
    offsets."""
    dia = seed % 2 == 1
    rp, col, val, x = random_pattern(seed, small_values=dia, max_offsets=16 if dia else 257)
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == expect_layout(rp, col, val, layout)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


@pytest.mark.parametrize("layout", LAYOUTS)
def test_spmv_long_and_empty_rows(layout):
    """Rows longer than one LDS window (dense rows: the chunked path; in DIA
    the wide-row slices), empty rows, a 4-row matrix: bit-exact."""
    n = 6000
    rng = np.random.default_rng(5)
    rows = [np.arange(n) if i in (0, 1, 2500, n - 1) else
            np.unique(np.concatenate([[max(i - 1, 0), i, min(i + 1, n - 1)], rng.integers(0, n, 4)]))
            for i in range(n)]
    rp = np.zeros(n + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    x = rng.standard_normal(n)
    with cgx.Solver(0, layout=layout) as s:
        for val in (rng.standard_normal(len(col)),
                    rng.choice(np.array([-1.0, 4.0]), size=len(col))):  # few values
            s.set_matrix(rp, col, val)
            assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        rp = np.array([0, 0, 2, 2, 3], np.int32)
        col = np.array([0, 3, 1], np.int32)
        val = np.array([2.0, -1.0, 5.0])
        x = np.array([1.0, 2.0, 3.0, 4.0])
        s.set_matrix(rp, col, val)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


@pytest.mark.parametrize("layout", LAYOUTS)
def test_spmv_f32_bit_exact(layout):
    rng = np.random.default_rng(1)
    with cgx.Solver(0, layout=layout) as s:
        rp, col, val = cgx.random_spd(20000, 16, 11, f32=True)
        x = rng.standard_normal(20000).astype(np.float32)
        s.set_matrix(rp, col, val)
        assert same32(s.spmv(x), H.o_spmv_f32(rp, col, val, x))
        g = H.load_golden("lap3d_12")
        v = g["val"].astype(np.float32)
        s.set_matrix(g["row_ptr"], g["col"], v)
        assert s.info()["layout_name"] == expect_layout(g["row_ptr"], g["col"], v, layout)
        x = rng.standard_normal(len(g["row_ptr"]) - 1).astype(np.float32)
        assert same32(s.spmv(x), H.o_spmv_f32(g["row_ptr"], g["col"], v, x))
        rp, col, v32 = banded_spd(6000, [1, 77, 500], 9, f32=True)
        s.set_matrix(rp, col, v32)
        x = rng.standard_normal(6000).astype(np.float32)
        assert same32(s.spmv(x), H.o_spmv_f32(rp, col, v32, x))


def test_layout_selection_limits():
    """The documented limits of each layout, bit-exact throughout: 255
    offsets -> DC (256-entry dictionary), 257 -> CSR; 16 diagonals with 15
    values each -> DIA, a 17th diagonal or a 16th value -> DC; a row whose
    columns descend -> not DIA; a row of 256 entries -> CSR (DC's byte row
    lengths)."""
    rng = np.random.default_rng(5)

    def check(s, rp, col, val, want):
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == want
        x = rng.standard_normal(len(rp) - 1)
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))

    with cgx.Solver(0) as s:
        offs = sorted(rng.choice(np.arange(1, 3000), 127, replace=False).tolist())
        rp, col, val = banded_spd(5000, offs, 7)
        check(s, rp, col, val, "dc")
        assert s.info()["n_dict"] == 255
        rp, col, val = banded_spd(3000, list(range(1, 129)), 8)
        check(s, rp, col, val, "csr")
        n = 20000

        def band(extra, nv):
            """diagonals 0, +-1..+-7 and `extra`; value k of a diagonal from a
            table of nv values (entry-dependent, so every value occurs)"""
            rows = [[c for c in range(r - 7, r + 8) if 0 <= c < n] +
                    [r + e for e in extra if 0 <= r + e < n] for r in range(n)]
            rows = [sorted(cs) for cs in rows]
            rp = np.zeros(n + 1, np.int32)
            rp[1:] = np.cumsum([len(c) for c in rows])
            col = np.array([c for cs in rows for c in cs], np.int32)
            off = col - np.repeat(np.arange(n), np.diff(rp))
            val = np.linspace(-2, 2, 16)[:nv][(np.arange(len(col)) * 7 + off) % nv]
            return rp, col, val

        for extra, nv, want in (([500], 15, "dia"), ([500], 16, "dc"), ([-500, 500], 15, "dc")):
            rp, col, val = band(extra, nv)
            assert expect_layout(rp, col, val) == want
            check(s, rp, col, val, want)
            if want == "dia":
                i = s.info()
                assert i["n_dict"] == 16 and i["code_bytes_per_row"] == 8
                assert i["n_values"] == 16 * 15
        # descending columns in one row: same diagonals, but not in row order
        rp, col, val = banded_spd(3000, [1, 2], 4)
        col = col.copy()
        col[rp[10]:rp[11]] = col[rp[10]:rp[11]][::-1]
        val = np.where(np.arange(len(val)) >= 0, np.round(val), val)
        check(s, rp, col, val, expect_layout(rp, col, val))
        assert s.info()["layout_name"] != "dia"
        n = 700
        rows = [list(range(0, 256))] + [[] if r % 5 == 0 else [r] for r in range(1, n)]
        rp = np.zeros(n + 1, dtype=np.int32)
        rp[1:] = np.cumsum([len(c) for c in rows])
        col = np.array([c for cs in rows for c in cs], dtype=np.int32)
        check(s, rp, col, rng.standard_normal(len(col)), "csr")


def diag_values_matrix(n, offsets, nvs, seed):
    """Rows hold the diagonals `offsets` (ascending, 0 included) where they
    fit; diagonal k draws its entries from nvs[k] distinct values, each
    value used (entry-dependent choice); the main diagonal dominates."""
    rng = np.random.default_rng(seed)
    tabs = []
    for d, nv in zip(offsets, nvs):
        base = 60.0 if d == 0 else 0.0
        tabs.append(base + rng.choice(np.linspace(-1, 1, 64), nv, replace=False))
    r = np.repeat(np.arange(n), len(offsets))
    k = np.tile(np.arange(len(offsets)), n)
    c = r + np.asarray(offsets)[k]
    keep = (c >= 0) & (c < n)
    r, k, c = r[keep], k[keep], c[keep]
    nv = np.asarray(nvs)[k]
    vidx = (r * 7 + k * 3) % nv
    val = np.array([tabs[kk][vv] for kk, vv in zip(k, vidx)])
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, r + 1, 1)
    return np.cumsum(rp).astype(np.int32), c.astype(np.int32), val


@pytest.mark.parametrize("offsets,nvs,cb", [
    ([-7, -1, 0, 1, 7], [1] * 5, 1),                        # a 2-D stencil: 5 bits
    ([-40, -9, -3, -1, 0, 1, 3, 9, 40], [1] * 9, 2),        # 9 one-value diagonals
    ([-3, -1, 0, 1, 3], [3, 2, 3, 2, 3], 2),                # 2-bit fields
    ([-1500, -2, -1, 0, 1, 2, 3, 1500], [2] + [15] * 6 + [3], 4),  # 28 bits, far pair
    ([-4, -3, -2, -1, 0, 1, 2, 3], [15] * 8, 4),            # 32 bits
    (list(range(-8, 8)), [1] * 16, 2),                      # 16 one-value diagonals
    ([-4, -3, -2, -1, 0, 1, 2, 3, 4], [15] * 9, 8),         # 36 bits
])
def test_dia_code_widths(offsets, nvs, cb):
    """DIA-VI packs a row's value indices into fields of 1-4 bits (by each
    diagonal's value count), the word 1, 2, 4 or 8 bytes: every width is
    bit-exact against the oracle SpMV (odd n: a half row pair at the end),
    and the fused HS step (words <= 4 bytes) is bit-identical to the
    unfused iteration."""
    n = 6001
    rp, col, val = diag_values_matrix(n, offsets, nvs, seed=len(offsets) * 10 + cb)
    assert expect_layout(rp, col, val) == "dia"
    x = np.random.default_rng(1).standard_normal(n)
    b = np.random.default_rng(2).standard_normal(n)
    out = []
    for fused in (True, False):
        with cgx.Solver(0, layout="dia", fused=fused) as s:
            s.set_matrix(rp, col, val)
            i = s.info()
            assert i["layout_name"] == "dia" and i["code_bytes_per_row"] == cb
            assert i["n_values"] == sum(nvs)
            assert i["fused"] == (1 if fused and cb <= 4 else 0)
            assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
            s.set_rhs(b)
            its = s.run(21, 0.0)
            out.append((its, s.x(), s.history(its)))
    assert out[0][0] == out[1][0] == 22
    assert H.same_bits_or_both_nan(out[0][1], out[1][1])
    assert H.same_bits_or_both_nan(out[0][2], out[1][2])


def test_bad_column_rejected():
    """A column outside [0, n) would be an out-of-bounds device gather: the
    upload refuses it on the host."""
    with cgx.Solver(0) as s:
        with pytest.raises(cgx.CgxError):
            s.set_matrix(np.array([0, 1, 2], np.int32), np.array([0, 2], np.int32), np.ones(2))
        with pytest.raises(cgx.CgxError):
            s.set_matrix(np.array([0, 2, 1], np.int32), np.array([0, 1], np.int32), np.ones(2))


@pytest.mark.parametrize("layout", ["auto", "csr", "dc", "dia"])
def test_spmv_c3_full_size_bit_exact(layout):
    """BASELINE config C3 (3-D 7-pt 216^3, 10,077,696 rows): one SpMV,
    bit-exact against the oracle at full size in every layout; the automatic
    choice is DIA (7 diagonals, one value each: one 1-bit field per diagonal,
    1 code byte per row), found
    from the sampled rows without an exact host scan."""
    rp, col, val = cgx.laplacian3d(216, 216, 216)
    x = np.random.default_rng(2).standard_normal(len(rp) - 1)
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        assert i["layout_name"] == {"auto": "dia"}.get(layout, layout)
        assert i["encode_fallback"] == 0 and i["nt"] == 1
        if i["layout_name"] == "dia":
            assert i["n_dict"] == 7 and i["code_bytes_per_row"] == 1 and i["n_values"] == 7
            assert i["spmv_grid"] == -(-(len(rp) - 1) // 512)
        else:
            assert i["gathers_per_chunk"] == 7
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))


@pytest.mark.parametrize("layout", ["auto", "csr", "dc"])
def test_c2_full_size(layout):
    """BASELINE config C2 (2-D 5-pt 1000^2, the cache-resident 328-entry
    window case): bit-exact SpMV at full size and solve(1e-8) reaches a true
    relative residual below tol."""
    rp, col, val = cgx.laplacian2d(1000, 1000)
    n = len(rp) - 1
    x = np.random.default_rng(7).standard_normal(n)
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        assert i["layout_name"] == {"auto": "dia"}.get(layout, layout)
        assert i["nt"] == 0  # the whole iteration fits the Infinity Cache
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        b = np.ones(n)
        s.set_rhs(b)
        its = s.run(6000, 1e-8)
        xs = s.x()
    r = b - H.o_spmv(rp, col, val, xs)
    assert np.linalg.norm(r) <= 1.5e-8 * np.linalg.norm(b)
    assert its < 6000


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


def test_mv_mult_matrix_residency():
    """the op-level drop-in keeps A on the device.  The
    reference's conj_grad calls mv_mult once per iteration on the same A
    (cg.c:111): the second call reuses the upload; changing a value in place
    (same pointers) or passing another matrix uploads again; y stays
    bit-exact throughout."""
    rp, col, val = cgx.laplacian3d(40, 30, 20)
    x = np.random.default_rng(3).standard_normal(len(rp) - 1)
    A = cgx.Mv(val, col, rp)
    b = cgx.Mv(x)
    u0, r0 = cgx.ops_counters()
    y1 = cgx.mv_mult(A, b)
    y2 = cgx.mv_mult(A, b)
    u1, r1 = cgx.ops_counters()
    assert (u1 - u0, r1 - r0) == (1, 1)
    assert H.same_bits_or_both_nan(y1, H.o_spmv(rp, col, val, x))
    assert H.same_bits_or_both_nan(y2, y1)
    A.values[17] = 2.5  # in place: same pointers, new contents
    y3 = cgx.mv_mult(A, b)
    u2, r2 = cgx.ops_counters()
    assert (u2 - u1, r2 - r1) == (1, 0)
    assert H.same_bits_or_both_nan(y3, H.o_spmv(rp, col, A.values, x))
    # conj_grad after mv_mult on the same A: no second upload
    x_cg = cgx.conj_grad(5, A, b)
    u3, r3 = cgx.ops_counters()
    assert (u3 - u2, r3 - r2) == (0, 1)
    assert np.all(np.isfinite(x_cg))
    # edits that cancelled in the round-2 hash: a symmetric pair
    # a_ij / a_ji negated in place, then every value negated (even length);
    # each is detected (one upload, the call redone on the new A)
    i = 1000
    k = rp[i]  # first entry of row i (its -nx neighbour, column 960)
    j = int(col[k])
    kt = rp[j] + int(np.searchsorted(col[rp[j]:rp[j + 1]], i))
    assert col[kt] == i
    A.values[k] = -A.values[k]
    A.values[kt] = -A.values[kt]
    y4 = cgx.mv_mult(A, b)
    u4, r4 = cgx.ops_counters()
    assert (u4 - u3, r4 - r3) == (1, 0)
    assert H.same_bits_or_both_nan(y4, H.o_spmv(rp, col, A.values, x))
    assert len(A.values) % 2 == 0
    A.values[:] = -A.values
    x_cg2 = cgx.conj_grad(5, A, b)
    u5, r5 = cgx.ops_counters()
    assert (u5 - u4, r5 - r4) == (1, 0)
    x_ref, _ = H.o_conj_grad(5, rp, col, A.values, x)
    assert rel(x_cg2, x_ref) <= FAST_RTOL


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
    cgx.ops_set_mode(cgx.CGX_MODE_FAST)
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
    cgx.ops_set_mode(cgx.CGX_MODE_FAST)
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
    assert cgx.ops_last_timing()["breakdown"] == 0
    assert np.all(np.isnan(cgx.conj_grad(5, A, b)))
    # SURVEY.md 5 (failure detection): r is exactly 0 after the 5th x update,
    # so p = 0 and p.s = 0 at the 6th: the breakdown the reference turns into
    # NaN (cg.c:113) is reported, the IEEE result kept
    assert cgx.ops_last_timing()["breakdown"] == 6
    with cgx.Solver(0, mode=cgx.CGX_MODE_EXACT) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        s.run(5)
        assert s.info()["breakdown"] == 6 and np.all(np.isnan(s.x()))
        s.run(3)
        assert s.info()["breakdown"] == 0


def test_fuse_status_reports_why():
    """cgx_info.fuse_status names why the fused step does or does not run
    (the refusal was silent)."""
    rp, col, val = cgx.laplacian3d(40, 30, 24)
    cases = [(dict(), cgx.CGX_FUSE_STATUS_CACHED), (dict(fused=True), cgx.CGX_FUSE_STATUS_RUNS),
             (dict(fused=False), cgx.CGX_FUSE_STATUS_OFF),
             (dict(mode=cgx.CGX_MODE_EXACT), cgx.CGX_FUSE_STATUS_EXACT),
             (dict(layout="csr", fused=True), cgx.CGX_FUSE_STATUS_NOT_DIA)]
    for kw, want in cases:
        with cgx.Solver(0, **kw) as s:
            s.set_matrix(rp, col, val)
            i = s.info()
            assert i["fuse_status"] == want, (kw, i["fuse_status"])
            assert i["fused"] == (1 if want == cgx.CGX_FUSE_STATUS_RUNS else 0)


def test_dropin_sr_every_matrix():
    """cgx_ops_set_mode(FAST, SR) through the
    drop-in solve() (cg.c:72's caller): a matrix without the plane-marched
    DIA step (the random-pattern CSR fixture) runs the unfused two-launch SR
    step (SpMV with (p.s, s.s) pairs, k_update_sr) -- within 1e-9 of the HS
    goldens at the tolerance stop (the stop iteration within 1) and within
    1e-10 of oracle_solve_sr; a 3-D Laplacian whose planes are 8 slices
    apart runs the one-launch SR step, against oracle_solve_sr and the HS
    oracle (the bars of test_sr_single_launch_vs_oracle).
    cgx_ops_last_timing() reports SR for both."""
    cgx.ops_set_mode(cgx.CGX_MODE_FAST, cgx.CGX_ALG_SR)
    try:
        g = H.load_golden("rand_spd_2000")
        A = cgx.Mv(g["val"], g["col"], g["row_ptr"])
        b = cgx.Mv(g["b"])
        x, its = cgx.solve(A, b, 1e-10, 1000)
        assert cgx.ops_last_timing()["alg"] == cgx.CGX_ALG_SR
        x_o, its_o, _ = H.o_solve(1000, 1e-10, g["row_ptr"], g["col"], g["val"], g["b"])
        x_sr, its_sr, _ = H.o_solve(1000, 1e-10, g["row_ptr"], g["col"], g["val"], g["b"],
                                    sr=True)
        assert abs(its - its_o) <= 1 and its == its_sr, (its, its_o, its_sr)
        assert rel(x, x_o) <= 1e-9 and rel(x, x_sr) <= 1e-10
        rp, col, val = H.laplacian3d(64, 64, 40)
        bv = np.random.default_rng(23).standard_normal(len(rp) - 1)
        A, b = cgx.Mv(val, col, rp), cgx.Mv(bv)
        for tol, maxit in ((0.0, 30), (1e-9, 3000)):
            x, its = cgx.solve(A, b, tol, maxit)
            assert cgx.ops_last_timing()["alg"] == cgx.CGX_ALG_SR
            x_sr, its_sr, _ = H.o_solve(maxit, tol, rp, col, val, bv, sr=True)
            x_hs, its_hs, _ = H.o_solve(maxit, tol, rp, col, val, bv)
            assert its == its_sr and abs(its - its_hs) <= 1, (tol, its, its_sr, its_hs)
            assert rel(x, x_sr) <= 1e-10 and rel(x, x_hs) <= 1e-9, tol
        # general coefficients (round 5): the drop-in's matrix on DIA-V, the
        # one-launch SR step over streamed values
        rp, col, val = cgx.varcoef3d(32, 48, 20, seed=4)
        bv = np.random.default_rng(29).standard_normal(len(rp) - 1)
        A, b = cgx.Mv(val, col, rp), cgx.Mv(bv)
        for tol, maxit in ((0.0, 25), (1e-9, 3000)):
            x, its = cgx.solve(A, b, tol, maxit)
            assert cgx.ops_last_timing()["alg"] == cgx.CGX_ALG_SR
            x_sr, its_sr, _ = H.o_solve(maxit, tol, rp, col, val, bv, sr=True)
            x_hs, its_hs, _ = H.o_solve(maxit, tol, rp, col, val, bv)
            assert its == its_sr and abs(its - its_hs) <= 1, (tol, its, its_sr, its_hs)
            assert rel(x, x_sr) <= 1e-10 and rel(x, x_hs) <= 1e-9, tol
    finally:
        cgx.ops_set_mode(cgx.CGX_MODE_FAST, cgx.CGX_ALG_HS)


def sr_unfused_cases():
    # (name, system): every layout the unfused SR step runs on
    for name in ("rand_spd_2000", "lap2d_32", "lap3d_12", "dense128"):
        g = H.load_golden(name)
        yield name, g["row_ptr"], g["col"], g["val"], g["b"], "auto"
    rp, col, val = H.laplacian3d(40, 30, 24)
    b = np.random.default_rng(5).standard_normal(len(rp) - 1)
    for layout in ("csr", "dc", "dia"):
        yield f"lap3d_40x30x24_{layout}", rp, col, val, b, layout


@pytest.mark.parametrize("case", list(sr_unfused_cases()), ids=lambda c: c[0] + "_" + c[5])
def test_sr_unfused_vs_oracle(case):
    """CGX_ALG_SR without the plane march -- two launches
    and ONE reduction per iteration on any layout (CSR, DC, DIA without a
    march, column panels): at fixed max_iter within 1e-10 of
    oracle_solve_sr (the recurrence it restates; only the grouping of the
    dot products differs) with its r.r history within 1e-8; at a 1e-10
    tolerance stop the iteration count of oracle_solve_sr, within 1 of the
    HS oracle's, x within 1e-9 of HS."""
    name, rp, col, val, b, layout = case
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR, layout=layout) as s:
        s.set_matrix(rp, col, val)
        s.set_march(0)  # the unfused step even where a march plan exists
        i = s.info()
        assert i["fused"] == 0 and i["alg"] == cgx.CGX_ALG_SR
        for maxit in (0, 1, 2, 7, 20):
            s.set_rhs(b)
            its = s.run(maxit)
            x_sr, its_sr, h_sr = H.o_solve(maxit, 0.0, rp, col, val, b, sr=True)
            assert its == its_sr == maxit + 1
            assert rel(s.x(), x_sr) <= 1e-10, (maxit, rel(s.x(), x_sr))
            assert np.allclose(s.history(its), h_sr[:its], rtol=1e-8, atol=0)
        s.set_rhs(b)
        its = s.run(5000, 1e-10)
        x = s.x()
    x_sr, its_sr, _ = H.o_solve(5000, 1e-10, rp, col, val, b, sr=True)
    x_hs, its_hs, _ = H.o_solve(5000, 1e-10, rp, col, val, b)
    assert its == its_sr and abs(its - its_hs) <= 1, (its, its_sr, its_hs)
    assert rel(x, x_sr) <= 1e-9 and rel(x, x_hs) <= 1e-9


def test_sr_unfused_graph_and_bench():
    """The unfused SR step graph-replayed and eager bit-identical, and its
    bench loop (the bench's general-coefficient leg) runs."""
    rp, col, val = cgx.varcoef3d(40, 30, 24, seed=3)
    b = np.random.default_rng(9).standard_normal(len(rp) - 1)
    xs = []
    for graph in (True, False):
        with cgx.Solver(0, alg=cgx.CGX_ALG_SR, layout="dc") as s:
            s.set_matrix(rp, col, val)
            assert s.info()["fused"] == 0
            s.set_rhs(b)
            s.bench_prepare(0)
            s.bench_run(33, graph=graph)
            xs.append(s.x())
    assert H.same_bits_or_both_nan(xs[0], xs[1])
    assert np.all(np.isfinite(xs[0]))
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR, layout="dc") as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        s.bench_prepare(3)
        ms, sp = s.bench_run(20, graph=False, spmv_events=True)
        assert ms > 0 and 0 < sp <= ms / 20 * 1.01
        assert s.bench_run(20)[0] > 0


def test_sr_fuse_status():
    """cgx_info.fuse_status follows fused()'s SR rules -- SR
    ignores the Infinity Cache rule (a cache-resident system runs it) and
    needs the march plan (NO_MARCH after set_march(0) or without a plan).
    Round 6: a matrix whose diagonals all lie within the window's halo (a
    2-D grid) has a near-only plan and runs the one-launch step; one whose
    far diagonals are two distances (1,500 and 3,000) has none."""
    rp, col, val = H.laplacian3d(64, 64, 10)
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        assert i["fused"] == 1 and i["fuse_status"] == cgx.CGX_FUSE_STATUS_RUNS
        s.set_march(0)
        i = s.info()
        assert i["fused"] == 0 and i["fuse_status"] == cgx.CGX_FUSE_STATUS_NO_MARCH
        s.set_rhs(np.ones(len(rp) - 1))
        assert s.run(5) == 6  # round 5: the unfused SR step runs instead
    rp, col, val = H.laplacian2d(300, 200)
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        assert i["fused"] == 1 and i["fuse_status"] == cgx.CGX_FUSE_STATUS_RUNS
        assert i["fuse_march"] > 0
    rp, col, val, _ = band_sym_rhs(20000, [1, 1500, 3000], 8)
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == "dia"
        assert s.info()["fuse_status"] == cgx.CGX_FUSE_STATUS_NO_MARCH


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


@pytest.mark.parametrize("layout", ["csr", "dc", "dia", "panel"])
def test_exact_mode_history_identical_across_layouts(layout):
    """Exact mode (sequential dots): x and the r.r history equal the oracle's
    bit for bit in every layout -- the layouts differ only in how A is
    stored."""
    g = H.load_golden("lap3d_12")
    with cgx.Solver(0, mode=cgx.CGX_MODE_EXACT, layout=layout) as s:
        s.set_matrix(g["row_ptr"], g["col"], g["val"])
        s.set_rhs(g["b"])
        assert s.run(40) == 41
        x, h = s.x(), s.history(41)
    x_ref, hist = H.o_conj_grad(40, g["row_ptr"], g["col"], g["val"], g["b"])
    assert H.same_bits_or_both_nan(h, hist)
    assert H.same_bits_or_both_nan(x, x_ref)


@pytest.mark.parametrize("layout", ["auto", "csr", "dc", "dia"])
def test_fast_mode_reproducible_and_stops(layout):
    """Fast mode in each layout: within FAST_RTOL of the reference order,
    bit-reproducible run to run (fixed-order reductions, no fp64 atomics),
    the tolerance stop within one iteration of the oracle's, the stop
    iteration's x update applied once (maxit 0, 1, 37 and tol stops that
    land inside a replayed batch)."""
    cases = [H.random_spd(30000, 9, seed=21)]
    g = H.load_golden("lap3d_12")
    cases.append((g["row_ptr"], g["col"], g["val"], g["b"]))
    for rp, col, val, b in cases:
        with cgx.Solver(0, layout=layout) as s:
            s.set_matrix(rp, col, val)
            for maxit, tol in [(0, 0.0), (1, 0.0), (37, 0.0), (2000, 1e-9), (2000, 1e-6)]:
                runs = []
                for _ in range(2):
                    s.set_rhs(b)
                    its = s.run(maxit, tol)
                    runs.append((its, s.x(), s.history(its)))
                assert runs[0][0] == runs[1][0]
                assert H.same_bits_or_both_nan(runs[0][1], runs[1][1])
                assert H.same_bits_or_both_nan(runs[0][2], runs[1][2])
                if tol == 0.0:
                    assert runs[0][0] == maxit + 1
                    x_ref, _ = H.o_conj_grad(maxit, rp, col, val, b)
                    assert rel(runs[0][1], x_ref) <= FAST_RTOL
                else:
                    _, its_o, _ = H.o_solve(maxit, tol, rp, col, val, b)
                    assert abs(runs[0][0] - its_o) <= 1
                    r = b - H.o_spmv(rp, col, val, runs[0][1])
                    assert np.linalg.norm(r) <= 1.01 * tol * np.linalg.norm(b)


def test_graph_and_eager_agree():
    """The hipGraph-replayed iterations and the eager launches are the same
    kernels in the same order: bit-identical x and history."""
    g = H.load_golden("lap2d_32")
    out = []
    for graph in (True, False):
        with cgx.Solver(0) as s:
            s.set_matrix(g["row_ptr"], g["col"], g["val"])
            s.set_rhs(g["b"])
            s.bench_prepare(0)
            s.bench_run(32, graph=graph)
            out.append(s.x())
    assert H.same_bits_or_both_nan(out[0], out[1])
    assert np.all(np.isfinite(out[0]))


def band_sym_rhs(n, offsets, seed):
    """Symmetric banded matrix on the diagonals +-offsets (and 0), a few
    distinct values per diagonal, strictly diagonally dominant."""
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    dsum = np.zeros(n)
    for d in offsets:
        i = np.arange(n - d)
        v = -rng.choice([0.25, 0.5, 0.75, 1.0], size=n - d)
        for rr, cc in ((i, i + d), (i + d, i)):
            rows.append(rr)
            cols.append(cc)
            vals.append(v)
            np.add.at(dsum, rr, np.abs(v))
    rows.append(np.arange(n))
    cols.append(np.arange(n))
    vals.append(np.ceil(dsum) + 1.0)
    r, c, v = (np.concatenate(a) for a in (rows, cols, vals))
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, r + 1, 1)
    return (np.cumsum(rp).astype(np.int32), c.astype(np.int32), v.astype(np.float64),
            rng.standard_normal(n))


def fused_cases():
    yield "lap3d_24x20x17", (*H.laplacian3d(24, 20, 17), None), True   # all near, NF 2
    yield "lap3d_40x30x9", (*H.laplacian3d(40, 30, 9), None), True     # +-1200 far, NF 3
    yield "band_1_37", band_sym_rhs(9001, [1, 37], 3), True              # odd halo (rounded)
    yield "band_far2", band_sym_rhs(20000, [1, 1100, 2100], 4), True    # 2 far a side
    yield "band_wide", band_sym_rhs(20000, [1, 1000, 1500], 7), True    # NF 5, 1 far a side
    yield "band_one_far", band_sym_rhs(20000, [1, 1500], 5), True        # near + 1 far a side
    yield "band_9", band_sym_rhs(8000, [1, 2, 3, 4, 5], 6), False        # 11 diagonals: unfused


@pytest.mark.parametrize("case", list(fused_cases()), ids=lambda c: c[0])
def test_fused_step_bit_identical_to_unfused(case):
    """The fused HS step (k_spmv_dia_h: x / p update + s = A p in one
    launch, p_new of the slice and its halo in LDS) computes every value
    of the unfused SpMV + k_update_rf + k_xpay_xf sequence with the same
    roundings: x, the iteration count and the r.r history are bit-identical
    (maxit 0 / 1 / even / odd batch remainders, a tolerance stop, graph and
    eager replays in bench_run)."""
    _, (rp, col, val, b), fusable = case
    n = len(rp) - 1
    if b is None:
        b = np.random.default_rng(9).standard_normal(n)
    out = {}
    for fused in (True, False):
        res = []
        with cgx.Solver(0, layout="dia", fused=fused) as s:
            s.set_matrix(rp, col, val)
            info = s.info()
            assert info["layout_name"] == "dia"
            assert info["fused"] == (1 if fused and fusable else 0)
            for maxit, tol in [(0, 0.0), (1, 0.0), (16, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-9)]:
                s.set_rhs(b)
                its = s.run(maxit, tol)
                res.append((its, s.x(), s.history(its)))
            # bench_run: fused launch j >= 2 finishes iteration j - 2 and
            # applies x updates in pairs (odd iterations), so 35 fused
            # launches hold x of 34 iterations
            for graph in (True, False):
                s.set_rhs(b)
                s.bench_prepare(0)
                s.bench_run(35 if fused and fusable else 34, graph=graph)
                res.append((34, s.x(), None))
        out[fused] = res
    for j, ((i0, x0, h0), (i1, x1, h1)) in enumerate(zip(out[True], out[False])):
        assert i0 == i1, j
        assert H.same_bits_or_both_nan(x0, x1), j
        if h0 is not None:
            assert H.same_bits_or_both_nan(h0, h1), j
    its, x, _ = out[True][5]
    assert its < 3000
    assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 1.01e-9 * np.linalg.norm(b)


def march_cases():
    # (name, system, two-slice super-items)
    yield "lap3d_32x48x20", (*H.laplacian3d(32, 48, 20), None), False   # F 1536 = 3 slices
    yield "lap3d_64x64x10", (*H.laplacian3d(64, 64, 10), None), False   # F 4096 = 8 slices
    yield "lap3d_300x7x20", (*H.laplacian3d(300, 7, 20), None), True    # F 2100 = 4 * 512 + 52
    yield "band_1_200_1100", band_sym_rhs(20000, [1, 200, 1100], 8), False  # 2 * 512 + 76


def sr_march_cases():
    # the one-launch SR step also runs near-only plans (round 6): a 2-D grid
    # whose +-1000 diagonals lie within the window's halo, C2's shape in 60 rows
    yield from march_cases()
    yield "lap2d_1000x60", (*H.laplacian2d(1000, 60), None), False


@pytest.mark.parametrize("case", list(march_cases()), ids=lambda c: c[0])
def test_fused_march_bit_identical_to_unfused(case):
    """The plane march of the fused step (k_spmv_dia_m: a workgroup walks
    slices F apart, the +-F neighbours read from an LDS ring of windows)
    computes every value of the unfused iteration with the same roundings
    and writes each slice's p.s partial at the unfused slot: x, iteration
    counts and the r.r history bit-identical to the unfused path for every
    segment length (1 step, a few, the auto length, whole chains), with
    ragged last slices and chains of unequal length."""
    _, (rp, col, val, b), two = case
    n = len(rp) - 1
    if b is None:
        b = np.random.default_rng(11).standard_normal(n)
    runs = [(0, 0.0), (1, 0.0), (16, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-9)]

    def solve(fused, march):
        res = []
        with cgx.Solver(0, layout="dia", fused=fused) as s:
            s.set_march(march)
            s.set_matrix(rp, col, val)
            info = s.info()
            for maxit, tol in runs:
                s.set_rhs(b)
                its = s.run(maxit, tol)
                res.append((its, s.x(), s.history(its)))
            s.set_rhs(b)
            s.bench_prepare(0)
            s.bench_run(35 if fused else 34)
            res.append((34, s.x(), None))
        return info, res

    _, ref = solve(False, -1)
    for march in (-1, 1, 3, 100000, 0):
        info, res = solve(True, march)
        assert info["fused"] == 1
        assert (info["fuse_march"] > 0) == (march != 0), (march, info["fuse_march"])
        for j, ((i0, x0, h0), (i1, x1, h1)) in enumerate(zip(res, ref)):
            assert i0 == i1, (march, j)
            assert H.same_bits_or_both_nan(x0, x1), (march, j)
            if h0 is not None:
                assert H.same_bits_or_both_nan(h0, h1), (march, j)


@pytest.mark.parametrize("case", list(sr_march_cases()), ids=lambda c: c[0])
def test_sr_single_launch_vs_oracle(case):
    """CGX_ALG_SR on one GPU (k_sr1_dia_m: the r update of the previous
    iteration, the p update and s = A p in ONE plane-marched launch, one
    reduction of (p.s, s.s, r.r)) against oracle_solve_sr, the recurrence it
    restates, and the HS oracle: same iteration counts at fixed maxit (+-1 at
    a tolerance stop), x within 1e-10 (fixed maxit; only the dot products'
    summation order differs), the r.r estimates within 1e-6, segment lengths
    1 / auto / whole chains, and graph vs eager replays bit-identical."""
    _, (rp, col, val, b), _ = case
    n = len(rp) - 1
    if b is None:
        b = np.random.default_rng(13).standard_normal(n)
    # (march, chain width): auto; one step per segment with the narrowest
    # chains (a quarter step, the ragged last chain); whole chains at a width
    # that is not a multiple of 64 rows; four-slice steps (2,048 / 1,536 /
    # 1,200-row chains)
    for march, chain in ((-1, 0), (1, 1), (100000, 0), (-1, 458), (-1, 2048), (1, 1536),
                         (3, 1200)):
        with cgx.Solver(0, alg=cgx.CGX_ALG_SR, layout="dia") as s:
            s.set_march(march)
            s.set_sr_chain(chain)
            s.set_matrix(rp, col, val)
            info = s.info()
            assert info["fused"] == 1 and info["fuse_march"] > 0
            for maxit in (0, 1, 2, 3, 16, 17, 18, 19, 40):  # every k % 4 at the stop
                s.set_rhs(b)
                its = s.run(maxit)
                x, h = s.x(), s.history(its)
                x_ref, its_ref, h_ref = H.o_solve(maxit, 0.0, rp, col, val, b, sr=True)
                assert its == its_ref == maxit + 1, (march, chain, maxit)
                assert rel(x, x_ref) <= 1e-10, (march, chain, maxit)
                assert np.allclose(h, h_ref, rtol=1e-6, atol=0), (march, chain, maxit)
            s.set_rhs(b)
            its = s.run(3000, 1e-10)
            x = s.x()
            x_sr, its_sr, _ = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
            x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
            assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
            assert rel(x, x_sr) <= 1e-9 and rel(x, x_hs) <= 1e-9
            assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 2e-10 * np.linalg.norm(b)
            out = []
            for graph in (True, False):
                s.set_rhs(b)
                s.bench_prepare(0)
                s.bench_run(35, graph=graph)
                out.append(s.x())
            assert H.same_bits_or_both_nan(out[0], out[1])


@pytest.mark.parametrize("shape", [(32, 48, 20), (13, 11, 9), (64, 48, 10), (40, 30, 24)])
def test_dia_v_general_coefficients(shape):
    """DIA-V (round 5): general coefficients on <= 8 diagonals
    (cgx_gen_varcoef3d: every off-diagonal value distinct, mv_ops.h:17-23's
    arbitrary values) keep a presence byte per row and stream the values
    diagonal-major on one GPU.  The SpMV bit-exact to the oracle
    (mv_ops.c:187-197) and the matrix read back identical; HS runs unfused
    (fuse_status VALUE_STREAM: the fused HS kernels read value tables)
    within 1e-12 of oracle_conj_grad; the one-launch SR step
    (k_sr1_dia_m<..., DV>) at every segment shape as
    test_sr_single_launch_vs_oracle: within 1e-10 of oracle_solve_sr at
    fixed maxit, within 1e-9 of both oracles at a tolerance stop, graph and
    eager replays bit-identical.  A plane of <= 1,024 rows has no far
    diagonal: 13 x 11 runs the near-only plan (round 6); without any plan
    (40 x 30 = 1,200 rows lie 176 rows off two slices, outside the 40-row
    halo) SR runs unfused (k_spmv_dia's (p.s, s.s) pairs + k_update_sr) to
    the same bars."""
    rp, col, val = cgx.varcoef3d(*shape, seed=11)
    march_plan = shape[:2] in ((32, 48), (64, 48), (13, 11))  # 3 and 6 slices; near-only
    n = len(rp) - 1
    b = np.random.default_rng(23).standard_normal(n)
    with cgx.Solver(0, fused=True) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        assert (i["layout_name"], i["dia_value_stream"], i["code_bytes_per_row"]) == ("dia", 1, 1)
        assert i["fused"] == 0 and i["fuse_status"] == cgx.CGX_FUSE_STATUS_VALUE_STREAM
        assert H.same_bits_or_both_nan(s.spmv(b), H.o_spmv(rp, col, val, b))
        rp2, col2, val2 = s.matrix()
        assert np.array_equal(rp2, rp) and np.array_equal(col2, col)
        assert H.same_bits_or_both_nan(val2, val)
        s.set_rhs(b)
        s.run(20)
        x = s.x()
    x_ref, h_ref = H.o_conj_grad(20, rp, col, val, b)
    assert rel(x, x_ref) <= 1e-12
    # exact mode (the reference's sequential dots): bit-identical x and history
    with cgx.Solver(0, mode=cgx.CGX_MODE_EXACT) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["dia_value_stream"] == 1
        s.set_rhs(b)
        assert s.run(20) == 21
        assert H.same_bits_or_both_nan(s.x(), x_ref)
        assert H.same_bits_or_both_nan(s.history(21), h_ref)
    # CG1 (unfused on DIA-V) at a tolerance stop
    with cgx.Solver(0, alg=cgx.CGX_ALG_CG1) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        its = s.run(3000, 1e-10)
        x = s.x()
    x_o, its_o, _ = H.o_solve(3000, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its - its_o) <= 1 and rel(x, x_o) <= 1e-9
    # (-1, 2048): wider than DIA-V's widest step (two slices, no four-slice
    # kernel) -- clamped to 1,024-row chains with balanced segments (ADVICE
    # r05), not one segment per chain
    shapes = ((-1, 0), (1, 1), (100000, 0), (-1, 458), (2, 1000), (-1, 2048)) if march_plan else ((-1, 0),)
    for march, chain in shapes:
        with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
            s.set_march(march)
            s.set_sr_chain(chain)
            s.set_matrix(rp, col, val)
            info = s.info()
            assert info["dia_value_stream"] == 1
            assert info["fused"] == int(march_plan) and (info["fuse_march"] > 0) == march_plan, info
            if chain == 2048:  # segments (steps each) shorter than a whole chain (nz steps)
                assert info["fuse_march"] < shape[2], info
            for maxit in (0, 1, 2, 3, 16, 17, 18, 19, 40):  # every k % 4 at the stop
                s.set_rhs(b)
                its = s.run(maxit)
                x, h = s.x(), s.history(its)
                x_ref, its_ref, h_ref = H.o_solve(maxit, 0.0, rp, col, val, b, sr=True)
                assert its == its_ref == maxit + 1, (march, chain, maxit)
                assert rel(x, x_ref) <= 1e-10, (march, chain, maxit)
                assert np.allclose(h, h_ref, rtol=1e-6, atol=0), (march, chain, maxit)
            s.set_rhs(b)
            its = s.run(3000, 1e-10)
            x = s.x()
            x_sr, its_sr, _ = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
            x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
            assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
            assert rel(x, x_sr) <= 1e-9 and rel(x, x_hs) <= 1e-9
            out = []
            for graph in (True, False):
                s.set_rhs(b)
                s.bench_prepare(0)
                s.bench_run(35, graph=graph)
                out.append(s.x())
            assert H.same_bits_or_both_nan(out[0], out[1])


@pytest.mark.parametrize("seed", range(6))
def test_dia_v_random_patterns(seed):
    """DIA-V's encoder and kernel on random patterns: n not a multiple of 512,
    ragged and empty rows, 1-7 random offsets out to +-3000 (far diagonals,
    no plane-march plan), values drawn from a distinct-valued set with signed
    zeros, a denormal-range value and stored explicit zeros -- the layout is
    DIA-V when its bytes do not exceed DC's (else DC) and y is bit-identical
    to the oracle."""
    rng = np.random.default_rng(700 + seed)
    n = int(rng.integers(600, 7000))
    nd = int(rng.integers(1, 8))
    offs = np.sort(rng.choice(np.arange(-3000, 3001), size=nd, replace=False))
    rows = []
    for r in range(n):
        cand = r + offs
        cand = cand[(cand >= 0) & (cand < n)]
        keep = cand[rng.random(len(cand)) < 0.97] if rng.random() > 0.02 else cand[:0]
        rows.append(keep)
    rp = np.zeros(n + 1, dtype=np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.standard_normal(len(col))
    special = rng.random(len(col))
    val[special < 0.01] = -0.0
    val[(special >= 0.01) & (special < 0.02)] = 0.0
    val[(special >= 0.02) & (special < 0.025)] = 1e-310
    x = rng.standard_normal(n)
    x[rng.random(n) < 0.01] = -0.0
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        i = s.info()
        want = expect_layout(rp, col, val)
        assert i["layout_name"] == want, (i["layout_name"], want)
        if want == "dia":
            assert i["dia_value_stream"] == 1
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        rp2, col2, val2 = s.matrix()
        assert np.array_equal(rp2, rp) and np.array_equal(col2, col)
        assert H.same_bits_or_both_nan(val2, val)


def test_dia_v_layout_rules():
    """DIA-V only where it applies: a forced DC stays DC; more than 8
    diagonals (a 9-point 2-D pattern of general values) -> DC; a row whose
    columns descend -> not DIA; fp32 general coefficients -> DIA-V too; the
    partitioned solver never builds it (its ranks' kernels read value
    tables) -- every one bit-exact."""
    rng = np.random.default_rng(31)
    rp, col, val = cgx.varcoef3d(20, 18, 16, seed=2)
    n = len(rp) - 1
    x = rng.standard_normal(n)
    with cgx.Solver(0, layout="dc") as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == "dc"
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
    with cgx.Solver(0) as s:
        v32 = val.astype(np.float32)
        s.set_matrix(rp, col, v32)
        i = s.info()
        assert (i["layout_name"], i["dia_value_stream"]) == ("dia", 1)
        x32 = x.astype(np.float32)
        assert same32(s.spmv(x32), H.o_spmv_f32(rp, col, v32, x32))
        rp9, col9, val9 = banded_spd(5000, [1, 69, 70, 71], 3)
        s.set_matrix(rp9, col9, val9)
        assert s.info()["layout_name"] == expect_layout(rp9, col9, val9) == "dc"
        x9 = rng.standard_normal(5000)
        assert H.same_bits_or_both_nan(s.spmv(x9), H.o_spmv(rp9, col9, val9, x9))
        col_d = col.copy()
        col_d[rp[40]:rp[41]] = col_d[rp[40]:rp[41]][::-1]
        val_d = val.copy()
        val_d[rp[40]:rp[41]] = val_d[rp[40]:rp[41]][::-1]
        s.set_matrix(rp, col_d, val_d)
        assert s.info()["layout_name"] == expect_layout(rp, col_d, val_d) == "dc"
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col_d, val_d, x))


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


@pytest.mark.parametrize("shape", [(12, 12, 12), (40, 30, 24), (7, 5, 9), (64, 48, 10)])
def test_fused_cg1_step(shape):
    """The fused Chronopoulos-Gear step (k_cg1_dia_h: the p / s / x / r
    recurrences and w = A r_new with both partials in one launch, r / s / w
    double-buffered, replayed graphs of both parities): within 1e-9 of the
    oracle's CG1 solve (same iteration count within 1), within 1e-12 of the
    unfused CG1 iteration at fixed max_iter (the two differ only in how the
    gamma partials are grouped), every max_iter parity of the graph batches."""
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(8).standard_normal(len(rp) - 1)
    out = {}
    for fused in (True, False):
        with cgx.Solver(0, alg=cgx.CGX_ALG_CG1, layout="dia", fused=fused) as s:
            s.set_matrix(rp, col, val)
            assert s.info()["fused"] == (1 if fused else 0)
            res = []
            for maxit, tol in [(0, 0.0), (1, 0.0), (16, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]:
                s.set_rhs(b)
                its = s.run(maxit, tol)
                res.append((its, s.x()))
            out[fused] = res
    for (i0, x0), (i1, x1) in zip(out[True][:-1], out[False][:-1]):
        assert i0 == i1
        assert rel(x0, x1) <= 1e-12
    its, x = out[True][-1]
    x_o, its_o, _ = H.o_solve(3000, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its - its_o) <= 1 and its < 3000
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


def test_history_after_buffer_growth():
    """Cached hipGraphs are dropped when a longer run reallocates the r.r
    history buffer (regression: r01, the graph kept the freed pointer)."""
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
    fractions of the 8 TB/s spec."""
    t = cgx.stream_bench(0, 16 * 2**20, 3, cgx.CGX_STREAM_TRIAD)
    r = cgx.stream_bench(0, 16 * 2**20, 3, cgx.CGX_STREAM_READ)
    assert 2000.0 < t < 8000.0 and 2000.0 < r < 8000.0
    # the tuned read/write mixes, every kind through the ABI
    for name in ("copy", "copy_nt", "triad_tuned", "triad_nt", "mix33", "mix33_nt"):
        g = cgx.stream_bench(0, 16 * 2**20, 3, cgx.STREAM_KINDS[name])
        assert 2000.0 < g < 8000.0, (name, g)


def test_bench_state_dropped_on_recurrence_change():
    """bench_prepare under HS, then set_mode(FAST, SR) (whose
    second r / s / w buffers HS never allocated) -- bench_run must refuse
    (CGX_EINVAL) until the next bench_prepare, not launch on null buffers."""
    rp, col, val = cgx.laplacian3d(32, 48, 20)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(np.ones(len(rp) - 1))
        s.bench_prepare(2)
        s.bench_run(4)
        for change in (lambda: s.set_mode(cgx.CGX_MODE_FAST, cgx.CGX_ALG_SR),
                       lambda: s.set_fused(True), lambda: s.set_march(3)):
            s.set_mode(cgx.CGX_MODE_FAST, cgx.CGX_ALG_HS)
            s.set_fused("auto")
            s.set_march(-1)
            s.bench_prepare(2)
            s.bench_run(2)
            change()
            with pytest.raises(cgx.CgxError):
                s.bench_run(2)
        s.bench_prepare(2)  # prepared again (HS, march 3): runs
        s.bench_run(4)


def test_spmv_only_bench():
    """CGX_BENCH_SPMV_ONLY: back-to-back SpMVs, the iteration state untouched."""
    rp, col, val = cgx.laplacian3d(64, 64, 64)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(np.ones(len(rp) - 1))
        s.bench_prepare(2)
        ms, sp = s.bench_run(10, graph=False, spmv_events=True, spmv_only=True)
        assert ms > 0 and 0 < sp <= ms / 10 * 1.01
        ms2, _ = s.bench_run(10)
        assert ms2 > 0


# ------------------------------------------------------------ column panels

def rows_with_dense(n, dense, seed):
    """Tridiagonal band + 4 random columns per row, plus fully dense rows."""
    rng = np.random.default_rng(seed)
    r = np.repeat(np.arange(n, dtype=np.int64), 7)
    c = np.stack([np.arange(n) - 1, np.arange(n), np.arange(n) + 1] +
                 [rng.integers(0, n, n) for _ in range(4)], axis=1).reshape(-1)
    keep = (c >= 0) & (c < n)
    r, c = r[keep], c[keep]
    for d in dense:
        r = np.concatenate([r, np.full(n, d)])
        c = np.concatenate([c, np.arange(n)])
    key = np.unique(r * n + c)
    r, c = key // n, key % n
    rp = np.zeros(n + 1, np.int32)
    np.add.at(rp, r + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    return rp, c.astype(np.int32), rng.standard_normal(len(c)), rng.standard_normal(n)


def test_column_panels_bit_exact():
    """Column-panel layout: rows continue their sequential sums panel after
    panel, so SpMV stays bit-exact in fp64 and fp32, rows longer than a window
    (dense rows crossing every panel) included; CG matches the oracle."""
    rp, col, val = cgx.random_spd(600000, 9, 31)  # x: 4.8 MB, two 3.5 MiB panels
    b = np.random.default_rng(31).standard_normal(600000)
    with cgx.Solver(0, layout="panel") as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == "panel" and s.info()["n_panels"] > 1
        assert H.same_bits_or_both_nan(s.spmv(b), H.o_spmv(rp, col, val, b))
        s.set_rhs(b)
        s.run(40)
        x_ref, _ = H.o_conj_grad(40, rp, col, val, b)
        assert rel(s.x(), x_ref) <= FAST_RTOL
        rp2, col2, val2, x2 = rows_with_dense(600000, (0, 17, 599999), 9)
        s.set_matrix(rp2, col2, val2)
        assert s.info()["n_panels"] > 1
        assert H.same_bits_or_both_nan(s.spmv(x2), H.o_spmv(rp2, col2, val2, x2))
        rp32, col32, v32 = cgx.random_spd(1200000, 20, 9, f32=True)
        x32 = np.random.default_rng(2).standard_normal(1200000).astype(np.float32)
        s.set_matrix(rp32, col32, v32)
        assert s.info()["n_panels"] > 1
        assert same32(s.spmv(x32), H.o_spmv_f32(rp32, col32, v32, x32))


def test_column_panels_auto_c5():
    """C5 (random SPD, 5 M rows, fp32) selects column panels by itself and is
    bit-exact at full size; a large Laplacian does not."""
    rp, col, val = cgx.random_spd(5_000_000, 32, 42, f32=True)
    x = np.random.default_rng(3).standard_normal(len(rp) - 1).astype(np.float32)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == "panel" and s.info()["n_panels"] == 6
        assert same32(s.spmv(x), H.o_spmv_f32(rp, col, val, x))
    del rp, col, val
    rp, col, val = cgx.laplacian3d(128, 128, 128)
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["n_panels"] == 1


# ------------------------------------------- generators, stencil, big configs

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
    generator's CSR bit for bit (C3 at full size included), encoded to
    DIA-VI on the device against the stencil's pairs, and solves alike."""
    nx, ny, nz = shape
    host = cgx.laplacian3d(nx, ny, nz) if dim == 3 else cgx.laplacian2d(nx, ny)
    with cgx.Solver(0) as s:
        s.gen_laplacian(dim, nx, ny, nz)
        rp, col, val = s.matrix()
        assert np.array_equal(rp, host[0]) and np.array_equal(col, host[1])
        assert H.same_bits_or_both_nan(val, host[2])
        assert s.info()["layout_name"] == "dia"
        assert s.info()["n_dict"] == len(lap_dict(dim, nx, ny, nz))
        n = len(rp) - 1
        x = np.random.default_rng(6).standard_normal(n)
        if n <= 200_000:
            assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(*host, x))
        if n <= 2000:
            b = np.random.default_rng(4).standard_normal(n)
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
        assert s.info()["nnz"] == len(col) and s.info()["layout_name"] == "stencil"
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


@pytest.mark.parametrize("layout", ["dia", "dc", "csr"])
def test_tiled_item_order_bit_exact(layout):
    """L2-tiled work-item order for a stencil whose plane exceeds the L2
    budget (600 x 600 planes: 3 planes of x = 8.6 MB > 1.5 MiB per XCD; plain
    CSR too, its reach taken from the sampled offsets): only the order changes, so the SpMV is bit-identical to the oracle and a CG run
    stays within the fast-mode tolerance."""
    rp, col, val = cgx.laplacian3d(600, 600, 5)
    n = len(rp) - 1
    x = np.random.default_rng(8).standard_normal(n)
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(rp, col, val)
        assert s.info()["layout_name"] == layout
        assert s.info()["tile_bands"] == 6
        assert H.same_bits_or_both_nan(s.spmv(x), H.o_spmv(rp, col, val, x))
        s.set_rhs(x)
        s.run(10)
        x_ref, _ = H.o_conj_grad(10, rp, col, val, x)
        assert rel(s.x(), x_ref) <= FAST_RTOL


def test_c4_full_size_spmv_device_generated():
    """C4 at full size (400^3: 64,000,000 rows, 447,040,000 nnz -- the largest
    BASELINE config): the device-generated DIA-VI SpMV equals the matrix-free
    stencil bit for bit (the stencil is pinned to the oracle's CSR SpMV at
    small sizes by test_matrix_free_stencil_bit_exact)."""
    x = np.random.default_rng(11).standard_normal(400 ** 3)
    with cgx.Solver(0) as s:
        s.gen_laplacian(3, 400, 400, 400)
        assert s.info()["nnz"] == 447_040_000
        assert s.info()["layout_name"] == "dia" and s.info()["tile_bands"] > 0
        y = s.spmv(x)
    with cgx.Solver(0) as s:
        s.set_stencil(3, 400, 400, 400)
        y2 = s.spmv(x)
    assert H.same_bits_or_both_nan(y, y2)


def test_c4_full_size_csr_tiled_spmv():
    """C4 at full size in the reference's plain CSR (the roofline layout,
    SURVEY.md 8d): the generated CSR runs in the L2-tiled block order and its
    SpMV equals the matrix-free stencil bit for bit."""
    x = np.random.default_rng(12).standard_normal(400 ** 3)
    with cgx.Solver(0, layout="csr") as s:
        s.gen_laplacian(3, 400, 400, 400)
        i = s.info()
        assert i["layout_name"] == "csr" and i["tile_bands"] > 0
        y = s.spmv(x)
    with cgx.Solver(0) as s:
        s.set_stencil(3, 400, 400, 400)
        y2 = s.spmv(x)
    assert H.same_bits_or_both_nan(y, y2)


def test_fused_step_fp32_bit_identical_to_unfused():
    """The fused step's fp32 instances (C5's precision on a DIA matrix): x
    and the history bit-identical to the unfused fp32 iteration, and the
    solve converges."""
    rp, col, val = cgx.laplacian3d(40, 36, 30)
    v32 = val.astype(np.float32)
    b = np.random.default_rng(12).standard_normal(len(rp) - 1).astype(np.float32)
    out = []
    for fused in (True, False):
        with cgx.Solver(0, layout="dia", fused=fused) as s:
            s.set_matrix(rp, col, v32)
            assert s.info()["fused"] == (1 if fused else 0) and s.info()["dtype"] == cgx.CGX_F32
            res = []
            for maxit, tol in [(17, 0.0), (40, 0.0), (500, 1e-5)]:
                s.set_rhs(b)
                its = s.run(maxit, tol)
                res.append((its, s.x(), s.history(its)))
            out.append(res)
    for (i0, x0, h0), (i1, x1, h1) in zip(*out):
        assert i0 == i1
        assert np.array_equal(x0.view(np.uint32), x1.view(np.uint32))
        assert H.same_bits_or_both_nan(h0, h1)
    its, x, _ = out[0][-1]
    r = b.astype(np.float64) - H.o_spmv(rp, col, val, x.astype(np.float64))
    assert its < 500 and np.linalg.norm(r) <= 2e-5 * np.linalg.norm(b)
