"""Pin the CPU oracle (oracle/cg_oracle.c) to the compiled reference.

Every golden vector in tests/golden/ was produced by the reference itself
(tests/golden/make_golden.py).  The oracle must reproduce them bit for bit
on chained matrices, and its literal dense-row restatement must reproduce the
reference's documented divergence on the non-chained diagonal case.
"""
import numpy as np
import pytest

import helpers as H

NAMES = H.golden_names()
CHAINED = [n for n in NAMES if H.load_golden(n)["chained"]]


def test_fixture_set_complete():
    assert set(NAMES) >= {"kat_tridiag10", "dense128", "lap2d_32", "lap3d_12",
                          "rand_spd_2000", "diag5_divergence"}


def test_kat_values():
    # tridiagonal n = 10, b = 1
    g = H.load_golden("kat_tridiag10")
    assert np.all(g["iters"][0] == 5.0)
    assert list(g["iters"][1]) == [5, 9, 9, 9, 9, 9, 9, 9, 9, 5]
    assert list(g["iters"][4]) == [5, 9, 12, 14, 15, 15, 14, 12, 9, 5]
    assert np.all(np.isnan(g["iters"][5]))   # beta = 0/0 at cg.c:129


@pytest.mark.parametrize("name", CHAINED)
def test_oracle_conj_grad_bit_exact(name):
    g = H.load_golden(name)
    for it, want in g["iters"].items():
        x, _ = H.o_conj_grad(it, g["row_ptr"], g["col"], g["val"], g["b"])
        assert H.same_bits_or_both_nan(x, want), (name, it)


@pytest.mark.parametrize("name", ["kat_tridiag10", "dense128", "diag5_divergence"])
def test_oracle_dense_expand_bit_exact(name):
    """The literal O(n^2) restatement matches the reference everywhere,
    including the non-chained divergence case."""
    g = H.load_golden(name)
    for it, want in g["iters"].items():
        x, _ = H.o_conj_grad(it, g["row_ptr"], g["col"], g["val"], g["b"],
                             dense_expand=True)
        assert H.same_bits_or_both_nan(x, want), (name, it)


def test_divergence_documented():
    """diag(1..5), b = 1, max_iter 0: correct CSR CG gives 1/3 (x = (rr/pAp) b),
    the reference's greedy row scan gives 1/11 = 0.0909..."""
    g = H.load_golden("diag5_divergence")
    ref = g["iters"][0]
    assert np.allclose(ref, 5.0 / 55.0)
    x, _ = H.o_conj_grad(0, g["row_ptr"], g["col"], g["val"], g["b"])
    assert np.allclose(x, 5.0 / 15.0)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_ops_bit_exact(name):
    """test_mv_ops' list (cg.c:368-384) on (A, b)."""
    g = H.load_golden(name)
    b, ops = g["b"], g["ops"]
    if g["chained"]:
        assert H.same_bits_or_both_nan(H.o_spmv(g["row_ptr"], g["col"], g["val"], b),
                                       ops["mv_mult"])
    assert H.same_bits_or_both_nan(H.o_spmv_dense(g["row_ptr"], g["col"], g["val"], b),
                                   ops["mv_mult"])
    assert H.same_bits_or_both_nan(4.0 * b, ops["sv_mult"])
    assert H.same_bits_or_both_nan([H.o_dot(b, b)], ops["dot_product"])
    assert H.same_bits_or_both_nan(b + b, ops["vec_add"])
    assert H.same_bits_or_both_nan(b - b, ops["vec_sub"])


@pytest.mark.parametrize("name", ["lap2d_32", "lap3d_12", "dense128"])
def test_oracle_solve_tol_is_prefix_of_conj_grad(name):
    """solve(tol) stops at the first k with r.r <= tol^2 b.b and returns exactly
    conj_grad(k)'s x; tol <= 0 equals conj_grad(maxit)."""
    g = H.load_golden(name)
    rp, col, val, b = g["row_ptr"], g["col"], g["val"], g["b"]
    x0, its0, _ = H.o_solve(20, 0.0, rp, col, val, b)
    xr, _ = H.o_conj_grad(20, rp, col, val, b)
    assert its0 == 21 and H.same_bits_or_both_nan(x0, xr)
    tol = 1e-6
    x, its, hist = H.o_solve(500, tol, rp, col, val, b)
    bb = H.o_dot(b, b)
    assert hist[-1] <= tol * tol * bb and np.all(hist[:-1] > tol * tol * bb)
    xk, _ = H.o_conj_grad(its - 1, rp, col, val, b)
    assert H.same_bits_or_both_nan(x, xk)


@pytest.mark.parametrize("name", ["lap2d_32", "lap3d_12", "rand_spd_2000"])
def test_oracle_cg1_matches_hs(name):
    """Chronopoulos-Gear (one reduction/iteration) agrees with HS-CG to
    rounding-level differences."""
    g = H.load_golden(name)
    rp, col, val, b = g["row_ptr"], g["col"], g["val"], g["b"]
    x1, its1, h1 = H.o_solve(400, 1e-10, rp, col, val, b)
    x2, its2, h2 = H.o_solve(400, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its1 - its2) <= 1
    assert np.linalg.norm(x1 - x2) <= 1e-8 * np.linalg.norm(x1)


def test_oracle_mt_matches_serial():
    g = H.load_golden("lap3d_12")
    rp, col, val, b = g["row_ptr"], g["col"], g["val"], g["b"]
    x1, its1, _ = H.o_solve(50, 0.0, rp, col, val, b)
    x2, its2 = H.o_solve_mt(50, 0.0, rp, col, val, b, 4)
    assert its1 == its2 == 51
    assert np.linalg.norm(x1 - x2) <= 1e-10 * np.linalg.norm(x1)


def test_oracle_f32_pinned_on_the_kats():
    """oracle_solve_f32 (C5's fp32 iteration; the reference is fp64 only,
    mv_ops.h:20) against the reference's own golden KATs: on the n = 10
    tridiagonal system every alpha, beta and iterate is a small dyadic or
    integer value, exact in float, so the fp32 iteration reproduces the
    reference's x bit for bit (as floats) for max_iter 0..4."""
    g = H.load_golden("kat_tridiag10")
    rp, col = g["row_ptr"], g["col"]
    val, b = g["val"].astype(np.float32), g["b"].astype(np.float32)
    for it in range(5):
        x, its, _ = H.o_solve_f32(it, 0.0, rp, col, val, b)
        assert its == it + 1
        assert np.array_equal(x, g["iters"][it].astype(np.float32)), it


@pytest.mark.parametrize("name", ["lap2d_32", "lap3d_12", "rand_spd_2000", "dense128"])
def test_oracle_f32_tracks_the_reference(name):
    """On the other fixtures the fp32 iteration stays within fp32 rounding of
    the reference's fp64 x (the golden vectors) for its first iterations,
    and stops at a tolerance within 1 iteration of the fp64 oracle."""
    g = H.load_golden(name)
    rp, col = g["row_ptr"], g["col"]
    val, b = g["val"].astype(np.float32), g["b"].astype(np.float32)
    for it, want in g["iters"].items():
        if it > 10:
            continue
        x, _, _ = H.o_solve_f32(it, 0.0, rp, col, val, b)
        assert np.linalg.norm(x - want) <= 1e-4 * np.linalg.norm(want), (name, it)
    x, its, hist = H.o_solve_f32(500, 1e-4, rp, col, val, b)
    _, its64, _ = H.o_solve(500, 1e-4, rp, col, g["val"], g["b"])
    assert abs(its - its64) <= 1
    assert hist[-1] <= 1e-8 * H.o_dot(g["b"], g["b"]) * 1.0001
