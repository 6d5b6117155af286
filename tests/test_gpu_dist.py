"""GPU: the partitioned solver (cgx_dist).  On one MI355X the in-process
transport runs P = 1..8 partitions with the exact phase code of the RCCL
path (halo copies + fixed-order all-reduce); RCCL itself is exercised at
world size 1 here and at N = 2/4/8 by bench.py on a full node.

Bar: x within 1e-9 (relative) of the serial oracle's Chronopoulos-Gear
solve, iteration count within 1, true residual below the tolerance."""
import numpy as np
import pytest

import cgx
import helpers as H

pytestmark = pytest.mark.gpu


def system(kind):
    if kind == "lap3d":
        rp, col, val = cgx.laplacian3d(24, 20, 30)
        b = np.ones(len(rp) - 1)
    elif kind == "lap2d":
        rp, col, val = cgx.laplacian2d(90, 70)
        b = np.random.default_rng(4).standard_normal(len(rp) - 1)
    else:
        rp, col, val = cgx.random_spd(20000, 8, 21)
        b = np.random.default_rng(5).standard_normal(20000)
    return rp, col, val, b


def solve_local(rp, col, val, b, P, maxit, tol, alg=cgx.CGX_ALG_CG1, layout="auto"):
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, P)
    try:
        parts[0].set_alg(alg)
        for g, d in enumerate(parts):
            d.set_layout(layout)
            rb, re_ = cgx.partition_rows(n, P, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]],
                         val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        its = parts[0].run(maxit, tol)
        x = np.concatenate([d.x() for d in parts])
        hist = parts[0].history(its)
        stats = [d.info() for d in parts]
    finally:
        parts[0].close()
    return x, its, hist, stats


@pytest.mark.parametrize("kind", ["lap3d", "lap2d", "rand"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_local_partitions_match_oracle(kind, P):
    rp, col, val, b = system(kind)
    x, its, hist, stats = solve_local(rp, col, val, b, P, 2000, 1e-10)
    x_ref, its_ref, hist_ref = H.o_solve(2000, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)
    m = min(len(hist), len(hist_ref)) - 2
    assert np.allclose(hist[:m], hist_ref[:m], rtol=1e-6, atol=0)
    res = b - H.o_spmv(rp, col, val, x)
    assert np.linalg.norm(res) <= 2e-10 * np.linalg.norm(b)
    if P > 1:
        assert all(s["n_ghost"] > 0 for s in stats)
        assert sum(s["n_send"] for s in stats) == sum(s["n_ghost"] for s in stats)


def test_fixed_iterations_agree_across_partition_counts():
    """tol = 0: exactly maxit+1 x-updates whatever P; P only changes the
    reduction order, so x agrees to rounding."""
    rp, col, val, b = system("lap3d")
    xs = [solve_local(rp, col, val, b, P, 60, 0.0) for P in (1, 2, 4, 8)]
    assert all(x[1] == 61 for x in xs)
    for x in xs[1:]:
        assert np.linalg.norm(x[0] - xs[0][0]) <= 1e-11 * np.linalg.norm(xs[0][0])


def test_rccl_world1():
    rp, col, val, b = system("rand")
    d = cgx.DistSolver(0, 1, 0, None)
    try:
        d.set_matrix(len(rp) - 1, rp, col, val)
        d.set_rhs(b)
        its = d.run(1000, 1e-10)
        x = d.x()
        d.bench_prepare(3)
        ms, sp = d.bench_run(5, spmv_events=True)
        assert ms > 0 and 0 < sp < ms
    finally:
        d.close()
    x_ref, its_ref, _ = H.o_solve(1000, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)


def test_local_group_bench_and_interior_split():
    rp, col, val = cgx.laplacian3d(32, 32, 64)
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, 4)
    try:
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, 4, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(np.ones(re_ - rb))
        parts[0].bench_prepare(2)
        assert parts[0].bench_run(5)[0] > 0
        st = [d.info() for d in parts]
    finally:
        parts[0].close()
    # z-slabs of 16 planes: one ghost plane per neighbour, boundary blocks
    # are the first and last plane's 64-row blocks
    # DIA slices of 512 rows: the first and last plane's 2 slices per face
    assert [s["n_ghost"] for s in st] == [1024, 2048, 2048, 1024]
    assert [s["layout_name"] for s in st] == ["dia"] * 4
    assert [s["boundary_items"] for s in st] == [2, 4, 4, 2]
    assert all(s["interior_items"] > 0 for s in st)


def test_history_after_buffer_growth():
    """A replayed graph must not keep the old history pointer when a later,
    longer run reallocates the history buffer (regression: r01)."""
    rp, col, val, b = system("lap3d")
    n = len(rp) - 1

    def fresh():
        d = cgx.DistSolver.local_group(0, 1)[0]
        d.set_matrix(n, rp, col, val)
        d.set_rhs(b)
        return d

    d = fresh()
    try:
        d.run(40)                    # captures the replay graph (short history)
        its = d.run(5000, 1e-10)     # longer history: buffer reallocated
        h = d.history(its)
    finally:
        d.close()
    d = fresh()
    try:
        its2 = d.run(5000, 1e-10)
        h2 = d.history(its2)
    finally:
        d.close()
    assert its == its2
    assert H.same_bits_or_both_nan(h, h2)


@pytest.mark.parametrize("P", [1, 2, 4])
def test_layouts_partitions_identical_in_exact_sums(P):
    """Partitions of a Laplacian keep a small set of local column offsets
    (owned rows: the stencil's; ghost columns: one more constant offset per
    face), so every part runs CSR-DC or DIA-VI like the single-GPU solver.
    With tol = 0 the layouts only change how A is stored and how the SpMV
    partials are grouped: x agrees to rounding (1e-12) across CSR, DC, DIA."""
    rp, col, val, b = system("lap3d")
    out = {}
    for layout in ("csr", "dc", "dia"):
        x, its, hist, stats = solve_local(rp, col, val, b, P, 50, 0.0, layout=layout)
        assert all(s["layout_name"] == layout for s in stats)
        if layout != "csr":
            assert all(0 < s["n_dict"] <= 21 for s in stats)  # <= 7 stencil + 7 per ghost face
            assert all(s["spmv_iter_bytes"] < s["spmv_bytes"] for s in stats)
        out[layout] = x
    for layout in ("dc", "dia"):
        assert np.linalg.norm(out[layout] - out["csr"]) <= 1e-12 * np.linalg.norm(out["csr"])


@pytest.mark.parametrize("kind", ["lap3d", "lap2d", "rand"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_hs_partitions_match_oracle(kind, P):
    """The HS recurrence across partitions (two all-reduced scalars per
    iteration, the single-GPU folded kernels): x within 1e-9 of the oracle's
    HS solve (the reference's recurrence), stop iteration within 1."""
    rp, col, val, b = system(kind)
    x, its, hist, stats = solve_local(rp, col, val, b, P, 2000, 1e-10, alg=cgx.CGX_ALG_HS)
    x_ref, its_ref, hist_ref = H.o_solve(2000, 1e-10, rp, col, val, b)
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)
    m = min(len(hist), len(hist_ref)) - 2
    assert np.allclose(hist[:m], hist_ref[:m], rtol=1e-6, atol=0)
    res = b - H.o_spmv(rp, col, val, x)
    assert np.linalg.norm(res) <= 2e-10 * np.linalg.norm(b)


def test_hs_single_part_identical_to_solver():
    """One partition, no transport: the HS recurrence runs the single-GPU
    solver's kernels with the same grids, so x and the r.r history are
    bit-identical to cgx.Solver's."""
    rp, col, val, b = system("lap3d")
    x, its, hist, _ = solve_local(rp, col, val, b, 1, 40, 0.0, alg=cgx.CGX_ALG_HS)
    d = cgx.DistSolver(0, 1, 0, None)
    try:
        d.set_alg(cgx.CGX_ALG_HS)
        d.set_matrix(len(rp) - 1, rp, col, val)
        d.set_rhs(b)
        its2 = d.run(40)
        x2 = d.x()
    finally:
        d.close()
    with cgx.Solver(0) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        its3 = s.run(40)
        x3 = s.x()
        h3 = s.history(41)
    assert its == its2 == its3 == 41
    assert H.same_bits_or_both_nan(x, x3)
    assert H.same_bits_or_both_nan(x2, x3)
    assert H.same_bits_or_both_nan(hist, h3[:len(hist)])


def test_hs_fixed_iterations_and_bench():
    rp, col, val, b = system("lap3d")
    xs = [solve_local(rp, col, val, b, P, 60, 0.0, alg=cgx.CGX_ALG_HS) for P in (1, 2, 4)]
    assert all(x[1] == 61 for x in xs)
    for x in xs[1:]:
        assert np.linalg.norm(x[0] - xs[0][0]) <= 1e-11 * np.linalg.norm(xs[0][0])
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, 3)
    try:
        parts[0].set_alg(cgx.CGX_ALG_HS)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, 3, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        parts[0].bench_prepare(2)
        ms, sp = parts[0].bench_run(5, spmv_events=True)
        assert ms > 0 and 0 < sp < ms
    finally:
        parts[0].close()


@pytest.mark.parametrize("alg", [cgx.CGX_ALG_CG1, cgx.CGX_ALG_HS])
def test_rccl_one_rank_communicator(alg):
    """A 1-rank RCCL communicator (an id at world size 1) runs the multi-GPU
    phase code on one GPU: pack, grouped send/recv loop (no peers), local
    sums by the producing kernels' last workgroups, ncclAllReduce, scalar
    steps -- replayed as a hipGraph (RCCL calls captured) and eagerly, the
    two bit-identical.  Bit-identical to the in-process 1-partition group
    (the same phases with a fixed-order group sum), within tolerance of the
    oracle."""
    rp, col, val, b = system("lap3d")
    n = len(rp) - 1
    res = {}
    for graph in (True, False):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(alg)
            d.set_graph(graph)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            its = d.run(500, 1e-10)
            x = d.x()
            h = d.history(its)
            assert d.info()["graph"] == (1 if graph else 0)
            d.bench_prepare(2)
            ms, sp = d.bench_run(5, spmv_events=True)
            assert ms > 0 and 0 < sp < ms
            ms2, _ = d.bench_run(32, graph=graph)
            assert ms2 > 0
        finally:
            d.close()
        res[graph] = (its, x, h)
    assert res[True][0] == res[False][0]
    assert H.same_bits_or_both_nan(res[True][1], res[False][1])
    assert H.same_bits_or_both_nan(res[True][2], res[False][2])
    its, x, _ = res[True]
    x1, its1, _, _ = solve_local(rp, col, val, b, 1, 500, 1e-10, alg=alg)
    assert its == its1
    assert H.same_bits_or_both_nan(x, x1)
    x_ref, its_ref, _ = H.o_solve(500, 1e-10, rp, col, val, b, cg1=alg == cgx.CGX_ALG_CG1)
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)


def test_local_group_sums_match_solver_bit_exact():
    """One in-process partition WITH the transport phases: the local sums are
    the SpMV's / k_update_rf's last-arriver canonical sums (cgx_kernels.hip
    canon_sum), fed to the same folded kernels through a one-value
    all-reduce.  x and the history are bit-identical to cgx.Solver, whose
    folded kernels sum the partials directly (sum_parts<1024>): the in-kernel
    local sums reproduce the finalize order exactly, in every layout."""
    rp, col, val, b = system("lap3d")
    for layout in ("csr", "dc", "dia"):
        x, its, hist, _ = solve_local(rp, col, val, b, 1, 40, 0.0, alg=cgx.CGX_ALG_HS,
                                      layout=layout)
        with cgx.Solver(0, layout=layout) as s:
            s.set_matrix(rp, col, val)
            s.set_rhs(b)
            assert s.run(40) == its == 41
            assert H.same_bits_or_both_nan(x, s.x()), layout
            assert H.same_bits_or_both_nan(hist, s.history(41)), layout


def solve_local_fz(rp, col, val, b, P, runs, fused):
    """A local HS group with the fused step on or off; (its, x, hist) per
    (maxit, tol) of `runs`, and the partitions' stats."""
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, P)
    out = []
    try:
        parts[0].set_alg(cgx.CGX_ALG_HS)
        parts[0].set_fused(fused)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, P, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        for maxit, tol in runs:
            its = parts[0].run(maxit, tol)
            out.append((its, np.concatenate([d.x() for d in parts]), parts[0].history(its)))
        stats = [d.info() for d in parts]
    finally:
        parts[0].close()
    return out, stats


@pytest.mark.parametrize("shape,P", [((24, 20, 30), 1), ((24, 20, 30), 2), ((24, 20, 30), 3),
                                     ((24, 20, 30), 8), ((40, 30, 16), 2), ((40, 30, 16), 4),
                                     ((40, 30, 24), 8)])
def test_fused_partitions_bit_identical_to_unfused(shape, P):
    """The fused partitioned HS step (halo of p_new = r + beta p_old packed
    at the send rows, k_spmv_dia_h over interior then boundary items, ghost
    diagonals reading the received p_new, x every other iteration) computes
    every value of the unfused phases with the same roundings: x, the
    iteration count and the history are bit-identical at every partition
    count (24x20x30: +-nx*ny near, read through the LDS window, partitions
    cutting planes at P = 8; 40x30x16 / x24: +-1200 far, plane-aligned slabs
    of >= 3 planes with four far diagonals including the ghost faces, as
    C4's 400^3 slabs)."""
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(3).standard_normal(len(rp) - 1)
    runs = [(0, 0.0), (1, 0.0), (16, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]
    fz, st_f = solve_local_fz(rp, col, val, b, P, runs, True)
    uf, st_u = solve_local_fz(rp, col, val, b, P, runs, False)
    assert all(s["fused"] == 1 for s in st_f) and all(s["layout_name"] == "dia" for s in st_f)
    assert all(s["fused"] == 0 for s in st_u)
    for j, ((i0, x0, h0), (i1, x1, h1)) in enumerate(zip(fz, uf)):
        assert i0 == i1, j
        assert H.same_bits_or_both_nan(x0, x1), j
        assert H.same_bits_or_both_nan(h0, h1), j
    its, x, _ = fz[-1]
    assert its < 3000
    assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 1.01e-10 * np.linalg.norm(b)


def test_fused_rccl_one_rank_graph_parity():
    """The fused step through a 1-rank RCCL communicator: replayed graphs of
    both p-buffer parities (odd batch remainders) and eager launches give
    bit-identical x; equal to the unfused communicator's."""
    rp, col, val = cgx.laplacian3d(24, 20, 30)
    b = np.random.default_rng(6).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for fused, graph in ((True, True), (True, False), (False, True)):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(cgx.CGX_ALG_HS)
            d.set_fused(fused)
            d.set_graph(graph)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            out = []
            for maxit in (17, 33, 40):
                its = d.run(maxit, 0.0)
                out.append((its, d.x(), d.history(its)))
            its = d.run(3000, 1e-10)
            out.append((its, d.x(), d.history(its)))
            assert d.info()["fused"] == (1 if fused else 0)
            assert d.info()["graph"] == (1 if graph else 0)
        finally:
            d.close()
        res[(fused, graph)] = out
    for key in ((True, False), (False, True)):
        for (i0, x0, h0), (i1, x1, h1) in zip(res[(True, True)], res[key]):
            assert i0 == i1
            assert H.same_bits_or_both_nan(x0, x1), key
            assert H.same_bits_or_both_nan(h0, h1), key


@pytest.mark.parametrize("shape,P", [((24, 20, 30), 1), ((24, 20, 30), 3), ((24, 20, 30), 8),
                                     ((40, 30, 16), 2), ((40, 30, 24), 8)])
def test_fused_cg1_partitions(shape, P):
    """The fused CG1 step across partitions (halo of r_new = r - alpha (w +
    beta s) packed at the send rows, k_cg1_dia_h over interior then
    boundary items, ghost diagonals reading the received r_new, ONE
    all-reduce of (gamma, delta) per iteration): within 1e-9 of the oracle's
    CG1 solve, stop iteration within 1, and within 1e-12 of the unfused
    partitioned CG1 at fixed max_iter."""
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(13).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for fused in (True, False):
        parts = cgx.DistSolver.local_group(0, P)
        try:
            parts[0].set_alg(cgx.CGX_ALG_CG1)
            parts[0].set_fused(fused)
            for g, d in enumerate(parts):
                rb, re_ = cgx.partition_rows(n, P, g)
                d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
                d.set_rhs(b[rb:re_])
            out = []
            for maxit, tol in [(0, 0.0), (1, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]:
                its = parts[0].run(maxit, tol)
                out.append((its, np.concatenate([d.x() for d in parts])))
            assert all(d.info()["fused"] == (1 if fused else 0) for d in parts)
        finally:
            parts[0].close()
        res[fused] = out
    for (i0, x0), (i1, x1) in zip(res[True][:-1], res[False][:-1]):
        assert i0 == i1
        assert np.linalg.norm(x0 - x1) <= 1e-12 * np.linalg.norm(x1)
    its, x = res[True][-1]
    x_ref, its_ref, _ = H.o_solve(3000, 1e-10, rp, col, val, b, cg1=True)
    assert abs(its - its_ref) <= 1 and its < 3000
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)


def test_fused_cg1_rccl_one_rank_graph_parity():
    """The fused CG1 step through a 1-rank RCCL communicator: replayed graphs
    of both buffer parities and eager launches bit-identical."""
    rp, col, val = cgx.laplacian3d(24, 20, 30)
    b = np.random.default_rng(14).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for graph in (True, False):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(cgx.CGX_ALG_CG1)
            d.set_fused(True)
            d.set_graph(graph)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            out = []
            for maxit in (17, 33, 40):
                its = d.run(maxit, 0.0)
                out.append((its, d.x()))
            its = d.run(3000, 1e-10)
            out.append((its, d.x()))
            assert d.info()["fused"] == 1 and d.info()["graph"] == (1 if graph else 0)
        finally:
            d.close()
        res[graph] = out
    for (i0, x0), (i1, x1) in zip(res[True], res[False]):
        assert i0 == i1
        assert H.same_bits_or_both_nan(x0, x1)


def _sr_group(rp, col, val, b, P, runs, alg=cgx.CGX_ALG_SR, fused="auto", layout="auto",
              march=-1, chain=0):
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, P)
    out = []
    try:
        parts[0].set_alg(alg)
        parts[0].set_fused(fused)
        parts[0].set_march(march)
        parts[0].set_sr_chain(chain)
        for g, d in enumerate(parts):
            d.set_layout(layout)
            rb, re_ = cgx.partition_rows(n, P, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        for maxit, tol in runs:
            its = parts[0].run(maxit, tol)
            out.append((its, np.concatenate([d.x() for d in parts]), parts[0].history(its)))
        stats = [d.info() for d in parts]
    finally:
        parts[0].close()
    return out, stats


@pytest.mark.parametrize("shape,P", [((24, 20, 30), 1), ((24, 20, 30), 2), ((24, 20, 30), 3),
                                     ((24, 20, 30), 8), ((40, 30, 16), 2), ((40, 30, 16), 4),
                                     ((40, 30, 24), 8)])
def test_sr_partitions(shape, P):
    """CGX_ALG_SR, the fused HS step with ONE reduction of (p.s, s.s, r.r)
    per iteration (beta and the stop test from alpha^2 s.s - r.r): the fused
    step runs under AUTO even on these cache-resident sizes (SR has no
    unfused form); within 1e-9 of oracle_solve_sr (the restated variant) and
    of the HS oracle, stop iteration within 1 of both, true residual below
    the tolerance; at fixed max_iter within 1e-10 of the fused HS group (the
    recurrences differ only in how r_new.r_new is formed)."""
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(23).standard_normal(len(rp) - 1)
    runs = [(0, 0.0), (1, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]
    sr, st = _sr_group(rp, col, val, b, P, runs)
    hs, _ = _sr_group(rp, col, val, b, P, runs, alg=cgx.CGX_ALG_HS, fused="on")
    assert all(s["fused"] == 1 and s["alg"] == cgx.CGX_ALG_SR for s in st)
    for (i0, x0, _), (i1, x1, _) in zip(sr[:-1], hs[:-1]):
        assert i0 == i1
        assert np.linalg.norm(x0 - x1) <= 1e-10 * np.linalg.norm(x1)
    its, x, hist = sr[-1]
    x_sr, its_sr, hist_sr = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
    x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
    assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
    assert np.linalg.norm(x - x_sr) <= 1e-9 * np.linalg.norm(x_sr)
    assert np.linalg.norm(x - x_hs) <= 1e-9 * np.linalg.norm(x_hs)
    m = min(len(hist), len(hist_sr)) - 2
    assert np.allclose(hist[:m], hist_sr[:m], rtol=1e-6, atol=0)
    assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 2e-10 * np.linalg.norm(b)


SR1_CASES = [((32, 48, 20), 1), ((32, 48, 20), 2), ((32, 48, 20), 3), ((32, 48, 20), 8),
             ((64, 64, 12), 2), ((64, 64, 12), 5), ((64, 64, 12), 8), ((64, 64, 12), 16),
             ((300, 7, 20), 4), ((41, 25, 20), 3), ((41, 25, 20), 4)]


@pytest.mark.parametrize("shape,P", SR1_CASES)
def test_sr_one_launch_partitions(shape, P):
    """CGX_ALG_SR on partitioned ranks as ONE k_sr1_dia_m step
    per iteration -- the ranks' rows in the in-place numbering (ghost planes
    below 0 and from n_loc), every step marched while the halo of p_k is in
    flight, s of the edge rows recomputed after it (k_sr1_edge) -- on
    plane-aligned and
    plane-cutting slabs, odd planes and odd slabs (41 x 25: F = 1,025, 5,125
    rows per part at P = 4, both edge bounds rounded to row pairs), and thin
    slabs (P = 8 at 32 x 48 x 20: 2.5 planes per
    part; P = 16 at 64 x 64 x 12: 0.75 of a plane, whose ghost rows are not
    contiguous, so it runs the two-launch step -- to the same oracle bars).
    Against the two-launch fused SR group (set_march(0)) within 1e-10 at
    fixed max_iter (the same recurrence, the dot products grouped otherwise)
    where the slabs allow that step (plane-aligned); against oracle_solve_sr
    within 1e-10 at fixed max_iter and within 1e-9 with the stop iteration
    within 1 (and of the HS oracle) at a tolerance, true residual below it;
    segment lengths 1, 3 and auto (balanced) and chain widths (a quarter step,
    458 rows) within 1e-12 of each other."""
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(27).standard_normal(len(rp) - 1)
    runs = [(0, 0.0), (1, 0.0), (2, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]
    one, st1 = _sr_group(rp, col, val, b, P, runs)
    # in place needs each side's ghost rows contiguous: a slab at least one
    # plane thick (thinner ones, P = 16 here, run the two-launch fused step)
    thick = (len(rp) - 1) // P >= shape[0] * shape[1]
    assert all(s["march"] > 0 and s["inplace"] == 1 and s["fused"] == 1 if thick
               else s["march"] == 0 and s["fused"] == 1 for s in st1), \
        [(s["march"], s["inplace"], s["fused"], s["layout_name"]) for s in st1]
    try:  # a plane-cutting slab has > 4 far (ghost) diagonals: no two-launch SR
        two, st2 = _sr_group(rp, col, val, b, P, runs, march=0)
    except cgx.CgxError as e:
        assert "fused DIA step" in str(e)
        two = None
    if two is not None:
        for (i0, x0, _), (i1, x1, _) in zip(one[:-1], two[:-1]):
            assert i0 == i1
            assert np.linalg.norm(x0 - x1) <= 1e-10 * np.linalg.norm(x1), i0
        assert abs(one[-1][0] - two[-1][0]) <= 1
    its, x, hist = one[-1]
    x_sr, its_sr, hist_sr = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
    x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
    assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
    assert np.linalg.norm(x - x_sr) <= 1e-9 * np.linalg.norm(x_sr)
    for (i0, x0, _), (maxit, _) in zip(one[:-1], runs[:-1]):
        x_o, _, _ = H.o_solve(maxit, 0.0, rp, col, val, b, sr=True)
        assert i0 == maxit + 1 and np.linalg.norm(x0 - x_o) <= 1e-10 * np.linalg.norm(x_o)
    m = min(len(hist), len(hist_sr))
    assert np.allclose(hist[:m], hist_sr[:m], rtol=1e-6, atol=0)
    assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 2e-10 * np.linalg.norm(b)
    # segment lengths, and chain widths (round 5: the narrowest, a quarter
    # step, with a ragged last chain; a width not a multiple of 64 rows)
    for march, chain in ((1, 0), (3, 0), (1, 1), (-1, 458)):
        seg, _ = _sr_group(rp, col, val, b, P, runs[:-1], march=march, chain=chain)
        for (i0, x0, _), (i1, x1, _) in zip(seg, one[:-1]):
            assert i0 == i1
            assert np.linalg.norm(x0 - x1) <= 1e-12 * np.linalg.norm(x1), (march, chain, i0)


def test_sr_one_launch_rccl_one_rank_graph_parity():
    """The one-launch SR step through a 1-rank RCCL communicator (FIN_SUM3,
    the all-reduce of three doubles, FIN_SR1 in the replayed graphs), eager,
    and without a communicator (FIN_SR1 on the partials, as the single-GPU
    solver): bit-identical x, iteration counts and histories; and the
    single-GPU solver's SR within 1e-12 (its partials are grouped otherwise)."""
    rp, col, val = cgx.laplacian3d(32, 48, 20)
    b = np.random.default_rng(25).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for key in (("rccl", True), ("rccl", False), ("solo", True)):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id() if key[0] == "rccl" else None)
        try:
            d.set_alg(cgx.CGX_ALG_SR)
            d.set_graph(key[1])
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            out = []
            for maxit in (17, 33, 40):
                its = d.run(maxit, 0.0)
                out.append((its, d.x(), d.history(its)))
            its = d.run(3000, 1e-10)
            out.append((its, d.x(), d.history(its)))
            i = d.info()
            assert i["fused"] == 1 and i["march"] > 0 and i["alg"] == cgx.CGX_ALG_SR
        finally:
            d.close()
        res[key] = out
    for key in (("rccl", False), ("solo", True)):
        for (i0, x0, h0), (i1, x1, h1) in zip(res[("rccl", True)], res[key]):
            assert i0 == i1
            assert H.same_bits_or_both_nan(x0, x1), key
            assert H.same_bits_or_both_nan(h0, h1), key
    with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
        s.set_matrix(rp, col, val)
        s.set_rhs(b)
        for (its, x, _), maxit in zip(res[("solo", True)], (17, 33, 40)):
            assert s.run(maxit) == its
            assert np.linalg.norm(s.x() - x) <= 1e-12 * np.linalg.norm(x)


@pytest.mark.parametrize("alg", [cgx.CGX_ALG_SR, cgx.CGX_ALG_HS])
def test_capture_refusal_is_collective(alg):
    """Graph or eager is decided by all ranks together (ensure_graphs: the
    capture results MIN- and MAX-all-reduced).  On a 1-rank RCCL
    communicator: a capture refused before any RCCL call was recorded (mode
    1), or after the iteration's RCCL calls were (mode 2) -- every rank
    refused at the same point -- drops the graphs and runs eager, with x,
    iteration counts and histories bit-identical to the replayed graphs; a
    mix of ranks that recorded RCCL calls and ranks that did not (mode 3:
    this rank refused after recording, its peers taken to have captured)
    fails with CGX_ECOMM and leaves the communicator unusable (no eager run
    on a possibly desynchronised comm)."""
    rp, col, val = cgx.laplacian3d(32, 48, 20)
    b = np.random.default_rng(31).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for mode in (0, 1, 2):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(alg)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            if mode:
                d.debug_refuse_capture(mode)
            out = []
            for maxit in (17, 40):
                its = d.run(maxit, 0.0)
                out.append((its, d.x(), d.history(its)))
            its = d.run(3000, 1e-10)
            out.append((its, d.x(), d.history(its)))
            assert d.info()["graph"] == (1 if mode == 0 else -1), mode
        finally:
            d.close()
        res[mode] = out
    for mode in (1, 2):
        for (i0, x0, h0), (i1, x1, h1) in zip(res[0], res[mode]):
            assert i0 == i1, mode
            assert H.same_bits_or_both_nan(x0, x1), mode
            assert H.same_bits_or_both_nan(h0, h1), mode
    d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
    try:
        d.set_alg(alg)
        d.set_matrix(n, rp, col, val)
        d.set_rhs(b)
        d.debug_refuse_capture(3)
        with pytest.raises(cgx.CgxError, match="RCCL calls were recorded"):
            d.run(17, 0.0)
        d.debug_refuse_capture(0)
        with pytest.raises(cgx.CgxError, match="unusable"):
            d.run(17, 0.0)
    finally:
        d.close()


def test_sr_rccl_one_rank_graph_parity():
    """SR through a 1-rank RCCL communicator (the all-reduce of three doubles
    in the replayed graphs), eager, and without a communicator (local sums
    straight into k_update_rf): bit-identical x, iteration counts and
    histories."""
    rp, col, val = cgx.laplacian3d(24, 20, 30)
    b = np.random.default_rng(24).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    res = {}
    for key in (("rccl", True), ("rccl", False), ("solo", True)):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id() if key[0] == "rccl" else None)
        try:
            d.set_alg(cgx.CGX_ALG_SR)
            d.set_graph(key[1])
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            out = []
            for maxit in (17, 33, 40):
                its = d.run(maxit, 0.0)
                out.append((its, d.x(), d.history(its)))
            its = d.run(3000, 1e-10)
            out.append((its, d.x(), d.history(its)))
            i = d.info()
            assert i["fused"] == 1 and i["alg"] == cgx.CGX_ALG_SR
        finally:
            d.close()
        res[key] = out
    for key in (("rccl", False), ("solo", True)):
        for (i0, x0, h0), (i1, x1, h1) in zip(res[("rccl", True)], res[key]):
            assert i0 == i1
            assert H.same_bits_or_both_nan(x0, x1), key
            assert H.same_bits_or_both_nan(h0, h1), key


@pytest.mark.parametrize("layout,fused,P", [("csr", "auto", 1), ("csr", "auto", 2),
                                            ("dc", "auto", 3), ("auto", "off", 2),
                                            ("csr", "auto", 8)])
def test_sr_unfused_partitions(layout, fused, P):
    """CGX_ALG_SR on ranks whose layout takes no fused step
    (CSR, DC, CGX_FUSE_OFF) runs the unfused SR step -- the SpMV's (p.s, s.s)
    pairs, ONE all-reduce of (p.s, s.s, r.r) per iteration, k_update_sr with
    p in place and x every iteration -- within 1e-10 of oracle_solve_sr at
    fixed max_iter, and at a 1e-10 stop the iteration count within 1 of it
    and of the HS oracle, x within 1e-9, true residual below the tolerance."""
    rp, col, val = cgx.laplacian3d(24, 20, 30)
    b = np.random.default_rng(31).standard_normal(len(rp) - 1)
    runs = [(0, 0.0), (1, 0.0), (2, 0.0), (17, 0.0), (3000, 1e-10)]
    out, st = _sr_group(rp, col, val, b, P, runs, layout=layout, fused=fused)
    assert all(s["alg"] == cgx.CGX_ALG_SR and s["fused"] == 0 and s["march"] == 0 for s in st)
    for (maxit, _), (its, x, hist) in zip(runs[:-1], out[:-1]):
        x_sr, its_sr, h_sr = H.o_solve(maxit, 0.0, rp, col, val, b, sr=True)
        assert its == its_sr == maxit + 1
        assert np.linalg.norm(x - x_sr) <= 1e-10 * np.linalg.norm(x_sr), maxit
        assert np.allclose(hist, h_sr[:its], rtol=1e-8, atol=0)
    its, x, _ = out[-1]
    x_sr, its_sr, _ = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
    x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
    assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
    assert np.linalg.norm(x - x_sr) <= 1e-9 * np.linalg.norm(x_sr)
    assert np.linalg.norm(x - x_hs) <= 1e-9 * np.linalg.norm(x_hs)
    assert np.linalg.norm(b - H.o_spmv(rp, col, val, x)) <= 2e-10 * np.linalg.norm(b)


@pytest.mark.parametrize("P", [1, 2, 3])
def test_sr_one_launch_partitions_general_coefficients(P):
    """Round 5: general coefficients (cgx_gen_varcoef3d, every value distinct)
    on partitioned ranks run the one-launch SR step too -- each rank's
    in-place matrix is DIA-V (values streamed beside a presence byte per row),
    k_sr1_dia_m<..., DV> marches the slab and k_sr1_edge reads the values of
    the edge rows.  Against oracle_solve_sr within 1e-10 at fixed max_iter
    (every residue of the depth-4 x deferral at the stop) and within 1e-9 with
    the stop iteration within 1 (and of the HS oracle) at a tolerance."""
    rp, col, val = cgx.varcoef3d(32, 48, 20, seed=9)
    b = np.random.default_rng(41).standard_normal(len(rp) - 1)
    runs = [(0, 0.0), (1, 0.0), (2, 0.0), (17, 0.0), (40, 0.0), (3000, 1e-10)]
    out, st = _sr_group(rp, col, val, b, P, runs)
    assert all(s["march"] > 0 and s["inplace"] == 1 and s["fused"] == 1 for s in st), \
        [(s["march"], s["inplace"], s["fused"], s["layout_name"]) for s in st]
    for (its, x, _), (maxit, tol) in zip(out[:-1], runs[:-1]):
        x_sr, its_sr, _ = H.o_solve(maxit, tol, rp, col, val, b, sr=True)
        assert its == its_sr == maxit + 1, (maxit, its, its_sr)
        assert np.linalg.norm(x - x_sr) <= 1e-10 * np.linalg.norm(x_sr), maxit
    its, x, _ = out[-1]
    x_sr, its_sr, _ = H.o_solve(3000, 1e-10, rp, col, val, b, sr=True)
    x_hs, its_hs, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
    assert abs(its - its_sr) <= 1 and abs(its - its_hs) <= 1 and its < 3000
    assert np.linalg.norm(x - x_sr) <= 1e-9 * np.linalg.norm(x_sr)
    assert np.linalg.norm(x - x_hs) <= 1e-9 * np.linalg.norm(x_hs)


def test_sr_one_launch_rccl_one_rank_general_coefficients():
    """The same over a 1-rank RCCL communicator (pack, all-reduce, the sums
    applied privately), graph-replayed and eager bit-identical, within 1e-10
    of oracle_solve_sr."""
    rp, col, val = cgx.varcoef3d(32, 48, 20, seed=13)
    n = len(rp) - 1
    b = np.random.default_rng(5).standard_normal(n)
    res = {}
    for graph in (True, False):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(cgx.CGX_ALG_SR)
            d.set_graph(graph)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            its = d.run(25)
            i = d.info()
            assert i["fused"] == 1 and i["march"] > 0 and i["inplace"] == 1, i
            res[graph] = (its, d.x())
        finally:
            d.close()
    assert res[True][0] == res[False][0] == 26
    assert H.same_bits_or_both_nan(res[True][1], res[False][1])
    x_sr, _, _ = H.o_solve(25, 0.0, rp, col, val, b, sr=True)
    assert np.linalg.norm(res[True][1] - x_sr) <= 1e-10 * np.linalg.norm(x_sr)


def test_sr_unfused_rccl_one_rank_graph_parity():
    """The unfused SR step over a 1-rank RCCL communicator (every transport
    phase: pack, all-reduce of the three sums, the privately applied scalar
    step) graph-replayed and eager, bit-identical, within 1e-10 of
    oracle_solve_sr."""
    rp, col, val = cgx.varcoef3d(30, 20, 16, seed=5)
    n = len(rp) - 1
    b = np.random.default_rng(3).standard_normal(n)
    res = {}
    for graph in (True, False):
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
        try:
            d.set_alg(cgx.CGX_ALG_SR)
            d.set_layout("csr")
            d.set_graph(graph)
            d.set_matrix(n, rp, col, val)
            d.set_rhs(b)
            its = d.run(25)
            assert d.info()["fused"] == 0
            res[graph] = (its, d.x())
        finally:
            d.close()
    assert res[True][0] == res[False][0] == 26
    assert H.same_bits_or_both_nan(res[True][1], res[False][1])
    x_sr, _, _ = H.o_solve(25, 0.0, rp, col, val, b, sr=True)
    assert np.linalg.norm(res[True][1] - x_sr) <= 1e-10 * np.linalg.norm(x_sr)


def test_fuse_refusal_reported_for_plane_cutting_partitions():
    """slabs that do not start on a plane boundary add ghost
    diagonals, so some partition's layout cannot take the fused step and the
    group runs unfused -- now reported per partition (fuse_status: the
    partition's own reason, or PEER when another partition refused), and
    the result still matches the oracle."""
    rp, col, val = cgx.laplacian3d(40, 30, 16)
    n = len(rp) - 1
    b = np.random.default_rng(15).standard_normal(n)
    P = 7
    parts = cgx.DistSolver.local_group(0, P)
    try:
        parts[0].set_alg(cgx.CGX_ALG_HS)
        parts[0].set_fused(True)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, P, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        its = parts[0].run(3000, 1e-10)
        x = np.concatenate([d.x() for d in parts])
        st = [d.info() for d in parts]
    finally:
        parts[0].close()
    assert all(s["fused"] == 0 for s in st)
    codes = [s["fuse_status"] for s in st]
    own = {cgx.CGX_FUSE_STATUS_NOT_DIA, cgx.CGX_FUSE_STATUS_WIDE_CODES,
           cgx.CGX_FUSE_STATUS_FAR_DIAGS}
    assert any(c in own for c in codes), codes
    assert all(c in own | {cgx.CGX_FUSE_STATUS_PEER} for c in codes), codes
    x_ref, its_ref, _ = H.o_solve(3000, 1e-10, rp, col, val, b)
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)


def test_capture_fork_join_shape():
    """The multi-rank iteration's stream shape (phase_pack / phase_halo /
    phase_spmv: fork of the communication stream by an event, pack + copy
    on it, join by an event before the boundary kernel) captured as a
    hipGraph with real work on the forked stream -- the shape a 1-rank
    communicator cannot produce (no peers, no fork) -- replayed bit-identical
    to eager (tests/native/capture_fork.hip)."""
    import subprocess
    exe = H.REPO / "conjugate-gradient_amd" / "bin" / "capture_fork"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-identical" in r.stdout


def test_bench_dist_path_rehearsal(tmp_path):
    """bench.py's N > 1 path at one rank (torch.distributed.run, a 1-rank
    RCCL communicator): the parity gate (HS, fused HS, CG1 against the
    single-GPU solve) passes and the timed line is well formed."""
    import json
    import os
    import socket
    import subprocess
    import sys
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(H.REPO / "bench.py"),
           "--gpus", "1", "--dist-rehearsal", "--workload", "c3", "--steps", "10", "--warmup", "2"]
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["parity"]["ok"] and set(line["parity"]) >= {"hs", "hs_fused", "sr", "cg1"}
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["config"]["fused"] in (0, 1)
