"""Partition layer: row ranges, ownership, ghost discovery,
local renumbering and halo send lists, checked bit-exactly against a Python
restatement, and the halo exchange checked by a simulated multi-rank SpMV
(host only, no GPU)."""
import bisect

import numpy as np
import pytest

import cgx
import helpers as H


def py_rows(n, G, g):
    return (g * n) // G, ((g + 1) * n) // G


def py_owner(n, G, c):
    begins = [py_rows(n, G, g)[0] for g in range(G)]
    return bisect.bisect_right(begins, c) - 1 if n else 0


def py_partition(n, G, g, rp, col):
    rb, re_ = py_rows(n, G, g)
    ghosts = sorted({int(c) for c in col if c < rb or c >= re_})
    pos = {c: i for i, c in enumerate(ghosts)}
    n_loc = re_ - rb
    local = [int(c) - rb if rb <= c < re_ else n_loc + pos[int(c)] for c in col]
    counts = [0] * G
    for c in ghosts:
        counts[py_owner(n, G, c)] += 1
    return ghosts, np.array(local, np.int32), counts


_MAKERS = {
    "lap3d_9x7x8": lambda: cgx.laplacian3d(9, 7, 8),
    "lap2d_40x30": lambda: cgx.laplacian2d(40, 30),
    "rand1500": lambda: cgx.random_spd(1500, 6, 5),
    "tiny5": lambda: cgx.laplacian2d(5, 1),
}
MAT_NAMES = sorted(_MAKERS)
_CACHE = {}


def mat(name):
    """Built on first use, not at import: the generators call libcgx, which
    the session fixture in conftest.py builds only after collection (a fresh
    checkout has no libcgx.so when this module is imported)."""
    if name not in _CACHE:
        _CACHE[name] = tuple(_MAKERS[name]())
    return _CACHE[name]


@pytest.mark.parametrize("n,G", [(10, 3), (64_000_000, 8), (80_621_568, 8), (7, 8),
                                 (1, 4), (2**31 - 1, 7)])
def test_rows_and_owner_64bit(n, G):
    ends = [cgx.partition_rows(n, G, g) for g in range(G)]
    assert ends == [py_rows(n, G, g) for g in range(G)]
    assert ends[0][0] == 0 and ends[-1][1] == n
    assert all(ends[g][1] == ends[g + 1][0] for g in range(G - 1))
    rng = np.random.default_rng(0)
    probes = {0, n - 1} | {int(c) for c in rng.integers(0, n, 50)}
    probes |= {e[0] for e in ends if e[0] < n} | {e[1] - 1 for e in ends if e[1] > e[0]}
    for c in probes:
        assert cgx.lib().cgx_partition_owner(n, G, c) == py_owner(n, G, c)


@pytest.mark.parametrize("name", MAT_NAMES)
@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_partition_bit_exact_vs_restatement(name, G):
    rp, col, val = mat(name)
    n = len(rp) - 1
    for g in range(G):
        rb, re_ = py_rows(n, G, g)
        lrp = rp[rb:re_ + 1] - rp[rb]
        lcol = col[rp[rb]:rp[re_]]
        P = cgx.Partition(n, G, g, lrp, lcol)
        ghosts, local, counts = py_partition(n, G, g, lrp, lcol)
        info = P.info()
        assert info["n_loc"] == re_ - rb and info["row_begin"] == rb
        assert list(P.ghosts()) == ghosts
        assert np.array_equal(P.local_cols(), local)
        assert list(P.recv_counts()) == counts


@pytest.mark.parametrize("name", MAT_NAMES)
@pytest.mark.parametrize("G", [2, 3, 5, 8])
def test_halo_exchange_reproduces_global_spmv(name, G):
    """Exchange requests between G simulated ranks, move halo values by the
    send lists, and check every rank's local SpMV against the global one bit
    for bit (same products, same order)."""
    rp, col, val = mat(name)
    n = len(rp) - 1
    x = np.random.default_rng(1).standard_normal(n)
    y_ref = H.o_spmv(rp, col, val, x)
    parts, rows = [], []
    for g in range(G):
        rb, re_ = py_rows(n, G, g)
        lrp = (rp[rb:re_ + 1] - rp[rb]).astype(np.int32)
        parts.append(cgx.Partition(n, G, g, lrp, col[rp[rb]:rp[re_]]))
        rows.append((rb, re_, lrp))
    ghosts = [p.ghosts() for p in parts]
    recv = [p.recv_counts() for p in parts]
    roff = [np.concatenate([[0], np.cumsum(r)[:-1]]) for r in recv]
    for q in range(G):  # rank q receives each rank p's request list for q
        counts = [int(recv[p][q]) for p in range(G)]
        glob = np.concatenate([ghosts[p][roff[p][q]:roff[p][q] + recv[p][q]]
                               for p in range(G)] + [np.zeros(0, np.int32)])
        parts[q].set_requests(counts, glob)
    sends = [(p.send_counts(), p.send_local()) for p in parts]
    soff = [np.concatenate([[0], np.cumsum(c)[:-1]]) for c, _ in sends]
    for g in range(G):
        rb, re_, lrp = rows[g]
        x_ext = np.concatenate([x[rb:re_], np.zeros(len(ghosts[g]))])
        for q in range(G):
            cnt = int(recv[g][q])
            if cnt == 0:
                continue
            sc, sl = sends[q]
            assert sc[g] == cnt
            xq = x[rows[q][0]:rows[q][1]]
            x_ext[re_ - rb + roff[g][q]: re_ - rb + roff[g][q] + cnt] = \
                xq[sl[soff[q][g]: soff[q][g] + cnt]]
        y = H.o_spmv(lrp, parts[g].local_cols(), val[rp[rb]:rp[re_]], x_ext)
        assert H.same_bits_or_both_nan(y, y_ref[rb:re_])


def test_partition_rejects_wrong_range():
    rp, col, _ = mat("lap2d_40x30")
    with pytest.raises(cgx.CgxError):
        cgx.Partition(len(rp) - 1, 4, 1, rp[:11] - rp[0], col[:rp[10]])


@pytest.mark.parametrize("shape,G", [((32, 48, 20), 2), ((32, 48, 20), 3), ((32, 48, 20), 8),
                                     ((64, 64, 12), 5), ((64, 64, 12), 16), ((400, 400, 8), 8)])
def test_slab_ghosts_are_neighbouring_planes(shape, G):
    """The precondition of the one-launch SR step's in-place numbering
    (cgx_dist.cpp build_inplace): on a 3-D Laplacian cut into
    row slabs at least one plane (F = nx ny rows) thick, each partition's
    ghost columns are EXACTLY the rows [row_begin - F, row_begin) and
    [row_end, row_end + F) inside [0, n) -- plane-aligned or not -- so the
    columns global - row_begin put them in place below 0 and after n_loc;
    thinner slabs leave holes (and keep the two-launch step)."""
    nx, ny, nz = shape
    F, n = nx * ny, nx * ny * nz
    for g in range(G):
        rb, re_ = cgx.partition_rows(n, G, g)
        rp, col, _ = cgx.laplacian3d(nx, ny, nz, rb, re_)
        p = cgx.Partition(n, G, g, rp, col)
        ghosts = list(p.ghosts())
        want = list(range(max(0, rb - F), rb)) + list(range(re_, min(n, re_ + F)))
        if re_ - rb >= F:
            assert ghosts == want, g
        else:
            assert set(ghosts) < set(want) and ghosts != want, g
