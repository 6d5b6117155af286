"""Next rows of SURVEY.md 8f: the reader for the reference's 4-line input
format (cg.c:146-218) and the drop-in `cg` CLI (cg.c:42-85)."""
import ctypes
import gzip
import subprocess

import numpy as np
import pytest

import cgx
import helpers as H

CLI = H.REPO / "conjugate-gradient_amd" / "bin" / "cg"


def read(path, cache=None):
    A, b = cgx.lib().new_mv_struct(), cgx.lib().new_mv_struct()
    hit = ctypes.c_int(-1)
    if cache is None:
        rc = cgx.lib().cgx_read_input_file(str(path).encode(), A, b)
    else:
        rc = cgx.lib().cgx_read_input_cached(str(path).encode(), str(cache).encode(), A, b,
                                             ctypes.byref(hit))
    if rc != 0:
        return None
    a, bb = A.contents, b.contents
    rp = np.ctypeslib.as_array(a.row_ptr, shape=(a.size + 1,)).copy()
    col = np.ctypeslib.as_array(a.col_indices, shape=(max(rp[-1], 1),))[:rp[-1]].copy()
    val = np.ctypeslib.as_array(a.values, shape=(max(a.nnz, 1),))[:a.nnz].copy()
    bv = np.ctypeslib.as_array(bb.values, shape=(max(bb.size, 1),))[:bb.size].copy()
    out = dict(n=a.size, nnz=a.nnz, rp=rp, col=col, val=val, b=bv, bsize=bb.size, bnnz=bb.nnz,
               from_cache=hit.value)
    cgx.lib().cgx_free_mv_deep(A)
    cgx.lib().cgx_free_mv_deep(b)
    return out


@pytest.mark.parametrize("name", H.golden_names())
def test_reader_matches_fixture(name, tmp_path):
    src = tmp_path / f"{name}.txt"
    src.write_bytes(gzip.open(H.GOLDEN / f"{name}.txt.gz").read())
    g = H.load_golden(name)
    for _ in range(2):  # re-entrant: the reference's reader works once per process
        r = read(src)
        assert r["n"] == g["n"] and r["nnz"] == g["nnz"]
        assert r["bsize"] == r["bnnz"] == len(g["b"])
        assert np.array_equal(r["rp"], g["row_ptr"]) and np.array_equal(r["col"], g["col"])
        assert H.same_bits_or_both_nan(r["val"], g["val"])
        assert H.same_bits_or_both_nan(r["b"], g["b"])


def test_reader_edge_cases(tmp_path):
    p = tmp_path / "eof.txt"
    p.write_text("0,1\n0,1,2\n2.5,-1e-3\n1,2")  # no final newline
    r = read(p)
    assert r["n"] == 2 and list(r["b"]) == [1.0, 2.0] and list(r["val"]) == [2.5, -1e-3]
    p.write_text("0,,1\n0,2,3\n1,2,3\n4,5\n")  # empty token parses as 0 (cg.c:350)
    r = read(p)
    assert list(r["col"]) == [0, 0, 1]
    assert read(tmp_path / "missing.txt") is None


def test_reader_token_rules(tmp_path):
    """The reference's token rules (cg.c:317-350): a line ended by a newline
    has one token more than commas (empty -> 0, also after a trailing
    comma); the unterminated last line drops a trailing empty token; text
    after the fourth line is ignored."""
    p = tmp_path / "t.txt"
    p.write_text("0,1,\n0,2,3\n1,,3\n4,5,\n7,8\n")
    r = read(p)
    assert list(r["col"]) == [0, 1, 0] and list(r["val"]) == [1.0, 0.0, 3.0]
    assert list(r["b"]) == [4.0, 5.0, 0.0]
    p.write_text("0,1\n0,1,2\n1,2\n4,5,")
    assert list(read(p)["b"]) == [4.0, 5.0]
    p.write_text("0\n0,1\n\n")  # an empty third line: one 0 token; no b line
    r = read(p)
    assert list(r["val"]) == [0.0] and r["bsize"] == 0


def _big_text(n, seed):
    """A random CSR as the reference's text, lines of several MB (the
    reader's threaded chunking) with every number format %.17g writes."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 12, n)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = rng.integers(0, n, int(rp[-1]))
    val = rng.standard_normal(len(col)) * 10.0 ** rng.integers(-30, 30, len(col))
    val[::97] = 0.0
    b = rng.standard_normal(n)
    lines = [",".join(map(str, col)), ",".join(map(str, rp)),
             ",".join("%.17g" % v for v in val), ",".join("%.17g" % v for v in b)]
    return "\n".join(lines) + "\n", rp, col, val, b


def test_reader_large_lines_and_cache(tmp_path):
    """Multi-MB lines parse identically through the threaded chunks; the
    binary cache returns the same arrays without parsing, and a changed
    input invalidates it."""
    txt, rp, col, val, b = _big_text(300000, 5)
    p, c = tmp_path / "big.txt", tmp_path / "big.cgxbin"
    p.write_text(txt)
    for want_hit in (0, 1, 1):
        r = read(p, cache=c)
        assert r["from_cache"] == want_hit
        assert np.array_equal(r["rp"], rp) and np.array_equal(r["col"], col)
        assert np.array_equal(r["val"].view(np.uint64), val.view(np.uint64))
        assert np.array_equal(r["b"].view(np.uint64), b.view(np.uint64))
    r0 = read(p)
    assert np.array_equal(r0["val"].view(np.uint64), val.view(np.uint64))
    txt2, rp2, _, _, _ = _big_text(1000, 6)
    p.write_text(txt2)
    r = read(p, cache=c)
    assert r["from_cache"] == 0 and np.array_equal(r["rp"], rp2)
    assert read(tmp_path / "missing.txt", cache=c) is None


def test_reader_cache_keyed_on_content(tmp_path):
    """the cache is keyed on the text's content (a 64-bit hash of
    every byte), not on size + mtime: a rewrite with same-width numbers and
    the old timestamp restored, or another file of the same size behind the
    same cache path, is parsed again."""
    import os
    txt, rp, col, val, b = _big_text(20000, 7)
    p, c = tmp_path / "a.txt", tmp_path / "a.cgxbin"
    p.write_text(txt)
    st = os.stat(p)
    assert read(p, cache=c)["from_cache"] == 0
    assert read(p, cache=c)["from_cache"] == 1
    i = txt.index("\n") + 1  # first row_ptr entry "0" -> "1": same size
    assert txt[i] == "0"
    txt2 = txt[:i] + "1" + txt[i + 1:]
    p.write_text(txt2)
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert os.stat(p).st_size == st.st_size and os.stat(p).st_mtime_ns == st.st_mtime_ns
    r = read(p, cache=c)
    assert r["from_cache"] == 0 and r["rp"][0] == 1
    q = tmp_path / "b.txt"  # another input of the same size, same cache path
    q.write_text(txt)
    r = read(q, cache=c)
    assert r["from_cache"] == 0 and r["rp"][0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,it", [("kat_tridiag10", 4), ("lap2d_32", 25), ("dense128", 11)])
def test_cli_output_matches_reference(name, it, tmp_path):
    """Same stdout as the reference CLI: 'CG took approx %d seconds' then
    print_sparse(x) with %f values (mv_ops.c:77-95)."""
    src = tmp_path / f"{name}.txt"
    src.write_bytes(gzip.open(H.GOLDEN / f"{name}.txt.gz").read())
    out = subprocess.run([str(CLI), str(src), str(it)], capture_output=True, text=True,
                         check=True, env={**__import__("os").environ, "CGX_MODE": "exact"}).stdout
    lines = out.splitlines()
    want = H.load_golden(name)["iters"][it]
    assert lines[0].startswith("CG took approx ") and lines[0].endswith(" seconds")
    assert lines[1] == "Sparse Object:"
    assert lines[2] == f"\tSize: {len(want)}" and lines[3] == f"\tNNZ: {len(want)}"
    assert lines[4].startswith("\tValues: ")
    assert lines[5:] == ["\t%f" % v for v in want]


def test_cli_usage_and_missing_input():
    r = subprocess.run([str(CLI)], capture_output=True, text=True)
    assert r.returncode != 0 and "Usage:" in r.stderr
    r = subprocess.run([str(CLI), "/nonexistent/input.txt", "3"], capture_output=True, text=True)
    assert r.returncode != 0 and "Failed to open input file" in r.stderr
