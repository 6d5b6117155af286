#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the COMPILED REFERENCE.

The reference (rnelias/Conjugate-Gradient) ships no fixtures (.gitignore:1-3
excludes *.txt), so every golden vector is produced here:

  1. each fixture matrix is generated (seeded numpy, tests/helpers.py) and
     written in the reference's own 4-line input format (cg.c:146-218);
  2. oracle/Makefile `ref` compiles /root/reference/{cg.c,mv_ops.c} unchanged
     (reference flags `-Wall -g`) and links oracle/ref_harness.c, which calls
     the reference's read_input_file + conj_grad (cg.c:23-24) and the
     mv_ops.h op list of test_mv_ops (cg.c:368-384);
  3. the harness prints x (and op results) as C99 hex floats, stored here as
     <name>.json.gz next to the gzipped input <name>.txt.gz.

Run in the build container (the reference is not present on the GPU box):
    python tests/golden/make_golden.py
"""
from __future__ import annotations

import gzip
import json
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import helpers  # noqa: E402

HARNESS = helpers.ORACLE_DIR / "_ref" / "ref_harness"

FIXTURES = {
    # SURVEY.md 4 KATs: n = 10 tridiagonal [-1 2 -1], b = 1; max_iter 5 -> NaN
    "kat_tridiag10": dict(make=lambda: (*helpers.tridiag(10), [1.0] * 10),
                          iters=[0, 1, 2, 3, 4, 5, 6], chained=True),
    # C1 shape: dense 128 SPD, diagonally dominant, seeded
    "dense128": dict(make=lambda: helpers.dense_spd(128, seed=1),
                     iters=[0, 1, 2, 3, 5, 8, 10, 11, 15, 20, 40, 60],
                     chained=True),
    "lap2d_32": dict(make=lambda: (*helpers.laplacian2d(32, 32), [1.0] * 1024),
                     iters=[0, 1, 2, 5, 10, 25, 50, 80, 120], chained=True),
    "lap3d_12": dict(make=lambda: (*helpers.laplacian3d(12, 12, 12), [1.0] * 1728),
                     iters=[0, 1, 2, 5, 10, 20, 40, 60], chained=True),
    "rand_spd_2000": dict(make=lambda: helpers.random_spd(2000, 7, seed=7),
                          iters=[0, 1, 2, 5, 10, 20, 30], chained=True),
    # Documented divergence: diagonal matrices are not
    # chained; the reference's mat_get_row scan gives a wrong SpMV.
    "diag5_divergence": dict(
        make=lambda: (*helpers.csr_from_dense(
            __import__("numpy").diag([1.0, 2.0, 3.0, 4.0, 5.0])), [1.0] * 5),
        iters=[0, 1], chained=False),
}


def parse_blocks(text):
    out, cur, key = {}, None, None
    for line in text.splitlines():
        parts = line.split()
        if len(parts) >= 2 and not parts[0].startswith(("0x", "-0x", "nan", "-nan", "inf", "-inf")):
            key = " ".join(parts[:-1])
            cur = out.setdefault(key, [])
            continue
        v = float.fromhex(line) if "0x" in line else float(line)
        cur.append(v.hex())
    return out


def main():
    subprocess.run(["make", "-s", "-C", str(helpers.ORACLE_DIR), "ref"], check=True)
    for name, fx in FIXTURES.items():
        rp, col, val, b = fx["make"]()
        with tempfile.TemporaryDirectory() as td:
            src = Path(td) / f"{name}.txt"
            helpers.write_ref_format(src, rp, col, val, b)
            solve = subprocess.run([str(HARNESS), "solve", str(src),
                                    ",".join(map(str, fx["iters"]))],
                                   check=True, capture_output=True, text=True).stdout
            ops = subprocess.run([str(HARNESS), "ops", str(src)], check=True,
                                 capture_output=True, text=True).stdout
            with open(src, "rb") as fi, gzip.GzipFile(HERE / f"{name}.txt.gz", "wb",
                                                      mtime=0) as fo:
                fo.write(fi.read())
        blocks = parse_blocks(solve)
        golden = {
            "name": name,
            "n": len(rp) - 1,
            "nnz": len(col),
            "chained": fx["chained"],
            "source": "compiled reference: /root/reference/{cg.c,mv_ops.c} "
                      "via oracle/ref_harness.c (gcc -Wall -g)",
            "iters": {k.split()[1]: v for k, v in blocks.items()},
            "ops": {k: v for k, v in parse_blocks(ops).items()},
        }
        with gzip.GzipFile(HERE / f"{name}.json.gz", "wb", mtime=0) as f:
            f.write(json.dumps(golden).encode())
        print(f"{name}: n={golden['n']} nnz={golden['nnz']} iters={fx['iters']}")


if __name__ == "__main__":
    main()
