"""C4 partitioned-path diagnosis: x of the in-process group (P partitions,
fused / unfused HS) against the single-GPU solver at several max_iter.

  python tools/c4_diag.py [nx ny nz] [P ...]
"""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
import cgx  # noqa: E402

MAXITS = (0, 1, 2, 3, 10)


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    a = sys.argv[1:]
    nx, ny, nz = (int(v) for v in a[:3]) if len(a) >= 3 else (400, 400, 400)
    Ps = [int(v) for v in a[3:]] or [8]
    n = nx * ny * nz
    b = np.ones(n)
    ref = {}
    for fused in (True, False):
        with cgx.Solver(0, fused=fused) as s:
            s.gen_laplacian(3, nx, ny, nz)
            s.set_rhs(b)
            for m in MAXITS:
                s.run(m)
                ref[(fused, m)] = s.x()
            print(f"single fused={fused} info fused={s.info()['fused']} tile_bands={s.info()['tile_bands']}",
                  flush=True)
    for m in MAXITS:
        print(f"single m={m}: fused vs unfused rel {rel(ref[(True, m)], ref[(False, m)]):.3e}", flush=True)
    for P in Ps:
        for fused in (True, False):
            t0 = time.time()
            parts = cgx.DistSolver.local_group(0, P)
            try:
                parts[0].set_alg(cgx.CGX_ALG_HS)
                parts[0].set_fused(fused)
                for g, d in enumerate(parts):
                    rb, re_ = cgx.partition_rows(n, P, g)
                    rp, col, val = cgx.laplacian3d(nx, ny, nz, rb, re_)
                    d.set_matrix(n, rp, col, val)
                    d.set_rhs(b[rb:re_])
                for m in MAXITS:
                    parts[0].run(m, 0.0)
                    x = np.concatenate([d.x() for d in parts])
                    bad = np.nonzero(np.abs(x - ref[(False, m)]) > 1e-9 * np.abs(ref[(False, m)]).max())[0]
                    where = f"first bad row {bad[0]} ({len(bad)} rows)" if len(bad) else ""
                    print(f"P={P} fused={fused} m={m}: rel vs single {rel(x, ref[(False, m)]):.3e} {where}",
                          flush=True)
                st = [d.info() for d in parts]
                print(f"  fused flags {[s['fused'] for s in st]} layouts {[s['layout_name'] for s in st]} "
                      f"ghost {[s['n_ghost'] for s in st]} int/bnd "
                      f"{[(s['interior_items'], s['boundary_items']) for s in st]} ({time.time() - t0:.1f} s)",
                      flush=True)
            finally:
                parts[0].close()


if __name__ == "__main__":
    main()
