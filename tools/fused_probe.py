"""Fused vs unfused HS iteration time on one GPU (cgx.Solver, graph-replayed),
C3 (216^3) and C4 (400^3): same box, same build, back to back."""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

for nx in [int(a) for a in sys.argv[1:]] or [216, 400]:
    for fused in (True, False, True, False):
        with cgx.Solver(0, fused=fused) as s:
            s.gen_laplacian(3, nx, nx, nx)
            s.set_rhs(np.ones(nx ** 3))
            s.bench_prepare(5)
            ms = s.bench_run(100)[0]
            _, sp = s.bench_run(30, graph=False, spmv_events=True)
            print("nx %d fused %d: %.1f us/iter, spmv launch %.1f us" % (nx, s.info()["fused"], 1e3 * ms / 100, 1e3 * sp), flush=True)
