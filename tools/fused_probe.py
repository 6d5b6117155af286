"""Fused vs unfused HS iteration time on one GPU (cgx.Solver, graph-replayed,
device-generated Laplacian), same box, same build, back to back.
  python tools/fused_probe.py [dim:nx ...]      default 3:216 3:400 (C3, C4); 2:1000 = C2"""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

for spec in sys.argv[1:] or ["3:216", "3:400"]:
    dim, nx = (int(v) for v in spec.split(":"))
    n = nx ** dim
    for fused in (True, False, True, False):
        with cgx.Solver(0, fused=fused) as s:
            s.gen_laplacian(dim, nx, nx, nx if dim == 3 else 1)
            s.set_rhs(np.ones(n))
            s.bench_prepare(5)
            ms = s.bench_run(200)[0]
            _, sp = s.bench_run(30, graph=False, spmv_events=True)
            print("%dD nx %d fused %d: %.1f us/iter, spmv launch %.1f us" %
                  (dim, nx, s.info()["fused"], 1e3 * ms / 200, 1e3 * sp), flush=True)
