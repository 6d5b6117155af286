"""Fused vs unfused HS iteration time on one GPU (cgx.Solver, graph-replayed,
device-generated Laplacian), same box, same build, back to back.
  python tools/fused_probe.py [dim:nx[:ny:nz] ...]   default 3:216 3:400 (C3, C4); 2:1000 = C2"""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

for spec in sys.argv[1:] or ["3:216", "3:400"]:
    v = [int(t) for t in spec.split(":")]
    dim, nx = v[0], v[1]
    ny, nz = (v[2], v[3]) if len(v) > 2 else (nx, nx if dim == 3 else 1)
    n = nx * ny * nz
    for fused in (True, False, True, False):
        with cgx.Solver(0, fused=fused) as s:
            s.gen_laplacian(dim, nx, ny, nz)
            s.set_rhs(np.ones(n))
            s.bench_prepare(5)
            ms = s.bench_run(200)[0]
            _, sp = s.bench_run(30, graph=False, spmv_events=True)
            print("%dD nx %d fused %d: %.1f us/iter, spmv launch %.1f us" %
                  (dim, nx, s.info()["fused"], 1e3 * ms / 200, 1e3 * sp), flush=True)
