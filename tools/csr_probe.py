"""In-iteration CSR SpMV, alternating, one box: bench.py's solver_leg
(graph-replayed CG it/s, HIP-event SpMV launch average, back-to-back SpMV).
  python tools/csr_probe.py [rounds]           C3 Laplacian and the C3 variable-coefficient
                                               matrix (same pattern, same bytes)
  python tools/csr_probe.py [rounds] 3:400     a device-generated Laplacian in plain CSR
                                               (C4), with its tile_bands"""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np
import bench, cgx

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
if len(sys.argv) > 2:
    dim, nx = (int(t) for t in sys.argv[2].split(":"))
    n = nx ** dim
    for r in range(rounds):
        with cgx.Solver(0, layout="csr") as s:
            s.gen_laplacian(dim, nx, nx, nx if dim == 3 else 1)
            s.set_rhs(np.ones(n))
            s.bench_prepare(5)
            ms = s.bench_run(50, graph=True)[0]
            _, sp = s.bench_run(20, graph=False, spmv_events=True)
            _, b2b = s.bench_run(20, graph=False, spmv_events=True, spmv_only=True)
            i = s.info()
        print("%d %dD nx %d csr tile_bands %d: %.1f it/s, in-CG SpMV %.2f us, b2b %.2f us" %
              (r, dim, nx, i["tile_bands"], 50 / (ms * 1e-3), 1e3 * sp, 1e3 * b2b), flush=True)
    sys.exit(0)
lap = bench.make_system(bench.WORKLOADS["c3"])
rp, col, val = cgx.varcoef3d(216, 216, 216, seed=7)
var = dict(rp=rp, col=col, val=val, b=np.ones(len(rp) - 1))
for r in range(rounds):
    for name, sysm, layout in (("laplacian", lap, "csr"), ("varcoef", var, "csr"),
                               ("varcoef", var, "dc")):
        leg = bench.solver_leg(sysm, 100, 10, layout, b2b=True)
        print("%d %-9s %s: %.1f it/s, in-CG SpMV %.2f us, b2b %.2f us" %
              (r, name, layout, leg["value"], leg["spmv_us"], leg["b2b_spmv_us"]), flush=True)
