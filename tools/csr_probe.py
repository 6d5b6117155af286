"""In-iteration CSR SpMV on the C3 Laplacian and on the C3 variable-coefficient
matrix (same pattern, same bytes), alternating, one box: bench.py's solver_leg
(graph-replayed CG it/s, HIP-event SpMV launch average, back-to-back SpMV).
  python tools/csr_probe.py [rounds]"""
import sys
sys.path.insert(0, ".")
import numpy as np
import bench, cgx

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
lap = bench.make_system(bench.WORKLOADS["c3"])
rp, col, val = cgx.varcoef3d(216, 216, 216, seed=7)
var = dict(rp=rp, col=col, val=val, b=np.ones(len(rp) - 1))
for r in range(rounds):
    for name, sysm in (("laplacian", lap), ("varcoef", var)):
        leg = bench.solver_leg(sysm, 100, 10, "csr", b2b=True)
        print("%d %-9s csr: %.1f it/s, in-CG SpMV %.2f us, b2b %.2f us" %
              (r, name, leg["value"], leg["spmv_us"], leg["b2b_spmv_us"]), flush=True)
