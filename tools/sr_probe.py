"""HS against the unfused SR step (two launches, one reduction) on layouts
without a plane march, alternating, one box: CG it/s (graph replay) and the
SpMV launch in the iteration.
  python tools/sr_probe.py [rounds]
C3's pattern with general coefficients (DC and CSR), C3 in CSR, C2 (DIA,
cache-resident)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np
import bench, cgx

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rp, col, val = cgx.varcoef3d(216, 216, 216, seed=7)
var = dict(rp=rp, col=col, val=val, b=np.ones(len(rp) - 1))
lap3 = bench.make_system(bench.WORKLOADS["c3"])
lap2 = bench.make_system(bench.WORKLOADS["c2"])
cases = [("varcoef", var, "auto"), ("varcoef", var, "csr"), ("lap3d", lap3, "csr"),
         ("lap2d", lap2, "auto")]
for r in range(rounds):
    for name, sysm, layout in cases:
        for alg in ("hs", "sr"):
            leg = bench.solver_leg(sysm, 100, 10, layout, alg=alg)
            i = leg["info"]
            print("%d %-8s %-4s %s (%s, fused %d): %.1f it/s, SpMV %.2f us" %
                  (r, name, layout, alg, i["layout_name"], i["fused"], leg["value"],
                   leg["spmv_us"]), flush=True)
