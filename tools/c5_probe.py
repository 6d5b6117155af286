"""C5 (random SPD, 5 M rows, fp32, column panels): CG it/s and the SpMV in the
iteration, back to back with the product library and the ab/ variants
(tools/ab_probe.sh), one box.
  python tools/c5_probe.py [rounds]"""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "conjugate-gradient_amd")
import bench

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 1
sysm = bench.make_system(bench.WORKLOADS["c5"])
for r in range(rounds):
    leg = bench.solver_leg(sysm, 50, 5, "auto", b2b=True)
    i = leg["info"]
    print("%d c5 %s panels %d: %.1f it/s, in-CG SpMV %.1f us, b2b %.1f us" %
          (r, i["layout_name"], i["n_panels"], leg["value"], leg["spmv_us"], leg["b2b_spmv_us"]),
          flush=True)
