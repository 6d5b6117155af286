"""the unfused SR step (k_update_sr with FIN_SR1 folded in: every
update workgroup re-reads all of the SpMV's (p.s, s.s) pairs) against HS on
layouts with many SpMV workgroups -- C5's column panels (fp32) and C4's plain
CSR -- same box, alternating: CG it/s (graph replay), the SpMV launch in the
iteration, and the SpMV's pair count (= partials the fold re-reads per
update workgroup).
  python tools/sr_fold_probe.py [rounds] [c5,c4csr]"""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "conjugate-gradient_amd")
import bench

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
which = (sys.argv[2] if len(sys.argv) > 2 else "c5,c4csr").split(",")
cases = []
if "c5" in which:
    cases.append(("c5", bench.make_system(bench.WORKLOADS["c5"]), "auto"))
if "c4csr" in which:
    cases.append(("c4csr", bench.make_system(bench.WORKLOADS["c4"]), "csr"))
for r in range(rounds):
    for name, sysm, layout in cases:
        for alg in ("hs", "sr"):
            leg = bench.solver_leg(sysm, 50, 5, layout, alg=alg)
            i = leg["info"]
            print("%d %-6s %s (%s, fused %d, spmv workgroups %d): %.2f it/s, SpMV %.1f us" %
                  (r, name, alg, i["layout_name"], i["fused"], i["spmv_grid"],
                   leg["value"], leg["spmv_us"]), flush=True)
