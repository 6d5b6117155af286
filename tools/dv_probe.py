"""DIA-V one-launch SR step on the C3 general-coefficient system
(cgx_gen_varcoef3d 216^3, seed 7): us per iteration (graph) and per SR
launch (HIP events), for A/B builds (tools/ab_probe.sh).

  python tools/dv_probe.py [--chains=0,1024,...] [--marches=-1,...]"""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
chains = [int(c) for c in opts.get("chains", "0").split(",")]
marches = [int(c) for c in opts.get("marches", "-1").split(",")]
rp, col, val = cgx.varcoef3d(216, 216, 216, seed=7)
b = np.ones(len(rp) - 1)
for march in marches:
    for chain in chains:
        with cgx.Solver(0, alg=cgx.CGX_ALG_SR) as s:
            s.set_march(march)
            s.set_sr_chain(chain)
            s.set_matrix(rp, col, val)
            s.set_rhs(b)
            s.bench_prepare(5)
            ms, _ = s.bench_run(100)
            _, sp = s.bench_run(30, graph=False, spmv_events=True)
            i = s.info()
            print("march %d chain %d: %.1f us/iter (%.0f it/s)  launch %.1f us  %.3f of 8 TB/s  "
                  "dv %d fused %d seg %d" % (march, chain, 1e3 * ms / 100, 1e5 / ms, 1e3 * sp,
                                             i["spmv_iter_bytes"] / (sp * 1e-3) / 8e12,
                                             i["dia_value_stream"], i["fused"], i["fuse_march"]),
                  flush=True)
