"""Fused vs unfused iteration time on one GPU (cgx.Solver, graph-replayed,
device-generated Laplacian), same box, same build, back to back; HS, or the
CG1 recurrence with --cg1.
  python tools/fused_probe.py [--cg1|--sr] [--modes=on,off,...] [--march=-1,0,...]
                              [--chain=0,1888,...] [dim:nx[:ny:nz] ...]
default 3:216 3:400 (C3, C4); 2:1000 = C2.  --march: cgx_solver_set_march values tried
for each mode (-1 auto, 0 off, > 0 steps per segment)."""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

args = [a for a in sys.argv[1:] if not a.startswith("--")]
alg = (cgx.CGX_ALG_CG1 if "--cg1" in sys.argv else cgx.CGX_ALG_SR if "--sr" in sys.argv
       else cgx.CGX_ALG_HS)
modes = [True, False, True, False]
for a in sys.argv[1:]:
    if a.startswith("--modes="):  # e.g. --modes=on,off,on,off (cgx.fuse_mode names)
        modes = a.split("=", 1)[1].split(",")
marches = [-1]
chains = [0]
for a in sys.argv[1:]:
    if a.startswith("--march="):
        marches = [int(t) for t in a.split("=", 1)[1].split(",")]
    if a.startswith("--chain="):  # SR: cgx_solver_set_sr_chain widths (0 auto)
        chains = [int(t) for t in a.split("=", 1)[1].split(",")]
for spec in args or ["3:216", "3:400"]:
    v = [int(t) for t in spec.split(":")]
    dim, nx = v[0], v[1]
    ny, nz = (v[2], v[3]) if len(v) > 2 else (nx, nx if dim == 3 else 1)
    n = nx * ny * nz
    for fused, march, chain in [(f, m, c) for f in modes for m in marches for c in chains]:
        with cgx.Solver(0, alg=alg, fused=fused) as s:
            s.set_march(march)
            s.set_sr_chain(chain)
            s.gen_laplacian(dim, nx, ny, nz)
            s.set_rhs(np.ones(n))
            s.bench_prepare(5)
            ms = s.bench_run(200)[0]
            _, sp = s.bench_run(30, graph=False, spmv_events=True)
            i = s.info()
            print("%s %dD nx %d mode %s march %d (runs %d) chain %d fused %d: %.1f us/iter, "
                  "spmv launch %.1f us" %
                  (["hs", "cg1", "sr"][alg], dim, nx, fused, march, i["fuse_march"], chain,
                   i["fused"], 1e3 * ms / 200, 1e3 * sp), flush=True)
