"""Per-rank iteration time of the partitioned solver on ONE GPU: a 1-rank
RCCL communicator (the multi-GPU phase code: pack, halo loop with no peers,
ncclAllReduce) on a slab of C4 (400 x 400 x nz planes, 8M rows at nz = 50 =
C4's slab at N = 8), HS, SR (HS with one all-reduce) and CG1, fused and
unfused, graph-replayed (HS fused and SR twice, alternating)."""
import sys, time
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

nz = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rp, col, val = cgx.laplacian3d(400, 400, nz)
n = len(rp) - 1
b = np.ones(n)
for name, alg, fused in (("hs_fused", cgx.CGX_ALG_HS, True), ("sr", cgx.CGX_ALG_SR, "auto"),
                         ("hs", cgx.CGX_ALG_HS, False), ("cg1", cgx.CGX_ALG_CG1, False),
                         ("hs_fused", cgx.CGX_ALG_HS, True), ("sr", cgx.CGX_ALG_SR, "auto")):
    d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
    try:
        d.set_alg(alg)
        d.set_fused(fused)
        d.set_matrix(n, rp, col, val)
        d.set_rhs(b)
        d.bench_prepare(5)
        ms, _ = d.bench_run(100)
        _, sp = d.bench_run(30, graph=False, spmv_events=True)
        i = d.info()
        print("%-9s n %d  %.1f us/iter  spmv(launches) %.1f us  fused %d layout %s" %
              (name, n, 1e3 * ms / 100, 1e3 * sp, i["fused"], i["layout"]), flush=True)
    finally:
        d.close()

# partitions with ghost faces: an in-process group of 3 slabs of nz planes
# each (part 0's SpMV launches timed: its far slots are -nx*ny, +nx*ny and
# the ghost face above, NFAR = 4 instances)
if len(sys.argv) > 2 and sys.argv[2] == "local3":
    rp, col, val = cgx.laplacian3d(400, 400, 3 * nz)
    n = len(rp) - 1
    for fused in (True, False):
        parts = cgx.DistSolver.local_group(0, 3)
        try:
            parts[0].set_alg(cgx.CGX_ALG_HS)
            parts[0].set_fused(fused)
            for g, d in enumerate(parts):
                rb, re_ = cgx.partition_rows(n, 3, g)
                d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
                d.set_rhs(np.ones(re_ - rb))
            parts[0].bench_prepare(3)
            ms, sp = parts[0].bench_run(20, spmv_events=True)
            print("local3 fused %d: part-0 SpMV launches %.1f us, group iteration %.1f us" %
                  (parts[0].info()["fused"], 1e3 * sp, 1e3 * ms / 20), flush=True)
        finally:
            parts[0].close()
