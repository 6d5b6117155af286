"""Per-rank iteration time of the partitioned solver on ONE GPU: a 1-rank
RCCL communicator (the multi-GPU phase code: pack, halo loop with no peers,
ncclAllReduce) on a slab of C4 (400 x 400 x nz planes, 8M rows at nz = 50 =
C4's slab at N = 8), graph-replayed.

  python tools/dist_probe.py [nz] [local3] [--cases=a,b,...]

cases: hs_fused, hs, cg1, sr (auto: the one-launch k_sr1_dia_m step where it
applies), sr2 (the two-launch fused SR step, set_march(0)), srN (one-launch
with N steps per workgroup), srcW (one-launch, chain width W rows), one / oneN (the single-GPU solver's SR
step on the same slab: auto or N steps per workgroup -- the rank step's base).  Default: hs_fused, sr, sr2, hs, cg1,
then hs_fused, sr, sr2 again (alternating)."""
import sys
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx

args = [a for a in sys.argv[1:] if not a.startswith("--")]
opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
nz = int(args[0]) if args else 50
cases = (opts.get("cases") or "hs_fused,sr,sr2,hs,cg1,hs_fused,sr,sr2").split(",")
rp, col, val = cgx.laplacian3d(400, 400, nz)
n = len(rp) - 1
b = np.ones(n)


def case(name):
    if name == "hs_fused":
        return cgx.CGX_ALG_HS, True, -1
    if name == "hs":
        return cgx.CGX_ALG_HS, False, -1
    if name == "cg1":
        return cgx.CGX_ALG_CG1, False, -1
    if name == "sr":
        return cgx.CGX_ALG_SR, "auto", -1
    if name == "sr2":
        return cgx.CGX_ALG_SR, "auto", 0
    if name.startswith("src"):  # srcW: auto segments, chain width W rows
        return cgx.CGX_ALG_SR, "auto", -1
    return cgx.CGX_ALG_SR, "auto", int(name[2:])


def one(name):
    with cgx.Solver(alg=cgx.CGX_ALG_SR) as s:
        s.gen_laplacian(3, 400, 400, nz)
        s.set_march(int(name[3:]) if len(name) > 3 else -1)
        s.set_rhs(b)
        s.bench_prepare(5)
        ms, _ = s.bench_run(100)
        _, sp = s.bench_run(30, graph=False, spmv_events=True)
        i = s.info()
        print("%-9s n %d  %.1f us/iter  spmv(launches) %.1f us  fused %d layout %s" %
              (name, n, 1e3 * ms / 100, 1e3 * sp, i["fused"], i["layout_name"]), flush=True)


for name in cases:
    if name.startswith("one"):
        one(name)
        continue
    alg, fused, march = case(name)
    d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id())
    try:
        d.set_alg(alg)
        d.set_fused(fused)
        d.set_march(march)
        if name.startswith("src"):
            d.set_sr_chain(int(name[3:]))
        d.set_matrix(n, rp, col, val)
        d.set_rhs(b)
        d.bench_prepare(5)
        ms, _ = d.bench_run(100)
        _, sp = d.bench_run(30, graph=False, spmv_events=True)
        ph = d.bench_phases()
        i = d.info()
        print("%-9s n %d  %.1f us/iter  spmv(launches) %.1f us  fused %d march %d layout %s" %
              (name, n, 1e3 * ms / 100, 1e3 * sp, i["fused"], i["march"], i["layout"]), flush=True)
        # the eager iteration's phases (HIP events): first launch, gap to the
        # second (halo wait), second launch (edge / boundary), tail to the next iteration's
        # first launch (local sums, all-reduce, pack, launch gaps), period
        if ph:
            print("          phases (eager, us): " + "  ".join(
                "%s %.1f" % (k, 1e3 * ph[k]) for k in ("first_launch", "halo_wait_gap",
                                                        "second_launch", "tail", "period")),
                  flush=True)
    finally:
        d.close()

# partitions with ghost faces: an in-process group of 2 slabs of nz planes
# (SR: each part's k_sr1_dia_m over its own steps, then k_sr1_edge of its
# ghost-facing plane after the D2D halo; part 0's launches timed)
if len(sys.argv) > 2 and sys.argv[2] == "local2sr":
    rp, col, val = cgx.laplacian3d(400, 400, 2 * nz)
    n = len(rp) - 1
    for march in (-1, 0):
        parts = cgx.DistSolver.local_group(0, 2)
        try:
            parts[0].set_alg(cgx.CGX_ALG_SR)
            parts[0].set_march(march)
            for g, d in enumerate(parts):
                rb, re_ = cgx.partition_rows(n, 2, g)
                d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
                d.set_rhs(np.ones(re_ - rb))
            parts[0].bench_prepare(3)
            ms, sp = parts[0].bench_run(20, spmv_events=True)
            i = parts[0].info()
            print("local2sr march %d: part-0 SR launches %.1f us, group iteration %.1f us (march %d inplace %d)" %
                  (march, 1e3 * sp, 1e3 * ms / 20, i["march"], i["inplace"]), flush=True)
        finally:
            parts[0].close()

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
