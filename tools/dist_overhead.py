#!/usr/bin/env python3
"""Per-iteration cost of the multi-GPU phase code on one GPU: the C3 system
through cgx_dist solo (no transport, graph replay) vs a 1-rank RCCL
communicator (pack, send/recv loop, local-sum launches, ncclAllReduce on one
rank, eager), for both recurrences.  The difference is what N > 1 adds
besides the real all-reduce latency and the peer halo."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
import bench  # noqa: E402
import cgx  # noqa: E402

sysm = bench.make_system(bench.WORKLOADS["c3"])
for name in ("solo", "comm1"):
    for alg in (cgx.CGX_ALG_HS, cgx.CGX_ALG_CG1):
        # an id serves one communicator: a fresh one per solver
        d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id() if name == "comm1" else None)
        d.set_alg(alg)
        d.set_matrix(sysm["n_global"], sysm["rp"], sysm["col"], sysm["val"])
        d.set_rhs(sysm["b"])
        d.bench_prepare(10)
        ts = sorted(d.bench_run(100)[0] / 100 * 1e3 for _ in range(3))
        print(f"{name:6s} {'hs' if alg == cgx.CGX_ALG_HS else 'cg1':4s} us/iter "
              f"{ts[1]:.1f} (min {ts[0]:.1f})", flush=True)
        d.close()
