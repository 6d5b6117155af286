#!/usr/bin/env python3
"""One variant of tools/dist_overhead.py (for rocprofv3): argv[1] = solo|comm1,
argv[2] = hs|cg1."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
import bench  # noqa: E402
import cgx  # noqa: E402

sysm = bench.make_system(bench.WORKLOADS["c3"])
d = cgx.DistSolver(0, 1, 0, cgx.dist_unique_id() if sys.argv[1] == "comm1" else None)
d.set_alg(cgx.CGX_ALG_HS if sys.argv[2] == "hs" else cgx.CGX_ALG_CG1)
d.set_matrix(sysm["n_global"], sysm["rp"], sysm["col"], sysm["val"])
d.set_rhs(sysm["b"])
d.bench_prepare(10)
print(sys.argv[1], sys.argv[2], d.bench_run(50)[0] / 50 * 1e3, "us/iter")
d.close()
