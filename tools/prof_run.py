#!/usr/bin/env python3
"""Workload driver for rocprofv3: builds a bench workload, runs `--iters` CG
iterations eagerly (every kernel a separate dispatch), optionally with
alternative SpMV settings via the CGX_* environment knobs."""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
sys.path.insert(0, str(REPO / "tests"))

import bench  # noqa: E402
import cgx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--alg", default="hs")
ap.add_argument("--graph", action="store_true")
a = ap.parse_args()
sysm = bench.make_system(bench.WORKLOADS[a.workload])
s = cgx.Solver(0, alg=cgx.CGX_ALG_CG1 if a.alg == "cg1" else cgx.CGX_ALG_HS)
s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
s.set_rhs(sysm["b"])
s.bench_prepare(2)
tot, spmv = s.bench_run(a.iters, graph=a.graph, spmv_events=not a.graph)
info = s.info()
print(f"{a.workload} {a.alg}: {tot / a.iters:.4f} ms/iter, spmv {spmv * 1e3:.2f} us "
      f"= {info['spmv_bytes'] / (spmv * 1e-3) / 1e9:.1f} GB/s")
s.close()
