#!/usr/bin/env python3
"""Interleaved A/B of SpMV/solver knobs in ONE process (methodology rule 24).

  python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
      --variant base: --variant vec4:CGX_SPMV_VEC=4 --variant nt:CGX_SPMV_NT=1

Each variant is a solver created with its CGX_* environment; the matrix is
uploaded once per variant.  Prints per-variant median/min SpMV time and
iteration time over the rounds."""
import argparse
import os
import statistics
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
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--alg", default="hs")
ap.add_argument("--variant", action="append", default=[])
ap.add_argument("--instances", type=int, default=1,
                help="solvers per variant (device placement varies by +-5%% between "
                     "allocations; the report is the median over instances)")
ap.add_argument("--control", action="store_true",
                help="append a second copy of the first variant (placement/order control)")
a = ap.parse_args()
variants = a.variant or ["base:"]
if a.control:
    n0, _, e0 = variants[0].partition(":")
    variants = variants + [f"{n0}_ctl:{e0}"]

sysm = bench.make_system(bench.WORKLOADS[a.workload])
solvers = []
for v in variants:
    name, _, envs = v.partition(":")
    saved = {}
    for kv in filter(None, envs.split(",")):
        k, _, val = kv.partition("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = val
    for inst in range(a.instances):
        s = cgx.Solver(0, alg=cgx.CGX_ALG_CG1 if a.alg == "cg1" else cgx.CGX_ALG_HS)
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        s.set_rhs(sysm["b"])
        s.bench_prepare(3)
        solvers.append((name, inst, s))
    for k, old in saved.items():
        if old is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = old
info = solvers[0][2].info()
infos = {n: s.info() for n, _, s in solvers}
res = {(n, i): {"spmv": [], "iter": []} for n, i, _ in solvers}
for r in range(a.rounds):
    k = r % len(solvers)  # rotate the order so no solver always runs first
    for name, inst, s in solvers[k:] + solvers[:k]:
        tot, sp = s.bench_run(a.iters, graph=False, spmv_events=True)
        res[(name, inst)]["spmv"].append(sp * 1e3)
        tot, _ = s.bench_run(a.iters, graph=True)
        res[(name, inst)]["iter"].append(tot / a.iters * 1e3)
print(f"workload {a.workload}: n={info['n']} nnz={info['nnz']} spmv_bytes={info['spmv_bytes']:.0f} "
      f"iter_bytes={info['iter_bytes']:.0f} grid={info['spmv_grid']} rowblocks={info['n_rowblocks']}"
      f" instances={a.instances}")
names = list(dict.fromkeys(n for n, _, _ in solvers))
for name in names:
    sp = [statistics.median(res[(name, i)]["spmv"]) for i in range(a.instances)]
    it = [statistics.median(res[(name, i)]["iter"]) for i in range(a.instances)]
    sm, si = statistics.median(sp), statistics.median(it)
    sb = infos[name]["spmv_iter_bytes"]
    spread = f" [{min(sp):.1f}-{max(sp):.1f}]" if a.instances > 1 else ""
    print(f"{name:>14}: spmv med {sm:8.2f} us{spread} ({sb / sm / 1e3:7.1f} GB/s)   iter med "
          f"{si:8.2f} us ({1e6 / si:7.1f} it/s, {info['iter_bytes'] / si / 1e3:7.1f} GB/s)")
