#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python - <<'PY'
import os, sys, time
sys.path.insert(0, "conjugate-gradient_amd")
import torch, numpy as np, cgx
for g in ("", "4096"):
    if g: os.environ["CGX_STENCIL_GRID"] = g
    else: os.environ.pop("CGX_STENCIL_GRID", None)
    with cgx.Solver(0) as s:
        s.set_stencil(3, 216, 216, 216)
        s.set_rhs(np.ones(216 ** 3))
        s.bench_prepare(10)
        tot, _ = s.bench_run(200, graph=True)
        _, sp = s.bench_run(50, graph=False, spmv_events=True)
        print(f"grid {g or 'n/256'}: {200/tot*1e3:.1f} it/s, spmv {sp*1e3:.1f} us = {16*216**3/sp/1e6:.0f} GB/s")
PY
