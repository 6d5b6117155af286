#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "generated or stencil" > gpurun_out/gen_tests.log 2>&1 || { tail -30 gpurun_out/gen_tests.log; exit 1; }
tail -2 gpurun_out/gen_tests.log
timeout -k 10 300 python - <<'PY'
import sys, time
sys.path.insert(0, "conjugate-gradient_amd")
import torch, cgx
for kind in ("csr-gen", "stencil"):
    with cgx.Solver(0) as s:
        t0 = time.perf_counter()
        if kind == "stencil":
            s.set_stencil(3, 216, 216, 216)
        else:
            s.gen_laplacian(3, 216, 216, 216)
        t1 = time.perf_counter()
        import numpy as np
        s.set_rhs(np.ones(216 ** 3))
        s.bench_prepare(10)
        tot, _ = s.bench_run(200, graph=True)
        _, sp = s.bench_run(50, graph=False, spmv_events=True)
        print(f"{kind}: setup {1e3*(t1-t0):.1f} ms, {200/tot*1e3:.1f} it/s, spmv {sp*1e3:.1f} us")
PY
