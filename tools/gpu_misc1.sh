#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "exact or golden or conj_grad or panels" > gpurun_out/misc1_tests.log 2>&1 || { tail -30 gpurun_out/misc1_tests.log; exit 1; }
tail -1 gpurun_out/misc1_tests.log
timeout -k 10 300 python - <<'PY'
import sys, time
sys.path.insert(0, "conjugate-gradient_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import torch, numpy as np, cgx, bench
sysm = bench.make_system(bench.WORKLOADS["c3"])
with cgx.Solver(0, mode=cgx.CGX_MODE_EXACT) as s:
    s.set_matrix(sysm["rp"], sysm["col"], sysm["val"]); s.set_rhs(sysm["b"])
    t0 = time.perf_counter(); s.run(4); dt = time.perf_counter() - t0
    print(f"exact mode C3: {dt/5*1e3:.1f} ms per iteration")
PY
timeout -k 10 600 python tools/sweep.py --workload c5 --rounds 3 --iters 10 \
  --variant u4: --variant u8:CGX_PANEL_U8=1 > gpurun_out/misc1_c5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/misc1_c5.log | tail -2
