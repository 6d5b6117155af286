#!/bin/bash
# window sizes on C2 (cache-resident) and C3, two allocations each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants" > gpurun_out/sweep28_tests.log 2>&1 || { tail -30 gpurun_out/sweep28_tests.log; exit 1; }
tail -1 gpurun_out/sweep28_tests.log
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --instances 2 \
  --variant w512: --variant w456:CGX_SPMV_CAPW=456 --variant w328:CGX_SPMV_CAPW=328 \
  > gpurun_out/sweep28.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep28.log | tail -4
