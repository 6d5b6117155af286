#!/bin/bash
# 456-entry LDS-DMA windows (7 WGs/CU instead of 6): parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or c3_full or long_rows" > gpurun_out/sweep26_tests.log 2>&1 || { tail -30 gpurun_out/sweep26_tests.log; exit 1; }
tail -1 gpurun_out/sweep26_tests.log
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 10 --iters 40 --control \
  --variant base: --variant w456:CGX_SPMV_CAPW=456 \
  > gpurun_out/sweep26.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep26.log | tail -4; exit $rc
