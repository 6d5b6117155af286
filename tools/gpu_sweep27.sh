#!/bin/bash
# 456-entry windows vs 512, four allocations each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 8 --iters 30 --instances 4 \
  --variant w456:CGX_SPMV_CAPW=456 --variant base: \
  > gpurun_out/sweep27.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep27.log | tail -3; exit $rc
