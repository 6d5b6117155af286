#!/bin/bash
# 16-wave coded-column kernel: parity, then C3 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "wide_workgroups or c3_full" > gpurun_out/w16_tests.log 2>&1 || { tail -30 gpurun_out/w16_tests.log; exit 1; }
tail -1 gpurun_out/w16_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 3 --control \
  --variant w4: --variant w8:CGX_SPMV_WPB=8 --variant w16:CGX_SPMV_WPB=16 > gpurun_out/w16.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/w16.log | tail -5
