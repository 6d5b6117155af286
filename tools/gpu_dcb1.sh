#!/bin/bash
# block-contiguous coded columns (k_spmv_dcb): parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "dictionary or coded or c3_full" > gpurun_out/dcb1_tests.log 2>&1 || { tail -30 gpurun_out/dcb1_tests.log; exit 1; }
tail -1 gpurun_out/dcb1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant dc: --variant dcb:CGX_DC_BLOCKED=1 > gpurun_out/dcb1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dcb1.log | tail -4
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 2 \
  --variant dc: --variant dcb:CGX_DC_BLOCKED=1 > gpurun_out/dcb1_c2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dcb1_c2.log | tail -3
