#!/bin/bash
# pipelined coded-column SpMV (k_spmv_dcp): parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "dictionary or coded or c3_full" > gpurun_out/dcp1_tests.log 2>&1 || { tail -30 gpurun_out/dcp1_tests.log; exit 1; }
tail -1 gpurun_out/dcp1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant dc: --variant dcp:CGX_DC_PIPE=1 > gpurun_out/dcp1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dcp1.log | tail -4
