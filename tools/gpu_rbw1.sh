#!/bin/bash
# coded-column SpMV, row blocks per wave in sequence: parity, then C3 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "blocks_per_wave or c3_full" > gpurun_out/rbw1_tests.log 2>&1 || { tail -30 gpurun_out/rbw1_tests.log; exit 1; }
tail -1 gpurun_out/rbw1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant r1: --variant r2:CGX_DC_RBW=2 --variant r4:CGX_DC_RBW=4 --variant r8:CGX_DC_RBW=8 > gpurun_out/rbw1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/rbw1.log | tail -6
