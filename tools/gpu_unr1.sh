#!/bin/bash
# folded vector kernels, two elements per trip: parity, then C3/C2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "deferred_x" > gpurun_out/unr1_tests.log 2>&1 || { tail -30 gpurun_out/unr1_tests.log; exit 1; }
tail -1 gpurun_out/unr1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant base: --variant unr:CGX_VEC_UNR=1 > gpurun_out/unr1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/unr1.log | tail -4
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 2 \
  --variant base: --variant unr:CGX_VEC_UNR=1 > gpurun_out/unr1_c2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/unr1_c2.log | tail -3
