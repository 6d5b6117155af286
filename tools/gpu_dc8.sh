#!/bin/bash
# coded-column SpMV with 8 waves per workgroup (half the epilogue partials)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "dictionary or coded or c3_full or variants_bit_exact" > gpurun_out/dc8_tests.log 2>&1 || { tail -30 gpurun_out/dc8_tests.log; exit 1; }
tail -1 gpurun_out/dc8_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant w4: --variant w8:CGX_SPMV_WPB=8 > gpurun_out/dc8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dc8.log | tail -4
