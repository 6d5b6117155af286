#!/bin/bash
# exact-size LDS-DMA windows vs full 6 KiB windows (both nt), order-rotated
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or c3_full or long_rows or reduction" > gpurun_out/sweep17_tests.log 2>&1 || { tail -30 gpurun_out/sweep17_tests.log; exit 1; }
tail -2 gpurun_out/sweep17_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant exact: --variant full:CGX_SPMV_DMA=3 --variant wave:CGX_SPMV_DMA=0 \
  > gpurun_out/sweep17.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep17.log | tail -5; exit $rc
