#!/bin/bash
# 32-row LDS-DMA blocks (2x waves per CU) vs 64-row, C3 and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or c3_full or long_rows" > gpurun_out/sweep19_tests.log 2>&1 || { tail -30 gpurun_out/sweep19_tests.log; exit 1; }
tail -2 gpurun_out/sweep19_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant dma: --variant dma32:CGX_SPMV_DMA=4 --variant dma32_nont:CGX_SPMV_DMA=4,CGX_SPMV_NT=0 \
  > gpurun_out/sweep19.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep19.log | tail -5
timeout -k 10 500 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --control \
  --variant dma: --variant dma32:CGX_SPMV_DMA=4 \
  > gpurun_out/sweep19b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep19b.log | tail -4; exit $rc
