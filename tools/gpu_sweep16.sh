#!/bin/bash
# branch-free row chunks: parity, then order-rotated A/B with control
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/sweep16_tests.log 2>&1 || { tail -30 gpurun_out/sweep16_tests.log; exit 1; }
tail -2 gpurun_out/sweep16_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant wave: --variant dma:CGX_SPMV_DMA=1 --variant dma8:CGX_SPMV_DMA=8 \
  --variant dma8nt:CGX_SPMV_DMA=8,CGX_SPMV_NT=1 --variant dmant:CGX_SPMV_DMA=1,CGX_SPMV_NT=1 \
  > gpurun_out/sweep16.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep16.log | tail -7; exit $rc
