#!/bin/bash
# LDS-DMA producer/consumer engine SpMV (CGX_SPMV_DMA=5): parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "eng or c3_full" > gpurun_out/sweep32_tests.log 2>&1 || { tail -30 gpurun_out/sweep32_tests.log; exit 1; }
tail -1 gpurun_out/sweep32_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 4 --iters 30 --instances 2 \
  --variant base: --variant eng0:CGX_SPMV_DMA=5 --variant eng1:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=1 --variant eng2:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=2 --variant eng3:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=3 > gpurun_out/sweep32.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep32.log | tail -3
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 2 \
  --variant base: --variant eng1:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=1 --variant eng2:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=2 > gpurun_out/sweep32b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep32b.log | tail -3; exit $rc
