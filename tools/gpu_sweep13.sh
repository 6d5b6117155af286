#!/bin/bash
# cache-policy A/B: nt matrix stream (wave / LDS-DMA kernels), nt x in update_xr
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or c3_full" > gpurun_out/sweep13_tests.log 2>&1 || { tail -30 gpurun_out/sweep13_tests.log; exit 1; }
tail -2 gpurun_out/sweep13_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 4 --iters 40 \
  --variant base: --variant nt:CGX_SPMV_NT=1 --variant xnt:CGX_VEC_XNT=1 \
  --variant nt_xnt:CGX_SPMV_NT=1,CGX_VEC_XNT=1 \
  --variant dma:CGX_SPMV_DMA=1 --variant dma_nt:CGX_SPMV_DMA=1,CGX_SPMV_NT=1 \
  --variant dma_nt_xnt:CGX_SPMV_DMA=1,CGX_SPMV_NT=1,CGX_VEC_XNT=1 \
  --variant w8_nt:CGX_SPMV_WPB=8,CGX_SPMV_NT=1 \
  > gpurun_out/sweep13.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sweep13.log | tail -12; exit $rc
