#!/bin/bash
# order-rotated A/B with a duplicate control: stream policy x kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant nt: --variant nont:CGX_SPMV_NT=0 --variant dma_nt:CGX_SPMV_DMA=1 \
  --variant dma_nont:CGX_SPMV_DMA=1,CGX_SPMV_NT=0 \
  > gpurun_out/sweep15.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep15.log | tail -7; exit $rc
