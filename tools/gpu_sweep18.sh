#!/bin/bash
# C2 (cache-resident, latency-bound): kernel and reduction-path A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 500 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --control \
  --variant dma: --variant wave:CGX_SPMV_DMA=0 --variant wave_ticket:CGX_SPMV_DMA=0,CGX_TICKET=1 \
  --variant dma_nt:CGX_SPMV_NT=1 --variant pipe4:CGX_SPMV_DMA=2,CGX_SPMV_RBW=4 \
  --variant wave_w8:CGX_SPMV_DMA=0,CGX_SPMV_WPB=8 \
  > gpurun_out/sweep18.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep18.log | tail -8; exit $rc
