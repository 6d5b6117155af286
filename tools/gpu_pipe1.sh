#!/bin/bash
# pipelined LDS-DMA SpMV: parity subset, then interleaved A/B on C3
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "pipe or c3_full or long_rows" > gpurun_out/pipe1_tests.log 2>&1 || { tail -30 gpurun_out/pipe1_tests.log; exit 1; }
tail -3 gpurun_out/pipe1_tests.log
timeout -k 10 300 python tools/sweep.py --workload c3 --rounds 3 --iters 40 \
  --variant base: --variant dma1:CGX_SPMV_DMA=1 \
  --variant pipe4:CGX_SPMV_DMA=2,CGX_SPMV_RBW=4 --variant pipe8:CGX_SPMV_DMA=2,CGX_SPMV_RBW=8 \
  --variant pipe16:CGX_SPMV_DMA=2,CGX_SPMV_RBW=16 --variant pipe32:CGX_SPMV_DMA=2,CGX_SPMV_RBW=32 \
  > gpurun_out/pipe1_sweep.log 2>&1
rc=$?
cat gpurun_out/pipe1_sweep.log | tail -20
exit $rc
