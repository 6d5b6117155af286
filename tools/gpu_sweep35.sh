#!/bin/bash
# engine SpMV with chunked descriptor prefetch: parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "eng or c3_full" > gpurun_out/sweep35_tests.log 2>&1 || { tail -30 gpurun_out/sweep35_tests.log; exit 1; }
tail -1 gpurun_out/sweep35_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 4 --iters 30 --instances 2 \
  --variant base: --variant eng4:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=4 \
  --variant eng6:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=6 \
  --variant eng7:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=7 > gpurun_out/sweep35.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep35.log | tail -7
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 4 --iters 200 --instances 2 \
  --variant base: --variant eng4:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=4 --variant eng7:CGX_SPMV_DMA=5,CGX_ENG_SHAPE=7 > gpurun_out/sweep35b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep35b.log | tail -4; exit $rc
