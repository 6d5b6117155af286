#!/bin/bash
# barrier-free SpMV epilogue (last-arriving wave writes the partial)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or reduction or deferred" > gpurun_out/sweep30_tests.log 2>&1 || { tail -30 gpurun_out/sweep30_tests.log; exit 1; }
tail -1 gpurun_out/sweep30_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 8 --iters 30 --instances 3 \
  --variant base: --variant last:CGX_SPMV_EPI_LAST=1 > gpurun_out/sweep30.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep30.log | tail -3
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --instances 2 \
  --variant base: --variant last:CGX_SPMV_EPI_LAST=1 > gpurun_out/sweep30b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep30b.log | tail -3; exit $rc
