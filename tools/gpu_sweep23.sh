#!/bin/bash
# 8-wave LDS-DMA SpMV workgroups (half the partials for the folded alpha)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or panels or deferred" > gpurun_out/sweep23_tests.log 2>&1 || { tail -30 gpurun_out/sweep23_tests.log; exit 1; }
tail -2 gpurun_out/sweep23_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant base: --variant w8:CGX_SPMV_WPB=8 \
  > gpurun_out/sweep23.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep23.log | tail -4
timeout -k 10 500 python tools/sweep.py --workload c2 --rounds 8 --iters 200 \
  --variant base: --variant w8:CGX_SPMV_WPB=8 \
  > gpurun_out/sweep23b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep23b.log | tail -3; exit $rc
