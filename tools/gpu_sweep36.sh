#!/bin/bash
# folded vector kernels: first loads issued before the partial sums (CGX_VEC_PF)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "deferred or fold or c3_full" > gpurun_out/sweep36_tests.log 2>&1 || { tail -30 gpurun_out/sweep36_tests.log; exit 1; }
tail -1 gpurun_out/sweep36_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 3 \
  --variant base: --variant pf:CGX_VEC_PF=1 > gpurun_out/sweep36.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep36.log | tail -3
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 3 \
  --variant base: --variant pf:CGX_VEC_PF=1 > gpurun_out/sweep36b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep36b.log | tail -3; exit $rc
