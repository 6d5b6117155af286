#!/bin/bash
# folded HS (no finalize launches): parity, then A/B on C3 and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "deferred or history or reduction or solve" > gpurun_out/sweep22_tests.log 2>&1 || { tail -30 gpurun_out/sweep22_tests.log; exit 1; }
tail -2 gpurun_out/sweep22_tests.log
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant base: --variant fold:CGX_FOLD=1 \
  > gpurun_out/sweep22.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep22.log | tail -4
timeout -k 10 500 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --control \
  --variant base: --variant fold:CGX_FOLD=1 \
  > gpurun_out/sweep22b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep22b.log | tail -4; exit $rc
