#!/bin/bash
# adaptive LDS window: full GPU suite, then auto vs forced-512 on C2 and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/sweep29_tests.log 2>&1 || { tail -30 gpurun_out/sweep29_tests.log; exit 1; }
tail -1 gpurun_out/sweep29_tests.log
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 8 --iters 200 --instances 2 \
  --variant auto: --variant w512:CGX_SPMV_CAPW=512 > gpurun_out/sweep29a.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep29a.log | tail -3
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 8 --iters 30 --instances 3 \
  --variant auto: --variant w512:CGX_SPMV_CAPW=512 > gpurun_out/sweep29b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep29b.log | tail -3; exit $rc
