#!/bin/bash
# coded-column SpMV knobs: XCD order, nt stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant base: --variant noxcd:CGX_SPMV_XCD=0 --variant nont:CGX_SPMV_NT=0 \
  > gpurun_out/dc5.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dc5.log | tail -5; exit $rc
