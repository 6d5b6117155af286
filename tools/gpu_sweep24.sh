#!/bin/bash
# confirmation: w8 first (its own control), base, w8 + nt off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 10 --iters 40 --control \
  --variant w8:CGX_SPMV_WPB=8 --variant base: --variant w8_nont:CGX_SPMV_WPB=8,CGX_SPMV_NT=0 \
  > gpurun_out/sweep24.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep24.log | tail -5; exit $rc
