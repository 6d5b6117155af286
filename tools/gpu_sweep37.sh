#!/bin/bash
# folded vector kernels: grid size (1024-thread workgroups per CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 \
  --variant base: --variant g512:CGX_VEC_GRID=512 --variant g2048:CGX_VEC_GRID=2048 --variant g3072:CGX_VEC_GRID=3072 \
  > gpurun_out/sweep37.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep37.log | tail -5
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 2 \
  --variant base: --variant g512:CGX_VEC_GRID=512 --variant g2048:CGX_VEC_GRID=2048 > gpurun_out/sweep37b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep37b.log | tail -4; exit $rc
