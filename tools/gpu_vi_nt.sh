#!/bin/bash
# CSR-VI: code-stream cache policy (nt on by size vs off) and XCD order, C3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant nt1: --variant nty:CGX_SPMV_NT=2 > gpurun_out/vi_nt.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/vi_nt.log | tail -5
