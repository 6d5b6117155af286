#!/bin/bash
# block-contiguous coded columns: larger A/B (4 allocations per variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 8 --iters 30 --instances 4 --control \
  --variant dc: --variant dcb:CGX_DC_BLOCKED=1 > gpurun_out/dcb2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dcb2.log | tail -4
