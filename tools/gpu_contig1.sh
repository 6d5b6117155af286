#!/bin/bash
# physically contiguous allocations: does the placement spread shrink / median move?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 4 --control \
  --variant contig:CGX_CONTIG=1 --variant base: > gpurun_out/contig1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/contig1.log | tail -4
