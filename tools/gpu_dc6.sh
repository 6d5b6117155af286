#!/bin/bash
# diagnostic: coded-column SpMV at 8 / 6 / 4 / 3 workgroups per CU (extra dynamic LDS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 5 --iters 30 --instances 2 \
  --variant wg8: --variant wg6:CGX_DC_LDS_PAD=8000 --variant wg5:CGX_DC_LDS_PAD=13500 --variant wg4:CGX_DC_LDS_PAD=21500 --variant wg3:CGX_DC_LDS_PAD=35000 \
  > gpurun_out/dc6.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dc6.log | tail -6; exit $rc
