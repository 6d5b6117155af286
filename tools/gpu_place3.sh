#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for off in 0 8 64 256 512 1024 1280 1536; do
  CGX_ARENA=1 CGX_ARENA_COL_KB=$off timeout -k 10 300 python tools/placement.py 4 > gpurun_out/place_$off.log 2>&1 || exit 1
  echo "col +${off}KB: $(grep inst gpurun_out/place_$off.log | awk '{print $4}' | tr '\n' ' ')"
done
