#!/bin/bash
# rocprofv3 kernel trace + single-counter PMC passes of the default C3 bench (coded columns)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/profile.sh c3_dc python3 bench.py --steps 50 --warmup 10 --no-cpu
