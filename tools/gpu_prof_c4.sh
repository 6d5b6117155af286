#!/bin/bash
# rocprofv3 + PMC passes of the C4 bench line (coded columns, L2-tiled block order)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/profile.sh c4_dc python3 bench.py --workload c4 --steps 20 --warmup 5 --no-cpu || exit 3
