#!/bin/bash
# rocprofv3 + PMC passes of the C2 and C4 bench lines (coded columns)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/profile.sh c2_dc python3 bench.py --workload c2 --steps 200 --warmup 10 --no-cpu || exit 3
bash tools/profile.sh c4_dc python3 bench.py --workload c4 --steps 20 --warmup 5 --no-cpu || exit 3
