#!/bin/bash
# rocprofv3 kernel trace + single-counter PMC passes of the C2 and C4 benches (value-indexed pairs)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/profile.sh c2_vi python3 bench.py --workload c2 --steps 50 --warmup 10 --no-cpu || exit 3
bash tools/profile.sh c4_vi python3 bench.py --workload c4 --steps 10 --warmup 3 --no-cpu || exit 3
