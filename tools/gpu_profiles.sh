#!/bin/bash
# rocprofv3 trace + PMC passes for the other workloads and the partitioned path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
bash tools/profile.sh c2_bench python3 bench.py --workload c2 --steps 100 --warmup 10 --no-cpu || exit 1
bash tools/profile.sh c5_bench python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu || exit 1
bash tools/profile.sh c4_bench python3 bench.py --workload c4 --steps 20 --warmup 5 --no-cpu || exit 1
bash tools/profile.sh c3_dist1 python3 bench.py --alg cg1-dist --steps 50 --warmup 10 --no-cpu || exit 1
