#!/bin/bash
# rocprofv3 kernel trace of the partitioned HS path on a 1-rank RCCL communicator
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof_dist; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dist/comm1 -o run -- python3 tools/dist_overhead1.py comm1 hs > gpurun_out/prof_dist/comm1.log 2>&1 || { tail gpurun_out/prof_dist/comm1.log; exit 3; }
grep us/iter gpurun_out/prof_dist/comm1.log
