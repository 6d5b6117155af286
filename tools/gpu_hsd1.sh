#!/bin/bash
# partitioned HS recurrence + 1-rank RCCL communicator path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hsd1_tests.log 2>&1 || { tail -40 gpurun_out/hsd1_tests.log; exit 1; }
tail -3 gpurun_out/hsd1_tests.log
