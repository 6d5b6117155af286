#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "c4_full" --durations=3 > gpurun_out/c4test.log 2>&1; rc=$?
tail -6 gpurun_out/c4test.log; exit $rc
