#!/bin/bash
# coded columns for device-generated matrices + dist paths; full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/dc4_tests.log 2>&1 || { tail -30 gpurun_out/dc4_tests.log; exit 1; }
tail -1 gpurun_out/dc4_tests.log
