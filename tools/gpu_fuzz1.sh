#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "random_patterns" > gpurun_out/fuzz1.log 2>&1 || { tail -30 gpurun_out/fuzz1.log; exit 1; }
tail -1 gpurun_out/fuzz1.log
