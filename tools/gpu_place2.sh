#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python tools/placement.py 8 > gpurun_out/place_sep.log 2>&1 || exit 1
CGX_ARENA=1 timeout -k 10 600 python tools/placement.py 8 > gpurun_out/place_arena.log 2>&1; rc=$?
echo "== separate"; grep inst gpurun_out/place_sep.log
echo "== arena"; grep inst gpurun_out/place_arena.log
exit $rc
