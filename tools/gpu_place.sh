#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python tools/placement.py 8 > gpurun_out/place.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/place.log | tail -20; exit $rc
