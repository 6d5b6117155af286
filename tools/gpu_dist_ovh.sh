#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python tools/dist_overhead.py > gpurun_out/dist_ovh.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dist_ovh.log | tail -6; exit $rc
