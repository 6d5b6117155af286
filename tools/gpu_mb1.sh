#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out tools/mb/bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/mb/bin/mb_stream tools/mb/mb_stream.hip || exit 1
timeout -k 10 120 tools/mb/bin/mb_stream > gpurun_out/mb1.log 2>&1; rc=$?
cat gpurun_out/mb1.log; exit $rc
