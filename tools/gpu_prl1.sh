#!/bin/bash
# column panels with byte row lengths per pass: parity, then C5 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "column_panels" > gpurun_out/prl1_tests.log 2>&1 || { tail -30 gpurun_out/prl1_tests.log; exit 1; }
tail -1 gpurun_out/prl1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c5 --rounds 5 --iters 10 --instances 2 --control \
  --variant rl: --variant rp:CGX_PANEL_RLEN=0 > gpurun_out/prl1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/prl1.log | tail -4
