#!/bin/bash
# column panels: parity, then C5 A/B (CSR vs panel sizes) and C3 unchanged
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "panels or variants or c3_full" > gpurun_out/sweep21_tests.log 2>&1 || { tail -30 gpurun_out/sweep21_tests.log; exit 1; }
tail -2 gpurun_out/sweep21_tests.log
timeout -k 10 600 python tools/sweep.py --workload c5 --rounds 3 --iters 10 \
  --variant auto: --variant w512:CGX_PANEL_WIN512=1 --variant w512_1m:CGX_PANEL_WIN512=1,CGX_PANEL_KB=1024 \
  --variant w512_4m:CGX_PANEL_WIN512=1,CGX_PANEL_KB=4096 \
  > gpurun_out/sweep21.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep21.log | tail -6; exit $rc
