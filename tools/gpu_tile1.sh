#!/bin/bash
# L2-tiled block order: parity, then C4 A/B (C3 is below the budget: untiled)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "tiled" > gpurun_out/tile1_tests.log 2>&1 || { tail -30 gpurun_out/tile1_tests.log; exit 1; }
tail -1 gpurun_out/tile1_tests.log
timeout -k 10 900 python tools/sweep.py --workload c4 --rounds 6 --iters 10 --instances 2 --control \
  --variant tile: --variant notile:CGX_DC_TILE=0 --variant kb768:CGX_DC_TILE_KB=768 > gpurun_out/tile1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/tile1.log | tail -5
