#!/bin/bash
# coded columns + byte row lengths: parity, then C3/C2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 \
  -k "dictionary or coded or c3_full or variants_bit_exact" > gpurun_out/dc3_tests.log 2>&1 || { tail -30 gpurun_out/dc3_tests.log; exit 1; }
tail -1 gpurun_out/dc3_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 \
  --variant csr:CGX_LAYOUT=csr --variant dc8:CGX_DC_BITS=8 --variant dc4: \
  > gpurun_out/dc3_sweep.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dc3_sweep.log | tail -4
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 6 --iters 200 --instances 2 \
  --variant csr:CGX_LAYOUT=csr --variant dc8:CGX_DC_BITS=8 --variant dc4: > gpurun_out/dc3_sweep_c2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dc3_sweep_c2.log | tail -4; exit $rc
