#!/bin/bash
# coded-column SpMV with the one-round-trip prologue: parity, then A/B vs plain CSR
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 \
  -k "dictionary or coded or c3_full or variants_bit_exact or generated" > gpurun_out/dc7_tests.log 2>&1 || { tail -30 gpurun_out/dc7_tests.log; exit 1; }
tail -1 gpurun_out/dc7_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant dc: --variant csr:CGX_LAYOUT=csr > gpurun_out/dc7.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dc7.log | tail -4
