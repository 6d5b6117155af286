#!/bin/bash
# value-indexed pairs (CSR-VI): parity (single GPU + partitions), then C3 A/B of workgroup widths
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "dictionary or coded or value_indexed or c3_full or tiled or wide_workgroups" > gpurun_out/vi_tests.log 2>&1 || { tail -40 gpurun_out/vi_tests.log; exit 1; }
tail -1 gpurun_out/vi_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/vi_dist.log 2>&1 || { tail -40 gpurun_out/vi_dist.log; exit 1; }
tail -1 gpurun_out/vi_dist.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant vw1: --variant vw2:CGX_VI_BPW=2 --variant vs:CGX_VI_WIN=0 > gpurun_out/vi.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/vi.log | tail -6
