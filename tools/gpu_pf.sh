#!/bin/bash
# folded vector kernels: prefetch depth before the partial sum (CGX_VEC_PF 1/2/4)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "prefetch_depth or deferred_x or value_indexed_cg" > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
timeout -k 10 900 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 --control \
  --variant pf1: --variant pf2:CGX_VEC_PF=2 --variant pf4:CGX_VEC_PF=4 > gpurun_out/pf.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pf.log | tail -5
