#!/bin/bash
# full GPU suite + A/B of the finalize change and stream policy, then the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/check6_tests.log 2>&1 || { tail -30 gpurun_out/check6_tests.log; exit 1; }
tail -2 gpurun_out/check6_tests.log
timeout -k 10 400 python tools/sweep.py --workload c3 --rounds 8 --iters 40 \
  --control --variant nt: --variant nont:CGX_SPMV_NT=0 --variant dma_nt:CGX_SPMV_DMA=1 --variant dma_nont:CGX_SPMV_DMA=1,CGX_SPMV_NT=0 \
  > gpurun_out/sweep14.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sweep14.log | tail -4
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
