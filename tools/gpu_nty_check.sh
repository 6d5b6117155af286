#!/bin/bash
# nt=2 by-size default (CSR-VI y store past caches): gpu tests, C4 A/B, C3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nty_tests.log 2>&1 || { tail -20 gpurun_out/nty_tests.log; exit 1; }
tail -2 gpurun_out/nty_tests.log
timeout -k 10 400 python tools/sweep.py --workload c4 --rounds 4 --iters 20 --instances 1 \
  --variant nty: --variant nt1:CGX_SPMV_NT=1 > gpurun_out/nty_c4.log 2>&1 || { tail gpurun_out/nty_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/nty_c4.log | tail -3
timeout -k 10 400 python bench.py > gpurun_out/nty_bench_c3.json 2> gpurun_out/nty_bench_c3.err || { tail gpurun_out/nty_bench_c3.err; exit 1; }
cut -c1-600 gpurun_out/nty_bench_c3.json
