#!/bin/bash
# default bench line (with triad + CPU legs) and C4 strong-scaling at N = 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "stream_ceilings" > gpurun_out/bf_tests.log 2>&1 || { tail -20 gpurun_out/bf_tests.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
true
true
