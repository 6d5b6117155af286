#!/bin/bash
# default bench line (with CPU legs), then C4 and C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 30 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 1; }
cut -c1-400 gpurun_out/bench_c4.json
timeout -k 10 400 python bench.py --workload c2 --no-cpu --steps 200 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
cut -c1-400 gpurun_out/bench_c2.json
