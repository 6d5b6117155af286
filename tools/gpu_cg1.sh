#!/bin/bash
# CG1 (single solver) and the single-rank partitioned path with coded columns, C3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for a in cg1 cg1-dist; do
  timeout -k 10 300 python bench.py --alg $a --no-cpu > gpurun_out/bench_$a.json 2> gpurun_out/bench_$a.err || { tail gpurun_out/bench_$a.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$a.json'));print('$a', d['value'], d['ms_per_step'], d['roofline']['spmv_us'], d['config']['layout'])"
done
