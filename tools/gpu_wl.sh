#!/bin/bash
# numbers for DESIGN.md: other workloads / recurrences at N = 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for args in "--workload c2 --no-cpu" "--workload c5 --no-cpu" "--alg cg1 --no-cpu" "--alg cg1-dist --no-cpu" "--no-cpu --steps 200"; do
  echo "== $args"
  timeout -k 10 300 python bench.py $args > gpurun_out/wl.json 2> gpurun_out/wl.err || { tail gpurun_out/wl.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/wl.json'))
r=d['roofline']
print(d['value'], d['ms_per_step'], d['config']['alg'], 'spmv', r['spmv_us'], r['achieved'], r['frac'], 'upload_ms', d['upload_ms'], d['iter_gbs'])"
done
