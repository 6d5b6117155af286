#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dist -o run -- python3 bench.py --alg cg1-dist --no-cpu --steps 50 > gpurun_out/prof_dist.log 2>&1 || { tail -20 gpurun_out/prof_dist.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_dist/run_kernel_stats.csv")):
    print(r["Calls"], round(float(r["AverageNs"])/1e3,2), r["Percentage"][:5], r["Name"][:110])
PY
