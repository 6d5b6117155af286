#!/bin/bash
# bench paths of the partitioned solver at one rank: HS, CG1, auto trial
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for a in hs-dist cg1-dist auto-dist; do
  timeout -k 10 300 python bench.py --alg $a --no-cpu > gpurun_out/bench_$a.json 2> gpurun_out/bench_$a.err || { tail gpurun_out/bench_$a.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$a.json'));print('$a', d['value'], d['ms_per_step'], d['roofline']['spmv_us'], d['config']['alg'], d['config']['alg_trial_ms_per_iter'])"
done
