#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q -m gpu -k "dist or local or rccl or c3_full or reduction" > gpurun_out/c2c3_tests.log 2>&1 || { tail -30 gpurun_out/c2c3_tests.log; exit 1; }
tail -2 gpurun_out/c2c3_tests.log
for args in "--workload c2 --no-cpu --steps 500" "--no-cpu --steps 200" "--alg cg1-dist --no-cpu --steps 200"; do
  timeout -k 10 300 python bench.py $args > gpurun_out/wl.json 2> gpurun_out/wl.err || { tail gpurun_out/wl.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/wl.json')); r=d['roofline']
print('$args', d['value'], d['ms_per_step'], 'spmv', r['spmv_us'], r['frac'], r['kernel'])"
done
