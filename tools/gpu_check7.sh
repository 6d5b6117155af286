#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "generated or stencil" > gpurun_out/c7_tests.log 2>&1 || { tail -30 gpurun_out/c7_tests.log; exit 1; }
tail -1 gpurun_out/c7_tests.log
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3.json')); print(d['value'], d['roofline']['spmv_us'], d['matrix_free_upper_bound'])"
timeout -k 10 400 python bench.py --no-cpu --workload c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print(d['value'], d['roofline']['spmv_us'], d['matrix_free_upper_bound'])"
