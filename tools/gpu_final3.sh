#!/bin/bash
# checkpoint after CSR-VI: full GPU suite, smoke, rocprofv3 profile of the default bench, bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final3_tests.log 2>&1 || { tail -30 gpurun_out/final3_tests.log; exit 1; }
tail -1 gpurun_out/final3_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/profile.sh c3_vi python3 bench.py --steps 50 --warmup 10 --no-cpu || exit 1
timeout -k 10 500 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cut -c1-400 gpurun_out/bench_c3.json
