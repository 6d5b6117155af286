#!/bin/bash
# checkpoint: full GPU suite, smoke, default bench line, rocprofv3 trace + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/rb_tests.log 2>&1 || { tail -30 gpurun_out/rb_tests.log; exit 1; }
tail -2 gpurun_out/rb_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
bash tools/profile.sh c3_bench python3 bench.py --steps 50 --warmup 10 --no-cpu
