set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x --maxfail=10 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --alg cg1 --no-cpu > gpurun_out/bench_cg1.log 2>&1; rc=$?; echo "bench cg1 rc=$rc"; tail -3 gpurun_out/bench_cg1.log
