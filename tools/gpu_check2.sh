set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench_hs.log 2>&1; rc=$?; echo "bench hs rc=$rc"; tail -1 gpurun_out/bench_hs.log | cut -c1-900
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --alg cg1-dist > gpurun_out/bench_dist1.log 2>&1; rc=$?; echo "bench dist rc=$rc"; tail -3 gpurun_out/bench_dist1.log | cut -c1-900
