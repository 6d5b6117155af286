set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_dist.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dist.log
[ $rc -le 1 ] || exit $rc
for a in hs cg1-dist hs cg1-dist; do
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --alg $a > gpurun_out/bench_$a.log 2>&1; rc=$?; echo "bench $a rc=$rc"; tail -1 gpurun_out/bench_$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['spmv_us'], d['roofline']['frac'])"
[ $rc -eq 0 ] || exit $rc
done
