set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_dist.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dist.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --alg cg1-dist > gpurun_out/bench_dist1.log 2>&1; rc=$?; echo "bench dist rc=$rc"; tail -1 gpurun_out/bench_dist1.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
# two RCCL ranks sharing the one GPU (validation of the N>1 path; may be refused by RCCL)
HIP_VISIBLE_DEVICES=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/dist_same_gpu.py > gpurun_out/dist2same.log 2>&1; rc=$?; echo "2 ranks/1 GPU rc=$rc"; tail -12 gpurun_out/dist2same.log
