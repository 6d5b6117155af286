set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant b256v4:CGX_SPMV_VEC=4 --variant w64v4:CGX_SPMV_BS=64,CGX_SPMV_VEC=4 --variant w64v2:CGX_SPMV_BS=64,CGX_SPMV_VEC=2 \
  --variant w64v1:CGX_SPMV_BS=64,CGX_SPMV_VEC=1 --variant w64v4nt:CGX_SPMV_BS=64,CGX_SPMV_VEC=4,CGX_SPMV_NT=1 \
  > gpurun_out/sweep3.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep3.log | grep -v amdgpu.ids
