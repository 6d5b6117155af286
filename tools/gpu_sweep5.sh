set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant rbw1:CGX_SPMV_RBW=1 --variant rbw2:CGX_SPMV_RBW=2 --variant rbw4:CGX_SPMV_RBW=4 --variant rbw8:CGX_SPMV_RBW=8 \
  --variant p2:CGX_SPMV_RBW=2,CGX_SPMV_PIPE=1 --variant p4:CGX_SPMV_RBW=4,CGX_SPMV_PIPE=1 --variant p8:CGX_SPMV_RBW=8,CGX_SPMV_PIPE=1 \
  --variant rbw4w8:CGX_SPMV_RBW=4,CGX_SPMV_WPB=8 \
  > gpurun_out/sweep5.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep5.log | grep -v amdgpu.ids
