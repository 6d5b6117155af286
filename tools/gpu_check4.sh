set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant tg:CGX_SPMV_TG=1 --variant notg:CGX_SPMV_TG=0 --variant tg_fused:CGX_SPMV_TG=1,CGX_FUSE_XPAY=1 \
  --variant tg_v2:CGX_SPMV_TG=1,CGX_SPMV_VEC=2 --variant tg_w8:CGX_SPMV_TG=1,CGX_SPMV_WPB=8 --variant tg_nt:CGX_SPMV_TG=1,CGX_SPMV_NT=1 \
  > gpurun_out/sweep7.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep7.log | grep -v amdgpu.ids
