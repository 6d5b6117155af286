set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant v2:CGX_SPMV_VEC=2 --variant v4:CGX_SPMV_VEC=4 --variant v1:CGX_SPMV_VEC=1 \
  --variant v2nt:CGX_SPMV_VEC=2,CGX_SPMV_NT=1 --variant v4nt:CGX_SPMV_VEC=4,CGX_SPMV_NT=1 \
  --variant v2noxcd:CGX_SPMV_XCD=0 --variant g1024:CGX_SPMV_GRID=1024 --variant g4096:CGX_SPMV_GRID=4096 \
  --variant g40k:CGX_SPMV_GRID=100000 > gpurun_out/sweep1.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep1.log | grep -v amdgpu.ids
