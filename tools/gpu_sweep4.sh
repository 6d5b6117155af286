set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant xcd:CGX_SPMV_XCD=1 --variant noxcd:CGX_SPMV_XCD=0 --variant xcdnt:CGX_SPMV_NT=1 \
  --variant wpb8:CGX_SPMV_WPB=8 --variant wpb8nt:CGX_SPMV_WPB=8,CGX_SPMV_NT=1 \
  > gpurun_out/sweep4.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep4.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh c3_w64 --workload c3 --iters 20
