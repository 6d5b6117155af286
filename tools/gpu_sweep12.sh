set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 4 --iters 30 \
  --variant base: --variant dma:CGX_SPMV_DMA=1 --variant dma_fused:CGX_SPMV_DMA=1,CGX_FUSE_XPAY=1 \
  > gpurun_out/sweep12.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep12.log | grep -v amdgpu.ids
