set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 3 --iters 30 \
  --variant base:CGX_SPMV_XCD=0 --variant xcd:CGX_SPMV_XCD=1 --variant xcdnt:CGX_SPMV_XCD=1,CGX_SPMV_NT=1 \
  --variant xcd_notg:CGX_SPMV_XCD=1,CGX_SPMV_TG=0 --variant xcd_w8:CGX_SPMV_XCD=1,CGX_SPMV_WPB=8 --variant xcd_v2:CGX_SPMV_XCD=1,CGX_SPMV_VEC=2 \
  --variant xcd_fused:CGX_SPMV_XCD=1,CGX_FUSE_XPAY=1 \
  > gpurun_out/sweep8.log 2>&1; rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep8.log | grep -v amdgpu.ids
