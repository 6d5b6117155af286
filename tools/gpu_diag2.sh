set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
for v in normal diag1 diag2 diag3; do
  if [ $v = normal ]; then L=conjugate-gradient_amd/lib/libcgx.so; else L=diaglibs/libcgx_$v.so; fi
  CGX_LIB=$L CGX_SPMV_DMA=1 timeout -k 10 120 python tools/prof_run.py --workload c3 --iters 30 2>&1 | grep -v amdgpu | sed "s/^/$v: /"
done; done
