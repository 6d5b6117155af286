set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --workload c2 --rounds 3 --iters 50 --variant csr: --variant sell:CGX_LAYOUT=sell --variant notg:CGX_SPMV_TG=0 > gpurun_out/sweep_c2.log 2>&1; rc=$?; echo "c2 rc=$rc"; grep -v amdgpu.ids gpurun_out/sweep_c2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/sweep.py --workload c5 --rounds 2 --iters 20 --variant csr: --variant notg:CGX_SPMV_TG=0 --variant sell:CGX_LAYOUT=sell --variant b256:CGX_SPMV_BS=256,CGX_SPMV_VEC=4 > gpurun_out/sweep_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; grep -v amdgpu.ids gpurun_out/sweep_c5.log
