#!/bin/bash
# non-temporal vector streams: HS x (k_xpay_xf), CG1 x/p/s (k_cg1_update)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --workload c3 --rounds 6 --iters 30 --instances 2 \
  --variant base: --variant xnt:CGX_VEC_NT=1 > gpurun_out/nt1_hs.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/nt1_hs.log | tail -3
timeout -k 10 900 python tools/sweep.py --workload c3 --alg cg1 --rounds 6 --iters 30 --instances 2 \
  --variant base: --variant x:CGX_CG1_NT=1 --variant xp:CGX_CG1_NT=3 --variant xs:CGX_CG1_NT=5 --variant xps:CGX_CG1_NT=7 \
  > gpurun_out/nt1_cg1.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/nt1_cg1.log | tail -6; exit $rc
