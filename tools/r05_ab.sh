#!/bin/bash
# Round-5 A/B session on the GPU box (each step its own time limit, chained):
#   1. the SR tests on the product build (-k "sr or march")
#   2. the SR step-width / chain-width sweep (tools/fused_probe.py, dist_probe)
#   3. the CSR tests on the ab/1 variant (pair gathers), then the in-iteration
#      CSR SpMV alternated between the product and ab/1 (tools/csr_probe.py)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
what=${1:-all}
if [ "$what" = all ] || [ "$what" = sr ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sr or march" > gpurun_out/t_sr.log 2>&1 || { tail -30 gpurun_out/t_sr.log; exit 1; }
  tail -1 gpurun_out/t_sr.log
  timeout -k 10 400 python -u tools/fused_probe.py --sr --modes=on --chain=0,512,1024,2048,1312,0 \
    3:216 3:400 > gpurun_out/probe_sr.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/dist_probe.py 50 --cases=sr,src2048,sr >> gpurun_out/probe_sr.log 2>&1 || exit $?
  grep -v "version\|Hostname\|path" gpurun_out/probe_sr.log
fi
if [ "$what" = all ] || [ "$what" = csr ]; then
  AB_LIBS=ab/1/libcgx.so bash tools/ab_check.sh "csr or spmv" || exit $?
  AB_LIBS="conjugate-gradient_amd/lib/libcgx.so ab/1/libcgx.so" timeout -k 10 600 \
    bash tools/ab_probe.sh 2 tools/csr_probe.py 1 > gpurun_out/ab_csr_c3.log 2>&1 || exit $?
  AB_LIBS="conjugate-gradient_amd/lib/libcgx.so ab/1/libcgx.so" timeout -k 10 600 \
    bash tools/ab_probe.sh 2 tools/csr_probe.py 1 3:400 > gpurun_out/ab_csr_c4.log 2>&1 || exit $?
  cat gpurun_out/ab_csr_c3.log gpurun_out/ab_csr_c4.log
fi
