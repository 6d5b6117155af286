#!/bin/bash
# XCD-contiguous block order on the LDS-DMA kernel: parity, EA read requests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variants or c3_full" > gpurun_out/sweep25_tests.log 2>&1 || { tail -30 gpurun_out/sweep25_tests.log; exit 1; }
tail -2 gpurun_out/sweep25_tests.log
for x in 0 1; do
  CGX_SPMV_XCD=$x timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/pmc3/x$x -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/pmc3/x$x.log 2>&1 || { echo "pmc x$x failed"; tail -5 gpurun_out/pmc3/x$x.log; exit 1; }
done
python3 - <<'PY'
import csv
for x in (0, 1):
    v=[float(r["Counter_Value"]) for r in csv.DictReader(open(f"gpurun_out/pmc3/x{x}/run_counter_collection.csv")) if "k_spmv_dma" in r["Kernel_Name"]]
    print(f"xcd={x}: k_spmv_dma EA read {sum(v)/len(v)*128/1e6:.1f} MB per launch")
PY
timeout -k 10 500 python tools/sweep.py --workload c3 --rounds 8 --iters 40 --control \
  --variant base: --variant xcd:CGX_SPMV_XCD=1 \
  > gpurun_out/sweep25.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep25.log | tail -4; exit $rc
