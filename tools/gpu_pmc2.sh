#!/bin/bash
# EA read-request counters by size, one --pmc pass each (kernel-trace only),
# over bench.py: k_stream_read (exactly 512 MiB read) calibrates bytes/request
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
for c in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc2/$c -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/pmc2/$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmc2/$c.log; exit 1; }
  echo "pass $c ok"
done
