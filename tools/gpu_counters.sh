#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1
grep -i -E "mall|dram|hbm|ea0_rd|ea0_wr|EA_|_MC_|umc|df_" gpurun_out/counters.txt | head -80
wc -l gpurun_out/counters.txt
