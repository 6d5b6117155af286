# Unit-level PMC passes of a command (rocprofv3), each pass its own run and
# within gfx950's per-pass slots (MI355X_MICROARCH.md: <= 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 TD, 2 GRBM), counters never combined with other tracing:
#   bash tools/pmc_passes.sh <tag> <program> [args...]
# -> gpurun_out/pmcu_<tag>/p<i>/run_counter_collection.csv, summarised per
# kernel by tools/pmc_units.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmcu_$TAG
mkdir -p $OUT
echo "$*" > $OUT/cmd.txt
PASSES=(
  "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum"
  "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
)
i=0
for p in "${PASSES[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 \
    || { echo "pmc pass $i ($p) failed"; tail -5 $OUT/p$i.log; exit 3; }
  i=$((i + 1))
done
echo "pmc passes $TAG done"
