#!/bin/bash
# Round-5 profile collection on the GPU box (each step its own time limit,
# chained with &&): the C4 headline SR launch (trace + single-counter byte
# passes), its unit counters, and C4's N = 8 slab on a 1-rank RCCL
# communicator (the rank kernel the N > 1 line prices).  Summaries:
#   python tools/pmc_summary.py c4sr r05 c4_sr1 3904000000 "k_sr1_dia_m<double, 4"
#   python tools/pmc_summary.py c4n8 r05 c4n8_sr1 488000000 "k_sr1_dia_m<double, 4"
#   python tools/pmc_units.py c4sr "k_sr1_dia_m<double, 4"
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
what=${1:-all}
if [ "$what" = all ] || [ "$what" = c4sr ]; then
  bash tools/profile.sh c4sr python3 bench.py --no-legs --no-cpu --steps 30 --warmup 5 --alg sr || exit $?
fi
if [ "$what" = all ] || [ "$what" = c4n8 ]; then
  bash tools/profile.sh c4n8 python3 tools/dist_probe.py 50 --cases=sr || exit $?
fi
if [ "$what" = all ] || [ "$what" = units ]; then
  bash tools/pmc_passes.sh c4sr python3 bench.py --no-legs --no-cpu --steps 30 --warmup 5 --alg sr || exit $?
fi
echo "r05 profiles done"
