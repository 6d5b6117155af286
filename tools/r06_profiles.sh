#!/bin/bash
# Round-6 profile collection on the GPU box (each step its own time limit,
# chained: a failed step ends the call).  Unit counters (tools/pmc_passes.sh,
# the counter set of profiles/r05_c4sr_units.md) of
#   c3u    C3's headline launch (k_sr1_dia_m<double, 2, ...>, bench --workload c3)
#   slabu  C4's N = 8 slab on a 1-rank RCCL communicator (tools/dist_probe.py 50)
#   c4u    C4's headline launch (the comparison row)
#   c5u    C5's column-panel SpMV (k_spmv_csr<float ...>, 6 launches per SpMV)
# and rocprofv3 traces + byte passes (tools/profile.sh) of
#   c3sr / c4sr / c4n8 / c4csr / c5   as tools/r05_profiles.sh
# Summaries:
#   python tools/pmc_units.py r06c3u "k_sr1_dia_m<double, 2"
#   python tools/pmc_units.py r06slabu "k_sr1_dia_m<double, 4"
#   python tools/pmc_units.py r06c5u "k_spmv_csr<float" 6
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --no-legs --no-cpu --steps 30 --warmup 5"
steps=${*:-c3u slabu}
for what in $steps; do
  case $what in
    c3u)   bash tools/pmc_passes.sh r06c3u $B --workload c3 --alg sr || exit $? ;;
    slabu) bash tools/pmc_passes.sh r06slabu python3 tools/dist_probe.py 50 --cases=sr || exit $? ;;
    c4u)   bash tools/pmc_passes.sh r06c4u $B --alg sr || exit $? ;;
    c5u)   bash tools/pmc_passes.sh r06c5u $B --workload c5 || exit $? ;;
    c3sr)  bash tools/profile.sh r06c3sr $B --workload c3 --alg sr || exit $? ;;
    c4sr)  bash tools/profile.sh r06c4sr $B --alg sr || exit $? ;;
    c4n8)  bash tools/profile.sh r06c4n8 python3 tools/dist_probe.py 50 --cases=sr || exit $? ;;
    c4csr) bash tools/profile.sh r06c4csr $B --layout csr --alg hs || exit $? ;;
    c5)    bash tools/profile.sh r06c5 $B --workload c5 || exit $? ;;
  esac
done
echo "r06 profiles done"
