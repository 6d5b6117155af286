#!/bin/bash
# Round-5 profile collection on the GPU box (each step its own time limit,
# chained with &&): the C4 headline SR launch (trace + single-counter byte
# passes), its unit counters, C4's N = 8 slab on a 1-rank RCCL communicator
# (the rank kernel the N > 1 line prices), the plain-CSR SpMV at C3 / C4
# (the north-star figure) and C5's column-panel SpMV.  Summaries:
#   python tools/pmc_summary.py r05c4sr r05 c4_sr1 3904000000 "k_sr1_dia_m<double, 4"
#   python tools/pmc_summary.py r05c4n8 r05 c4n8_sr1 488000000 "k_sr1_dia_m<double, 4"
#   (c4n4 / c4n2: 976000000 / 1952000000 bytes, the N = 4 / 2 slabs)
#   python tools/pmc_units.py r05c4sr "k_sr1_dia_m<double, 4"
#   python tools/pmc_summary.py r05c3csr r05 c3_csr 1044721156 "k_spmv_csr<double, 456, 7, true"
#   python tools/pmc_summary.py r05c4csr r05 c4_csr 6644480004 "k_spmv_csr<double, 456, 7, true"
#   python tools/pmc_summary.py r05c5 r05 c5_panel <bytes> "k_spmv_csr<float" r05 sum
#   python tools/pmc_summary.py r05c3dv r05 c3dv_sr1 <bytes> "k_sr1_dia_m<double, 2"
#   (C3 general coefficients on DIA-V: 1,159 MB = 115 B per row x 10,077,696)
#   python tools/pmc_summary.py r05c3sr r05 c3_sr1 594584064 "k_sr1_dia_m<double, 2"
#   (C3's headline launch: 59 B per row x 10,077,696)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --no-legs --no-cpu --steps 30 --warmup 5"
steps=${*:-c4sr c4n8 units c3csr c4csr c5}
for what in $steps; do
  case $what in
    c4sr)  bash tools/profile.sh r05c4sr $B --alg sr || exit $? ;;
    c4n8)  bash tools/profile.sh r05c4n8 python3 tools/dist_probe.py 50 --cases=sr || exit $? ;;
    c4n4)  bash tools/profile.sh r05c4n4 python3 tools/dist_probe.py 100 --cases=sr || exit $? ;;
    c4n2)  bash tools/profile.sh r05c4n2 python3 tools/dist_probe.py 200 --cases=sr || exit $? ;;
    units) bash tools/pmc_passes.sh r05c4sr $B --alg sr || exit $? ;;
    c3csr) bash tools/profile.sh r05c3csr $B --workload c3 --layout csr --alg hs || exit $? ;;
    c4csr) bash tools/profile.sh r05c4csr $B --layout csr --alg hs || exit $? ;;
    c5)    bash tools/profile.sh r05c5 $B --workload c5 || exit $? ;;
    c3dv)  bash tools/profile.sh r05c3dv python3 tools/dv_probe.py || exit $? ;;
    c3sr)  bash tools/profile.sh r05c3sr $B --workload c3 --alg sr || exit $? ;;
  esac
done
echo "r05 profiles done"
