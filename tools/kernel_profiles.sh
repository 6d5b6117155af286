#!/bin/bash
# tools/kernel_profiles.sh <round> -- the rocprofv3 evidence bench.py prices
# its kernels with: for each headline-path kernel, a kernel
# trace + single-counter PMC passes (tools/profile.sh) of a short
# device-generated run (tools/fused_probe.py), and the unit counters of the
# N = 1 headline kernel (tools/pmc_passes.sh).  Summarise afterwards with
# tools/pmc_summary.py / tools/pmc_units.py (see tools/README.md).
#   c3_sr1     k_sr1_dia_m at C3 (the c3 leg's SR launch)
#   c4_march   k_spmv_dia_m at C4 (the hs_recurrence leg's fused HS launch)
#   c4_sr1     k_sr1_dia_m at C4 (the N = 1 headline launch)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rnd=${1:-r04}
bash tools/profile.sh ${rnd}c3sr python3 tools/fused_probe.py --sr --modes=auto 3:216 &&
bash tools/profile.sh ${rnd}c4hs python3 tools/fused_probe.py --modes=auto 3:400 &&
bash tools/profile.sh ${rnd}c4sr python3 tools/fused_probe.py --sr --modes=auto 3:400 &&
bash tools/pmc_passes.sh ${rnd}c4sr python3 tools/fused_probe.py --sr --modes=auto 3:400
