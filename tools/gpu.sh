#!/bin/bash
# tools/gpu.sh -- the GPU-side steps of this repo, one parameterised script
# (run on the MI355X box: gpurun -- bash tools/gpu.sh <step> [args]).
# Every step runs under its own timeout and writes under gpurun_out/.
#
#   tests [pytest args]          pytest -m gpu (thread timeouts, stops at the first failure)
#   smoke                        __graft_entry__.smoke()
#   bench [bench.py args]        one bench line -> gpurun_out/bench.json
#   lab [N rounds insitu list]   tools/mb/spmv_lab (build it first: see its header)
#   profile <tag> [bench args]   rocprofv3 trace + single-counter PMC passes (tools/profile.sh)
#
# Steps chain with &&: a failed, killed or timed-out step ends the call.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step=${1:-}; shift || true
case "$step" in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
      --timeout-method thread "$@" > gpurun_out/gputest.log 2>&1
    rc=$?; tail -5 gpurun_out/gputest.log; exit $rc ;;
  smoke)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?; tail -c 600 gpurun_out/bench.json; exit $rc ;;
  lab)
    timeout -k 10 300 tools/mb/bin/spmv_lab "$@" > gpurun_out/lab.log 2>&1
    rc=$?; cat gpurun_out/lab.log; exit $rc ;;
  profile)
    tag=$1; shift
    bash tools/profile.sh "$tag" python3 bench.py "$@" ;;
  *)
    sed -n '2,14p' "$0"; exit 2 ;;
esac
