#!/bin/bash
# tools/ab_probe.sh <rounds> <probe.py> [probe args] -- a probe alternated
# between the product build and the ab/<exp> variant builds present
# (tools/ab_build.sh) -- or the libraries listed in AB_LIBS -- same box, e.g.
#   gpurun -- bash tools/ab_probe.sh 2 tools/fused_probe.py --modes=on 3:216 3:400
set -u
cd "$(dirname "$0")/.."
rounds=$1; probe=$2; shift 2
for r in $(seq "$rounds"); do
  for lib in ${AB_LIBS:-conjugate-gradient_amd/lib/libcgx.so ab/*/libcgx.so}; do
    echo "== $lib"
    CGX_LIB=$PWD/$lib timeout -k 10 150 python3 "$probe" "$@" || exit $?
  done
done
