#!/bin/bash
# tools/ab_check.sh <pytest -k expr> -- the selected GPU tests against the
# product build and every ab/<exp> variant (tools/ab_build.sh), one pytest
# process per library, each under its own time limit; stops at the first
# failure.  Output: gpurun_out/abcheck_<lib>.log
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in ${AB_LIBS:-conjugate-gradient_amd/lib/libcgx.so ab/*/libcgx.so}; do
  tag=$(echo "$lib" | tr '/' '_')
  CGX_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "$1" > gpurun_out/abcheck_$tag.log 2>&1
  rc=$?
  echo "$lib: $(tail -1 gpurun_out/abcheck_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
done
