# rocprofv3 collection for a command: kernel trace + stats, then the HBM
# counters in separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one
# pass on gfx950; counters never combined with other tracing).
#   bash tools/profile.sh <tag> <program> [args...]      (program = python3 ...)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 3; }
grep '"metric"' $OUT/trace.log | tail -1 | cut -c1-300
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- "$@" > $OUT/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $OUT/fetch.log; exit 3; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- "$@" > $OUT/write.log 2>&1 || { echo "write failed"; tail -20 $OUT/write.log; exit 3; }
echo "profile $TAG done"
