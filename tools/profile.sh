# rocprofv3 collection for one workload: kernel trace + stats, then the HBM
# counters in separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one
# pass on gfx950).  Usage: bash tools/profile.sh <tag> [prof_run.py args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_run.py "$@" > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 3; }
tail -2 $OUT/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/prof_run.py "$@" > $OUT/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $OUT/fetch.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/prof_run.py "$@" > $OUT/write.log 2>&1 || { echo "write failed"; tail -20 $OUT/write.log; exit 3; }
find $OUT -name "*.csv" | head -20
