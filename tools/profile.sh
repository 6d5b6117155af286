# rocprofv3 collection for a command: kernel trace + stats, then memory-side
# counters in separate --pmc passes (counters never combined with other
# tracing; one counter per pass).
#   bash tools/profile.sh <tag> <program> [args...]      (program = python3 ...)
# Bytes: FETCH_SIZE / WRITE_SIZE (KiB; the guide's gfx950 rule doubles
# FETCH_SIZE for 16-B streams) and the size-resolved EA request counters
# (TCC_EA0_RDREQ_{32B,64B,128B}, TCC_EA0_WRREQ{,_64B}), calibrated on the
# bench's own k_stream_read (exactly 512 MiB read = RDREQ_128B x 128 B).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
echo "$*" > $OUT/cmd.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 3; }
grep '"metric"' $OUT/trace.log | tail -1 | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- "$@" > $OUT/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $OUT/pmc_$c.log; exit 3; }
done
echo "profile $TAG done"
