set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base:CGX_SPMV_XCD=0 xcd:CGX_SPMV_XCD=1 xcdnt:CGX_SPMV_XCD=1,CGX_SPMV_NT=1 nt:CGX_SPMV_NT=1; do
  name=${v%%:*}; envs=${v#*:}
  for kv in ${envs//,/ }; do export $kv; done
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/l2_$name -o run -- python3 tools/prof_run.py --workload c3 --iters 10 > gpurun_out/l2_$name.log 2>&1 || { echo "fail $name"; tail -5 gpurun_out/l2_$name.log; exit 3; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_$name -o run -- python3 tools/prof_run.py --workload c3 --iters 10 > gpurun_out/f_$name.log 2>&1 || { echo "fail f $name"; exit 3; }
  grep "spmv" gpurun_out/l2_$name.log | tail -1
  unset CGX_SPMV_XCD CGX_SPMV_NT
done
