set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/profile.sh c3_bench python3 bench.py --steps 50 --warmup 10 --no-cpu
