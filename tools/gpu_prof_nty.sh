#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the default C3 bench after the nt=2 default; smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/profile.sh c3_nty python3 bench.py --steps 50 --warmup 10 --no-cpu || exit 1
