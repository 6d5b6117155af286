#!/bin/bash
# CSR-VI on the other Laplacian configs: C2 and C4 bench lines (with their coded_offsets /
# csr_plain legs), and the partitioned path on one GPU (1-rank RCCL communicator, HS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c2 --no-cpu > gpurun_out/bench_c2_vi.json 2> gpurun_out/bench_c2_vi.err || { tail gpurun_out/bench_c2_vi.err; exit 1; }
timeout -k 10 600 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_vi.json 2> gpurun_out/bench_c4_vi.err || { tail gpurun_out/bench_c4_vi.err; exit 1; }
timeout -k 10 300 python tools/dist_overhead1.py comm1 hs > gpurun_out/dist1_vi.log 2>&1 || { tail gpurun_out/dist1_vi.log; exit 1; }
grep us/iter gpurun_out/dist1_vi.log
for f in c2 c4; do python3 -c "
import json,sys;d=json.loads(open('gpurun_out/bench_${f}_vi.json').read().strip().splitlines()[-1])
r=d['roofline'];print('$f', d['value'], r['spmv_us'], r['kernel'][:20], (d.get('coded_offsets') or {}).get('value'), (d.get('coded_offsets') or {}).get('spmv_us'), (d.get('csr_plain') or {}).get('value'))"; done
