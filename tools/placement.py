"""Per-instance SpMV time vs device addresses: K identical C3 solvers in one
process, order-rotated rounds; prints each instance's median SpMV / iteration
time (the pointers come from CGX_DEBUG_PTRS on stderr)."""
import os, statistics, sys
sys.path.insert(0, "conjugate-gradient_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch  # noqa
import bench, cgx
K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
os.environ["CGX_DEBUG_PTRS"] = "1"
sysm = bench.make_system(bench.WORKLOADS["c3"])
S = []
for k in range(K):
    s = cgx.Solver(0)
    s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
    s.set_rhs(sysm["b"])
    s.bench_prepare(3)
    S.append(s)
res = [[] for _ in range(K)]
it = [[] for _ in range(K)]
for r in range(6):
    for j in range(K):
        k = (j + r) % K
        _, sp = S[k].bench_run(30, graph=False, spmv_events=True)
        tot, _ = S[k].bench_run(30, graph=True)
        res[k].append(sp * 1e3); it[k].append(tot / 30 * 1e3)
for k in range(K):
    print(f"inst {k}: spmv {statistics.median(res[k]):7.2f} us  iter {statistics.median(it[k]):7.2f} us", flush=True)
