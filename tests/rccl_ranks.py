"""Multi-rank RCCL runs for the GPU tests (tests/test_gpu_rccl_multi.py) and
tools/rccl_pair_probe.py: one fresh child process per rank, started with
subprocess -- a child imports neither torch nor pytest, so libcgx binds the
ROCm it was built against (an `import torch` first would bind PyTorch's
bundled HIP / RCCL copies, whose hipStreamEndCapture crashed on the ranks'
captured halo: profiles/r06_rccl_pair.log).

share=True (fewer GPUs than ranks): every rank on GPU 0 with a host id of
its own (NCCL_HOSTID), so RCCL's duplicate-GPU check does not apply and the
ranks connect over its socket transport on the loopback interface -- not the
xGMI path, but the ranks' ncclSend/Recv pairing, group calls, all-reduces
and the graph capture of all of them between real peers.

  python tests/rccl_ranks.py --child RANK WORLD OUT MODE SHARE   (internal)"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent

SHAPE = (40, 30, 24)   # plane-aligned slabs: the fused HS step applies
SHAPE1 = (32, 48, 24)  # planes 3 slices apart: SR runs the one-launch march step
CASES = [("hs", True, SHAPE), ("hs", False, SHAPE), ("sr", "auto", SHAPE), ("cg1", False, SHAPE),
         ("sr", "auto", SHAPE1)]
C4_ITERS = 50  # mode "c4": fixed iterations of the row-partitioned 400^3 system


def _cgx():
    sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
    import cgx
    return cgx


def algs(cgx):
    return {"hs": cgx.CGX_ALG_HS, "sr": cgx.CGX_ALG_SR, "cg1": cgx.CGX_ALG_CG1}


def fused_expected(alg, fused):
    return 1 if alg == "sr" or fused is True else 0


def rank_env(rank, share):
    e = dict(os.environ)
    if share:
        e.update(NCCL_HOSTID=f"cgx-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    return e


def run(world, out, mode="cases", share=False, timeout=180, extra_env=None):
    """Runs the `world` ranks to completion; returns their exit codes (a rank
    still running at `timeout` s has its process group killed: -9)."""
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    procs = []
    for r in range(world):
        env = rank_env(r, share)
        env.update(extra_env or {})
        procs.append(subprocess.Popen(
            [sys.executable, "-u", str(Path(__file__).resolve()), "--child", str(r), str(world),
             str(out), mode, "1" if share else "0"], env=env, start_new_session=True))
    t_end = time.time() + timeout
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=max(1.0, t_end - time.time())))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, signal.SIGKILL)
            rcs.append(-9)
    for p in procs:
        p.wait()
    return rcs


def local(alg, fused, world, shape):
    """The in-process group of the same partitions (device copies, fixed-order
    sums): (iterations, [x of each partition])."""
    import numpy as np
    cgx = _cgx()
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, world)
    try:
        parts[0].set_alg(algs(cgx)[alg])
        parts[0].set_fused(fused)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, world, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        its = parts[0].run(3000, 1e-10)
        return its, [d.x() for d in parts]
    finally:
        parts[0].close()


def _uids(cgx, rank, out):
    if rank == 0:
        for name in ("uid", "uid1"):
            (out / (name + ".tmp")).write_bytes(cgx.dist_unique_id())
            os.replace(out / (name + ".tmp"), out / name)
    t0 = time.time()
    while not (out / "uid1").exists():
        if time.time() - t0 > 60:
            raise RuntimeError("no unique id from rank 0")
        time.sleep(0.05)
    return (out / "uid").read_bytes(), (out / "uid1").read_bytes()


def child(rank, world, out, mode, share):
    # diagnosis (tools/rccl_pair_probe.py): CGX_PAIR_TORCH=first binds
    # PyTorch's ROCm copies as bench.py's ranks did before round 6
    if os.environ.get("CGX_PAIR_TORCH") == "first":
        import torch  # noqa: F401
    import numpy as np
    cgx = _cgx()
    out = Path(out)
    dev = 0 if share else rank
    uid, uid1 = _uids(cgx, rank, out)
    if mode == "c4":
        # C4 (400^3) row-partitioned over the ranks: SR (the one-launch step)
        # and HS, 50 iterations each, b = 1
        nx = 400
        n = nx ** 3
        rb, re_ = cgx.partition_rows(n, world, rank)
        rp, col, val = cgx.laplacian3d(nx, nx, nx, rb, re_)
        d = cgx.DistSolver(dev, world, rank, uid)
        try:
            d.set_matrix(n, rp, col, val)
            d.set_rhs(np.ones(re_ - rb))
            for alg in ("sr", "hs"):
                d.set_alg(algs(cgx)[alg])
                its = d.run(C4_ITERS, 0.0)
                i = d.info()
                np.save(out / f"x_c4_{alg}_{rank}.npy", d.x())
                np.save(out / f"its_c4_{alg}_{rank}.npy",
                        np.array([its, i["fused"], i["graph"], i["march"], rb, re_]))
                print(f"rank {rank}: c4 {alg} its {its} graph {i['graph']} march {i['march']}",
                      flush=True)
        finally:
            d.close()
        return 0
    if mode == "versions":
        v = cgx.runtime_versions()
        np.save(out / f"versions_{rank}.npy", np.array([v["hip_runtime"], v["hip_compiled"],
                                                        v["rccl"]]))
        return 0
    for shape in (SHAPE, SHAPE1):
        if mode == "refuse" and shape != SHAPE1:
            continue
        rp, col, val = cgx.laplacian3d(*shape)
        b = np.random.default_rng(11).standard_normal(len(rp) - 1)
        n = len(rp) - 1
        rb, re_ = cgx.partition_rows(n, world, rank)
        d = cgx.DistSolver(dev, world, rank, uid if shape == SHAPE else uid1)
        try:
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
            if os.environ.get("CGX_PAIR_GRAPH") == "0":
                d.set_graph(False)
            if mode == "refuse":
                # both ranks refused before any RCCL call is recorded: eager together
                d.set_alg(cgx.CGX_ALG_SR)
                d.debug_refuse_capture(1)
                its = d.run(3000, 1e-10)
                np.save(out / f"x_refused_{rank}.npy", d.x())
                np.save(out / f"its_refused_{rank}.npy", np.array([its, d.info()["graph"]]))
                continue
            for alg, fused, sh in CASES:
                if sh != shape:
                    continue
                d.set_alg(algs(cgx)[alg])
                d.set_fused(fused)
                its = d.run(3000, 1e-10)
                tag = f"{alg}_{fused}_{sh[0]}_{rank}"
                np.save(out / f"x_{tag}.npy", d.x())
                i = d.info()
                np.save(out / f"its_{tag}.npy", np.array([its, i["fused"], i["graph"], i["march"]]))
                print(f"rank {rank}: {tag} its {its} graph {i['graph']}", flush=True)
        finally:
            d.close()
    return 0


if __name__ == "__main__":
    if len(sys.argv) == 7 and sys.argv[1] == "--child":
        sys.exit(child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5],
                       sys.argv[6] == "1"))
    sys.exit(__doc__)
