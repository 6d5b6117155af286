"""Two RCCL ranks on ONE GPU: each rank's process sets a host id of its own
(NCCL_HOSTID) before RCCL initialises, so RCCL's duplicate-GPU check (same
host, same bus id) does not apply and the ranks connect over its socket
transport on the loopback interface.  Not the xGMI path -- but the ranks'
ncclSend/Recv pairing, the group calls, the all-reduces and the graph capture
of all of them then run between real peers on hardware.  The cases of
tests/test_gpu_rccl_multi.py; every rank's x must be bit-identical to the
in-process group of the same partitions.
  python tools/rccl_pair_probe.py [world]"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))


# tests/test_gpu_rccl_multi.py's cases and its in-process reference (the
# test module imports torch, which this probe does not need)
SHAPE = (40, 30, 24)
SHAPE1 = (32, 48, 24)
CASES = [("hs", True, SHAPE), ("hs", False, SHAPE), ("sr", "auto", SHAPE), ("cg1", False, SHAPE),
         ("sr", "auto", SHAPE1)]


def pair_env(rank):
    e = dict(os.environ)
    e.update(NCCL_HOSTID=f"cgx-pair-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
             MASTER_ADDR="127.0.0.1")
    return e


def local(alg, fused, world, shape):
    import numpy as np
    import cgx
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, world)
    try:
        parts[0].set_alg({"hs": cgx.CGX_ALG_HS, "sr": cgx.CGX_ALG_SR, "cg1": cgx.CGX_ALG_CG1}[alg])
        parts[0].set_fused(fused)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, world, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        its = parts[0].run(3000, 1e-10)
        return its, [d.x() for d in parts]
    finally:
        parts[0].close()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    os.environ.update(NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    import numpy as np
    out = Path(tempfile.mkdtemp(prefix="cgx_pair_"))
    # the children start before this process touches the GPU (rank 0 makes
    # the communicators' unique ids)
    procs = [subprocess.Popen([sys.executable, "-u", __file__, "--child", str(r), str(world), str(out)],
                              env=pair_env(r)) for r in range(world)]
    rcs = [p.wait() for p in procs]
    print("children:", rcs, flush=True)
    if any(rcs):
        return 1
    bad = 0
    for alg, fused, shape in CASES:
        its_l, xs_l = local(alg, fused, world, shape)
        for rank in range(world):
            tag = f"{alg}_{fused}_{shape[0]}_{rank}"
            its, fz, graph, march = np.load(out / f"its_{tag}.npy")
            x = np.load(out / f"x_{tag}.npy")
            same = np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64))
            rel = float(np.linalg.norm(x - xs_l[rank]) / np.linalg.norm(xs_l[rank]))
            # two ranks: bit-identical (a + b is the local group's fixed-order
            # sum); more: RCCL's ring adds the ranks' sums in its own order
            close = same if world == 2 else rel <= 1e-12
            ok = its == its_l and close and graph == (0 if os.environ.get("CGX_PAIR_GRAPH") == "0" else 1) and fz == (1 if alg == "sr" or fused is True else 0)
            bad += not ok
            print("%-4s fused %-5s shape %-12s rank %d: its %d (local %d) fused %d graph %d march %d "
                  "x bit-identical %s rel %.2e %s" % (alg, fused, shape, rank, its, its_l, fz, graph,
                                                     march, same, rel, "ok" if ok else "MISMATCH"),
                  flush=True)
    return 1 if bad else 0


def child(rank, world, out):
    order = os.environ.get("CGX_PAIR_TORCH", "")
    if order == "first":
        # as in bench.py's ranks: torch (and its bundled RCCL) loaded before libcgx
        import torch  # noqa: F401
    import numpy as np
    import cgx as c
    if order == "after":
        c.lib()
        import torch  # noqa: F401,F811
    c.lib()
    if os.environ.get("CGX_PAIR_BT"):  # native backtrace on SIGSEGV (tools/segv_bt.c)
        import ctypes
        ctypes.CDLL(str(REPO / "tools" / "segv_bt.so"))
    algs = {"hs": c.CGX_ALG_HS, "sr": c.CGX_ALG_SR, "cg1": c.CGX_ALG_CG1}
    out = Path(out)
    if rank == 0:
        for name in ("uid", "uid1"):
            (out / (name + ".tmp")).write_bytes(c.dist_unique_id())
            os.replace(out / (name + ".tmp"), out / name)
    import time
    t0 = time.time()
    while not (out / "uid1").exists():
        if time.time() - t0 > 60:
            raise RuntimeError("no unique id from rank 0")
        time.sleep(0.05)
    uid, uid1 = (out / "uid").read_bytes(), (out / "uid1").read_bytes()
    for shape in (SHAPE, SHAPE1):
        rp, col, val = c.laplacian3d(*shape)
        b = np.random.default_rng(11).standard_normal(len(rp) - 1)
        n = len(rp) - 1
        rb, re_ = c.partition_rows(n, world, rank)
        d = c.DistSolver(0, world, rank, uid if shape == SHAPE else uid1)
        try:
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
            if os.environ.get("CGX_PAIR_GRAPH") == "0":
                d.set_graph(False)
            for alg, fused, sh in CASES:
                if sh != shape:
                    continue
                d.set_alg(algs[alg])
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
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        sys.exit(child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]))
    sys.exit(main())
