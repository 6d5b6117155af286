"""GPU, >= 2 devices: the partitioned solver over a real multi-rank RCCL
communicator -- ncclSend/Recv halos between ranks and ncclAllReduce of both
recurrences, fused and unfused HS and SR (one all-reduce), graph-replayed -- one fresh child process
per GPU (spawned; the children initialise their own device).  Every rank's x
must be bit-identical to the in-process group of the same partitions (the
same phase code with device copies and a fixed-order sum).  Skipped on a
1-GPU box (RCCL refuses two ranks on one GPU); bench.py's parity gate runs
the same comparison on the driver's 8-GPU node."""
import os

import numpy as np
import pytest

import cgx

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

SHAPE = (40, 30, 24)  # plane-aligned slabs at 2 ranks: the fused step applies
CASES = [("hs", True), ("hs", False), ("sr", "auto"), ("cg1", False)]
ALGS = {"hs": cgx.CGX_ALG_HS, "sr": cgx.CGX_ALG_SR, "cg1": cgx.CGX_ALG_CG1}


def _fused_expected(alg, fused):
    return 1 if alg == "sr" or fused is True else 0


def _system():
    rp, col, val = cgx.laplacian3d(*SHAPE)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    return rp, col, val, b


def _worker(rank, world, uid, out_dir):
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo / "conjugate-gradient_amd"))
    import cgx as c
    rp, col, val = c.laplacian3d(*SHAPE)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    rb, re_ = c.partition_rows(n, world, rank)
    d = c.DistSolver(rank, world, rank, uid)
    try:
        d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
        d.set_rhs(b[rb:re_])
        for alg, fused in CASES:
            d.set_alg({"hs": c.CGX_ALG_HS, "sr": c.CGX_ALG_SR, "cg1": c.CGX_ALG_CG1}[alg])
            d.set_fused(fused)
            its = d.run(3000, 1e-10)
            np.save(os.path.join(out_dir, f"x_{alg}_{fused}_{rank}.npy"), d.x())
            np.save(os.path.join(out_dir, f"its_{alg}_{fused}_{rank}.npy"),
                    np.array([its, d.info()["fused"], d.info()["graph"]]))
    finally:
        d.close()


def _local(alg, fused, world):
    rp, col, val, b = _system()
    n = len(rp) - 1
    parts = cgx.DistSolver.local_group(0, world)
    try:
        parts[0].set_alg(ALGS[alg])
        parts[0].set_fused(fused)
        for g, d in enumerate(parts):
            rb, re_ = cgx.partition_rows(n, world, g)
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
        its = parts[0].run(3000, 1e-10)
        return its, [d.x() for d in parts]
    finally:
        parts[0].close()


def test_two_rank_rccl_bit_identical_to_local_group(tmp_path):
    if cgx.lib().cgx_device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    world = 2
    uid = cgx.dist_unique_id()
    mp.start_processes(_worker, args=(world, uid, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for alg, fused in CASES:
        its_l, xs_l = _local(alg, fused, world)
        for rank in range(world):
            its, fz, graph = np.load(tmp_path / f"its_{alg}_{fused}_{rank}.npy")
            assert its == its_l, (alg, fused)
            assert fz == _fused_expected(alg, fused) and graph == 1
            x = np.load(tmp_path / f"x_{alg}_{fused}_{rank}.npy")
            assert np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64)), (alg, fused)
