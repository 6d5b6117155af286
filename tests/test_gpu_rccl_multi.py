"""GPU, >= 2 devices: the partitioned solver over a real multi-rank RCCL
communicator -- ncclSend/Recv halos between ranks and ncclAllReduce of both
recurrences, fused and unfused HS and SR (one all-reduce; on a shape whose
planes the march fits, the one-launch k_sr1_dia_m step on the in-place
numbering), graph-replayed -- one fresh child process
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
SHAPE1 = (32, 48, 24)  # planes 3 slices apart: SR runs the one-launch march step
CASES = [("hs", True, SHAPE), ("hs", False, SHAPE), ("sr", "auto", SHAPE), ("cg1", False, SHAPE),
         ("sr", "auto", SHAPE1)]
ALGS = {"hs": cgx.CGX_ALG_HS, "sr": cgx.CGX_ALG_SR, "cg1": cgx.CGX_ALG_CG1}


def _fused_expected(alg, fused):
    return 1 if alg == "sr" or fused is True else 0


def _system(shape):
    rp, col, val = cgx.laplacian3d(*shape)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    return rp, col, val, b


def _worker(rank, world, uid, uid1, out_dir):
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo / "conjugate-gradient_amd"))
    import cgx as c
    for shape in (SHAPE, SHAPE1):
        rp, col, val = c.laplacian3d(*shape)
        b = np.random.default_rng(11).standard_normal(len(rp) - 1)
        n = len(rp) - 1
        rb, re_ = c.partition_rows(n, world, rank)
        d = c.DistSolver(rank, world, rank, uid if shape == SHAPE else uid1)
        try:
            d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
            d.set_rhs(b[rb:re_])
            for alg, fused, sh in CASES:
                if sh != shape:
                    continue
                d.set_alg({"hs": c.CGX_ALG_HS, "sr": c.CGX_ALG_SR, "cg1": c.CGX_ALG_CG1}[alg])
                d.set_fused(fused)
                its = d.run(3000, 1e-10)
                tag = f"{alg}_{fused}_{sh[0]}_{rank}"
                np.save(os.path.join(out_dir, f"x_{tag}.npy"), d.x())
                i = d.info()
                np.save(os.path.join(out_dir, f"its_{tag}.npy"),
                        np.array([its, i["fused"], i["graph"], i["march"]]))
        finally:
            d.close()


def _local(alg, fused, world, shape):
    rp, col, val, b = _system(shape)
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
    uid, uid1 = cgx.dist_unique_id(), cgx.dist_unique_id()
    mp.start_processes(_worker, args=(world, uid, uid1, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for alg, fused, shape in CASES:
        its_l, xs_l = _local(alg, fused, world, shape)
        for rank in range(world):
            tag = f"{alg}_{fused}_{shape[0]}_{rank}"
            its, fz, graph, march = np.load(tmp_path / f"its_{tag}.npy")
            assert its == its_l, (alg, fused, shape)
            assert fz == _fused_expected(alg, fused) and graph == 1
            assert (march > 0) == (shape == SHAPE1), (alg, shape)
            x = np.load(tmp_path / f"x_{tag}.npy")
            assert np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64)), (alg, fused, shape)


def _worker_refuse(rank, world, uid, out_dir):
    """Both ranks' captures refused before any RCCL call is recorded: the
    MIN / MAX agreement sends both eager with the results of the replayed
    graphs.  (The mixed case -- one rank refused, its peer captured, RCCL
    calls recorded on one side only -- is fatal by the same rule and is
    checked on a 1-rank communicator in test_gpu_dist.py: over real peers a
    one-sided capture may block in RCCL's lazy connection setup before the
    agreement is reached.)"""
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo / "conjugate-gradient_amd"))
    import cgx as c
    rp, col, val = c.laplacian3d(*SHAPE1)
    b = np.random.default_rng(11).standard_normal(len(rp) - 1)
    n = len(rp) - 1
    rb, re_ = c.partition_rows(n, world, rank)
    d = c.DistSolver(rank, world, rank, uid)
    try:
        d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
        d.set_rhs(b[rb:re_])
        d.set_alg(c.CGX_ALG_SR)
        d.debug_refuse_capture(1)
        its = d.run(3000, 1e-10)
        np.save(os.path.join(out_dir, f"x_refused_{rank}.npy"), d.x())
        np.save(os.path.join(out_dir, f"its_refused_{rank}.npy"), np.array([its, d.info()["graph"]]))
    finally:
        d.close()


def test_two_rank_capture_refusal_goes_eager_together(tmp_path):
    """VERDICT r05 #3 over real peers: graph or eager is one decision of all
    ranks (ensure_graphs' MIN / MAX all-reduce of the capture results)."""
    if cgx.lib().cgx_device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    world = 2
    uid = cgx.dist_unique_id()
    mp.start_processes(_worker_refuse, args=(world, uid, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    its_l, xs_l = _local("sr", "auto", world, SHAPE1)
    for rank in range(world):
        its, graph = np.load(tmp_path / f"its_refused_{rank}.npy")
        assert its == its_l and graph == -1
        x = np.load(tmp_path / f"x_refused_{rank}.npy")
        assert np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64))
