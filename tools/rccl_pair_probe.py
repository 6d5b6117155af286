"""RCCL ranks as separate processes, one per rank, sharing ONE GPU (or one
GPU each with --own-gpus): tests/rccl_ranks.py's cases, every rank's x
against the in-process group of the same partitions -- bit-identical at two
ranks, within 1e-12 at more (RCCL's ring adds the partial sums in its own
order).  Diagnosis switches (environment, read by the ranks):
  CGX_PAIR_TORCH=first  import torch before libcgx (binds PyTorch's bundled
                        HIP / RCCL: the hipStreamEndCapture crash of
                        profiles/r06_rccl_pair.log)
  CGX_PAIR_GRAPH=0      eager iterations (no capture)
  CGX_DIST_TRACE=1      libcgx prints its capture / replay steps
  python tools/rccl_pair_probe.py [world] [--own-gpus]"""
import os
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import rccl_ranks as R  # noqa: E402


def main():
    import numpy as np
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    world = int(args[0]) if args else 2
    out = Path(tempfile.mkdtemp(prefix="cgx_pair_"))
    # the ranks start before this process touches the GPU
    rcs = R.run(world, out, "cases", share="--own-gpus" not in sys.argv, timeout=240)
    print("ranks:", rcs, flush=True)
    if any(rcs):
        return 1
    want_graph = 0 if os.environ.get("CGX_PAIR_GRAPH") == "0" else 1
    bad = 0
    for alg, fused, shape in R.CASES:
        its_l, xs_l = R.local(alg, fused, world, shape)
        for rank in range(world):
            tag = f"{alg}_{fused}_{shape[0]}_{rank}"
            its, fz, graph, march = np.load(out / f"its_{tag}.npy")
            x = np.load(out / f"x_{tag}.npy")
            same = np.array_equal(x.view(np.uint64), xs_l[rank].view(np.uint64))
            rel = float(np.linalg.norm(x - xs_l[rank]) / np.linalg.norm(xs_l[rank]))
            close = same if world == 2 else rel <= 1e-12
            ok = (its == its_l and close and graph == want_graph and
                  fz == R.fused_expected(alg, fused))
            bad += not ok
            print("%-4s fused %-5s shape %-12s rank %d: its %d (local %d) fused %d graph %d march %d "
                  "x bit-identical %s rel %.2e %s" % (alg, fused, shape, rank, its, its_l, fz, graph,
                                                     march, same, rel, "ok" if ok else "MISMATCH"),
                  flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
