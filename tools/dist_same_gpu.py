"""Two RCCL ranks on ONE GPU (validation of the multi-process path on a
1-GPU box): each rank solves its half of a 3-D Laplacian with cgx_dist over
RCCL; rank 0 checks x against the in-process 2-partition solve."""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
sys.path.insert(0, str(REPO / "tests"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import numpy as np  # noqa: E402
import cgx  # noqa: E402
import helpers as H  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
uid = [cgx.dist_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
rp, col, val = cgx.laplacian3d(40, 30, 24)
n = len(rp) - 1
rb, re_ = cgx.partition_rows(n, world, rank)
d = cgx.DistSolver(0, world, rank, uid[0])
d.set_matrix(n, rp[rb:re_ + 1] - rp[rb], col[rp[rb]:rp[re_]], val[rp[rb]:rp[re_]])
d.set_rhs(np.ones(re_ - rb))
its = d.run(500, 1e-10)
xs = [None] * world
dist.all_gather_object(xs, d.x().tolist())
if rank == 0:
    x = np.array(sum(xs, []))
    x_ref, its_ref, _ = H.o_solve(500, 1e-10, rp, col, val, np.ones(n), cg1=True)
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    print(f"RCCL 2 ranks on one GPU: its {its} (oracle {its_ref}) rel err {err:.2e}")
    assert abs(its - its_ref) <= 1 and err < 1e-9
d.close()
dist.destroy_process_group()
