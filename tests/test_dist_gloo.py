"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): each process
builds its partition with libcgx's partition layer, exchanges ghost requests,
then runs the distributed recurrence with the same communication pattern as
the GPU solver -- Chronopoulos-Gear: halo of r point-to-point, ONE all-reduce
of (gamma, delta) per iteration; HS: halo of p, one all-reduce of p.s and one
of r.r; fused HS: the halo carries p_new = r + beta p_old computed at the send
rows, x updated in pairs; SR: the fused HS protocol with ONE all-reduce of
(p.s, s.s, r.r) per iteration, beta and the stop test from alpha^2 s.s - r.r --
and the gathered x is checked against the serial oracle (fused HS:
bit-identical to the HS protocol's; SR: against oracle_solve_sr)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, out_path, alg="cg1"):
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo / "conjugate-gradient_amd"))
    sys.path.insert(0, str(repo / "tests"))
    import cgx
    import helpers as H
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind == "lap3d":
        nx, ny, nz = 10, 9, 12
        n = nx * ny * nz
        rb, re_ = cgx.partition_rows(n, world, rank)
        rp, col, val = cgx.laplacian3d(nx, ny, nz, rb, re_)
        b = np.ones(re_ - rb)
    else:
        n = 1200
        rb, re_ = cgx.partition_rows(n, world, rank)
        rp, col, val = cgx.random_spd(n, 6, 3, rb, re_)
        b = np.random.default_rng(9).standard_normal(n)[rb:re_]
    P = cgx.Partition(n, world, rank, rp, col)
    ghosts, recv = P.ghosts(), P.recv_counts()
    roff = np.concatenate([[0], np.cumsum(recv)[:-1]])
    # exchange requests: everyone learns what everyone needs from it
    allg = [None] * world
    dist.all_gather_object(allg, (ghosts.tolist(), recv.tolist()))
    counts = [allg[p][1][rank] for p in range(world)]
    glob = []
    for p in range(world):
        gp, rc = allg[p]
        off = int(np.sum(rc[:rank]))
        glob += gp[off:off + rc[rank]]
    P.set_requests(counts, np.array(glob, np.int32))
    scount, slocal = P.send_counts(), P.send_local()
    soff = np.concatenate([[0], np.cumsum(scount)[:-1]])
    lcol = P.local_cols()
    n_loc = re_ - rb

    def halo(r):
        reqs, bufs = [], {}
        for q in range(world):
            if q == rank:
                continue
            if scount[q]:
                t = torch.from_numpy(r[slocal[soff[q]:soff[q] + scount[q]]].copy())
                reqs.append(dist.isend(t, q))
            if recv[q]:
                bufs[q] = torch.empty(int(recv[q]), dtype=torch.float64)
                reqs.append(dist.irecv(bufs[q], q))
        for rq in reqs:
            rq.wait()
        ext = np.zeros(len(ghosts))
        for q, t in bufs.items():
            ext[roff[q]:roff[q] + recv[q]] = t.numpy()
        return np.concatenate([r, ext])

    def allreduce(a, c):
        t = torch.tensor([a, c], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t[0]), float(t[1])

    def halo_vals(vals_for, own):
        # the fused step's halo: each rank sends values it computes at its
        # send rows (p_new = r + beta p_old), received into the ghost tail
        reqs, bufs = [], {}
        for q in range(world):
            if q == rank:
                continue
            if scount[q]:
                t = torch.from_numpy(vals_for(slocal[soff[q]:soff[q] + scount[q]]).copy())
                reqs.append(dist.isend(t, q))
            if recv[q]:
                bufs[q] = torch.empty(int(recv[q]), dtype=torch.float64)
                reqs.append(dist.irecv(bufs[q], q))
        for rq in reqs:
            rq.wait()
        ext = np.zeros(len(ghosts))
        for q, t in bufs.items():
            ext[roff[q]:roff[q] + recv[q]] = t.numpy()
        return np.concatenate([own, ext])

    maxit, tol = 500, 1e-10
    if alg == "sr":  # cgx_dist.cpp's CGX_ALG_SR: one all-reduce per iteration
        def allreduce3(a, c, e):
            t = torch.tensor([a, c, e], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t[0]), float(t[1]), float(t[2])
        x = np.zeros(n_loc)
        r = b.copy()
        rr_loc = float(np.dot(r, r))      # the prologue's local b.b
        t = torch.tensor([rr_loc], dtype=torch.float64)
        dist.all_reduce(t)
        bb = float(t[0])
        k, beta, first, p_old = 0, 0.0, True, None
        while True:
            if first:
                p_new = r.copy()
                ext = halo_vals(lambda idx: r[idx], p_new)
            else:
                p_new = r + beta * p_old
                ext = halo_vals(lambda idx: r[idx] + beta * p_old[idx], p_new)
            s = H.o_spmv(rp, lcol, val, ext)
            ps, ss, rr = allreduce3(float(np.dot(p_new, s)), float(np.dot(s, s)), rr_loc)
            # the previous iteration's stop test on the exact r.r, one
            # reduction late (cg.c:125's rule; oracle_solve_sr)
            if k >= 1 and (k - 1 == maxit or rr <= tol * tol * bb):
                break
            alpha = rr / ps
            x = x + alpha * p_new
            r = r - alpha * s
            rr_loc = float(np.dot(r, r))  # reduced with the next p.s, s.s
            est = max(alpha * (alpha * ss) - rr, 0.0)
            beta, first = est / rr, False  # the estimate: beta only
            p_old = p_new
            k += 1
        xs = [None] * world
        dist.all_gather_object(xs, x.tolist())
        if rank == 0:
            np.save(out_path, np.array(sum(xs, [])))
            np.save(out_path + ".its.npy", np.array([k]))
        dist.destroy_process_group()
        return
    if alg == "hs_fused":  # cgx_dist.cpp's fused step: pack p_new, x in pairs
        def allreduce1(a):
            t = torch.tensor([a], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t[0])
        x = np.zeros(n_loc)
        r = b.copy()
        p_old = b.copy()
        rr = allreduce1(float(np.dot(r, r)))
        bb, k, beta, first = rr, 0, 0.0, True
        pend = []  # deferred (alpha, p) x updates, applied in pairs
        while True:
            if first:
                p_new = r.copy()
                ext = halo_vals(lambda idx: r[idx], p_new)
            else:
                p_new = r + beta * p_old
                ext = halo_vals(lambda idx: r[idx] + beta * p_old[idx], p_new)
            s = H.o_spmv(rp, lcol, val, ext)
            alpha = rr / allreduce1(float(np.dot(p_new, s)))
            pend.append((alpha, p_new))
            r = r - alpha * s
            rr_new = allreduce1(float(np.dot(r, r)))
            stop = k == maxit or rr_new <= tol * tol * bb
            if len(pend) == 2 or stop:
                for a_, p_ in pend:
                    x = x + a_ * p_
                pend = []
            if stop:
                break
            beta, first = rr_new / rr, False
            p_old = p_new
            rr = rr_new
            k += 1
        xs = [None] * world
        dist.all_gather_object(xs, x.tolist())
        if rank == 0:
            np.save(out_path, np.array(sum(xs, [])))
            np.save(out_path + ".its.npy", np.array([k + 1]))
        dist.destroy_process_group()
        return
    if alg == "hs":  # cg.c:88-141 with the two dots all-reduced
        def allreduce1(a):
            t = torch.tensor([a], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t[0])
        x = np.zeros(n_loc)
        r = b.copy()
        p = b.copy()
        rr = allreduce1(float(np.dot(r, r)))
        bb, k = rr, 0
        while True:
            s = H.o_spmv(rp, lcol, val, halo(p))
            alpha = rr / allreduce1(float(np.dot(p, s)))
            x = x + alpha * p
            r = r - alpha * s
            rr_new = allreduce1(float(np.dot(r, r)))
            if k == maxit or rr_new <= tol * tol * bb:
                break
            p = r + (rr_new / rr) * p
            rr = rr_new
            k += 1
        xs = [None] * world
        dist.all_gather_object(xs, x.tolist())
        if rank == 0:
            np.save(out_path, np.array(sum(xs, [])))
            np.save(out_path + ".its.npy", np.array([k + 1]))
        dist.destroy_process_group()
        return
    x = np.zeros(n_loc)
    r = b.copy()
    p = np.zeros(n_loc)
    s = np.zeros(n_loc)
    w = H.o_spmv(rp, lcol, val, halo(r))
    gamma, delta = allreduce(float(np.dot(r, r)), float(np.dot(w, r)))
    bb = gamma
    alpha, beta, k = gamma / delta, 0.0, 0
    while True:
        p = r + beta * p
        s = w + beta * s
        x = x + alpha * p
        r = r - alpha * s
        w = H.o_spmv(rp, lcol, val, halo(r))
        g_new, delta = allreduce(float(np.dot(r, r)), float(np.dot(w, r)))
        if k == maxit or g_new <= tol * tol * bb:
            break
        beta = g_new / gamma
        alpha = g_new / (delta - beta * g_new / alpha)
        gamma = g_new
        k += 1
    xs = [None] * world
    dist.all_gather_object(xs, x.tolist())
    if rank == 0:
        np.save(out_path, np.array(sum(xs, [])))
        np.save(out_path + ".its.npy", np.array([k + 1]))
    dist.destroy_process_group()


@pytest.mark.parametrize("alg", ["cg1", "hs", "hs_fused", "sr"])
@pytest.mark.parametrize("kind", ["lap3d", "rand"])
def test_distributed_world2_gloo(kind, alg, tmp_path):
    import helpers as H
    import cgx
    out = str(tmp_path / "x.npy")
    mp.start_processes(_worker, args=(2, _free_port(), kind, out, alg), nprocs=2,
                       join=True, start_method="spawn")
    x = np.load(out)
    its = int(np.load(out + ".its.npy")[0])
    if kind == "lap3d":
        rp, col, val = cgx.laplacian3d(10, 9, 12)
        b = np.ones(len(rp) - 1)
    else:
        rp, col, val = cgx.random_spd(1200, 6, 3)
        b = np.random.default_rng(9).standard_normal(1200)
    x_ref, its_ref, _ = H.o_solve(500, 1e-10, rp, col, val, b, cg1=alg == "cg1", sr=alg == "sr")
    if alg == "hs_fused":  # the same values as the HS protocol's, bit for bit
        out2 = str(tmp_path / "x_hs.npy")
        mp.start_processes(_worker, args=(2, _free_port(), kind, out2, "hs"), nprocs=2,
                           join=True, start_method="spawn")
        assert its == int(np.load(out2 + ".its.npy")[0])
        assert np.array_equal(x.view(np.uint64), np.load(out2).view(np.uint64))
    assert abs(its - its_ref) <= 1
    assert np.linalg.norm(x - x_ref) <= 1e-9 * np.linalg.norm(x_ref)
    res = b - H.o_spmv(rp, col, val, x)
    assert np.linalg.norm(res) <= 2e-10 * np.linalg.norm(b)
