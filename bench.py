#!/usr/bin/env python3
"""bench.py -- fp64 CG iterations/s on MI355X, with the SpMV roofline and the
CPU baseline beside it (BASELINE.json metric).

A "step" is one CG iteration of the device-resident solver (SpMV + dot
products + vector updates) on a synthetic SPD system already resident in
HBM.  Default workload (N = 1): C3, the 7-point 3-D Laplacian 216^3
(10,077,696 rows, 70,263,936 nnz, fp64, b = 1) -- BASELINE.json's HBM
roofline configuration.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c5]

N > 1 is launched by torch.distributed.run (one process per GPU); each rank
owns a 216^3-row slab of a 216 x 216 x (216 N) Laplacian (weak scaling), the
solver exchanges halo planes and all-reduces its dot products over RCCL.

Output: ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
sys.path.insert(0, str(REPO / "tests"))

METRIC = "fp64 CG iterations/sec + SpMV HBM GB/s (% of roofline), 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

WORKLOADS = {
    "c3": dict(desc="C3: 7-point 3-D Laplacian 216^3 (10,077,696 rows), fp64, b = 1",
               kind="lap3d", dims=(216, 216, 216), dtype="f64"),
    "c2": dict(desc="C2: 5-point 2-D Laplacian 1000^2 (1,000,000 rows), fp64, b = 1 "
                    "(working set fits the 256 MiB Infinity Cache)",
               kind="lap2d", dims=(1000, 1000), dtype="f64"),
    "c4": dict(desc="C4: 7-point 3-D Laplacian 400^3 (64,000,000 rows), fp64, b = 1, "
                    "row-partitioned over the ranks (strong scaling)",
               kind="lap3d", dims=(400, 400, 400), dtype="f64", strong=True),
    "c5": dict(desc="C5: random SPD 5,000,000 rows, 32 partners/row symmetrised "
                    "(~64 nnz/row), splitmix64 seed 42, fp32",
               kind="rand", n=5_000_000, partners=32, seed=42, dtype="f32"),
}


def make_system(wl, rank=0, world=1):
    import numpy as np
    import cgx
    if wl["kind"] == "lap3d":
        nx, ny, nz = wl["dims"]
        nz_g = nz if wl.get("strong") else nz * world
        n_g = nx * ny * nz_g
        rb, re_ = n_g * rank // world, n_g * (rank + 1) // world
        rp, col, val = cgx.laplacian3d(nx, ny, nz_g, rb, re_)
        return dict(rp=rp, col=col, val=val, b=np.ones(re_ - rb), n_global=n_g,
                    row_begin=rb, row_end=re_)
    if wl["kind"] == "lap2d":
        nx, ny = wl["dims"]
        ny_g = ny * world
        n_g = nx * ny_g
        rb, re_ = n_g * rank // world, n_g * (rank + 1) // world
        rp, col, val = cgx.laplacian2d(nx, ny_g, rb, re_)
        return dict(rp=rp, col=col, val=val, b=np.ones(re_ - rb), n_global=n_g,
                    row_begin=rb, row_end=re_)
    n = wl["n"]
    rp, col, val = cgx.random_spd(n, wl["partners"], wl["seed"], f32=True)
    b = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    return dict(rp=rp, col=col, val=val, b=b, n_global=n, row_begin=0, row_end=n)


def load_traffic(workload, alg):
    """HBM bytes per SpMV launch from the committed rocprofv3 PMC summary
    (profiles/pmc_<workload>.json, written by profiles/collect_pmc.py), or None."""
    p = REPO / "profiles" / f"pmc_{workload}.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get("spmv_hbm_bytes_per_launch")
    except Exception:
        return None


def spmv_layout_label(info, stream_bytes):
    """Kernel label for the layout a solver picked (coded columns, pairs)."""
    nd = info.get("n_dict", 0)
    label = spmv_kernel_label(stream_bytes)
    if nd and info.get("dict_vals", 0):
        return (f"k_spmv_vi (LDS-DMA code stream, value-indexed (offset, value) pairs: "
                f"{nd} pairs, 1 B/nnz, no value stream; one 64-row block per wave)")
    if nd:
        return label.replace("k_spmv_dma (LDS-DMA CSR-stream",
                             f"k_spmv_dc (LDS-DMA CSR-stream, dictionary-coded columns: "
                             f"{nd} offsets, 1 B/nnz")
    return label


def spmv_kernel_label(stream_bytes):
    """The SpMV kernel the solver selects (cgx_solver.cpp defaults, CGX_* knobs;
    nt by default only above kNtStreamBytes = 160 MiB of val+col)."""
    if os.environ.get("CGX_LAYOUT") == "sell":
        return "k_spmv_sell (SELL-64)"
    dma = os.environ.get("CGX_SPMV_DMA", "1")
    nt_env = os.environ.get("CGX_SPMV_NT")
    nt = (nt_env == "1") if nt_env is not None else (dma in ("1", "3") and stream_bytes > 160 * 2**20)
    name = {"0": "k_spmv_wave (register-staged CSR-stream, LDS row sums)",
            "1": "k_spmv_dma (LDS-DMA CSR-stream, LDS row sums)",
            "2": "k_spmv_pipe (persistent waves, LDS-DMA prefetch)",
            "8": "k_spmv_dma (LDS-DMA CSR-stream, 8 gathers per chunk)"}.get(dma, f"dma={dma}")
    return name + (", nt stream" if nt else "")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_mt(sysm, budget_s):
    """SURVEY.md 8d leg (c): the same CSR-sequential HS-CG with its row loops
    split over all host cores this job may use (oracle_solve_mt, pthreads;
    OMP_NUM_THREADS on the GPU box = the box's CPU share)."""
    import numpy as np
    import helpers as H
    rp, col, val, b = sysm["rp"], sysm["col"], sysm["val"], sysm["b"]
    if val.dtype != np.float64:
        val = val.astype(np.float64)
        b = b.astype(np.float64)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    t0 = time.perf_counter()
    H.o_solve_mt(0, 0.0, rp, col, val, b, threads)
    t1 = time.perf_counter() - t0
    its = max(1, min(2000, int(budget_s / max(t1, 1e-6))))
    t0 = time.perf_counter()
    _, done = H.o_solve_mt(its - 1, 0.0, rp, col, val, b, threads)
    dt = time.perf_counter() - t0
    return dict(value=done / dt, unit="it/s", cores=threads, kind="port",
                sample=f"{done} HS-CG iterations, row loops on {threads} threads "
                       f"(oracle_solve_mt), {dt:.1f} s")


def reference_c1(budget_s=2.0):
    """SURVEY.md 8d leg (a): the reference ITSELF (oracle/_ref/ref_harness =
    the reference's cg.c + mv_ops.c at its Makefile flags, built by
    `make -C oracle ref`) timing conj_grad on C1, the dense 128 SPD system --
    the one configuration where its O(n^2) dense-row SpMV is feasible.
    Returns None when the binary was not built (no /root/reference)."""
    import subprocess
    import tempfile
    import helpers as H
    exe = REPO / "oracle" / "_ref" / "ref_harness"
    if not exe.exists():
        return None
    rp, col, val, b = H.dense_spd(128, seed=1)
    maxit = 11  # ~tol 1e-10 on C1; conj_grad does maxit+1 SpMVs
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "c1.txt"
        H.write_ref_format(f, rp, col, val, b)
        probe = float(subprocess.run([str(exe), "time", str(f), str(maxit), "20"],
                                     capture_output=True, text=True, timeout=60).stdout)
        reps = max(20, int(budget_s / max(probe, 1e-6)))
        sec = float(subprocess.run([str(exe), "time", str(f), str(maxit), str(reps)],
                                   capture_output=True, text=True, timeout=120).stdout)
    return dict(value=(maxit + 1) / sec, unit="it/s", cores=1, kind="reference",
                sample=f"C1 dense 128 SPD, conj_grad({maxit}) x {reps} in one process: "
                       f"{sec * 1e6:.1f} us per call, {maxit + 1} x-updates each "
                       f"(oracle/_ref/ref_harness, the reference's own sources and flags)")


def cpu_baseline(sysm, budget_s):
    """The oracle's CSR-sequential HS-CG (bit-exact to the reference on chained
    matrices) on ONE host core, on the same matrix, for as many iterations as
    fit in ~budget_s seconds."""
    import numpy as np
    import helpers as H
    rp, col, val, b = sysm["rp"], sysm["col"], sysm["val"], sysm["b"]
    if val.dtype != np.float64:
        val = val.astype(np.float64)
        b = b.astype(np.float64)
    t0 = time.perf_counter()
    H.o_solve(0, 0.0, rp, col, val, b)          # 1 iteration (probe)
    t1 = time.perf_counter() - t0
    its = max(1, min(1000, int(budget_s / max(t1, 1e-6))))
    t0 = time.perf_counter()
    _, done, _ = H.o_solve(its - 1, 0.0, rp, col, val, b)
    dt = time.perf_counter() - t0
    return dict(value=done / dt, unit="it/s", cores=1, kind="port",
                sample=f"{done} HS-CG iterations of the same system (oracle/cg_oracle.c "
                       f"CSR-sequential restatement, bit-exact to the reference's "
                       f"mv_mult on chained matrices), 1 host core, {dt:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--alg", default=None, choices=["hs", "cg1", "cg1-dist", "hs-dist", "auto-dist"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch  # loads the HIP runtime libcgx then shares (same SONAME)
    import torch.distributed as dist
    import numpy as np
    import cgx

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def barrier():
        if world > 1:
            dist.barrier()

    wl = WORKLOADS[args.workload]
    if world > 1 and wl["kind"] == "rand":
        raise SystemExit("bench: C5 (random SPD) is a single-GPU configuration (BASELINE.json)")
    # N > 1: the partitioned solver; its recurrence is chosen by a short
    # timed trial of both (below) unless --alg names one
    alg = args.alg or ("auto-dist" if world > 1 else "hs")
    sysm = make_system(wl, rank, world)

    use_dist = world > 1 or alg.endswith("-dist")
    torch.cuda.synchronize()
    t_up = time.perf_counter()  # host -> HBM upload + row-block plan (outside `value`)
    trial = None
    if use_dist:
        # one rank per GPU; RCCL communicator from an id rank 0 broadcasts
        uid = [cgx.dist_unique_id() if (rank == 0 and world > 1) else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        s = cgx.DistSolver(local_rank, world, rank, uid[0])
        s.set_matrix(sysm["n_global"], sysm["rp"], sysm["col"], sysm["val"])
        s.set_rhs(sysm["b"])
        dinfo = s.info()
        if alg == "auto-dist":
            # HS needs two all-reduces per iteration, CG1 one but 8 B/row more
            # vector traffic: which wins depends on the node's all-reduce
            # latency, so time both (max over ranks, same choice everywhere)
            trial = {}
            for name, a in (("hs-dist", cgx.CGX_ALG_HS), ("cg1-dist", cgx.CGX_ALG_CG1)):
                s.set_alg(a)
                s.bench_prepare(3)
                barrier()
                tms = s.bench_run(20)[0] / 20
                if world > 1:
                    t = torch.tensor([tms], device="cuda", dtype=torch.float64)
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                    tms = float(t.item())
                trial[name] = round(tms, 4)
            alg = min(trial, key=trial.get)
        s.set_alg(cgx.CGX_ALG_HS if alg == "hs-dist" else cgx.CGX_ALG_CG1)
        info = dict(spmv_bytes=dinfo["spmv_bytes"], iter_bytes=dinfo["iter_bytes"],
                    spmv_iter_bytes=dinfo["spmv_iter_bytes"], n_dict=dinfo["n_dict"],
                    dict_vals=dinfo["dict_vals"])
    else:
        s = cgx.Solver(local_rank, alg=cgx.CGX_ALG_CG1 if alg == "cg1" else cgx.CGX_ALG_HS)
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        s.set_rhs(sysm["b"])
        info = s.info()
        dinfo = None

    torch.cuda.synchronize()
    upload_ms = 1e3 * (time.perf_counter() - t_up)

    # ---- timed region: exactly K steps, barrier + sync on both sides
    s.bench_prepare(args.warmup)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev_ms = s.bench_run(args.steps)[0] if use_dist else s.bench_run(args.steps, graph=True)[0]
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    ms_per_step = 1e3 * wall / args.steps

    # ---- roofline of the dominant kernel (SpMV): HIP events around every
    # SpMV launch on the solver's stream over K more iterations.
    if use_dist:
        _, spmv_ms = s.bench_run(args.steps, spmv_events=True)
    else:
        _, spmv_ms = s.bench_run(args.steps, graph=False, spmv_events=True)
    # achieved: the bytes the SpMV must move in the layout it runs on (coded
    # columns: 1 byte per nonzero instead of 4) over its measured time; the
    # CSR-equivalent rate (SURVEY.md 8d's B_spmv over the same time) beside it
    achieved = info["spmv_iter_bytes"] / (spmv_ms * 1e-3) / 1e9
    traffic = load_traffic(args.workload, alg)
    label = spmv_layout_label(info, len(sysm["col"]) * (4 + sysm["val"].itemsize))
    roofline = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS,
                    unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4),
                    traffic=traffic, kernel=label,
                    spmv_us=round(spmv_ms * 1e3, 2),
                    algorithmic_bytes_per_launch=int(info["spmv_iter_bytes"]),
                    csr_bytes_per_launch=int(info["spmv_bytes"]),
                    csr_equivalent_gbs=round(info["spmv_bytes"] / (spmv_ms * 1e-3) / 1e9, 1))

    # on-box HBM ceilings: STREAM triad (1/3 writes) and a
    # read-only stream, 512 MiB arrays.  The SpMV is 92% reads (its only
    # write is y), so the read ceiling is the one it is compared with.
    triad = cgx.stream_bench(local_rank, 64 * 2**20, 10, cgx.CGX_STREAM_TRIAD)
    rd = cgx.stream_bench(local_rank, 64 * 2**20, 10, cgx.CGX_STREAM_READ)
    roofline["stream_triad_gbs"] = round(triad, 1)
    roofline["stream_read_gbs"] = round(rd, 1)
    roofline["frac_of_stream_read"] = round(achieved / rd, 4)

    # matrix-free upper bound for the Laplacian runs -- the same
    # operator as a stencil (bit-identical SpMV), only x and y move
    # the same solve with plain 4-byte CSR columns (CGX_LAYOUT=csr): the
    # layout SURVEY.md 8d's B_spmv prices, measured beside the coded one
    def alt_layout(env, note):
        """The same solve with other layout knobs (env), measured like the main line."""
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            with cgx.Solver(local_rank, alg=cgx.CGX_ALG_CG1 if alg == "cg1" else cgx.CGX_ALG_HS) as cs:
                cs.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
                cs.set_rhs(sysm["b"])
                cs.bench_prepare(args.warmup)
                c_ms = cs.bench_run(args.steps, graph=True)[0]
                _, c_spmv = cs.bench_run(args.steps, graph=False, spmv_events=True)
                cinfo = cs.info()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        c_gbs = cinfo["spmv_iter_bytes"] / (c_spmv * 1e-3) / 1e9
        return dict(value=round(args.steps / (c_ms * 1e-3), 2), unit="it/s",
                    spmv_us=round(c_spmv * 1e3, 2), spmv_gbs=round(c_gbs, 1),
                    frac=round(c_gbs / HBM_PEAK_GBS, 4),
                    algorithmic_bytes_per_launch=int(cinfo["spmv_iter_bytes"]),
                    kernel=spmv_layout_label(cinfo, len(sysm["col"]) * (4 + sysm["val"].itemsize)),
                    note=note)

    # the same solve with plain 4-byte CSR columns (CGX_LAYOUT=csr): the
    # layout SURVEY.md 8d's B_spmv prices, measured beside the coded one; and
    # with offset codes but the value stream kept (CGX_DC_VALS=0)
    csr_plain = coded_offsets = None
    if world == 1 and not use_dist and info.get("n_dict", 0) > 0:
        csr_plain = alt_layout({"CGX_LAYOUT": "csr"},
                               "same system, plain int32 CSR columns (CGX_LAYOUT=csr): "
                               "B_spmv of SURVEY.md 8d")
        if info.get("dict_vals", 0):
            coded_offsets = alt_layout({"CGX_DC_VALS": "0"},
                                       "same system, offset codes + the fp64 value stream "
                                       "(CGX_DC_VALS=0)")

    mf = None
    if world == 1 and wl["kind"] in ("lap3d", "lap2d"):
        with cgx.Solver(local_rank) as ms:
            dims = wl["dims"]
            ms.set_stencil(3 if wl["kind"] == "lap3d" else 2, dims[0], dims[1],
                           dims[2] if len(dims) > 2 else 1)
            ms.set_rhs(sysm["b"])
            ms.bench_prepare(args.warmup)
            mf_ms = ms.bench_run(args.steps, graph=True)[0]
            _, mf_spmv = ms.bench_run(min(args.steps, 50), graph=False, spmv_events=True)
        mf = dict(value=round(args.steps / (mf_ms * 1e-3), 2), unit="it/s",
                  spmv_us=round(mf_spmv * 1e3, 2),
                  note="matrix-free 7/5-point stencil SpMV (cgx_solver_set_stencil): "
                       "not the CSR path, an upper bound for it")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(sysm, args.cpu_seconds)
        cpu["cpu_model"] = cpu_model()
        cpu["nproc"] = os.cpu_count()
        cpu["all_cores"] = cpu_baseline_mt(sysm, args.cpu_seconds / 2)
        cpu["reference_c1"] = reference_c1()

    # weak scaling (default): every rank owns one slab, value = slab-iterations/s
    # summed over ranks; strong (c4): one system over all ranks, value = its it/s
    strong = bool(wl.get("strong"))
    value = (args.steps / wall) * (1 if strong else world)
    out = dict(
        metric=METRIC, value=round(value, 2), unit="it/s", n_gpus=world,
        steps=args.steps, warmup=args.warmup, ms_per_step=round(ms_per_step, 4),
        higher_is_better=True, scaling="strong" if strong else "weak", vs_baseline=None,
        dtype=wl["dtype"], data="synthetic",
        config=dict(workload=wl["desc"], n=sysm["n_global"], nnz_local=int(len(sysm["col"])),
                    alg=alg, alg_trial_ms_per_iter=trial if use_dist else None,
                    graph=not use_dist or world == 1,
                    parallelism=f"row-partition x{world}",
                    layout=(f"CSR-VI: value-indexed coded columns ({info['n_dict']} "
                            f"(col-row, value) pairs, 1 B/nnz, no value stream) + byte row lengths"
                            if info.get("dict_vals", 0) else
                            f"CSR with dictionary-coded columns ({info['n_dict']} col-row "
                            f"offsets, 1 B/nnz) + byte row lengths"
                            if info.get("n_dict", 0) else "CSR (int32 columns)"),
                    halo_bytes_per_iter=(dinfo or {}).get("halo_bytes")),
        device_ms_per_step=round(dev_ms / args.steps, 4),
        # the C boundary takes host CSR buffers: one-time upload + plan, not in `value`
        upload_ms=round(upload_ms, 1),
        iter_bytes=int(info["iter_bytes"]),
        iter_gbs=round(info["iter_bytes"] / (ms_per_step * 1e-3) / 1e9, 1),
        # the iteration's bytes in the layout it runs on (SpMV as above + the
        # vector kernels' 8d bytes) over the measured step
        iter_layout_gbs=round((info["iter_bytes"] - info["spmv_bytes"] + info["spmv_iter_bytes"])
                              / (ms_per_step * 1e-3) / 1e9, 1),
        roofline=roofline, cpu_baseline=cpu, csr_plain=csr_plain, coded_offsets=coded_offsets,
        matrix_free_upper_bound=mf,
    )
    if rank == 0:
        print(json.dumps(out), flush=True)
    s.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
