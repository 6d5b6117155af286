#!/usr/bin/env python3
"""bench.py -- fp64 CG iterations/s on MI355X, with the SpMV roofline and the
CPU baseline beside it (BASELINE.json metric).

A "step" is one CG iteration of the device-resident solver (SpMV + dot
products + vector updates) on a synthetic SPD system already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c4|c2|c5]

Every N runs the same workload (default C4), so the driver's per-N values form
one strong-scaling curve and BASELINE.json's ">= 6x single-GPU CG it/s at 8
GPUs" reads off it directly.

N = 1 (default workload C4): the 7-point 3-D Laplacian 400^3 (64,000,000 rows,
447,040,000 nnz, fp64, b = 1) on ONE GPU in the layout libcgx picks for it --
the base of the curve; in the same run the same solve on the reference's plain
CSR (SURVEY.md 8d's B_spmv: the roofline figure), with dictionary-coded
columns and matrix-free; then C3 (216^3, 10,077,696 rows -- BASELINE.json's
HBM roofline configuration, the north star's ">= 70 % on fp64 CSR SpMV for a
10M-row 3-D Laplacian") in the picked layout and in plain CSR, C3's pattern
with general coefficients, and the end-to-end drop-in call solve(A, b, &x,
1e-8, maxit) through the C ABI; the CPU baseline on a bounded sample of the
workload.  (--workload c3 makes C3 the timed line, as rounds 1-2 did.)

N > 1 (default workload C4): one process per GPU.  Without WORLD_SIZE in the
environment this script starts itself under torch.distributed.run as a child
process (before touching the GPU) and forwards rank 0's line.  Each rank owns
a contiguous row block of the 400^3 Laplacian (64,000,000 rows; strong
scaling); halo planes go point to point and the dot products are all-reduced
over RCCL.  Before the timed run a small 3-D Laplacian is solved across the N
ranks to tol 1e-10 and checked against a single-GPU solve of the same system
(the `parity` gate: the timed run happens only if it passes).

Output: ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
               kind="lap3d", dims=(400, 400, 400), dtype="f64"),
    "c5": dict(desc="C5: random SPD 5,000,000 rows, 32 partners/row symmetrised "
                    "(~64 nnz/row), splitmix64 seed 42, fp32",
               kind="rand", n=5_000_000, partners=32, seed=42, dtype="f32"),
}


# ----------------------------------------------------------------- launcher

def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(argv, nproc, port):
    """The child command for N > 1 without WORLD_SIZE: this script under
    torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
            str(REPO / "bench.py"), *argv]


def launch_ranks(argv, nproc):
    """Runs the ranks as a child process (never exec: this process has not
    touched the GPU and must not be replaced); rank 0 prints the line."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(launch_cmd(argv, nproc, free_port()), env=env).returncode


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: c4 (every N: one strong-scaling curve)")
    ap.add_argument("--alg", default=None, choices=["hs", "sr", "cg1"],
                    help="recurrence (default: a timed trial after a parity gate -- N > 1: HS, "
                         "SR, CG1; N = 1: HS and SR, SR only where the one-launch march runs)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="at one rank (under torch.distributed.run --nproc-per-node 1): run the "
                         "N > 1 path -- parity gate, RCCL communicator, C4 -- on one GPU")
    ap.add_argument("--ranks-share-gpu", action="store_true",
                    help="rehearsal on a box with fewer GPUs than ranks: every rank on GPU 0, "
                         "each with a host id of its own (NCCL_HOSTID) so that RCCL connects "
                         "them over its socket transport on the loopback interface -- the N > 1 "
                         "path's RCCL calls between real peers, not an xGMI or scaling number")
    ap.add_argument("--no-legs", action="store_true",
                    help="N = 1: only the headline solve (no CSR/DC/stencil/C3/e2e legs)")
    ap.add_argument("--layout", default="auto", choices=["auto", "csr", "dc", "dia"],
                    help="N = 1: the headline solve's layout (profiling one kernel)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ systems

def make_system(wl, rank=0, world=1):
    """Host CSR of this rank's rows (the C boundary takes host CSR)."""
    import numpy as np
    import cgx
    if wl["kind"] == "lap3d":
        nx, ny, nz = wl["dims"]
        n_g = nx * ny * nz
        rb, re_ = cgx.partition_rows(n_g, world, rank)
        rp, col, val = cgx.laplacian3d(nx, ny, nz, rb, re_)
    elif wl["kind"] == "lap2d":
        nx, ny = wl["dims"]
        n_g = nx * ny
        rb, re_ = cgx.partition_rows(n_g, world, rank)
        rp, col, val = cgx.laplacian2d(nx, ny, rb, re_)
    else:
        n_g = wl["n"]
        rb, re_ = 0, n_g
        rp, col, val = cgx.random_spd(n_g, wl["partners"], wl["seed"], f32=True)
        b = np.random.default_rng(1).standard_normal(n_g).astype(np.float32)
        return dict(rp=rp, col=col, val=val, b=b, n_global=n_g, row_begin=rb, row_end=re_)
    return dict(rp=rp, col=col, val=val, b=np.ones(re_ - rb), n_global=n_g, row_begin=rb,
                row_end=re_)


# kernel key -> the name prefix its rocprofv3 PMC summary must carry
KERNEL_PREFIX = {"sr1": "k_sr1_dia_m<", "dia_march": "k_spmv_dia_m<", "dia_fused": "k_spmv_dia_h<",
                 "dia": "k_spmv_dia<", "dc": "k_spmv_dc<", "csr": "k_spmv_csr<",
                 "panel": "k_spmv_csr<", "stencil": "k_stencil<"}


def load_traffic(wl_name, key):
    """L2->fabric bytes per launch of kernel `key` (KERNEL_PREFIX) at workload
    wl_name from the committed rocprofv3 PMC summary
    profiles/pmc_<wl_name>_<key>.json (tools/pmc_summary.py) -- only when the
    file's `kernel` IS that kernel (traffic was attributed by
    workload name, to another kernel).  (bytes, source) or (None, reason)."""
    p = REPO / "profiles" / f"pmc_{wl_name}_{key}.json"
    if not p.exists():
        return None, f"no profiles/{p.name}"
    try:
        d = json.loads(p.read_text())
    except Exception as e:  # a malformed summary prices nothing
        return None, f"profiles/{p.name}: {e}"
    kern = str(d.get("kernel", ""))
    if not kern.startswith(KERNEL_PREFIX[key]):
        return None, f"profiles/{p.name} is {kern}, not {KERNEL_PREFIX[key]}...>"
    return d.get("spmv_hbm_bytes_per_launch"), f"profiles/{p.name} ({kern}, {d.get('source', '')})"


def traffic_fields(wl_name, key, alg_bytes):
    """`traffic` (HBM bytes per launch, PMC) beside `achieved`, its source and
    its ratio to the algorithmic bytes of the same kernel."""
    t, src = load_traffic(wl_name, key)
    return dict(traffic=None if t is None else int(t), traffic_source=src,
                traffic_ratio=None if t is None else round(t / alg_bytes, 4))


KERNELS = {
    "dia": "k_spmv_dia (DIA-VI: value-indexed diagonal codes, two rows per thread, pair loads of x)",
    "dia_fused": "k_spmv_dia_h (fused HS step on DIA-VI: x / p update of the previous iteration, "
                 "p of the slice + halo in an LDS window, s = A p, p.s partials)",
    "dia_march": "k_spmv_dia_m (fused HS step on DIA-VI as a plane march: a workgroup walks "
                 "slices nx*ny apart, p of three consecutive slices + halos in an LDS ring, "
                 "x / p update, s = A p, p.s partials)",
    "sr1": "k_sr1_dia_m (one-launch SR iteration on DIA-VI as a plane march: the scalar step "
           "of the previous launch folded in (single GPU: no k_finalize), r = r - alpha s "
           "and p = r + beta p of the previous iteration for each window row, x update, "
           "s = A p from an LDS ring of three windows, (p.s, s.s, r.r) per workgroup)",
    "dc": "k_spmv_dc (LDS-DMA code window + value window per 64-row block, dictionary-coded columns)",
    "csr": "k_spmv_csr (LDS-DMA val/col window per 64-row block, lane-per-row sums from LDS)",
    "panel": "k_spmv_csr over column panels",
    "stencil": "k_stencil (matrix-free, two rows per thread)",
}


def kernel_key(info):
    if info["layout_name"] == "dia" and info.get("fused"):
        if info.get("alg") == 2 and (info.get("fuse_march", 0) > 0 or info.get("march", 0) > 0):
            return "sr1"  # single GPU (cgx_info.fuse_march) or a rank (cgx_dist_stats.march)
        return "dia_march" if info.get("fuse_march") else "dia_fused"
    return info["layout_name"]


def kernel_name(info):
    k = KERNELS.get(kernel_key(info), info["layout_name"])
    if info.get("dia_value_stream"):
        k += " -- its DIA-V instance: the values streamed per (row, diagonal), no value table"
    return k


def layout_desc(info):
    name = info["layout_name"]
    if name == "dia" and info.get("dia_value_stream"):
        return (f"DIA-V: {info['n_dict']} diagonals, 1 presence byte per row + the values "
                "streamed diagonal-major (general coefficients), no column stream")
    if name == "dia":
        return (f"DIA-VI: {info['n_dict']} diagonals, {info['n_values']} values, "
                f"{info['code_bytes_per_row']} code bytes per row, no column or value stream")
    if name == "dc":
        return f"CSR-DC: {info['n_dict']} column offsets, 1 code byte per nonzero + values"
    if name == "panel":
        return f"CSR in {info['n_panels']} column panels"
    return "CSR (int32 columns, fp64 values): the reference's struct"


def value_basis(info):
    """What `value` is an iteration rate OF: the layout the
    timed solve streams -- so no reader compares a DIA-VI rate with a CSR one."""
    if info["layout_name"] == "dia" and not info.get("dia_value_stream"):
        return (f"DIA-VI compressed stencil ({info['code_bytes_per_row']} B/row of matrix codes, "
                "no column or value stream; exact, bit-identical SpMV) -- NOT a CSR rate: the "
                "plain-CSR solve of the same system is csr_plain.value")
    return f"{layout_desc(info)}: the matrix bytes SURVEY 8d's CSR basis counts or fewer"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# -------------------------------------------------------------- CPU legs

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


def cpu_baseline_mt(sysm, budget_s):
    """SURVEY.md 8d leg (c): the same CSR-sequential HS-CG with its row loops
    split over the host cores this job may use (oracle_solve_mt, pthreads;
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
    None when the binary was not built (no /root/reference)."""
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


# ----------------------------------------------------------- single GPU

def spmv_roofline(bytes_, ms, peak=HBM_PEAK_GBS):
    gbs = bytes_ / (ms * 1e-3) / 1e9
    return round(gbs, 1), round(gbs / peak, 4)


def solver_leg(sysm, steps, warmup, layout, device=0, b2b=False, alg="hs"):
    """One solver on the system in `layout`: CG it/s (graph replay), the
    average in-iteration SpMV time (HIP events around every SpMV launch on
    the solver's stream) and, with b2b, back-to-back SpMVs y = A p (the
    standard SpMV benchmark, the kernel without the p.s epilogue).  alg:
    the recurrence (ALGS)."""
    import cgx
    with cgx.Solver(device, layout=layout, alg=ALGS[alg]) as s:
        t0 = time.perf_counter()
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        s.set_rhs(sysm["b"])
        setup_ms = 1e3 * (time.perf_counter() - t0)
        s.bench_prepare(warmup)
        dev_ms = s.bench_run(steps, graph=True)[0]
        _, spmv_ms = s.bench_run(steps, graph=False, spmv_events=True)
        out = dict(value=round(steps / (dev_ms * 1e-3), 2), unit="it/s",
                   device_ms_per_step=round(dev_ms / steps, 4),
                   spmv_us=round(spmv_ms * 1e3, 2), info=s.info(), setup_ms=round(setup_ms, 1))
        if b2b:
            _, b2b_ms = s.bench_run(steps, graph=False, spmv_events=True, spmv_only=True)
            out["b2b_spmv_us"] = round(b2b_ms * 1e3, 2)
    return out


def solve_e2e(sysm, tol=1e-8, maxit=20000, alg="hs", legs=("cold", "warm")):
    """What cg.c:71-75 times: the drop-in call solve(A, b, &x, tol, maxit)
    through the C ABI on host structs -- content hash of A, upload + layout
    encoding (first call), the device iterations, x back to the host -- cold
    (A not yet resident) and warm (A resident, the second call on the same
    struct).  The true residual is computed here on the host (scipy).
    alg "sr": cgx_ops_set_mode(FAST, SR) -- the one-launch SR step where the
    matrix takes it, HS otherwise (`alg_ran`, cgx_ops_last_timing)."""
    import numpy as np
    import scipy.sparse as sp
    import cgx
    A = cgx.Mv(sysm["val"], sysm["col"], sysm["rp"])
    b = cgx.Mv(sysm["b"])
    cgx.ops_set_mode(cgx.CGX_MODE_FAST, ALGS[alg])
    out = {}
    for leg in legs:
        t0 = time.perf_counter()
        x, its = cgx.solve(A, b, tol, maxit)
        wall = 1e3 * (time.perf_counter() - t0)
        t = cgx.ops_last_timing()
        n = len(sysm["b"])
        Am = sp.csr_matrix((sysm["val"], sysm["col"], sysm["rp"]), shape=(n, n))
        res = float(np.linalg.norm(sysm["b"] - Am @ x) / np.linalg.norm(sysm["b"]))
        out[leg] = dict(wall_ms=round(wall, 1), iters=its, true_rel_residual=res,
                        setup_ms=round(t["setup_ms"], 1), hash_ms=round(t["hash_ms"], 1),
                        solve_ms=round(t["solve_ms"], 1), download_ms=round(t["download_ms"], 1),
                        uploaded=bool(t["uploaded"]),
                        setup_frac=round(t["setup_ms"] / max(wall, 1e-9), 3),
                        alg_ran={v: k for k, v in ALGS.items()}[t["alg"]])
    cgx.ops_set_mode(cgx.CGX_MODE_FAST, cgx.CGX_ALG_HS)
    out["note"] = (f"solve(A,b,&x,{tol:g},{maxit}) through the C ABI on host structs "
                   f"(include/cgx.h), cgx_ops_set_mode(FAST, {alg.upper()}), wall time incl. "
                   "ctypes; cold = A uploaded and encoded, warm = A resident (op-level residency)")
    return out


def general_coefficients(steps, warmup, device=0):
    """the C3 grid with one random coefficient per edge
    (cgx_gen_varcoef3d: every off-diagonal value distinct, so no layout can
    index the values -- the general CSR case mv_ops.h:17-23 allows): the
    layout libcgx picks for it (coded columns + the value stream) and the
    plain CSR, each with its CG it/s and in-iteration SpMV on its own bytes
    and on the CSR basis (SURVEY.md 8d B_spmv)."""
    import numpy as np
    import cgx
    rp, col, val = cgx.varcoef3d(216, 216, 216, seed=7)
    sysm = dict(rp=rp, col=col, val=val, b=np.ones(len(rp) - 1))
    out = dict(matrix="7-point pattern of C3 (216^3), a_ij = a_ji = -(0.5 + U(0,1]) per edge, "
                      "diagonal = sum |a_ij| + 0.01 (cgx_gen_varcoef3d, seed 7), b = 1")
    gate = sr_gate(sysm, ("auto", "csr"), device=device)
    out["sr_gate"] = gate
    for name, layout, alg in (("auto", "auto", "hs"), ("auto_sr", "auto", "sr"),
                              ("csr", "csr", "hs"), ("csr_sr", "csr", "sr")):
        if alg == "sr" and not gate[layout]["ok"]:
            out[name] = dict(refused=f"SR failed its parity gate: {gate[layout]}")
            continue
        leg = solver_leg(sysm, steps, warmup, layout, device, b2b=True, alg=alg)
        i = leg["info"]
        own_gbs, own_frac = spmv_roofline(i["spmv_iter_bytes"], leg["spmv_us"] * 1e-3)
        csr_gbs, csr_frac = spmv_roofline(i["spmv_bytes"], leg["spmv_us"] * 1e-3)
        one_launch = kernel_key(i) == "sr1"  # DIA-V (round 5): the one-launch SR step
        out[name] = dict(layout=layout_desc(i), layout_name=i["layout_name"], value=leg["value"],
                         unit="it/s",
                         alg=(ALG_DESC[alg] if alg == "hs" or one_launch else ALG_DESC["sr_unfused"]),
                         spmv_us=leg["spmv_us"], b2b_spmv_us=leg["b2b_spmv_us"],
                         own_bytes_gbs=own_gbs, own_bytes_frac=own_frac,
                         csr_basis_equiv_rate=csr_gbs, csr_basis_frac=csr_frac,
                         kernel=kernel_name(i))
        if one_launch:  # PMC of k_sr1_dia_m<..., DV> on this system (profiles/r05_c3dv.md)
            out[name].update(traffic_fields("c3dv", "sr1", i["spmv_iter_bytes"]))
    ok = [k for k in ("auto", "auto_sr") if "value" in out.get(k, {})]
    out["best_auto"] = max(ok, key=lambda k: out[k]["value"])
    return out


def sr_gate(sysm, layouts, maxit=20, device=0):
    """The SR parity gate of a leg (as alg_trial's): SR x of `maxit`
    iterations within 1e-10 of HS x in each layout, on the device whose legs
    are timed."""
    import numpy as np
    import cgx
    out = {}
    for layout in layouts:
        xs = {}
        for alg in ("hs", "sr"):
            with cgx.Solver(device, layout=layout, alg=ALGS[alg]) as s:
                s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
                s.set_rhs(sysm["b"])
                s.run(maxit)
                xs[alg] = s.x()
        rel = float(np.linalg.norm(xs["sr"] - xs["hs"]) / np.linalg.norm(xs["hs"]))
        out[layout] = dict(sr_vs_hs_rel=rel, maxit=maxit, ok=rel <= 1e-10)
    return out


def c4_one_gpu(steps, warmup, device=0):
    """The N = 1 point of the C4 strong-scaling curve: 400^3 generated in
    device memory (cgx_solver_gen_laplacian), the layout libcgx picks."""
    import numpy as np
    import cgx
    nx = 400
    with cgx.Solver(device) as s:
        t0 = time.perf_counter()
        s.gen_laplacian(3, nx, nx, nx)
        s.set_rhs(np.ones(nx ** 3))
        setup = 1e3 * (time.perf_counter() - t0)
        s.bench_prepare(warmup)
        ms = s.bench_run(steps, graph=True)[0]
        _, spmv_ms = s.bench_run(min(steps, 30), graph=False, spmv_events=True)
        i = s.info()
    gbs, frac = spmv_roofline(i["spmv_iter_bytes"], spmv_ms)
    return dict(value=round(steps / (ms * 1e-3), 2), unit="it/s", n=nx ** 3,
                layout=i["layout_name"], spmv_us=round(spmv_ms * 1e3, 2), spmv_gbs=gbs,
                spmv_frac=frac, setup_ms=round(setup, 1),
                note="C4 (400^3) on ONE GPU, same code path as the N = 1 headline: the "
                     "base of the C4 strong-scaling curve (N > 1 lines run C4 across N ranks)")


ALGS = {"hs": 0, "cg1": 1, "sr": 2}  # cgx.CGX_ALG_*
ALG_DESC = {"hs": "hs (the reference recurrence, cg.c:88-141)",
            "sr": "sr (cg.c:88-141's recurrence with ONE reduction of (p.s, s.s, r.r) per "
                  "iteration, beta from r_new.r_new = alpha (alpha s.s) - r.r; on one GPU the "
                  "r update of iteration k runs inside the SpMV launch of k + 1: one launch per "
                  "iteration, k_sr1_dia_m; oracle_solve_sr)",
            "cg1": "cg1 (Chronopoulos-Gear)",
            "sr_unfused": "sr, unfused (any layout): the SpMV stores (p.s, s.s) per workgroup, "
                          "one reduction, then r, p and x in one pass (k_update_sr): two "
                          "launches per iteration; oracle_solve_sr"}


_ORACLE_GATE = {}


def oracle_gate(maxit=20):
    """the N = 1 parity gate against the ORACLE -- C3 (216^3,
    b = 1, the bench's system) solved for maxit + 1 SpMVs on the GPU with HS
    and with SR (the one-launch plane-marched step), each x within 1e-10 of
    oracle_conj_grad(maxit) (cg.c:88-141 restated, bit-exact to the
    reference).  Computed once per process."""
    if _ORACLE_GATE:
        return _ORACLE_GATE
    import numpy as np
    import cgx
    import helpers as H
    sysm = make_system(WORKLOADS["c3"])
    t0 = time.perf_counter()
    x_ref, _ = H.o_conj_grad(maxit, sysm["rp"], sysm["col"], sysm["val"], sysm["b"])
    out = dict(system="C3 216^3, b = 1", maxit=maxit,
               oracle="oracle_conj_grad (cg.c:88-141, the reference's HS order)",
               oracle_s=round(time.perf_counter() - t0, 2))
    with cgx.Solver(0) as s:
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        for name in ("hs", "sr"):
            s.set_mode(cgx.CGX_MODE_FAST, ALGS[name])
            if name == "sr" and not s.info()["fuse_march"]:
                out[name] = dict(ok=False, note="no plane-marched DIA step")
                continue
            s.set_rhs(sysm["b"])
            s.run(maxit)
            rel = float(np.linalg.norm(s.x() - x_ref) / np.linalg.norm(x_ref))
            out[name] = dict(rel_vs_oracle=rel, ok=rel <= 1e-10)
    _ORACLE_GATE.update(out)
    return out


def alg_trial(sysm, warmup, layout="auto", maxit=20, its=30):
    """N = 1: the recurrence of the headline, as the N > 1 path picks it --
    a parity gate (the oracle gate above at C3: HS and SR within 1e-10 of
    oracle_conj_grad(20); on this workload HS and SR solves of `maxit`
    iterations within 1e-10 of each other), then a timed trial of `its`
    graph-replayed iterations each; the faster passing one.  SR runs on one
    GPU only where the plane-marched DIA step applies (cgx_info.fuse_march)."""
    import numpy as np
    import cgx
    res, trial, xs = {"oracle_gate": oracle_gate()}, {}, {}
    with cgx.Solver(0, layout=layout) as s:
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        for name in ("hs", "sr"):
            s.set_mode(cgx.CGX_MODE_FAST, ALGS[name])
            if name == "sr" and not s.info()["fuse_march"]:
                res[name] = "refused: no plane-marched DIA step for this matrix"
                continue
            s.set_rhs(sysm["b"])
            s.run(maxit)
            xs[name] = s.x()
            s.set_rhs(sysm["b"])
            s.bench_prepare(warmup)
            trial[name] = round(s.bench_run(its, graph=True)[0] / its, 4)
    if "sr" in xs:
        rel = float(np.linalg.norm(xs["sr"] - xs["hs"]) / np.linalg.norm(xs["hs"]))
        res["sr_vs_hs_rel"] = rel
        if not (rel <= 1e-10 and res["oracle_gate"]["sr"]["ok"]):
            res["sr"] = f"parity gate failed: {rel:.3e} vs HS, oracle gate {res['oracle_gate']['sr']}"
            trial.pop("sr", None)
    if not res["oracle_gate"]["hs"]["ok"]:
        raise SystemExit(f"bench: HS failed the oracle gate: {res['oracle_gate']['hs']}")
    return min(trial, key=trial.get), dict(gate=res, ms_per_iter=trial, gate_maxit=maxit)


def headline_solve(sysm, steps, warmup, layout="auto", alg="hs"):
    """The timed solve: upload (not timed), W warmup iterations, exactly K
    graph-replayed iterations bracketed by device syncs, then K more with HIP
    events around every SpMV launch (its average time in the iteration)."""
    import torch
    import cgx
    t_up = time.perf_counter()
    s = cgx.Solver(0, layout=layout, alg=ALGS[alg])
    try:
        s.set_matrix(sysm["rp"], sysm["col"], sysm["val"])
        s.set_rhs(sysm["b"])
        info = s.info()
        upload_ms = 1e3 * (time.perf_counter() - t_up)
        s.bench_prepare(warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev_ms = s.bench_run(steps, graph=True)[0]
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        _, spmv_ms = s.bench_run(steps, graph=False, spmv_events=True)
    finally:
        s.close()
    return dict(info=info, upload_ms=upload_ms, wall=wall, dev_ms=dev_ms, spmv_ms=spmv_ms)


def csr_legs(sysm, steps, warmup, alg):
    """The plain-CSR solve of the system in the recurrence the line runs (HS,
    or SR: since round 5 two launches and one reduction on any layout) with
    back-to-back SpMVs, and -- when that is SR -- the HS iteration beside it."""
    a = alg if alg in ("hs", "sr") else "hs"
    gate = None
    if a == "sr":  # SR's x against HS's on this layout first (sr_gate); HS if it fails
        gate = sr_gate(sysm, ("csr",))["csr"]
        if not gate["ok"]:
            a = "hs"
    csr = solver_leg(sysm, steps, warmup, "csr", b2b=True, alg=a)
    csr["alg"] = a
    csr["sr_gate"] = gate
    if a != "hs":
        csr["hs"] = solver_leg(sysm, steps, warmup, "csr", alg="hs")
    return csr


def csr_roofline(csr, wl_name):
    """SURVEY.md 8d's roofline figure: the plain-CSR SpMV on B_spmv = 12 nnz +
    4 (n+1) + 16 n, in the CG iteration of the line's recurrence (csr_legs),
    in the HS iteration, and back to back."""
    ci = csr["info"]
    c_gbs, c_frac = spmv_roofline(ci["spmv_bytes"], csr["spmv_us"] * 1e-3)
    b_gbs, b_frac = spmv_roofline(ci["spmv_bytes"], csr["b2b_spmv_us"] * 1e-3)
    hs = csr.get("hs")
    hs_fields = {}
    if hs is not None:
        h_gbs, h_frac = spmv_roofline(ci["spmv_bytes"], hs["spmv_us"] * 1e-3)
        hs_fields = dict(in_hs_iteration=dict(frac=h_frac, achieved=h_gbs,
                                              spmv_us=hs["spmv_us"], cg_its=hs["value"]))
    return dict(
        bound="hbm", achieved=c_gbs, peak=HBM_PEAK_GBS, unit="GB/s", frac=c_frac,
        **traffic_fields(wl_name, "csr", ci["spmv_bytes"]),
        kernel=KERNELS["csr"] + ", in the CG iteration (" +
        ALG_DESC["sr_unfused" if csr.get("alg") == "sr" else "hs"] + ")",
        recurrence=csr.get("alg", "hs"), sr_gate=csr.get("sr_gate"), **hs_fields,
        basis="SURVEY.md 8d B_spmv = 12 nnz + 4 (n+1) + 16 n (CSR int32 col + fp64 val, "
              "row_ptr, x read once, y written once)",
        algorithmic_bytes_per_launch=int(ci["spmv_bytes"]), spmv_us=csr["spmv_us"],
        csr=dict(frac=c_frac, achieved=c_gbs, spmv_us=csr["spmv_us"],
                 b2b_spmv_us=csr["b2b_spmv_us"], b2b_achieved=b_gbs, b2b_frac=b_frac,
                 cg_its=csr["value"], gathers_per_chunk=ci["gathers_per_chunk"],
                 note="in_cg: average launch inside the CG iteration (HIP events); b2b: "
                      "back-to-back y = A p launches (the standard SpMV benchmark, "
                      "k_spmv_csr without the p.s epilogue)"))


def layout_roofline(info, spmv_ms, wl_name):
    """The picked layout's SpMV launch priced on the bytes it moves."""
    gbs, frac = spmv_roofline(info["spmv_iter_bytes"], spmv_ms)
    return dict(kernel=kernel_name(info), layout=layout_desc(info),
                spmv_us=round(spmv_ms * 1e3, 2), achieved=gbs, frac=frac,
                algorithmic_bytes_per_launch=int(info["spmv_iter_bytes"]),
                **traffic_fields(wl_name, kernel_key(info), info["spmv_iter_bytes"]),
                csr_basis_equiv_rate=round(info["spmv_bytes"] / (spmv_ms * 1e-3) / 1e9, 1),
                note="the SpMV launch of the headline solve, priced on the bytes it moves (its "
                     "layout; with the fused HS step also r, p_old, x, p_new; with the one-launch "
                     "SR step r, s, p read and written, x every other launch); "
                     "csr_basis_equiv_rate = SURVEY 8d's CSR B_spmv / this launch's time, a "
                     "CSR-equivalent rate in GB/s -- NOT HBM bandwidth (this layout never "
                     "streams those bytes)")


def stream_ceilings(n=64 * 2**20, reps=10):
    """The on-box stream ceilings (cgx_stream_bench, fp64 arrays of n = 64 Mi
    elements, 512 MiB each -- far beyond the Infinity Cache): the naive
    triad and read stream of rounds 1-4, and tuned
    read/write mixes -- copy (1 read : 1 write), triad (2 : 1) and 3 : 3 (the
    one-launch SR step's r, p, s), each with plain and non-temporal stores,
    4 x 16 B per lane in flight, grid = resident workgroup slots."""
    import cgx
    return {k: round(cgx.stream_bench(0, n, reps, v), 1) for k, v in cgx.STREAM_KINDS.items()}


def c2_leg(steps, warmup):
    """C2 (the 5-point 2-D Laplacian 1000^2, 1 M rows) in the
    default line -- its whole working set (~150 MB as CSR, ~40 MB as DIA-VI
    + vectors) stays in the 256 MiB Infinity Cache, so its SpMV rates are
    cache rates, not HBM bandwidth: reported as times and as fractions of the
    HBM peak only for comparison, labelled resident."""
    wl = WORKLOADS["c2"]
    sysm = make_system(wl)
    out = dict(workload=wl["desc"], residency="Infinity-Cache resident (not an HBM figure)")
    gate = sr_gate(sysm, ("auto",))
    out["sr_gate"] = gate
    for name, layout, alg in (("auto", "auto", "hs"), ("auto_sr", "auto", "sr"),
                              ("csr", "csr", "hs")):
        if alg == "sr" and not gate[layout]["ok"]:
            out[name] = dict(refused=f"SR failed its parity gate: {gate[layout]}")
            continue
        leg = solver_leg(sysm, steps, warmup, layout, b2b=True, alg=alg)
        i = leg["info"]
        _, own_frac = spmv_roofline(i["spmv_iter_bytes"], leg["spmv_us"] * 1e-3)
        _, csr_frac = spmv_roofline(i["spmv_bytes"], leg["spmv_us"] * 1e-3)
        out[name] = dict(value=leg["value"], unit="it/s", layout=layout_desc(i), alg=alg,
                         kernel=kernel_name(i), spmv_us=leg["spmv_us"],
                         b2b_spmv_us=leg["b2b_spmv_us"],
                         own_bytes=int(i["spmv_iter_bytes"]), own_bytes_frac_resident=own_frac,
                         csr_basis_bytes=int(i["spmv_bytes"]), csr_basis_frac_resident=csr_frac)
    return out


def matrix_free(wl, b, steps, warmup):
    import cgx
    dims = wl["dims"]
    with cgx.Solver(0) as ms:
        ms.set_stencil(3 if wl["kind"] == "lap3d" else 2, dims[0], dims[1],
                       dims[2] if len(dims) > 2 else 1)
        ms.set_rhs(b)
        ms.bench_prepare(warmup)
        mf_ms = ms.bench_run(steps, graph=True)[0]
        _, mf_spmv = ms.bench_run(min(steps, 50), graph=False, spmv_events=True)
    return dict(value=round(steps / (mf_ms * 1e-3), 2), unit="it/s",
                spmv_us=round(mf_spmv * 1e3, 2), kernel=KERNELS["stencil"],
                note="the same operator without a stored matrix (x and y only), run as the "
                     "unfused three-launch iteration; NOT an upper bound: the fused DIA step "
                     "of the headline moves fewer bytes per iteration")


def c3_legs(steps, warmup):
    """C3 inside a C4 line: BASELINE.json's HBM roofline configuration in the
    picked layout and in plain CSR (the north star's 70 % figure), the general
    coefficient matrix on its grid, and the end-to-end drop-in call."""
    wl = WORKLOADS["c3"]
    sysm = make_system(wl)
    alg, trial = alg_trial(sysm, warmup)
    h = headline_solve(sysm, steps, warmup, alg=alg)
    csr = csr_legs(sysm, steps, warmup, alg)
    out = dict(workload=wl["desc"], value=round(steps / h["wall"], 2), unit="it/s",
               alg=ALG_DESC[alg], alg_trial=trial,
               ms_per_step=round(1e3 * h["wall"] / steps, 4), layout=layout_desc(h["info"]),
               layout_name=h["info"]["layout_name"],
               default_layout=layout_roofline(h["info"], h["spmv_ms"], "c3"),
               outside_launch_us=round(1e3 * h["dev_ms"] / steps - 1e3 * h["spmv_ms"], 2),
               csr_roofline=csr_roofline(csr, "c3"),
               csr_plain=dict(value=csr["value"], unit="it/s", spmv_us=csr["spmv_us"],
                              b2b_spmv_us=csr["b2b_spmv_us"], kernel=KERNELS["csr"],
                              recurrence=csr["alg"],
                              hs_value=csr["hs"]["value"] if "hs" in csr else csr["value"]))
    out["general_coefficients"] = general_coefficients(steps, warmup)
    out["solve_e2e"] = solve_e2e(sysm)
    # cold first (the first SR call switches the recurrence and
    # captures its graphs), then the warm call on the resident matrix
    out["solve_e2e_sr"] = solve_e2e(sysm, alg="sr", legs=("cold", "warm"))
    return out


def c5_leg(steps, warmup):
    """C5 (random SPD, 5 M rows, ~64 nnz/row, fp32) inside the
    default line -- CG it/s in the layout libcgx picks (column panels) and its
    SpMV in the iteration on its own bytes and on SURVEY.md 8d's CSR basis."""
    t0 = time.perf_counter()
    sysm = make_system(WORKLOADS["c5"])
    gen_s = time.perf_counter() - t0
    leg = solver_leg(sysm, steps, warmup, "auto", b2b=True)
    i = leg["info"]
    own_gbs, own_frac = spmv_roofline(i["spmv_iter_bytes"], leg["spmv_us"] * 1e-3)
    csr_gbs, csr_frac = spmv_roofline(i["spmv_bytes"], leg["spmv_us"] * 1e-3)
    return dict(workload=WORKLOADS["c5"]["desc"], n=i["n"], nnz=i["nnz"], value=leg["value"],
                unit="it/s", dtype="f32", layout=layout_desc(i), kernel=kernel_name(i),
                spmv_us=leg["spmv_us"], b2b_spmv_us=leg["b2b_spmv_us"],
                own_bytes=int(i["spmv_iter_bytes"]), own_bytes_gbs=own_gbs,
                own_bytes_frac=own_frac, csr_basis_bytes=int(i["spmv_bytes"]),
                csr_basis_equiv_rate=csr_gbs, csr_basis_frac=csr_frac,
                **traffic_fields("c5", kernel_key(i), i["spmv_iter_bytes"]),
                host_gen_s=round(gen_s, 1), setup_ms=leg["setup_ms"])


def run_single(args, wl_name):
    import torch
    import cgx

    wl = WORKLOADS[wl_name]
    torch.cuda.set_device(0)
    sysm = make_system(wl)
    torch.cuda.synchronize()

    # ---- headline: the layout libcgx picks (default path of the drop-in), the
    # recurrence a parity-gated trial picks (HS or SR)
    if args.alg in ("hs", "sr"):
        alg, trial = args.alg, None
    else:
        alg, trial = alg_trial(sysm, args.warmup, args.layout)
    h = headline_solve(sysm, args.steps, args.warmup, args.layout, alg)
    info, spmv_ms, wall = h["info"], h["spmv_ms"], h["wall"]
    ms_per_step = 1e3 * wall / args.steps

    legs = {}
    if alg != "hs" and not args.no_legs:  # the reference recurrence's own figure beside it
        hh = headline_solve(sysm, args.steps, args.warmup, args.layout, "hs")
        legs["hs"] = dict(value=round(args.steps / hh["wall"], 2), unit="it/s",
                          ms_per_step=round(1e3 * hh["wall"] / args.steps, 4),
                          alg=ALG_DESC["hs"], kernel=kernel_name(hh["info"]),
                          default_layout=layout_roofline(hh["info"], hh["spmv_ms"], wl_name))
    if not args.no_legs:
        if info["layout_name"] != "csr":
            legs["csr"] = csr_legs(sysm, args.steps, args.warmup, alg)
        if wl["kind"] in ("lap3d", "lap2d") and info["layout_name"] != "dc":
            legs["dc"] = solver_leg(sysm, args.steps, args.warmup, "dc")
    csr = legs.get("csr")

    # ---- roofline: the plain-CSR SpMV of the workload (SURVEY.md 8d basis),
    # the picked layout's SpMV (its own bytes) beside it
    if csr is not None:
        roofline = csr_roofline(csr, wl_name)
        roofline["default_layout"] = layout_roofline(info, spmv_ms, wl_name)
    else:
        lr = layout_roofline(info, spmv_ms, wl_name)
        roofline = dict(bound="hbm", achieved=lr["achieved"], peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=lr["frac"], traffic=lr["traffic"], kernel=lr["kernel"],
                        traffic_source=lr["traffic_source"], traffic_ratio=lr["traffic_ratio"],
                        algorithmic_bytes_per_launch=lr["algorithmic_bytes_per_launch"],
                        spmv_us=lr["spmv_us"])
    # the headline's own launch (the kernel `value` runs) beside the 8d CSR
    # figure, with its bytes, duration, roofline fraction and PMC traffic
    hk = layout_roofline(info, spmv_ms, wl_name)
    headline_kernel = dict(bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s",
                           **{k: hk[k] for k in ("kernel", "spmv_us", "achieved", "frac",
                                                  "algorithmic_bytes_per_launch", "traffic",
                                                  "traffic_source", "traffic_ratio")},
                           timing="HIP events (hipExtLaunchKernel) around every launch of "
                                  f"{args.steps} eager iterations on the solver's stream")
    ceil = stream_ceilings()
    roofline["stream_triad_gbs"] = ceil.pop("triad")
    roofline["stream_read_gbs"] = ceil.pop("read")
    roofline["stream_tuned_gbs"] = ceil
    mix = max(ceil["copy"], ceil["copy_nt"], ceil["mix33"], ceil["mix33_nt"])
    headline_kernel["rw_mix_ceiling_gbs"] = mix
    headline_kernel["frac_of_rw_mix_ceiling"] = round(headline_kernel["achieved"] / mix, 4)
    # the per-iteration time outside the headline launch --
    # the graph-replayed period minus the launch itself (HIP events); with the
    # one-launch SR step's scalar step folded into the launch (round 6) that
    # is the kernel boundary alone, no k_finalize
    headline_kernel["outside_launch_us"] = round(1e3 * h["dev_ms"] / args.steps - hk["spmv_us"], 2)
    headline_kernel["launches_per_iteration"] = 1 if kernel_key(info) == "sr1" else None

    extra = {}
    if "hs" in legs:
        extra["hs_recurrence"] = legs["hs"]
    if not args.no_legs:
        if "dc" in legs:
            d = legs["dc"]
            g, f = spmv_roofline(d["info"]["spmv_iter_bytes"], d["spmv_us"] * 1e-3)
            extra["coded_offsets"] = dict(value=d["value"], unit="it/s", spmv_us=d["spmv_us"],
                                          spmv_gbs=g, frac=f, kernel=KERNELS["dc"],
                                          layout=layout_desc(d["info"]))
        if csr is not None:
            extra["csr_plain"] = dict(value=csr["value"], unit="it/s", spmv_us=csr["spmv_us"],
                                      b2b_spmv_us=csr["b2b_spmv_us"], kernel=KERNELS["csr"],
                                      recurrence=csr["alg"],
                                      hs_value=csr["hs"]["value"] if "hs" in csr else csr["value"],
                                      note="the same solve on the reference's CSR (layout csr), "
                                           "in the line's recurrence (sr: unfused, two launches "
                                           "and one reduction); hs_value: the HS iteration")
        if wl["kind"] in ("lap3d", "lap2d"):
            extra["matrix_free"] = matrix_free(wl, sysm["b"], args.steps, args.warmup)
        if wl_name == "c4":
            extra["c3"] = c3_legs(args.steps, args.warmup)
            extra["c5"] = c5_leg(args.steps, args.warmup)
            extra["c2"] = c2_leg(args.steps, args.warmup)
        if wl_name == "c3":
            extra["general_coefficients"] = general_coefficients(args.steps, args.warmup)
            extra["c4_1gpu"] = c4_one_gpu(min(args.steps, 50), args.warmup)
            extra["solve_e2e"] = solve_e2e(sysm)

    cpu = None
    if not args.no_cpu:
        cpu = cpu_baseline(sysm, args.cpu_seconds)
        cpu["cpu_model"] = cpu_model()
        cpu["nproc"] = os.cpu_count()
        cpu["all_cores"] = cpu_baseline_mt(sysm, args.cpu_seconds / 2)
        cpu["reference_c1"] = reference_c1()

    out = dict(
        metric=METRIC, value=round(args.steps / wall, 2), unit="it/s", n_gpus=1,
        steps=args.steps, warmup=args.warmup, ms_per_step=round(ms_per_step, 4),
        higher_is_better=True, scaling="strong", vs_baseline=None, dtype=wl["dtype"],
        data="synthetic",
        config=dict(workload=wl["desc"], n=sysm["n_global"], nnz=int(len(sysm["col"])),
                    alg=ALG_DESC[alg], alg_trial=trial, graph=True,
                    parallelism="single GPU", layout=layout_desc(info),
                    layout_name=info["layout_name"], value_basis=value_basis(info),
                    scaling_curve="the same workload at every N (N > 1: row-partitioned "
                                  "over RCCL), so value(N) / value(1) is the speedup"),
        device_ms_per_step=round(h["dev_ms"] / args.steps, 4),
        upload_ms=round(h["upload_ms"], 1),  # host CSR -> HBM + layout encoding, not in `value`
        iter_bytes=int(info["iter_bytes"]),
        roofline=roofline, headline_kernel=headline_kernel, cpu_baseline=cpu, **extra)
    print(json.dumps(out), flush=True)


# ------------------------------------------------------------ multi GPU

def gather_x(x_local, n_global, world, rank):
    """x of all ranks on every rank (all_gather over the default group)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import cgx
    sizes = [cgx.partition_rows(n_global, world, q) for q in range(world)]
    m = max(e - b for b, e in sizes)
    t = torch.zeros(m, dtype=torch.float64)  # host tensors: the gloo group
    t[:len(x_local)] = torch.from_numpy(x_local)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([parts[q][:e - b].numpy() for q, (b, e) in enumerate(sizes)])


def parity_gate(world, rank, local_rank, uid, tol=1e-10):
    """A small 3-D Laplacian (64 x 64 x 16 N rows: planes 8 slices apart, so
    SR runs the one-launch march step on the ranks, as at C4) solved across
    the N ranks to tol with every recurrence the trial may pick (HS unfused
    and fused, SR one-launch and two-launch, CG1) over RCCL; rank 0 checks the
    gathered x against a single-GPU solve of the same system (cgx.Solver, HS),
    the iteration count (within 1) and the true residual (scipy, on the host)."""
    import numpy as np
    import scipy.sparse as sp
    import cgx
    nx, ny, nz = 64, 64, 16 * world
    n = nx * ny * nz
    rb, re_ = cgx.partition_rows(n, world, rank)
    rp, col, val = cgx.laplacian3d(nx, ny, nz, rb, re_)
    b_full = np.random.default_rng(11).standard_normal(n)
    res = {}
    d = cgx.DistSolver(local_rank, world, rank, uid)
    try:
        d.set_matrix(n, rp, col, val)
        d.set_rhs(b_full[rb:re_])
        # the fused HS step forced on: the timed C4 run takes it (auto), this
        # small system would not; SR is always the fused step
        for name, alg, fused, march, want in (("hs", cgx.CGX_ALG_HS, False, -1, 0),
                                              ("hs_fused", cgx.CGX_ALG_HS, True, -1, 1),
                                              ("sr", cgx.CGX_ALG_SR, "auto", -1, 1),
                                              ("sr_two_launch", cgx.CGX_ALG_SR, "auto", 0, 1),
                                              ("cg1", cgx.CGX_ALG_CG1, False, -1, 0)):
            d.set_alg(alg)
            d.set_fused(fused)
            d.set_march(march)
            try:  # a refusal is collective (every rank alike): that recurrence fails the gate
                its = d.run(5000, tol)
            except cgx.CgxError as e:
                res[name] = (None, str(e), None, False)
                continue
            i = d.info()
            ok_shape = i["fused"] == want and (name != "sr" or i["march"] > 0)
            res[name] = (its, gather_x(d.x(), n, world, rank), i["graph"], ok_shape)
        d.set_fused("auto")
        d.set_march(-1)
    finally:
        d.close()
    if rank != 0:
        return None
    grp, gcol, gval = cgx.laplacian3d(nx, ny, nz)
    with cgx.Solver(local_rank) as s:
        s.set_matrix(grp, gcol, gval)
        s.set_rhs(b_full)
        its1 = s.run(5000, tol)
        x1 = s.x()
    A = sp.csr_matrix((gval, gcol, grp), shape=(n, n))
    out = dict(system=f"3-D Laplacian {nx}x{ny}x{nz} ({n} rows), b ~ N(0,1), tol {tol:g}",
               reference="single-GPU cgx.Solver (HS) on rank 0 + true residual (scipy)",
               single_gpu_iters=its1)
    ok = True
    for name, (its, x, graph, fused_ok) in res.items():
        if its is None:
            ok = False
            out[name] = dict(error=x, ok=False)
            continue
        rel = float(np.linalg.norm(x - x1) / np.linalg.norm(x1))
        tr = float(np.linalg.norm(b_full - A @ x) / np.linalg.norm(b_full))
        good = rel <= 1e-9 and abs(its - its1) <= 1 and tr <= 10 * tol and fused_ok
        ok = ok and good
        out[name] = dict(iters=its, rel_diff=rel, true_rel_residual=tr, graph=graph, ok=good)
    out["ok"] = ok
    return out


def gate_passed(gate):
    """The trial's recurrences whose parity-gate entries all passed (gate:
    entry name -> ok; "hs" needs the unfused and the fused HS runs, AUTO
    takes either at the timed size)."""
    needs = {"hs": ("hs", "hs_fused"), "sr": ("sr",), "sr_two_launch": ("sr_two_launch",),
             "cg1": ("cg1",)}
    return [a for a in needs if all(gate.get(g, False) for g in needs[a])]


def dist_line(args, wl, world, m):
    """The N > 1 JSON line from the measured pieces m (run_dist): the
    contract's fields, the trial, the roofline of the rank kernel (with its
    PMC traffic), the per-phase breakdown, the CPU baseline and the parity
    gate (parity_ok / gate_failed at the top level)."""
    info, value, mps, dev, parity = m["info"], m["value"], m["ms_per_step"], m["dev"], m["parity"]
    return dict(
        metric=METRIC, value=None if value is None else round(value, 2), unit="it/s",
        n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=None if mps is None else round(mps, 4),
        higher_is_better=True, scaling="strong", vs_baseline=None, dtype=wl["dtype"],
        data="synthetic",
        config=dict(workload=wl["desc"], n=m["n_global"], rows_per_rank=info["n_loc"],
                    nnz_rank0=info["nnz"], alg=m["alg"], march=info["march"],
                    alg_trial_ms_per_iter=m["trial"],
                    alg_refused=m["refused"] or None, fuse_status=info["fuse_status"],
                    graph=info["graph"], fused=info["fused"],
                    parallelism=f"row-partition x{world} (RCCL)",
                    scaling_curve="the same workload at every N (N = 1: the "
                                  "single-GPU solver), so value(N) / value(1) is the "
                                  "speedup",
                    layout=info["layout_name"], halo_bytes_per_iter_max_rank=m["halo"]),
        device_ms_per_step=None if dev is None else round(dev, 4),
        upload_ms=round(m["upload_ms"], 1), iter_bytes_rank0=int(info["iter_bytes"]),
        roofline=m["roofline"], phases=m["phases"], cpu_baseline=m["cpu"], parity=parity,
        parity_ok=bool(parity.get("ok")),
        gate_failed=[k for k, v in parity.items() if isinstance(v, dict) and not v.get("ok")],
        runtime=dict(m["runtime"], orchestration="torch.distributed gloo (host); data path: "
                                                 "libcgx's RCCL communicator"),
        **(dict(rehearsal="--ranks-share-gpu: every rank on GPU 0, RCCL over loopback sockets "
                          "-- a correctness rehearsal of the N > 1 path, not a scaling number")
           if args.ranks_share_gpu else {}))


def dist_traffic_key(alg, info):
    """KERNEL_PREFIX key of the rank's headline launch whose PMC summary
    prices `traffic` (profiles/pmc_c4n<N>_<key>.json: the slab kernel
    profiled on a 1-rank communicator, tools/dist_probe.py), or None."""
    if alg == "sr" and info.get("march", 0) > 0:
        return "sr1"
    return None


def run_dist(args, wl_name, world, rank, local_rank):
    """One rank.  The solver's data path is libcgx's RCCL communicator (the
    halos, the all-reduces); torch.distributed only orchestrates (the ids,
    barriers, max over ranks, the parity gate's x) over a host-side gloo
    group, and this process never touches torch's GPU runtime: libcgx is
    loaded BEFORE torch, so it binds the ROCm it was built against
    (/opt/rocm: HIP and RCCL of the same release).  Loaded after `import
    torch`, it would bind the older libamdhip64.so.7 / librccl.so.1 copies
    PyTorch bundles (same sonames), whose hipStreamEndCapture crashed on the
    ranks' captured halo (tools/rccl_pair_probe.py, profiles/r06_rccl_pair.log)."""
    import numpy as np
    import cgx

    wl = WORKLOADS[wl_name]
    if wl["kind"] == "rand":
        raise SystemExit("bench: C5 (random SPD) is a single-GPU configuration (BASELINE.json)")
    if args.ranks_share_gpu:
        # before the first RCCL call of this process (RCCL reads its
        # environment once): a host of its own per rank, loopback sockets
        os.environ.update(NCCL_HOSTID=f"cgx-rank{rank}", NCCL_SOCKET_IFNAME="lo",
                          NCCL_IB_DISABLE="1")
        local_rank = 0
    cgx.lib()
    import torch
    import torch.distributed as dist
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # one node: the ranks meet on loopback
    dist.init_process_group("gloo")
    runtime = cgx.runtime_versions()

    def allmax(v):
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allmin(v):
        return -allmax(-v)

    # one RCCL unique id per communicator (the parity system's, the bench's)
    uids = [[cgx.dist_unique_id(), cgx.dist_unique_id()] if rank == 0 else None]
    dist.broadcast_object_list(uids, src=0)
    uid_parity, uid = uids[0]

    # ---- parity gate (RCCL path, every recurrence) before anything is timed;
    # a recurrence that fails it is not timed, the others still are
    parity = parity_gate(world, rank, local_rank, uid_parity)
    gate = [{k: v["ok"] for k, v in parity.items() if isinstance(v, dict)} if rank == 0 else None]
    dist.broadcast_object_list(gate, src=0)
    passed = gate_passed(gate[0])
    ok = [bool(passed)]

    # ---- CPU baseline: the N = 1 line's one-core oracle
    # sample of the same whole system, on rank 0, before anything is timed
    cpu = None
    if rank == 0 and not args.no_cpu:
        full = make_system(wl)
        cpu = cpu_baseline(full, args.cpu_seconds)
        cpu["cpu_model"] = cpu_model()
        cpu["nproc"] = os.cpu_count()
        cpu["note"] = "rank 0, before the timed region, while the other ranks wait at a barrier"
        del full
    dist.barrier()

    sysm = make_system(wl, rank, world)
    t_up = time.perf_counter()
    s = cgx.DistSolver(local_rank, world, rank, uid)
    s.set_matrix(sysm["n_global"], sysm["rp"], sysm["col"], sysm["val"])
    s.set_rhs(sysm["b"])
    dist.barrier()
    upload_ms = 1e3 * (time.perf_counter() - t_up)

    # ---- recurrence: HS pays two all-reduce latencies per iteration, SR and
    # CG1 one (CG1 with 8-13 B/row more traffic); a timed trial (max over
    # ranks) picks
    trial = {}
    # name -> (recurrence, march): "sr" is SR's one-launch step on the ranks
    # where their rows take it (the C4 slabs), "sr_two_launch" its fused
    # two-launch form
    algs = {"hs": (cgx.CGX_ALG_HS, -1), "sr": (cgx.CGX_ALG_SR, -1),
            "sr_two_launch": (cgx.CGX_ALG_SR, 0), "cg1": (cgx.CGX_ALG_CG1, -1)}
    refused = {}
    for name in ([args.alg] if args.alg else ["hs", "sr", "sr_two_launch", "cg1"]):
        if name not in passed:
            refused[name] = "failed the parity gate"
            continue
        s.set_alg(algs[name][0])
        s.set_march(algs[name][1])
        try:
            s.bench_prepare(3)  # collective: every rank refuses SR alike (no fused step)
        except cgx.CgxError as e:
            refused[name] = str(e)
            continue
        dist.barrier()
        trial[name] = round(allmax(s.bench_run(20)[0] / 20), 4)
    if not trial:
        ok = [False]
    alg = min(trial, key=trial.get) if trial else (args.alg or "hs")
    s.set_alg(algs[alg][0])
    s.set_march(algs[alg][1])
    info = s.info()

    value = None
    ms_per_step = dev_ms = spmv_ms = None
    if ok[0]:
        # ---- timed region: exactly K steps, barrier + sync on both sides
        s.bench_prepare(args.warmup)
        cgx.device_synchronize(local_rank)
        dist.barrier()
        t0 = time.perf_counter()
        dev_ms = s.bench_run(args.steps)[0]
        cgx.device_synchronize(local_rank)
        dist.barrier()
        wall = allmax(time.perf_counter() - t0)
        ms_per_step = 1e3 * wall / args.steps
        value = args.steps / wall  # CG iterations of the one 64M-row system per second
        _, spmv_ms = s.bench_run(min(args.steps, 30), spmv_events=True)
        phases = s.bench_phases()
    info = s.info()
    s.close()

    # ---- per-phase breakdown, max over ranks of partition
    # 0's HIP events in the eager iterations: the march / interior launch, the
    # halo wait before the edge / boundary launch, that launch, and the tail
    # (local sums, all-reduce, next pack) -- so a curve below 6x says which
    phase_out = None
    if ok[0]:
        keys = ("first_launch", "halo_wait_gap", "second_launch", "tail", "period")
        mine = [phases[k] if phases else -1.0 for k in keys]
        phase_out = {k: round(allmax(v) * 1e3, 2) for k, v in zip(keys, mine)}
        phase_out.update(unit="us per iteration (max over ranks)",
                         timing="HIP events on each rank's stream, "
                                f"{min(args.steps, 30)} eager iterations (no graph)",
                         legend=dict(first_launch="k_sr1_dia_m march (one-launch SR) / "
                                                  "interior SpMV", halo_wait_gap="wait for the "
                                                  "halo before the edge / boundary launch",
                                     second_launch="k_sr1_edge / boundary SpMV",
                                     tail="local sums + RCCL all-reduce(s) + vector updates "
                                          "+ the next halo pack", period="iteration"))

    roofline = None
    if spmv_ms is not None:
        # per-rank SpMV (interior + boundary launches) on its own layout bytes
        gbs, frac = spmv_roofline(info["spmv_iter_bytes"], spmv_ms)
        tk = dist_traffic_key(alg, info)
        tf = traffic_fields(f"c4n{world}", tk, info["spmv_iter_bytes"]) if tk else dict(
            traffic=None, traffic_source="no PMC summary for this recurrence's rank kernel",
            traffic_ratio=None)
        roofline = dict(bound="hbm", achieved=gbs, peak=HBM_PEAK_GBS, unit="GB/s", frac=frac,
                        **tf, kernel=kernel_name(info) + " (per rank)",
                        algorithmic_bytes_per_launch=int(info["spmv_iter_bytes"]),
                        spmv_us=round(spmv_ms * 1e3, 2),
                        spmv_us_max_over_ranks=round(allmax(spmv_ms) * 1e3, 2),
                        frac_min_over_ranks=round(allmin(frac), 4),
                        csr_basis_bytes_per_rank=int(info["spmv_bytes"]))
    halo = allmax(info["halo_bytes"])
    dev = allmax(dev_ms / args.steps) if dev_ms is not None else None
    if rank == 0:
        out = dist_line(args, wl, world, dict(
            value=value, ms_per_step=ms_per_step, dev=dev, n_global=sysm["n_global"], info=info,
            alg=alg, trial=trial, refused=refused, halo=halo, upload_ms=upload_ms,
            roofline=roofline, phases=phase_out, cpu=cpu, parity=parity, runtime=runtime))
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    if not ok[0]:
        raise SystemExit(1)


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        # no GPU has been touched in this process: start the ranks as a child
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(env_world or 1)
    if world != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist_path = world > 1 or args.dist_rehearsal
    wl_name = args.workload or "c4"
    if not dist_path:
        run_single(args, wl_name)
    else:
        run_dist(args, wl_name, world, rank, local_rank)


if __name__ == "__main__":
    main()
