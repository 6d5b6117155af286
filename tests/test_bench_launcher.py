"""bench.py's N > 1 launcher (CPU only, no GPU touched): `--gpus N` without
WORLD_SIZE starts this script under torch.distributed.run as a CHILD process
(one rank per GPU, rendezvous on 127.0.0.1) and exits with its code; with
WORLD_SIZE set it runs as a rank; a WORLD_SIZE that disagrees with --gpus is
refused."""
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402  (module import must not touch torch / the GPU)


def test_module_import_is_gpu_free():
    assert "torch" not in bench.__dict__ and "cgx" not in bench.__dict__


def test_launch_cmd_for_two_gpus():
    cmd = bench.launch_cmd(["--gpus", "2", "--steps", "5", "--warmup", "1"], 2, 29123)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=2" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29123" in cmd
    i = cmd.index(str(REPO / "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "5", "--warmup", "1"]


def test_main_spawns_child_without_world_size(monkeypatch):
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "7"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3  # the child's exit code is forwarded
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-4:] == ["--gpus", "2", "--steps", "7"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_size_mismatch_refused(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=4" in str(e.value.code)


def test_default_workloads():
    a = bench.parse_args(["--gpus", "8"])
    assert a.workload is None and a.steps == 100 and a.warmup == 10
    assert bench.WORKLOADS["c4"]["dims"] == (400, 400, 400)
    assert bench.WORKLOADS["c3"]["dims"] == (216, 216, 216)


@pytest.mark.parametrize("argv,expect", [(["--gpus", "1"], ("single", "c4")),
                                         (["--gpus", "1", "--workload", "c3"], ("single", "c3")),
                                         (["--gpus", "1", "--dist-rehearsal"], ("dist", "c4")),
                                         (["--gpus", "1", "--workload", "c2"], ("single", "c2"))])
def test_rank_path_selection(monkeypatch, argv, expect):
    """Every N runs the same workload (C4: one strong-scaling curve); one rank
    runs the single-GPU solver unless --dist-rehearsal asks for the N > 1
    path (C4 over a 1-rank RCCL communicator)."""
    seen = {}
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    monkeypatch.setattr(bench, "run_single", lambda a, w: seen.update(path="single", wl=w))
    monkeypatch.setattr(bench, "run_dist", lambda a, w, *r: seen.update(path="dist", wl=w))
    bench.main()
    assert (seen["path"], seen["wl"]) == expect


def test_traffic_is_keyed_on_the_kernel(tmp_path, monkeypatch):
    """a PMC summary prices only the kernel it was collected
    on -- a file naming another kernel yields no `traffic` (and says why)."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", tmp_path)
    (prof / "pmc_c4_sr1.json").write_text(json.dumps(
        {"kernel": "k_sr1_dia_m<double, 2, 2, 1>", "spmv_hbm_bytes_per_launch": 4.1e9}))
    (prof / "pmc_c4_dia_march.json").write_text(json.dumps(
        {"kernel": "k_sr1_dia_m<double, 2, 2, 1>", "spmv_hbm_bytes_per_launch": 4.1e9}))
    t = bench.traffic_fields("c4", "sr1", 3.904e9)
    assert t["traffic"] == 4_100_000_000 and t["traffic_ratio"] == round(4.1 / 3.904, 4)
    t = bench.traffic_fields("c4", "dia_march", 2.88e9)
    assert t["traffic"] is None and "not k_spmv_dia_m<" in t["traffic_source"]
    assert bench.traffic_fields("c3", "sr1", 1.0)["traffic"] is None


def test_committed_pmc_summaries_name_their_kernel():
    """Every committed profiles/pmc_<workload>_<key>.json is a summary of the
    kernel its key names."""
    import json
    files = sorted((REPO / "profiles").glob("pmc_*_*.json"))
    assert files
    for f in files:
        key = f.stem.split("_", 2)[2]
        if key in bench.KERNEL_PREFIX:
            assert json.loads(f.read_text())["kernel"].startswith(bench.KERNEL_PREFIX[key]), f.name


def test_gate_decides_per_recurrence():
    """bench.py N > 1: a recurrence that fails the parity gate (or is refused
    there) is left out of the timed trial; the others still run."""
    import bench
    every = dict(hs=True, hs_fused=True, sr=True, sr_two_launch=True, cg1=True)
    assert bench.gate_passed(every) == ["hs", "sr", "sr_two_launch", "cg1"]
    assert bench.gate_passed(dict(every, sr=False)) == ["hs", "sr_two_launch", "cg1"]
    assert bench.gate_passed(dict(every, hs_fused=False)) == ["sr", "sr_two_launch", "cg1"]
    assert bench.gate_passed({}) == []


def test_dist_line_schema():
    """the N > 1 line explains itself -- per-phase breakdown,
    the CPU baseline, the rank kernel's PMC traffic, and the parity gate at
    the top level (parity_ok / gate_failed)."""
    args = bench.parse_args(["--gpus", "8", "--steps", "50", "--warmup", "5"])
    info = dict(n_loc=8_000_000, nnz=55_680_000, march=17, fuse_status=0, graph=1, fused=1,
                layout_name="dia", iter_bytes=1.4e9, alg=2, spmv_iter_bytes=4.9e8)
    phases = dict(first_launch=117.0, halo_wait_gap=0.5, second_launch=8.0, tail=14.0,
                  period=140.0, unit="us per iteration (max over ranks)")
    parity = dict(ok=False, hs=dict(ok=True), sr=dict(ok=False), system="...")
    cpu = dict(value=2.0, unit="it/s", cores=1, kind="port", sample="...")
    roof = dict(bound="hbm", achieved=4000.0, peak=8000.0, unit="GB/s", frac=0.5,
                traffic=5.0e8, traffic_source="profiles/pmc_c4n8_sr1.json", traffic_ratio=1.02)
    m = dict(value=7000.0, ms_per_step=0.1428, dev=0.14, n_global=64_000_000, info=info,
             alg="sr", trial={"sr": 0.14}, refused={}, halo=2.56e6, upload_ms=900.0,
             roofline=roof, phases=phases, cpu=cpu, parity=parity,
             runtime=dict(hip_runtime=70226015, hip_compiled=70226015, rccl=22707))
    line = bench.dist_line(args, bench.WORKLOADS["c4"], 8, m)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "phases", "cpu_baseline", "parity", "parity_ok", "gate_failed",
              "runtime"):
        assert k in line, k
    assert "rehearsal" not in line
    assert line["runtime"]["hip_runtime"] == line["runtime"]["hip_compiled"]
    # --ranks-share-gpu labels its line a rehearsal
    shared = bench.dist_line(bench.parse_args(["--gpus", "2", "--ranks-share-gpu"]),
                             bench.WORKLOADS["c4"], 2, m)
    assert "not a scaling number" in shared["rehearsal"]
    assert line["n_gpus"] == 8 and line["value"] == 7000.0
    assert line["cpu_baseline"]["cores"] == 1 and line["roofline"]["traffic"] == 5.0e8
    assert set(line["phases"]) >= {"first_launch", "halo_wait_gap", "second_launch", "tail",
                                   "period"}
    assert line["parity_ok"] is False and line["gate_failed"] == ["sr"]
    import json
    json.dumps(line)  # one JSON line
    assert bench.dist_traffic_key("sr", info) == "sr1"
    assert bench.dist_traffic_key("hs", info) is None
    assert bench.kernel_key(dict(info, fused=1)) == "sr1"
    assert bench.kernel_key(dict(info, march=0)) == "dia_fused"


def test_no_gbs_field_exceeds_peak():
    """no field named *gbs* in the committed bench lines of
    this build's schema may exceed the HBM peak -- CSR-basis rates of the
    compressed layouts are csr_basis_equiv_rate, C2's rates are fractions
    marked resident."""
    src = (REPO / "bench.py").read_text()
    assert "csr_equivalent_gbs" not in src and "csr_basis_gbs" not in src


def test_ranks_load_libcgx_before_torch():
    """Round 6: a rank process binds libcgx to the ROCm it was built against
    only if libcgx is loaded before `import torch` (PyTorch bundles older
    libamdhip64.so.7 / librccl.so.1 under the same sonames; with those the
    ranks' first capture with real peers crashed, profiles/r06_rccl_pair.log),
    and the rank's torch.distributed group is host-side gloo (no torch GPU
    runtime in the rank)."""
    import inspect
    src = inspect.getsource(bench.run_dist)
    assert src.index("cgx.lib()") < src.index("import torch")
    assert 'init_process_group("gloo")' in src and "torch.cuda" not in src
    g = inspect.getsource(bench.gather_x)
    assert "cuda" not in g
