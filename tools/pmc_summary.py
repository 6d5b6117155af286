#!/usr/bin/env python3
"""Summarise a tools/profile.sh collection into profiles/ (committed):
  profiles/<round>_<tag>_kernel_stats.csv   rocprofv3 --stats output, verbatim
  profiles/<round>_<tag>.md                 per-kernel time + memory-side bytes
  profiles/pmc_<workload>.json              read by bench.py (roofline.traffic)

Two byte estimates per launch, both from separate single-counter --pmc passes:
* EA bytes (used for `traffic`): the size-resolved L2->fabric requests,
  128 RDREQ_128B + 64 RDREQ_64B + 32 RDREQ_32B reads and 64 WRREQ_64B +
  32 (WRREQ - WRREQ_64B) writes.  Calibrated on the bench's k_stream_read,
  which reads exactly 512 MiB: 4,194,304 RDREQ_128B.
* the guide's rule (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
  2 x FETCH_SIZE + WRITE_SIZE (KiB; FETCH_SIZE reports half of a 16-B/lane
  stream on gfx950).  Agrees with the EA bytes on the streaming kernels.
Both count L2 misses, including those the Infinity Cache serves: an upper
bound of DRAM traffic.

  python tools/pmc_summary.py <tag> <round> <out> <algorithmic_spmv_bytes> <kernel>
writes profiles/pmc_<out>.json for the kernel whose name starts with <kernel>
(e.g. "k_spmv_dia<double, 1, true" or "k_spmv_csr<double, 456, 7, true") --
the one with the most launches when several match.
"""
import csv
import collections
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
tag, rnd, workload = sys.argv[1], sys.argv[2], sys.argv[3]
alg_bytes = float(sys.argv[4]) if len(sys.argv) > 4 else None
want = sys.argv[5] if len(sys.argv) > 5 else "k_spmv"
src = REPO / "gpurun_out" / f"prof_{tag}"
dst = REPO / "profiles"
dst.mkdir(exist_ok=True)

COUNTERS = ["FETCH_SIZE", "WRITE_SIZE", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
            "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"]


def short(name):
    name = name.replace("cgx::(anonymous namespace)::", "").replace("cgx::", "").replace("void ", "")
    return name.split("(")[0] if "(" in name and "<" not in name.split("(")[0][-1:] else name[:90]


stats = list(csv.DictReader(open(src / "trace" / "run_kernel_stats.csv")))
# per-dispatch durations: the average over the launches that did the work
# (a solve with a tolerance ends with launches that early-exit on the stop
# flag in ~5 us; they pull --stats' average down)
durs = collections.defaultdict(list)
for r in csv.DictReader(open(src / "trace" / "run_kernel_trace.csv")):
    durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def active(name):
    d = sorted(durs.get(name, []))
    if not d:
        return None, None, 0
    med = d[len(d) // 2]
    act = [x for x in d if x >= 0.25 * med]
    return med, sum(act) / len(act), len(d) - len(act)
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{rnd}_{tag}_kernel_stats.csv")
pmc = collections.defaultdict(dict)
for c in COUNTERS:
    f = src / f"pmc_{c}" / "run_counter_collection.csv"
    if not f.exists():
        continue
    acc = collections.defaultdict(list)
    rs = list(csv.DictReader(open(f)))
    pd = collections.defaultdict(list)
    for r in rs:
        pd[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in pd.items()}
    for r in rs:  # working launches only (not the early exits after a stop)
        if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) >= 0.25 * med[r["Kernel_Name"]]:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        pmc[k][c] = sum(v) / len(v)

rows, spmv, calib = [], None, None
cmdf = src / "cmd.txt"
cmd = cmdf.read_text().strip() if cmdf.exists() else ""
for s in stats:
    name = s["Name"]
    c = pmc.get(name, {})
    g = lambda k: c.get(k, 0.0)  # noqa: E731
    guide = 2 * g("FETCH_SIZE") * 1024 + g("WRITE_SIZE") * 1024
    ea_rd = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + \
        32 * g("TCC_EA0_RDREQ_32B_sum")
    ea_wr = 64 * g("TCC_EA0_WRREQ_64B_sum") + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum"))
    avg_ns = float(s["AverageNs"])
    ea = ea_rd + ea_wr
    work_us = active(name)[1] or avg_ns / 1e3  # EA GB/s over the working launches
    rows.append((short(name), int(s["Calls"]), avg_ns / 1e3, float(s["Percentage"]),
                 ea_rd / 1e6, ea_wr / 1e6, guide / 1e6, ea / (work_us * 1e3) if work_us else 0))
    if "k_stream_read" in name:
        calib = ea_rd
    if short(name).startswith(want) and (spmv is None or int(s["Calls"]) > spmv["calls"]):
        med, act_avg, n_exit = active(name)
        spmv = dict(kernel=short(name), calls=int(s["Calls"]), avg_us=avg_ns / 1e3,
                    median_us=med, avg_us_working_launches=act_avg, early_exit_launches=n_exit,
                    ea_read_bytes=ea_rd, ea_write_bytes=ea_wr,
                    guide_bytes_2fetch_plus_write=guide,
                    spmv_hbm_bytes_per_launch=ea)
md = [f"# {rnd} {tag}: rocprofv3 --kernel-trace --stats + single-counter --pmc passes",
      "", f"Command: `{cmd}`" if cmd else "",
      "", "EA = L2->fabric requests by size (see tools/pmc_summary.py); guide = 2 x FETCH_SIZE "
      "+ WRITE_SIZE.  Both include Infinity-Cache hits.", "",
      "median us: per-dispatch median from the kernel trace.  A solve with a tolerance ends "
      "with launches that early-exit on the stop flag (~5 us); --stats' avg includes them, "
      "the byte columns (per launch) do not.", "",
      "| kernel | calls | avg us | median us | % time | EA read MB | EA write MB | guide MB | EA GB/s |",
      "|---|---|---|---|---|---|---|---|---|"]
for r, s in zip(rows, stats):
    med = active(s["Name"])[0]
    md.append(f"| `{r[0]}` | {r[1]} | {r[2]:.2f} | {med:.2f} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.1f} | "
              f"{r[6]:.1f} | {r[7]:.0f} |")
if calib:
    md += ["", f"Calibration: k_stream_read reads 536.9 MB by construction; EA read = "
           f"{calib / 1e6:.1f} MB."]
if spmv and alg_bytes:
    md += ["", f"SpMV algorithmic bytes per launch: {alg_bytes:.0f}; EA bytes: "
           f"{spmv['spmv_hbm_bytes_per_launch']:.0f} "
           f"({spmv['spmv_hbm_bytes_per_launch'] / alg_bytes:.3f}x)."]
md_path = dst / f"{rnd}_{tag}.md"
if not md_path.exists() or len(sys.argv) <= 6:
    md_path.write_text("\n".join(md) + "\n")
agg = len(sys.argv) > 6 and sys.argv[6] == "sum"
if spmv and agg:
    # a multi-launch SpMV (column panels): the bytes of every matching
    # launch, per SpMV (= per launch of the least-launched variant, the
    # last pass with the epilogue)
    ms = [x for x in stats if short(x["Name"]).startswith(want.split("<")[0] + "<")]
    tot, per = 0.0, min(int(x["Calls"]) for x in ms)
    for x in ms:
        c = pmc.get(x["Name"], {})
        g = lambda k: c.get(k, 0.0)  # noqa: E731
        tot += int(x["Calls"]) * (128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum")
                                  + 32 * g("TCC_EA0_RDREQ_32B_sum") + 64 * g("TCC_EA0_WRREQ_64B_sum")
                                  + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum")))
    spmv["spmv_hbm_bytes_per_launch"] = tot / per
    spmv["aggregated"] = f"{len(ms)} kernel variants, {per} SpMVs"
    md += ["", f"Multi-launch SpMV: EA bytes per SpMV over {len(ms)} kernel variants: "
           f"{tot / per:.0f}" + (f" ({tot / per / alg_bytes:.3f}x algorithmic)" if alg_bytes else "")]
    md_path.write_text("\n".join(md) + "\n")
if spmv:
    spmv["algorithmic_bytes_per_launch"] = alg_bytes
    spmv["calibration_stream_read_bytes"] = calib
    spmv["source"] = f"profiles/{rnd}_{tag}_kernel_stats.csv + single-counter PMC passes ({rnd})"
    (dst / f"pmc_{workload}.json").write_text(json.dumps(spmv, indent=1) + "\n")
print("\n".join(md))
