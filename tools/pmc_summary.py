#!/usr/bin/env python3
"""Summarise a tools/profile.sh collection into profiles/ (committed):
  profiles/<round>_<tag>_kernel_stats.csv   rocprofv3 --stats output, verbatim
  profiles/<round>_<tag>.md                 per-kernel time + HBM bytes table
  profiles/pmc_<workload>.json              read by bench.py (roofline.traffic)

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
16-B-per-lane streaming read, so reads are doubled.  The calibration was
checked on this code's own streaming kernels (k_update_xr / k_xpay read
exactly 2 x FETCH_SIZE = the algorithmic bytes).  The SpMV's x gathers and
row_ptr loads are narrower accesses (uncalibrated); doubling them makes the
SpMV figure an upper bound.

  python tools/pmc_summary.py <tag> <round> <workload> [algorithmic_spmv_bytes]
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
src = REPO / "gpurun_out" / f"prof_{tag}"
dst = REPO / "profiles"
dst.mkdir(exist_ok=True)


def short(name):
    name = name.replace("cgx::(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name and "<" not in name.split("(")[0][-1:] else name[:90]


stats = list(csv.DictReader(open(src / "trace" / "run_kernel_stats.csv")))
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{rnd}_{tag}_kernel_stats.csv")
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in ("fetch", "write"):
    for r in csv.DictReader(open(src / f / "run_counter_collection.csv")):
        pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))

rows, spmv = [], None
for s in stats:
    name = s["Name"]
    c = pmc.get(name, {})
    fetch = sum(c.get("FETCH_SIZE", [0])) / max(len(c.get("FETCH_SIZE", [1])), 1) * 1024
    write = sum(c.get("WRITE_SIZE", [0])) / max(len(c.get("WRITE_SIZE", [1])), 1) * 1024
    avg_ns = float(s["AverageNs"])
    hbm = 2 * fetch + write
    rows.append((short(name), int(s["Calls"]), avg_ns / 1e3, float(s["Percentage"]),
                 fetch / 1e6, write / 1e6, hbm / 1e6, hbm / avg_ns if avg_ns else 0))
    if "k_spmv" in name and (spmv is None or int(s["Calls"]) > spmv["calls"]):
        spmv = dict(kernel=short(name), calls=int(s["Calls"]), avg_us=avg_ns / 1e3,
                    fetch_size_bytes_raw=fetch, write_size_bytes=write,
                    spmv_hbm_bytes_per_launch=hbm)
md = [f"# {rnd} {tag}: rocprofv3 --kernel-trace --stats + --pmc FETCH_SIZE / WRITE_SIZE",
      "", "| kernel | calls | avg us | % time | FETCH raw MB | WRITE MB | HBM MB (2F+W) | GB/s |",
      "|---|---|---|---|---|---|---|---|"]
for r in rows:
    md.append(f"| `{r[0]}` | {r[1]} | {r[2]:.2f} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.1f} | "
              f"{r[6]:.1f} | {r[7]:.0f} |")
if spmv and alg_bytes:
    md += ["", f"SpMV algorithmic bytes per launch: {alg_bytes:.0f}; measured HBM (upper "
           f"bound, see tools/pmc_summary.py): {spmv['spmv_hbm_bytes_per_launch']:.0f} "
           f"({spmv['spmv_hbm_bytes_per_launch'] / alg_bytes:.2f}x)"]
(dst / f"{rnd}_{tag}.md").write_text("\n".join(md) + "\n")
if spmv:
    spmv["algorithmic_bytes_per_launch"] = alg_bytes
    spmv["source"] = f"profiles/{rnd}_{tag}_kernel_stats.csv + PMC passes ({rnd})"
    (dst / f"pmc_{workload}.json").write_text(json.dumps(spmv, indent=1) + "\n")
print("\n".join(md))
