#!/usr/bin/env python3
"""Per-kernel unit counters from tools/pmc_passes.sh: the totals of every
launch whose name starts with <kernel>, divided by <per> (launches per
operation, e.g. a C5 SpMV = 6 panel launches), plus derived rates.
  python tools/pmc_units.py <tag> <kernel-prefix> [per] [--md out.md]"""
import csv
import collections
import glob
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
tag, want = sys.argv[1], sys.argv[2]
per = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else 1
tot = collections.defaultdict(float)
launches = collections.defaultdict(int)
for f in sorted(glob.glob(str(REPO / "gpurun_out" / f"pmcu_{tag}" / "p*" / "**" / "*counter_collection.csv"),
                          recursive=True)):
    seen = set()
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        short = name.replace("cgx::(anonymous namespace)::", "").replace("void ", "")
        if not short.startswith(want):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
        if key not in seen:
            seen.add(key)
            launches[r["Counter_Name"]] += 1
n_ops = max(launches.values()) / per if launches else 0
rows = []
for c in sorted(tot):
    rows.append((c, tot[c] / max(launches[c] / per, 1)))
d = dict(rows)
lines = [f"# PMC units: `{want}` ({tag}), per operation = {per} launch(es), {n_ops:.0f} operations", "",
         "| counter | per operation |", "|---|---|"]
lines += [f"| {c} | {v:,.0f} |" for c, v in rows]
derived = []
if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
    derived.append(("L2 hit rate", d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1)))
if "GRBM_GUI_ACTIVE" in d:
    # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (checked on k_stream_read:
    # 512 MiB in 1.82 M summed = 228 K cycles = 95 us at 2.4 GHz, 5.6 TB/s)
    cyc = d["GRBM_GUI_ACTIVE"] / 8
    derived.append(("GPU cycles (GRBM_GUI_ACTIVE / 8 XCDs)", cyc))
    derived.append(("time at 2.4 GHz (us)", cyc / 2400.0))
    if "TCC_REQ_sum" in d:
        derived.append(("L2 requests per XCD-cycle (16 channels: peak 16)", d["TCC_REQ_sum"] / 8 / cyc))
    if "TA_TA_BUSY_sum" in d:
        derived.append(("TA busy fraction (TA_BUSY_sum / 256 CUs / cycles)", d["TA_TA_BUSY_sum"] / 256 / cyc))
    if "TA_ADDR_STALLED_BY_TC_CYCLES_sum" in d:
        derived.append(("TA address path stalled by the TC (fraction of cycles)",
                        d["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / 256 / cyc))
    if "TD_TD_BUSY_sum" in d:
        derived.append(("TD busy fraction", d["TD_TD_BUSY_sum"] / 256 / cyc))
if "TCP_TCC_READ_REQ_LATENCY_sum" in d and "TCP_TCC_READ_REQ_sum" in d:
    derived.append(("TCP->TCC read latency (cycles per request)",
                    d["TCP_TCC_READ_REQ_LATENCY_sum"] / max(d["TCP_TCC_READ_REQ_sum"], 1)))
if "SQ_WAVE_CYCLES" in d:
    w = d["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
        if k in d:
            derived.append((f"{k} / SQ_WAVE_CYCLES", d[k] / w))
if "SQ_LDS_BANK_CONFLICT" in d and "SQ_INSTS_LDS" in d:
    derived.append(("LDS bank-conflict cycles per LDS instruction", d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_INSTS_LDS"], 1)))
if derived:
    lines += ["", "| derived | value |", "|---|---|"] + [f"| {k} | {v:.4g} |" for k, v in derived]
text = "\n".join(lines) + "\n"
print(text)
if "--md" in sys.argv:
    Path(sys.argv[sys.argv.index("--md") + 1]).write_text(text)
