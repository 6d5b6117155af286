"""Per-kernel durations from a rocprofv3 kernel trace, split by launch grid:
  python tools/kgrid.py <run_kernel_trace.csv> [name substring ...]
One row per (kernel, workgroups): launches, median / mean / min us.  The
partitioned SR step launches k_sr1_dia_m twice per iteration (interior
and boundary steps, different grids); this separates them."""
import csv
import re
import statistics as st
import sys
from collections import defaultdict


def short(k):
    k = re.sub(r"^void ", "", k.replace("(anonymous namespace)::", ""))
    return re.sub(r"\(.*$", "", k).replace("cgx::", "")


want = sys.argv[2:]
runs = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = short(r["Kernel_Name"])
    if want and not any(w in name for w in want):
        continue
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    runs[(name, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("| kernel | workgroups | launches | median us | mean us | min us |")
print("|---|---|---|---|---|---|")
for (name, wg), d in sorted(runs.items(), key=lambda kv: -sum(kv[1])):
    print("| %s | %d | %d | %.1f | %.1f | %.1f |" % (name[:70], wg, len(d), st.median(d), st.mean(d), min(d)))
