"""Device timeline of a replayed CG iteration from a rocprofv3 kernel trace:
are the kernels back to back (device-bound) or separated by host gaps?
  python tools/gaps.py <run_kernel_trace.csv> <anchor kernel> [...]
For each anchor (a kernel launched once per iteration, e.g. k_spmv_dia_h):
runs of anchors less than 600 us apart (one replayed graph, or one eager
call), >= 8 iterations each; the median anchor period inside the runs
against the summed median kernel durations of one iteration (equal = no
gaps inside a run), the gaps between consecutive kernels inside the runs
(next start - this end), the time from one run's last anchor to the next
run's first, and the median duration of each kernel of one iteration."""
import csv
import re
import statistics as st
import sys
from collections import defaultdict


def short(k):
    k = re.sub(r"^void ", "", k.replace("(anonymous namespace)::", ""))
    return re.sub(r"[<(].*$", "", k).split("::")[-1]


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
              for r in csv.DictReader(open(sys.argv[1])))
print("| anchor | runs x iterations | period us (median) | kernels us (sum of medians) | gap in run: median / p99 / max us | between runs us (median) | one iteration (median us) |")
print("|---|---|---|---|---|---|---|")
for anchor in sys.argv[2:]:
    idx = [i for i, r in enumerate(rows) if r[2] == anchor]
    runs, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if rows[b][0] - rows[a][0] > 600_000:  # a graph launch / host boundary
            runs.append(cur)
            cur = []
        cur.append(b)
    runs.append(cur)
    runs = [r for r in runs if len(r) >= 8]
    periods, gaps, per, order, between = [], [], defaultdict(list), [], []
    for run in runs:
        periods += [(rows[b][0] - rows[a][0]) / 1e3 for a, b in zip(run, run[1:])]
        for i in range(run[0], run[-1]):
            b, e, k = rows[i]
            gaps.append((rows[i + 1][0] - e) / 1e3)
            if k not in per:
                order.append(k)
            per[k].append((e - b) / 1e3)
    for r0, r1 in zip(runs, runs[1:]):
        between.append((rows[r1[0]][0] - rows[r0[-1]][0]) / 1e3)
    its = sum(len(r) - 1 for r in runs)
    gaps.sort()
    p99 = gaps[min(len(gaps) - 1, int(0.99 * len(gaps)))]
    ksum = sum(st.median(per[k]) * len(per[k]) / its for k in order)
    one = ", ".join(f"{k} {st.median(per[k]):.1f}" +
                    (f" x{round(len(per[k]) / its)}" if round(len(per[k]) / its) > 1 else "")
                    for k in order)
    print(f"| {anchor} | {len(runs)} x {its // max(1, len(runs))} | {st.median(periods):.1f} | "
          f"{ksum:.1f} | {st.median(gaps):.2f} / {p99:.2f} / {gaps[-1]:.2f} | "
          f"{st.median(between) if between else float('nan'):.0f} | {one} |")
