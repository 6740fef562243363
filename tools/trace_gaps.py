"""Median idle gap between consecutive kernels of a rocprofv3 kernel trace, per (previous,
next) kernel pair, and the median duration of each kernel.

    python tools/trace_gaps.py gpurun_out/prof_x/run_kernel_trace.csv
"""
import csv
import statistics
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    short = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pmenv_dev::", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
rows.sort()
dur, gap = defaultdict(list), defaultdict(list)
for i, (s, e, k) in enumerate(rows):
    dur[k].append((e - s) / 1e3)
    if i:
        ps, pe, pk = rows[i - 1]
        gap[(pk, k)].append((s - pe) / 1e3)
for k, v in sorted(dur.items()):
    print(f"{k:40s} n {len(v):5d}  median {statistics.median(v):8.2f} us")
for (a, b), v in sorted(gap.items()):
    if len(v) >= 20:
        print(f"gap {a} -> {b}: n {len(v)}  median {statistics.median(v):.2f} us")
