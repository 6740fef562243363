"""Per-shape kernel durations from a rocprofv3 kernel trace: average / median / min
duration per (kernel, grid, workgroup) — shapes of one kernel differ by grid size.

    python tools/trace_by_grid.py gpurun_out/prof_rows/rows_kernel_trace.csv [substring ...]
"""
import csv
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
keys = sys.argv[2:] or ["pmenv_dev"]
acc = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if not any(k in name for k in keys):
        continue
    short = name.split("(")[0].replace("void ", "").replace("pmenv_dev::", "")
    grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))
    acc[(short, grid, int(r["Workgroup_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, grid, wg), ts in sorted(acc.items()):
    print(f"{k:48s} grid {grid[0]:>10d}x{grid[1]:<4d} wg {wg:4d}  n {len(ts):4d}  "
          f"avg {sum(ts) / len(ts):9.2f}  med {statistics.median(ts):9.2f}  min {min(ts):9.2f} us")
