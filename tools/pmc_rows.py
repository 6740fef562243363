"""Per-(kernel, grid) HBM traffic of the §8f row kernels from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over tools/bench_rows.py:

    python tools/pmc_rows.py gpurun_out/pmc_rows_fetch gpurun_out/pmc_rows_write > profiles/.../pmc_rows.txt

Both counters are KiB per dispatch. FETCH_SIZE is shown raw and doubled: the guide's
gfx950 correction (MI355X_MICROARCH.md §HBM) is exact for 16-B-per-lane streaming
reads only, so for kernels with narrower loads the truth lies between the two.
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(d, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter or "pmenv_dev" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pmenv_dev::", "")
            acc[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in acc.items()}


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':50s} {'grid':>10s} {'FETCH MB':>10s} {'x2 MB':>10s} {'WRITE MB':>10s}")
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, float("nan")), write.get(k, float("nan"))
    print(f"{k[0]:50s} {k[1]:10d} {f * 1024 / 1e6:10.1f} {2 * f * 1024 / 1e6:10.1f} {w * 1024 / 1e6:10.1f}")
