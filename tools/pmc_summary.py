"""Summarise rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes into profiles/.

    python tools/pmc_summary.py TAG [B N W F]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of
a wide (16 B/lane) coalesced streaming read, so it is doubled before comparison;
WRITE_SIZE is exact for 16-B/lane streaming stores. Both counters are in KiB.
The dword-wide loads of the kernel (w', unshifted weight) are L1/L2 hits of lines
the 16-B stream also fetches, so the doubling is applied to the whole counter.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
shape = [int(x) for x in sys.argv[2:6]] if len(sys.argv) >= 6 else [65536, 30, 50, 5]
out = os.path.join(ROOT, "gpurun_out")


def per_kernel(path, counter):
    rows = list(csv.DictReader(open(path)))
    acc = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        acc.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel(os.path.join(out, f"pmc_fetch_{tag}", "run_counter_collection.csv"), "FETCH_SIZE")
write = per_kernel(os.path.join(out, f"pmc_write_{tag}", "run_counter_collection.csv"), "WRITE_SIZE")
B, N, W, F = shape
alg = (8 * N * W * F + 20) * B
res = {"tag": tag, "workload": shape, "algorithmic_bytes_per_launch": alg, "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if "advance_rows" not in k and "advance_flat" not in k and "scalar_step" not in k and "step_advance" not in k \
            and "step_env" not in k and "step_flat" not in k and "flat_prime" not in k:
        continue
    fb = fetch.get(k, 0.0) * 1024 * 2
    wb = write.get(k, 0.0) * 1024
    res["kernels"][k] = {"fetch_size_kib_raw": fetch.get(k), "write_size_kib": write.get(k),
                         "hbm_read_bytes_corrected": fb, "hbm_write_bytes": wb, "hbm_bytes": fb + wb}
main = [k for k in res["kernels"] if "step_flat_kernel" in k and ", false>" in k] or \
       [k for k in res["kernels"] if "step_env_kernel<4, false" in k] or \
       [k for k in res["kernels"] if "advance_flat_inplace_kernel" in k] or \
       [k for k in res["kernels"] if "advance_flat_wg_kernel" in k] or \
       [k for k in res["kernels"] if "advance_flat_kernel" in k] or \
       [k for k in res["kernels"] if "advance_rows_kernel" in k and "false" in k] or \
       [k for k in res["kernels"] if "advance_rows_kernel" in k]
if main:
    res["hbm_bytes_per_launch"] = res["kernels"][main[0]]["hbm_bytes"]
    res["dominant_kernel"] = main[0]
    res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / alg
# the library these counters were collected on (the in-tree build the GPU run loaded):
# bench.py reports roofline.traffic only while the running library has this sha256
import hashlib  # noqa: E402
lib = os.path.join(ROOT, "pm-rl_amd", "pmenv", "libpmenv.so")
res["lib_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None
# ... or a build of the same sources (hipcc output is not byte-reproducible: tools/libfp.py)
sys.path.insert(0, ROOT)
from tools.libfp import source_sha256  # noqa: E402
res["lib_src_sha256"] = source_sha256(ROOT)
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
json.dump(res, open(os.path.join(ROOT, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
for f in ("run_kernel_stats.csv",):
    src = os.path.join(out, f"prof_{tag}", f)
    if os.path.exists(src):
        shutil.copy(src, os.path.join(ROOT, "profiles", f"kernel_stats_{tag}.csv"))
bench = os.path.join(out, f"bench_{tag}.json")
if os.path.exists(bench):
    shutil.copy(bench, os.path.join(ROOT, "profiles", f"bench_{tag}.json"))
print(json.dumps(res, indent=1))
