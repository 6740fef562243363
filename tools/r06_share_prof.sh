#!/bin/bash
# Round 6, final build: config 4's 8-GPU share (8,192 x 30 in place, step_relay_kernel on 256 x 4
# tiles) under rocprofv3 — the kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own.
set -o pipefail
T=${1:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--envs-per-gpu 8192 --steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/share_prof_$T -o run --output-format csv -- python3 bench.py $A > gpurun_out/share_prof_$T.log 2>&1 || exit $?
grep -E "step_relay|relay_prime" gpurun_out/share_prof_$T/run_kernel_stats.csv | cut -c1-200
B="--envs-per-gpu 8192 --steps 10 --warmup 2 --cpu-baseline 0 --alt-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/share_fetch_$T -o run --output-format csv -- python3 bench.py $B > gpurun_out/share_fetch_$T.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/share_write_$T -o run --output-format csv -- python3 bench.py $B > gpurun_out/share_write_$T.log 2>&1 || exit $?
python3 - <<PY
import csv
for c, d in (("FETCH_SIZE", "share_fetch_$T"), ("WRITE_SIZE", "share_write_$T")):
    acc = {}
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == c and "step_relay_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Kernel_Name"][:100], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(c, k, "KiB per launch", sum(v) / len(v), "launches", len(v))
PY
