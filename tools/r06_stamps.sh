#!/bin/bash
# Round 6: (1) the relay step's stamped breakdown at 8,192 / 4,096 x 30 in place (tools build,
# tools/relay_stamps.py); (2) the surface step at 65,536 x 30 x 50 x 5: per-kernel durations
# (rocprofv3 kernel trace) and FETCH_SIZE / WRITE_SIZE passes, one counter per pass.
#   bash tools/r06_stamps.sh TAG
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/relay_stamps.py > $O/relay_stamps.json 2> $O/relay_stamps.err || { echo "stamps failed"; tail -30 $O/relay_stamps.err; exit 1; }
cat $O/relay_stamps.err | cut -c1-1500
export SURF_SHAPES=65536x30x50x5 SURF_LIBS=pm-rl_amd/pmenv/libpmenv.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/surf_trace -o run --output-format csv -- python3 tools/bench_surface.py > $O/surf_trace.log 2>&1 || { echo "trace failed"; tail -20 $O/surf_trace.log; exit 1; }
grep -E "surface|scalar" $O/surf_trace/run_kernel_stats.csv | cut -c1-200
export SURF_K=10 SURF_R=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/surf_fetch -o run --output-format csv -- python3 tools/bench_surface.py > $O/surf_fetch.log 2>&1 || { echo "fetch failed"; tail -20 $O/surf_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/surf_write -o run --output-format csv -- python3 tools/bench_surface.py > $O/surf_write.log 2>&1 || { echo "write failed"; tail -20 $O/surf_write.log; exit 1; }
python - <<PY
import csv, json
def pk(p, c):
    acc = {}
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == c:
            acc.setdefault(r["Kernel_Name"].split("(")[0][:90], []).append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}
f = pk("$O/surf_fetch/run_counter_collection.csv", "FETCH_SIZE")
w = pk("$O/surf_write/run_counter_collection.csv", "WRITE_SIZE")
res = {}
for k in sorted(set(f) | set(w)):
    res[k] = {"fetch_kib_raw": f.get(k, (None,))[0], "write_kib": w.get(k, (None,))[0], "launches": f.get(k, (0, 0))[1]}
json.dump(res, open("$O/surf_pmc.json", "w"), indent=1)
print(json.dumps(res)[:2500])
PY
