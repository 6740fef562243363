# §8f kernels: bench_rows under rocprofv3 kernel trace (per-kernel durations)
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rows -o rows --output-format csv -- python3 $R/tools/bench_rows.py --reps 10 --out $R/gpurun_out/rows_prof.json > $R/gpurun_out/rows_prof.log 2>&1 || exit 1
f=$(find $R/gpurun_out/prof_rows -name "*kernel_stats.csv" | head -1)
cp "$f" $R/gpurun_out/rows_kernel_stats.csv
python3 - "$R/gpurun_out/rows_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(__import__("sys").argv[1])))
for r in rows:
    print(f"{float(r['AverageNs'])/1e3:10.2f} us  x{r['Calls']:>5}  {r['Name'][:110]}")
PY
