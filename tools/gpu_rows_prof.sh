# §8f kernels: bench_rows (event-timed, back-to-back calls) and the same run under a
# rocprofv3 kernel trace (per-kernel, per-shape durations: tools/trace_by_grid.py)
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/bench_rows.py --reps 5 --out $R/gpurun_out/rows.json > $R/gpurun_out/rows.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rows -o rows --output-format csv -- python3 $R/tools/bench_rows.py --reps 2 --out $R/gpurun_out/rows_prof.json > $R/gpurun_out/rows_prof.log 2>&1 || exit 1
f=$(find $R/gpurun_out/prof_rows -name "*kernel_stats.csv" | head -1)
cp "$f" $R/gpurun_out/rows_kernel_stats.csv
t=$(find $R/gpurun_out/prof_rows -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py "$t" > $R/gpurun_out/rows_kernel_by_grid.txt
cat $R/gpurun_out/rows_kernel_by_grid.txt
