# f1 GAE: the tiled scan (product), its 64-VGPR form and the pipelined per-env walk,
# event-timed (bench_rows --only f1) and under a rocprofv3 kernel trace
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/bench_rows.py --only f1 --reps 7 --out $R/gpurun_out/gae_rows.json > $R/gpurun_out/gae_rows.log 2>&1 || { tail -20 $R/gpurun_out/gae_rows.log; exit 1; }
grep '"case": "gae' $R/gpurun_out/gae_rows.log | cut -c1-260
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gae -o gae --output-format csv -- python3 $R/tools/bench_rows.py --only f1 --reps 2 > $R/gpurun_out/gae_prof.log 2>&1 || exit 1
t=$(find $R/gpurun_out/prof_gae -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py "$t" > $R/gpurun_out/gae_kernel_by_grid.txt
grep gae $R/gpurun_out/gae_kernel_by_grid.txt
