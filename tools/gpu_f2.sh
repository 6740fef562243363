# f2 batched reward: GPU tests, then the one- vs two-launch forward A/B (event-timed) and
# the same run under a rocprofv3 kernel trace
set -u
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/f2_tests.log 2>&1 || { tail -30 gpurun_out/f2_tests.log; exit 1; }
tail -2 gpurun_out/f2_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/bench_rows.py --only f2 --reps 7 --out $R/gpurun_out/f2_rows.json > $R/gpurun_out/f2_rows.log 2>&1 || exit 1
grep case $R/gpurun_out/f2_rows.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f2 -o f2 --output-format csv -- python3 $R/tools/bench_rows.py --only f2 --reps 2 > $R/gpurun_out/f2_prof.log 2>&1 || exit 1
t=$(find $R/gpurun_out/prof_f2 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py "$t" > $R/gpurun_out/f2_kernel_by_grid.txt
grep batch_reward $R/gpurun_out/f2_kernel_by_grid.txt
