# round 3: kernel trace of the config-4 share (8,192 x 30, two launches) and config 2
# (4,096 x 30): scalar step, stream and the gap between them
set -u
export TMPDIR=/tmp
TAG=${1:-r03c4}
mkdir -p gpurun_out
for B in 8192 4096; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$B -o run --output-format csv -- \
    python3 bench.py --envs-per-gpu $B --steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 0 > gpurun_out/prof_${TAG}_$B.log 2>&1 || exit $?
  python3 tools/trace_gaps.py gpurun_out/prof_${TAG}_$B/run_kernel_trace.csv > gpurun_out/gaps_${TAG}_$B.txt 2>&1 && cat gpurun_out/gaps_${TAG}_$B.txt

done
