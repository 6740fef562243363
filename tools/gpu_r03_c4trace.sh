# round 3: kernel trace of the config-4 share (8,192 x 30, two launches) and config 2
# (4,096 x 30): scalar step, stream and the gap between them
set -u
export TMPDIR=/tmp
TAG=${1:-r03c4}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k small_n_paths_agree > gpurun_out/smalln_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/smalln_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/smalln_tests_$TAG.log
for B in 8192 4096; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$B -o run --output-format csv -- \
    python3 bench.py --envs-per-gpu $B --steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 0 > gpurun_out/prof_${TAG}_$B.log 2>&1 || exit $?
  python3 tools/trace_gaps.py gpurun_out/prof_${TAG}_$B/run_kernel_trace.csv > gpurun_out/gaps_${TAG}_$B.txt 2>&1 && cat gpurun_out/gaps_${TAG}_$B.txt

done
