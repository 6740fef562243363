# bench (default and the driver's short form) + rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes on the current tree; summarise here with: python tools/pmc_summary.py TAG
set -u
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
tail -c 600 gpurun_out/bench_$TAG.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_short_$TAG.json 2> gpurun_out/bench_short_$TAG.err || exit $?
ARGS="--steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 50"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --alt-steps 0 > gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --alt-steps 0 > gpurun_out/pmc_write_$TAG.log 2>&1 || exit $?
grep -E "step_env|step_flat|flat_prime|advance_|scalar_step" gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-170
