# rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -u
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 50 --warmup 5 --cpu-baseline 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/pmc_write_$TAG.log 2>&1 || exit $?
find gpurun_out/prof_$TAG gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG -name '*.csv' | head -20
