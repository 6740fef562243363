# the tiny register step: parity (register / generic / golden tests), then its A/B against
# step_small_kernel under a kernel trace, and the generic stream's shapes again
set -u
export TMPDIR=/tmp
TAG=${1:-r05u}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_dropin.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
PMENV_TINY_OFF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
    -- python3 tools/ab_tiny.py > gpurun_out/${TAG}_tiny.json 2> gpurun_out/${TAG}_tiny.err || { tail -5 gpurun_out/${TAG}_tiny.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_tiny.err | cut -c1-250 | tail -8
grep "step_tiny\|step_small" gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-160
