# config 1's register step: parity of the register / small-window paths, then phase stamps
# and ablations (tools build) beside the product kernel under a kernel trace
set -u
export TMPDIR=/tmp
TAG=${1:-r05s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_dropin.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
    -- python3 tools/small_stamps.py > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || exit $?
grep -v "^[WE]2" gpurun_out/${TAG}_stamps.err | tail -8
cut -c1-160 gpurun_out/${TAG}_prof/run_kernel_stats.csv | head -9
PMENV_GEN_OFF=1 timeout -k 10 400 python tools/ab_gen.py > gpurun_out/${TAG}_gen.json 2> gpurun_out/${TAG}_gen.err || { tail -5 gpurun_out/${TAG}_gen.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_gen.err | cut -c1-300 | tail -16
