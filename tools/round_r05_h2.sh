# the surface step with its independent loads issued first: host-I/O / surface parity, the
# driver-sequence bench, then a kernel trace of it
set -u
export TMPDIR=/tmp
TAG=${1:-r05h2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "host or surface or dropin or goldens or driver" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python tools/bench_hostio.py > gpurun_out/${TAG}_hostio.json 2> gpurun_out/${TAG}_hostio.err || { tail -5 gpurun_out/${TAG}_hostio.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_hostio.err | cut -c1-420 | tail -2
HOSTIO_T=500 HOSTIO_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 tools/bench_hostio.py > /dev/null 2>&1 || exit $?
grep "surface\|reset" gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-200
