# host-I/O per-step time (tools/bench_hostio.py) and the host-tensor tests
set -u
export TMPDIR=/tmp
TAG=${1:-r05h}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "host or dropin" -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/bench_hostio.py > gpurun_out/${TAG}_hostio.json 2> gpurun_out/${TAG}_hostio.err || exit $?
tail -2 gpurun_out/${TAG}_hostio.err
exit $rc
