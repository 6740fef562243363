# Round 5 GPU pass: the -m gpu suite, the relay / GAE A/B against the round-4 library, the
# shape table (any F, one env) and its rocprofv3 kernel trace. Logs under gpurun_out/.
set -u
TAG=${1:-r05}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_r05.py > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err || exit $?
tail -10 gpurun_out/${TAG}_ab.err
timeout -k 10 300 python tools/bench_shapes.py > gpurun_out/${TAG}_shapes.json 2> gpurun_out/${TAG}_shapes.err || exit $?
tail -8 gpurun_out/${TAG}_shapes.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_shapes_prof -o run --output-format csv \
    -- python3 tools/bench_shapes.py config1_1x5x50x5_ip base_1x32x32x8_ip feat8_65536x30x50x8_ip \
    > gpurun_out/${TAG}_shapes_prof.log 2>&1 || exit $?
find gpurun_out/${TAG}_shapes_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-160 {} | head -12
exit $rc
