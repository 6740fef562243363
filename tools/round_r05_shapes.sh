# The shape table (any F, one env; tools/bench_shapes.py) on the product library, the
# register step's one-wave geometry through the tools build, and kernel traces of both.
set -u
export TMPDIR=/tmp
TAG=${1:-r05}
timeout -k 10 300 python tools/bench_shapes.py > gpurun_out/${TAG}_shapes.json 2> gpurun_out/${TAG}_shapes.err || exit $?
tail -8 gpurun_out/${TAG}_shapes.err
PMENV_LIB=tools/libpmenv_ab.so PMENV_SMALL_GEOM=64x32 timeout -k 10 300 python tools/bench_shapes.py config1_1x5x50x5_ip \
    config1_1x5x50x5_db > gpurun_out/${TAG}_shapes_64x32.json 2> gpurun_out/${TAG}_shapes_64x32.err || exit $?
tail -2 gpurun_out/${TAG}_shapes_64x32.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_shapes_prof -o run --output-format csv \
    -- python3 tools/bench_shapes.py config1_1x5x50x5_ip base_1x32x32x8_ip feat8_65536x30x50x8_ip \
    > gpurun_out/${TAG}_shapes_prof.log 2>&1 || exit $?
cut -c1-150 gpurun_out/${TAG}_shapes_prof/run_kernel_stats.csv | head -5
# the cache-resident shares' copy floor: membench's read+write copies / in-place shifts of the
# same bytes as a 4,096 / 8,192 x 30 x 50 x 5 window
timeout -k 10 120 tools/membench 4096 > gpurun_out/${TAG}_membench_4096.txt 2>&1 || exit $?
timeout -k 10 120 tools/membench 8192 > gpurun_out/${TAG}_membench_8192.txt 2>&1 || exit $?
grep -E "copy chunk U8 |inplace env 256x8 shift5|inplace env 512x4 shift5|hipMemcpy" gpurun_out/${TAG}_membench_4096.txt gpurun_out/${TAG}_membench_8192.txt
