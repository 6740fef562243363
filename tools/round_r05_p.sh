# the generic stream at F = 3 / 8 (65,536 x 30 x 50): kernel trace and HBM traffic per kernel
set -u
export TMPDIR=/tmp
TAG=${1:-r05p}
mkdir -p gpurun_out
S="feat3_65536x30x50x3_ip feat8_65536x30x50x8_ip"
SHAPES_K=50 SHAPES_R=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
    -- python3 tools/bench_shapes.py $S > gpurun_out/${TAG}_shapes.json 2> gpurun_out/${TAG}_shapes.err || exit $?
grep -v "^[WE]2" gpurun_out/${TAG}_shapes.err | cut -c1-220 | tail -3
grep "advance_gen\|scalar_step" gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-170
SHAPES_K=5 SHAPES_R=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 tools/bench_shapes.py $S > gpurun_out/${TAG}_fetch.log 2>&1 || exit $?
SHAPES_K=5 SHAPES_R=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- python3 tools/bench_shapes.py $S > gpurun_out/${TAG}_write.log 2>&1 || exit $?
ls gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
