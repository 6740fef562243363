# env-aligned relay tiles A/B + the register step's config-1 kernel trace
set -u
export TMPDIR=/tmp
TAG=${1:-r05g}
mkdir -p gpurun_out
PMENV_RELAY_ENV=1 timeout -k 10 400 python tools/ab_relay_env.py > gpurun_out/${TAG}_relayenv.json 2> gpurun_out/${TAG}_relayenv.err || exit $?
tail -8 gpurun_out/${TAG}_relayenv.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c1prof -o run --output-format csv \
    -- python3 tools/bench_shapes.py config1_1x5x50x5_ip base_1x32x32x8_ip > gpurun_out/${TAG}_c1prof.log 2>&1 || exit $?
cut -c1-150 gpurun_out/${TAG}_c1prof/run_kernel_stats.csv | head -4
