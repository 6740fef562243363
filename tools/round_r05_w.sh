# the generic stream's two-level compose: parity, then A/B against its per-element form and the
# register step, with a kernel trace of the former
set -u
export TMPDIR=/tmp
TAG=${1:-r05w}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "generic or goldens or register" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
PMENV_GEN_PERELEM=1 AB_R=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
    -- python3 tools/ab_gen.py > gpurun_out/${TAG}_perelem.json 2> gpurun_out/${TAG}_perelem.err || { tail -5 gpurun_out/${TAG}_perelem.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_perelem.err | cut -c1-200 | tail -14
grep "advance_gen\|scalar_step" gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-180
PMENV_GEN_OFF=1 timeout -k 10 400 python tools/ab_gen.py > gpurun_out/${TAG}_gen.json 2> gpurun_out/${TAG}_gen.err || { tail -5 gpurun_out/${TAG}_gen.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_gen.err | cut -c1-200 | tail -15
