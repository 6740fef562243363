# Round 5's GPU measurements, one subcommand per record under profiles/ (logs and JSON go to
# gpurun_out/<TAG>_*; copy the ones kept into profiles/). Each step runs under its own time
# limit and the script stops at the first failure.
#
#   bash tools/round_r05_ab.sh relay_gae TAG   # relay / look-back GAE / graph A/B vs round 4 (ab_r05/relay_gae_*)
#   bash tools/round_r05_ab.sh shapes TAG      # the any-F / one-env shape table, a kernel trace, membench floors
#   bash tools/round_r05_ab.sh relay_env TAG   # env-aligned relay tiles (tools build) vs the product's
#   bash tools/round_r05_ab.sh hostio TAG      # host-tensor tests, the driver-sequence bench and its kernel trace
#   bash tools/round_r05_ab.sh stamps TAG      # the register step's wall-clock stamps and ablations (config 1)
#   bash tools/round_r05_ab.sh tiny TAG        # step_tiny_kernel vs step_small_kernel under a kernel trace
#   bash tools/round_r05_ab.sh gen TAG         # the generic F != 5 stream vs the register step / LDS fallback
#   bash tools/round_r05_ab.sh gen_geom TAG    # its tile geometries (256 x 4 / 256 x 2 / 512 x 2) and cache policy
#   bash tools/round_r05_ab.sh gen_prof TAG    # its kernel trace and FETCH_SIZE / WRITE_SIZE at F = 3 / 8
#   bash tools/round_r05_ab.sh gen_few TAG     # the generic stream vs the register step around AUTO's threshold
#   bash tools/round_r05_ab.sh gen_abl TAG     # its timing-only ablations (no side data / compose / shifted read)
#   bash tools/round_r05_ab.sh surface TAG     # the surface contract: the two-launch surface stream vs the per-env kernel
#   bash tools/round_r05_ab.sh surface_prev TAG  # the surface contract against another product build (SURF_PREV)
set -u
export TMPDIR=/tmp
CMD=${1:?subcommand}
TAG=${2:-r05}
mkdir -p gpurun_out
O=gpurun_out/${TAG}

summ() {   # one line per shape of an ab_gen / ab_tiny run: the product, the other leg, bits
    grep -v "^[WE]2" "$1" | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: o = json.loads(j)
    except Exception: continue
    legs = [n for n in o if isinstance(o[n], dict)]
    print(k, *[f\"{n} {o[n]['us']:.1f}\" for n in legs], 'windows', o.get('windows_equal'), 'rewards', o.get('rewards_equal'))
"
}
tests() {
    timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
        "$@" > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
    tail -1 ${O}_tests.log
}

case "$CMD" in
relay_gae)
    timeout -k 10 300 python tools/ab_r05.py > ${O}_ab.json 2> ${O}_ab.err || exit $?
    tail -10 ${O}_ab.err ;;
shapes)
    timeout -k 10 300 python tools/bench_shapes.py > ${O}_shapes.json 2> ${O}_shapes.err || exit $?
    tail -8 ${O}_shapes.err
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_shapes_prof -o run --output-format csv \
        -- python3 tools/bench_shapes.py config1_1x5x50x5_ip base_1x32x32x8_ip feat8_65536x30x50x8_ip \
        > ${O}_shapes_prof.log 2>&1 || exit $?
    cut -c1-150 ${O}_shapes_prof/run_kernel_stats.csv | head -5
    # the cache-resident shares' copy floor: read+write copies / in-place shifts of the same
    # bytes as a 4,096 / 8,192 x 30 x 50 x 5 window
    timeout -k 10 120 tools/membench 4096 > ${O}_membench_4096.txt 2>&1 || exit $?
    timeout -k 10 120 tools/membench 8192 > ${O}_membench_8192.txt 2>&1 || exit $? ;;
relay_env)
    PMENV_RELAY_ENV=1 timeout -k 10 400 python tools/ab_relay_env.py > ${O}_relayenv.json 2> ${O}_relayenv.err || exit $?
    tail -8 ${O}_relayenv.err ;;
hostio)
    tests tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "host or surface or dropin or goldens or driver"
    timeout -k 10 300 python tools/bench_hostio.py > ${O}_hostio.json 2> ${O}_hostio.err || exit $?
    grep -v "^[WE]2" ${O}_hostio.err | cut -c1-420 | tail -2
    HOSTIO_T=500 HOSTIO_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_hostio_prof -o run \
        --output-format csv -- python3 tools/bench_hostio.py > /dev/null 2>&1 || exit $?
    grep "surface\|reset" ${O}_hostio_prof/run_kernel_stats.csv | cut -c1-200 ;;
stamps)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_stamps_prof -o run --output-format csv \
        -- python3 tools/small_stamps.py > ${O}_stamps.json 2> ${O}_stamps.err || exit $?
    grep -v "^[WE]2" ${O}_stamps.err | tail -8
    cut -c1-160 ${O}_stamps_prof/run_kernel_stats.csv | head -9 ;;
tiny)
    tests tests/test_gpu_parity.py -k "register or any_F or goldens"
    PMENV_TINY_OFF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_tiny_prof -o run --output-format csv \
        -- python3 tools/ab_tiny.py > ${O}_tiny.json 2> ${O}_tiny.err || { tail -5 ${O}_tiny.err; exit 1; }
    summ ${O}_tiny.err
    grep "step_tiny\|step_small" ${O}_tiny_prof/run_kernel_stats.csv | cut -c1-160 ;;
gen)
    tests tests/test_gpu_parity.py -k "generic or goldens or register or any_F"
    PMENV_GEN_OFF=1 timeout -k 10 400 python tools/ab_gen.py > ${O}_gen.json 2> ${O}_gen.err || { tail -5 ${O}_gen.err; exit 1; }
    summ ${O}_gen.err
    AB_GEN_SHAPES=wide PMENV_GEN_OFF=1 timeout -k 10 300 python tools/ab_gen.py > ${O}_gen_wide.json 2> ${O}_gen_wide.err || exit $?
    summ ${O}_gen_wide.err ;;
gen_geom)
    for g in ${GEOMS:-256x4 256x2 512x2}; do
        PMENV_GEN_GEOM=$g AB_GEN_FORCE=1 AB_R=3 timeout -k 10 300 python tools/ab_gen.py > ${O}_geom_$g.json \
            2> ${O}_geom_$g.err || exit $?
        echo "tools leg at $g:"; summ ${O}_geom_$g.err
    done
    PMENV_GEN_POL0=1 AB_R=3 timeout -k 10 300 python tools/ab_gen.py > ${O}_pol.json 2> ${O}_pol.err || exit $?
    echo "tools leg with the default cache policy:"; summ ${O}_pol.err ;;
gen_abl)    # timing-only ablations of the generic stream at 65,536 x 30 x 50 x {3, 4, 8} in place
    for a in 1 2 3 6 7; do
        PMENV_GEN_ABL=$a AB_GEN_SHAPES=big AB_R=3 timeout -k 10 300 python tools/ab_gen.py > ${O}_abl$a.json \
            2> ${O}_abl$a.err || exit $?
        echo "ablation $a:"; summ ${O}_abl$a.err
    done ;;
gen_few)    # the generic stream against the register step around AUTO's threshold
    AB_GEN_SHAPES=few PMENV_GEN_OFF=1 timeout -k 10 300 python tools/ab_gen.py > ${O}_few.json 2> ${O}_few.err || exit $?
    summ ${O}_few.err ;;
gen_prof)
    S="feat3_65536x30x50x3_ip feat8_65536x30x50x8_ip"
    SHAPES_K=50 SHAPES_R=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_gen_prof -o run --output-format csv \
        -- python3 tools/bench_shapes.py $S > ${O}_gen_shapes.json 2> ${O}_gen_shapes.err || exit $?
    grep "advance_gen\|scalar_step" ${O}_gen_prof/run_kernel_stats.csv | cut -c1-170
    SHAPES_K=5 SHAPES_R=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d ${O}_gen_fetch -o run --output-format csv \
        -- python3 tools/bench_shapes.py $S > ${O}_gen_fetch.log 2>&1 || exit $?
    SHAPES_K=5 SHAPES_R=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d ${O}_gen_write -o run --output-format csv \
        -- python3 tools/bench_shapes.py $S > ${O}_gen_write.log 2>&1 || exit $? ;;
surface)
    tests tests/test_gpu_parity.py -k "surface or goldens"
    # the tools leg on the per-env kernel (dword channel writes)
    SURF_LIBS=pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_ab.so PMENV_SURF_STREAM=0 timeout -k 10 300 \
        python tools/bench_surface.py > ${O}_surf.json 2> ${O}_surf.err || exit $?
    grep -v "^[WE]2" ${O}_surf.err | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: o = json.loads(j)
    except Exception: continue
    legs = [n for n in o if isinstance(o[n], dict)]
    print(k, *[f\"{o[n]['us_per_step']:.1f}\" for n in legs], 'windows', o.get('windows_equal'), 'rewards', o.get('rewards_equal'))
" ;;
surface_prof)   # the surface stream's kernel trace and FETCH_SIZE / WRITE_SIZE at 65,536 x 30 x 50 x 5
    export SURF_SHAPES=65536x30x50x5
    SURF_K=20 SURF_R=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_surf_prof -o run --output-format csv \
        -- python3 tools/bench_surface.py > ${O}_surf_prof.log 2>&1 || exit $?
    grep "surface\|scalar_step" ${O}_surf_prof/run_kernel_stats.csv | cut -c1-170
    SURF_K=5 SURF_R=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d ${O}_surf_fetch -o run --output-format csv \
        -- python3 tools/bench_surface.py > ${O}_surf_fetch.log 2>&1 || exit $?
    SURF_K=5 SURF_R=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d ${O}_surf_write -o run --output-format csv \
        -- python3 tools/bench_surface.py > ${O}_surf_write.log 2>&1 || exit $? ;;
surface_prev)   # the surface contract against another product build (SURF_PREV, e.g. the last commit's)
    tests tests/test_gpu_parity.py -k "surface or goldens"
    SURF_LIBS=pm-rl_amd/pmenv/libpmenv.so,${SURF_PREV:-tools/libpmenv_prev.so} timeout -k 10 300 \
        python tools/bench_surface.py > ${O}_surf.json 2> ${O}_surf.err || exit $?
    grep -v "^[WE]2" ${O}_surf.err | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: o = json.loads(j)
    except Exception: continue
    legs = [n for n in o if isinstance(o[n], dict)]
    print(k, *[f\"{o[n]['us_per_step']:.1f}\" for n in legs], 'windows', o.get('windows_equal'), 'rewards', o.get('rewards_equal'))
" ;;
*)
    echo "unknown subcommand $CMD"; exit 2 ;;
esac
