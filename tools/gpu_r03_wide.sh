# round 3: the wide one-launch steps (flat tiles, walk) — parity, then A/B against two launches
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_wide_step.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/gpu_tests_wide.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_wide.log; [ $rc -eq 0 ] || exit $rc
NEW=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # tag libs paths envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03wide.err || { tail -5 gpurun_out/ab_r03wide.err; exit 1; }
}
ab wide $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8,$NEW two_launch,flat,flat,walk 8192 500 0 diff_sharpe --rounds 7 --steps 10
ab wide $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8 two_launch,flat,flat 8192 500 0.0025 diff_sharpe --rounds 5 --steps 10
ab widedb $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8 two_launch,flat,flat 8192 500 0 diff_sharpe --rounds 5 --steps 10 --out
ab wide $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8 two_launch,flat,flat 2048 200 0 log_returns --rounds 7 --steps 20
ab wide $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8 two_launch,flat,flat 16384 100 0 log_returns --rounds 5 --steps 10
ab wide $NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x8 two_launch,flat,flat 1024 500 0 log_returns --rounds 7 --steps 20
grep "^#" gpurun_out/ab_r03wide.err
