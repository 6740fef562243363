# round 3: row_bcast:15 group sums (same bits) — GPU suite, then A/B against the previous build
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03i || exit $?
PREV=tools/libpmenv_prev.so; NEW=pm-rl_amd/pmenv/libpmenv.so
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03bc.err || { tail -5 gpurun_out/ab_r03bc.err; exit 1; }
}
ab bc $PREV,$NEW,$PREV,$NEW,$NEW flat,flat,two_launch,two_launch,one_launch 4096 30 0 log_returns --rounds 9
ab bc $PREV,$NEW,$PREV,$NEW,$NEW flat,flat,two_launch,two_launch,one_launch 8192 30 0 log_returns --rounds 9
ab bc $PREV,$NEW flat,flat 65536 30 0 log_returns --rounds 9 --steps 20
ab bc $PREV,$NEW flat,flat 65536 30 0.0025 log_returns --rounds 7 --steps 20
grep "^#" gpurun_out/ab_r03bc.err
