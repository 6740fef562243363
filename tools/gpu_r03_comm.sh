# round 3: the active-set commission fixed point — GPU suite, then A/B against the previous build
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03f || exit $?
PREV=tools/libpmenv_prev.so; NEW=pm-rl_amd/pmenv/libpmenv.so
ab() {  # tag libs paths envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03comm.err || { tail -5 gpurun_out/ab_r03comm.err; exit 1; }
}
ab comm2 $PREV,$PREV,$NEW,$NEW,$NEW two_launch,flat,two_launch,flat,auto 65536 30 0.0025 log_returns --rounds 7 --steps 20
ab comm2 $PREV,$NEW,$NEW two_launch,two_launch,flat 65536 30 0.01 log_returns --rounds 5 --steps 20
ab comm2 $PREV,$NEW,$NEW two_launch,two_launch,flat 65536 16 0.0025 log_returns --rounds 5 --steps 20
ab comm2 $PREV,$NEW,$NEW two_launch,two_launch,flat 16384 30 0.0025 log_returns --rounds 7
ab comm2 $PREV,$NEW,$NEW,$NEW two_launch,two_launch,flat,one_launch 8192 30 0.0025 log_returns --rounds 7
ab comm2 $PREV,$NEW,$NEW two_launch,two_launch,flat 8192 500 0.0025 diff_sharpe --rounds 5 --steps 10
grep "^#" gpurun_out/ab_r03comm.err
