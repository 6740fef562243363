# round 3: uniform wave index in the flat steps (no waterfall loops around the scalar
# step's buffer loads) — A/B against the previous build at the in-place shares
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
PREV=tools/libpmenv_prev.so; NEW=pm-rl_amd/pmenv/libpmenv.so
ab() {  # tag libs paths envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03rfl.err || { tail -5 gpurun_out/ab_r03rfl.err; exit 1; }
}
ab rfl $PREV,$NEW,$PREV,$NEW,$NEW flat,flat,two_launch,two_launch,one_launch 4096 30 0 log_returns --rounds 9
ab rfl $PREV,$NEW,$PREV,$NEW,$NEW flat,flat,two_launch,two_launch,one_launch 8192 30 0 log_returns --rounds 9
ab rfl $PREV,$NEW,$NEW flat,flat,two_launch 16384 30 0 log_returns --rounds 7
ab rfl $PREV,$NEW flat,flat 65536 30 0 log_returns --rounds 9 --steps 20
ab rfl $PREV,$NEW,$NEW flat,flat,two_launch 65536 30 0.0025 log_returns --rounds 7 --steps 20
ab rfl $PREV,$NEW,$NEW flat,flat,two_launch 8192 500 0 diff_sharpe --rounds 5 --steps 10
grep "^#" gpurun_out/ab_r03rfl.err
