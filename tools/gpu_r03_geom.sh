# round 3: flat-step geometries on cache-resident in-place windows, and commission > 0 on
# the flat step vs two launches across shapes (uniform-wave build)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # tag libs paths envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03geom.err || { tail -5 gpurun_out/ab_r03geom.err; exit 1; }
}
G="$NEW,$NEW,$AB+PMENV_FLAT1_GEOM=128x4,$AB+PMENV_FLAT1_GEOM=256x2,$AB+PMENV_FLAT1_GEOM=256x4,$AB+PMENV_FLAT1_GEOM=128x8"
ab geom $G two_launch,flat,flat,flat,flat,flat 4096 30 0 log_returns --rounds 9
ab geom $G two_launch,flat,flat,flat,flat,flat 8192 30 0 log_returns --rounds 9
ab comm $NEW,$NEW two_launch,flat 16384 30 0.0025 log_returns --rounds 7
ab comm $NEW,$NEW two_launch,flat 65536 30 0.01 log_returns --rounds 5 --steps 20
ab comm $NEW,$NEW two_launch,flat 65536 16 0.0025 log_returns --rounds 5 --steps 20
ab comm $NEW,$NEW two_launch,flat 32768 64 0.0025 sharpe_ratio --rounds 5 --steps 20
ab comm $NEW,$NEW two_launch,flat 65536 30 0.0025 diff_sharpe --rounds 5 --steps 20
ab comm $NEW,$NEW,$NEW two_launch,flat,one_launch 8192 30 0.0025 log_returns --rounds 7
grep "^#" gpurun_out/ab_r03geom.err
