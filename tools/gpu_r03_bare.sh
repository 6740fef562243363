# round 3: where the cache-resident in-place stream's time goes (tools build; knobs read at
# create): no compose (timing only, with / without side data), bar rows via LDS, the
# direct-load form without the LDS image
set -u
export TMPDIR=/tmp
TAG=${1:-r03b}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
R=PMENV_K1=reg
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+$R,$AB+$R+PMENV_STREAM_BARE=1,$AB+$R+PMENV_STREAM_BARE=2,$AB+$R+PMENV_FLAT_LSIDE=1,$AB+$R+PMENV_FLAT_DIRECT=1,$AB+$R+PMENV_FLAT_DIRECT=1+PMENV_FLAT_DIRECT_ABL=15 \
    --path two_launch,two_launch,two_launch,two_launch,two_launch,two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_bare_${TAG}_$1x$2.json 2>> gpurun_out/ab_bare_$TAG.err || { tail -5 gpurun_out/ab_bare_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
ab 8192 16 7 40
grep "^#" gpurun_out/ab_bare_$TAG.err
