# round 3: the two-level compose of the flat stream (tools build, PMENV_FLAT_PATCH) against
# the product's per-element compose: bits and time, in place and double-buffered
set -u
export TMPDIR=/tmp
TAG=${1:-r03p}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
R=PMENV_K1=reg
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+$R,$AB+$R+PMENV_FLAT_PATCH=1 \
    --path two_launch,two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 "${@:5}" \
    > gpurun_out/ab_patch_${TAG}_$1x$2.json 2>> gpurun_out/ab_patch_$TAG.err || { tail -5 gpurun_out/ab_patch_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
ab 8192 16 9 40
ab 16384 8 9 40
ab 4096 48 9 40
ab 65536 30 3 10
ab 8192 30 7 40 --out
ab 65536 30 3 10 --out
ab 8192 30 7 40 --commission 0.0025 --reward sharpe_ratio
ab 3000 7 7 40
grep "^#" gpurun_out/ab_patch_$TAG.err
