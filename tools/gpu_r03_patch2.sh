# round 3: the product stream with the two-level compose against the per-element compose
# (tools build PMENV_FLAT_PERELEM), after the switch
set -u
export TMPDIR=/tmp
TAG=${1:-r03p2}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
R=PMENV_K1=reg
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+$R+PMENV_FLAT_PERELEM=1 \
    --path two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 "${@:5}" \
    > gpurun_out/ab_patch_${TAG}_$1x$2.json 2>> gpurun_out/ab_patch_$TAG.err || { tail -5 gpurun_out/ab_patch_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
ab 6144 30 9 40
ab 8192 30 7 40 --out
ab 8192 500 5 10 --reward diff_sharpe
grep "^#" gpurun_out/ab_patch_$TAG.err
