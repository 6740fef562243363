# round 3: where step_split_kernel's time goes (tools build: interleave R, timing-only ablations)
set -u
export TMPDIR=/tmp
TAG=${1:-r03t}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB,$AB+PMENV_SPLIT_R=1,$AB+PMENV_SPLIT_ABL=1,$AB+PMENV_SPLIT_ABL=2,$AB+PMENV_SPLIT_ABL=4,$AB+PMENV_SPLIT_ABL=5,$AB+PMENV_SPLIT_R=64,$AB+PMENV_SPLIT_R=4 \
    --path two_launch,split,split,split,split,split,split,split,split --envs $1 --assets 30 --rounds $2 --steps $3 \
    > gpurun_out/ab_splitab_${TAG}_$1.json 2>> gpurun_out/ab_splitab_$TAG.err || { tail -5 gpurun_out/ab_splitab_$TAG.err; exit 1; }
}
ab 8192 7 40
ab 4096 7 40
ab 65536 3 10
grep "^#" gpurun_out/ab_splitab_$TAG.err
