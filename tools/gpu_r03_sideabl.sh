# round 3: which side datum costs the cache-resident in-place stream (timing-only SKIP bits:
# 1 bar, 2 w', 4 counter, 15 all), the scalar kernel's halo copy kept
set -u
export TMPDIR=/tmp
TAG=${1:-r03sa}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_K1=reg,$AB+PMENV_K1=reg+PMENV_ABLATE=65,$AB+PMENV_K1=reg+PMENV_ABLATE=66,$AB+PMENV_K1=reg+PMENV_ABLATE=68,$AB+PMENV_K1=reg+PMENV_ABLATE=79 \
    --path two_launch,two_launch,two_launch,two_launch,two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_sideabl_${TAG}_$1x$2.json 2>> gpurun_out/ab_sideabl_$TAG.err || { tail -5 gpurun_out/ab_sideabl_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
grep "^#" gpurun_out/ab_sideabl_$TAG.err
