# round 3: the cache-resident two-launch step's scalar kernel: env groups per wave (P) of
# the register form, and the packed 16 x 2 form (another reduction order), against the product
set -u
export TMPDIR=/tmp
TAG=${1:-r03k1g}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; T=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$T+PMENV_K1=reg,$T+PMENV_K1=reg+PMENV_K1_GROUPS=2,$T+PMENV_K1=reg+PMENV_K1_GROUPS=4,$T+PMENV_K1=16x2,$T+PMENV_K1=16x2s \
    --path two_launch --envs $1 --assets $2 --rounds $3 --steps $4 > gpurun_out/ab_k1g_${TAG}_$1x$2.json 2>> gpurun_out/ab_k1g_$TAG.err \
    || { tail -5 gpurun_out/ab_k1g_$TAG.err; exit 1; }
}
ab 8192 30 7 40
ab 4096 30 7 40
grep "^#" gpurun_out/ab_k1g_$TAG.err | cut -c1-150
