# round 3: the in-place stream's workgroup geometry with the two-level compose body, on the
# cache-resident shapes (two launches), against the product (256 x 2)
set -u
export TMPDIR=/tmp
TAG=${1:-r03ipg}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; T=tools/libpmenv_ab.so
G() { echo "$T+PMENV_FLAT_IP_BLOCK=$1+PMENV_FLAT_IP_VEC=$2"; }
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$(G 512 1),$(G 256 1),$(G 1024 1),$(G 512 2),$(G 256 4) \
    --path two_launch --envs $1 --assets $2 --rounds $3 --steps $4 > gpurun_out/ab_ipg_${TAG}_$1x$2.json 2>> gpurun_out/ab_ipg_$TAG.err \
    || { tail -5 gpurun_out/ab_ipg_$TAG.err; exit 1; }
}
ab 8192 30 7 40
ab 4096 30 7 40
ab 16384 16 7 30
grep "^#" gpurun_out/ab_ipg_$TAG.err | cut -c1-140
