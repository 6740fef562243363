# round 3: cache-resident in-place windows — the one-WG-per-env step with fewer chunks per lane
# (more waves) and the in-place stream with other workgroup shapes, against the product
set -u
export TMPDIR=/tmp
TAG=${1:-r03r}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$L,$AB+PMENV_ONE_V=2,$AB+PMENV_ONE_V=3,$AB+PMENV_FLAT_IP_BLOCK=1024+PMENV_FLAT_IP_VEC=1,$AB+PMENV_FLAT_IP_BLOCK=512+PMENV_FLAT_IP_VEC=1,$AB+PMENV_FLAT_IP_BLOCK=256+PMENV_FLAT_IP_VEC=1 \
    --path two_launch,one_launch,one_launch,one_launch,two_launch,two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_res_${TAG}_$1x$2.json 2>> gpurun_out/ab_res_$TAG.err || { tail -5 gpurun_out/ab_res_$TAG.err; exit 1; }
}
ab 8192 30 7 40
ab 4096 30 7 40
ab 2048 30 7 40
ab 16384 30 5 20
grep "^#" gpurun_out/ab_res_$TAG.err
timeout -k 10 120 ./tools/membench 8192 > gpurun_out/membench_8192_$TAG.log 2>&1 || exit $?
timeout -k 10 120 ./tools/membench 4096 > gpurun_out/membench_4096_$TAG.log 2>&1 || exit $?
grep -E "inplace env|inplace unit  500|D2D" gpurun_out/membench_8192_$TAG.log
