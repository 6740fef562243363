# round 4: where the relay tiles' extra time goes: only the staging threads issue the side loads
# (PMENV_RELAY_PRIO=5, the same results), no halo_out stores (6, timing only), both (7)
set -u
export TMPDIR=/tmp
TAG=${1:-r04u}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
for B in 8192 4096; do
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_RELAY_PRIO=5,$AB+PMENV_RELAY_PRIO=6,$AB+PMENV_RELAY_PRIO=7,$L \
    --path relay,relay,relay,relay,two_launch --envs $B --assets 30 --rounds 7 --steps 40 \
    > gpurun_out/ab_rabl_${TAG}_$B.json 2>> gpurun_out/ab_rabl_$TAG.err || { tail -5 gpurun_out/ab_rabl_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_rabl_$TAG.err | cut -c1-150
