# round 4: what the relayed step's wait costs: the product against a timing-only ablation whose
# scalar blocks exit at once and whose tiles do not wait (PMENV_RELAY_PRIO=2, wrong results)
set -u
export TMPDIR=/tmp
TAG=${1:-r04s}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
for B in 4096 8192; do
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_RELAY_PRIO=2,$L --path relay,relay,two_launch \
    --envs $B --assets 30 --rounds 7 --steps 40 > gpurun_out/ab_nowait_${TAG}_$B.json 2>> gpurun_out/ab_nowait_$TAG.err || { tail -5 gpurun_out/ab_nowait_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_nowait_$TAG.err | cut -c1-150
