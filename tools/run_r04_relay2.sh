# round 4: the relay tiles' side loads by the staging threads only and one halo entry per 128-B
# line (the product) against the library before them (tools/libpmenv_r04l.so, rebuilt from the
# previous commit), then the relay GPU tests on the product
set -u
export TMPDIR=/tmp
TAG=${1:-r04v}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; O=tools/libpmenv_r04l.so
for S in 8192x30 4096x30 6144x30 2048x30 8192x16 16384x8 2048x64 4096x30/out; do
  B=${S%%x*}; R=${S#*x}; N=${R%%/*}; X=""; [ "$R" != "$N" ] && X="--out"
  timeout -k 10 300 python3 tools/ab_libs.py --libs $O,$L,$O,$L --path relay,relay,relay,relay --envs $B --assets $N $X \
    --rounds 7 --steps 40 > gpurun_out/ab_relay2_${TAG}_${B}_$N.json 2>> gpurun_out/ab_relay2_$TAG.err || { tail -5 gpurun_out/ab_relay2_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_relay2_$TAG.err | cut -c1-140
timeout -k 10 600 python -u -m pytest tests/test_gpu_relay.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_relay_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_relay_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_relay_$TAG.log
