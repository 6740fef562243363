# round 4: the relay step's scalar waves at issue priority 3 (tools build, PMENV_RELAY_PRIO)
# against the product; then the GPU tests added since r04l (bit fingerprints, GAE shapes)
set -u
export TMPDIR=/tmp
TAG=${1:-r04p}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
for S in 4096x30 8192x30 2048x30 6144x30 8192x30/out; do
  B=${S%%x*}; R=${S#*x}; N=${R%%/*}; O=""; [ "$R" != "$N" ] && O="--out"
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_RELAY_PRIO=1,$L,$AB+PMENV_RELAY_PRIO=1 \
    --path relay,relay,relay,relay --envs $B --assets $N $O --rounds 7 --steps 40 \
    > gpurun_out/ab_prio_${TAG}_${B}_$N.json 2>> gpurun_out/ab_prio_$TAG.err || { tail -5 gpurun_out/ab_prio_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_prio_$TAG.err | cut -c1-120
timeout -k 10 600 python -u -m pytest tests/test_gpu_bits.py tests/test_gpu_trainer.py "tests/test_gpu_parity.py::test_gpu_gae_horizon_split_matches_oracle" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_new_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_new_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_new_$TAG.log
