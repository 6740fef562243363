# round 3: step_split_kernel — parity (flat-step tests over both kernels, the C caller), then
# interleaved A/B against the other step paths on cache-resident and HBM windows
set -u
export TMPDIR=/tmp
TAG=${1:-r03s}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_flat_step.py tests/test_gpu_c_abi.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_split_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_split_$TAG.log; [ $rc -eq 0 ] || exit $rc
L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # tag paths envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$L,$L,$L --path $2 --envs $3 --assets $4 --commission $5 \
    --reward $6 "${@:7}" > gpurun_out/ab_$1_$3x$4_c$5.json 2>> gpurun_out/ab_split_$TAG.err || { tail -5 gpurun_out/ab_split_$TAG.err; exit 1; }
}
ab $TAG two_launch,split,flat,one_launch 4096 30 0 log_returns --rounds 9 --steps 40
ab $TAG two_launch,split,flat,one_launch 8192 30 0 log_returns --rounds 9 --steps 40
ab $TAG two_launch,split,flat,one_launch 8192 30 0.0025 log_returns --rounds 7 --steps 40
ab $TAG two_launch,split,flat,one_launch 2048 30 0 log_returns --rounds 9 --steps 40
ab $TAG two_launch,split,flat,one_launch 16384 30 0 log_returns --rounds 7 --steps 20
ab $TAG two_launch,split,flat,one_launch 65536 30 0 log_returns --rounds 5 --steps 10
ab $TAG two_launch,split,flat,one_launch 8192 8 0 log_returns --rounds 7 --steps 40
ab $TAG two_launch,split,flat,one_launch 4096 64 0 log_returns --rounds 7 --steps 40
grep "^#" gpurun_out/ab_split_$TAG.err
