# round 3: the packed scalar step specialised on commission (no fixed point's registers
# without it) and, at A = 8, its halo copied first (72 / 81 VGPRs instead of 100: 7 / 5
# waves per SIMD instead of 4), against the previous build
set -u
export TMPDIR=/tmp
TAG=${1:-r03k1w}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_wide_step.py \
  -k "k1_packed or wide or small_n or vec" > gpurun_out/k1w_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/k1w_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/k1w_tests_$TAG.log
B=tools/libpmenv_base.so; L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps commission reward
  timeout -k 10 300 python3 tools/ab_libs.py --libs $B,$L,$B,$L --path two_launch,two_launch,two_launch,two_launch --envs $1 --assets $2 \
    --rounds $3 --steps $4 --commission $5 --reward $6 > gpurun_out/ab_k1w_${TAG}_$1x$2_c$5.json 2>> gpurun_out/ab_k1w_$TAG.err \
    || { tail -5 gpurun_out/ab_k1w_$TAG.err; exit 1; }
}
ab 8192 500 5 20 0 diff_sharpe
ab 8192 500 5 20 0.0025 diff_sharpe
ab 8192 256 5 20 0 log_returns
ab 16384 100 5 20 0 log_returns
ab 16384 8 7 30 0 log_returns
grep "^#" gpurun_out/ab_k1w_$TAG.err
