# round 3: the two-launch step's K1 at N <= 16 in the packed one-asset-per-lane form
# (8 / 16 lanes per env) against the previous build (register form, 32 lanes per env)
set -u
export TMPDIR=/tmp
TAG=${1:-r03k1s}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "small_n_paths_agree or k1_packed_asset_counts or one_and_two_launch_agree or auto_path_rule" \
  > gpurun_out/k1s_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/k1s_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/k1s_tests_$TAG.log
B=tools/libpmenv_base.so; L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps commission
  timeout -k 10 300 python3 tools/ab_libs.py --libs $B,$L,$L --path two_launch,two_launch,flat --envs $1 --assets $2 \
    --rounds $3 --steps $4 --commission $5 > gpurun_out/ab_k1s_${TAG}_$1x$2_c$5.json 2>> gpurun_out/ab_k1s_$TAG.err \
    || { tail -5 gpurun_out/ab_k1s_$TAG.err; exit 1; }
}
ab 16384 8 9 40 0
ab 32768 8 7 30 0
ab 8192 16 9 40 0
ab 16384 16 7 30 0
ab 16384 16 7 30 0.0025
ab 32768 4 7 30 0
ab 65536 1 7 30 0
grep "^#" gpurun_out/ab_k1s_$TAG.err
