# round 4: config 5's scalar step (scalar_step_vec_kernel<64, 8, strided>, 102 VGPRs, 4 waves
# per SIMD) held to 6 / 8 waves per SIMD (tools build, PMENV_K1_OCC), two launches; the
# wrapper's host cost per step (tools/bench_wrapper.py)
set -u
export TMPDIR=/tmp
TAG=${1:-r04k}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_K1_OCC=6,$AB+PMENV_K1_OCC=8 \
  --path two_launch,two_launch,two_launch --envs 8192 --assets 500 --rounds 5 --steps 6 --reward diff_sharpe \
  > gpurun_out/ab_k1occ_$TAG.json 2> gpurun_out/ab_k1occ_$TAG.err || { tail -5 gpurun_out/ab_k1occ_$TAG.err; exit 1; }
grep "^#" gpurun_out/ab_k1occ_$TAG.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k1occ_$TAG -o run --output-format csv -- \
  python3 tools/ab_libs.py --libs $L,$AB+PMENV_K1_OCC=8 --path two_launch,two_launch --envs 8192 --assets 500 \
  --rounds 3 --steps 6 --reward diff_sharpe > gpurun_out/prof_k1occ_$TAG.log 2>&1 || exit $?
grep -E "scalar_step_vec" gpurun_out/prof_k1occ_$TAG/run_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python3 tools/bench_wrapper.py > gpurun_out/wrapper_$TAG.json 2> gpurun_out/wrapper_$TAG.err || exit $?
cat gpurun_out/wrapper_$TAG.err | grep -v amdgpu.ids
