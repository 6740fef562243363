# per-kernel times of the step paths with and without commission (one rocprofv3 run each)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in two_launch:0 two_launch:0.0025 flat:0 flat:0.0025 one_launch:0 one_launch:0.0025; do
  tag=$(echo $cfg | tr ':.' '__')
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/pc_$tag -o run --output-format csv -- python3 tools/prof_paths.py --configs $cfg --envs ${ENVS:-65536} > gpurun_out/pc_$tag.log 2>&1 || exit $?
  f=$(ls gpurun_out/pc_$tag/run_kernel_trace.csv 2>/dev/null || find gpurun_out/pc_$tag -name '*kernel_trace.csv' | head -1)
  echo "== $cfg"; python3 tools/trace_by_grid.py $f scalar_step advance_ step_flat step_env flat_prime
done
PREV=tools/libpmenv_prev.so; NEW=pm-rl_amd/pmenv/libpmenv.so
timeout -k 10 300 python3 tools/ab_libs.py --libs $PREV,$PREV,$NEW,$NEW,$NEW --path two_launch,flat,two_launch,flat,one_launch \
  --envs 65536 --assets 30 --commission 0.0025 --rounds 7 --steps 20 > gpurun_out/ab_comm3.json 2> gpurun_out/ab_comm3.err || exit 1
timeout -k 10 300 python3 tools/ab_libs.py --libs $NEW,$NEW,$NEW --path two_launch,flat,one_launch \
  --envs 8192 --assets 30 --commission 0.0025 --rounds 7 > gpurun_out/ab_comm3s.json 2>> gpurun_out/ab_comm3.err || exit 1
grep "^#" gpurun_out/ab_comm3.err
