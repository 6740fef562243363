# round 4: kernel durations of the relayed step against the two-launch path's stream and scalar
# kernels at the cache-resident shapes (rocprofv3 kernel trace of one ab_libs process)
set -u
export TMPDIR=/tmp
TAG=${1:-r04t}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so
for B in 8192 4096; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rtr_${TAG}_$B -o run --output-format csv -- \
  python3 tools/ab_libs.py --libs $L,$L --path relay,two_launch --envs $B --assets 30 --rounds 3 --steps 40 \
  > gpurun_out/rtr_${TAG}_$B.log 2>&1 || { tail -5 gpurun_out/rtr_${TAG}_$B.log; exit 1; }
grep -E "step_relay|advance_flat|scalar_step" gpurun_out/rtr_${TAG}_$B/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-150
done
