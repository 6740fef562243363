# round 4: the relay step back to one store phase (counter from the parity copy, w' relayed),
# lead sweep at the cache-resident shapes, config 5 with the 8-wave form
set -u
export TMPDIR=/tmp
TAG=${1:-r04t}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relay.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_relay_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_relay_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_relay_$TAG.log
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps libs paths [extra]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $5 --path $6 --envs $1 --assets $2 --rounds $3 --steps $4 ${7:-} \
    > gpurun_out/ab_relay3_${TAG}_$1x$2.json 2>> gpurun_out/ab_relay3_$TAG.err || { tail -5 gpurun_out/ab_relay3_$TAG.err; exit 1; }
}
ab 4096 30 7 40 $L,$AB+PMENV_RELAY_LEAD=8192,$AB+PMENV_RELAY_LEAD=1000000000 two_launch,relay,relay
ab 8192 30 7 40 $L,$AB+PMENV_RELAY_LEAD=16384,$AB+PMENV_RELAY_LEAD=1000000000 two_launch,relay,relay
ab 6144 30 5 40 $L,$AB+PMENV_RELAY_LEAD=16384,$AB+PMENV_RELAY_LEAD=1000000000 two_launch,relay,relay
ab 8192 16 5 40 $L,$AB+PMENV_RELAY_LEAD=16384,$AB+PMENV_RELAY_LEAD=1000000000 two_launch,relay,relay
ab 65536 30 3 10 $L,$AB+PMENV_RELAY_LEAD=4096,$L flat,relay,two_launch
ab 8192 500 3 6 $L,$AB+PMENV_RELAY_LEAD=8192,$AB+PMENV_RELAY_LEAD=1000000000 two_launch,relay,relay "--reward diff_sharpe"
grep "^#" gpurun_out/ab_relay3_$TAG.err
