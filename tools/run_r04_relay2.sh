# round 4: the split-store relay step (phase-1 stores before the relay words are read, the
# counter from a parity copy) — its GPU tests, then the lead sweep against two launches
set -u
export TMPDIR=/tmp
TAG=${1:-r04s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relay.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_relay_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_relay_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_relay_$TAG.log
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps libs paths [extra]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $5 --path $6 --envs $1 --assets $2 --rounds $3 --steps $4 ${7:-} \
    > gpurun_out/ab_relay2_${TAG}_$1x$2.json 2>> gpurun_out/ab_relay2_$TAG.err || { tail -5 gpurun_out/ab_relay2_$TAG.err; exit 1; }
}
ab 8192 30 7 40 $L,$L,$AB+PMENV_RELAY_LEAD=4096,$AB+PMENV_RELAY_LEAD=16384,$AB+PMENV_RELAY_LEAD=65536 two_launch,relay,relay,relay,relay
ab 4096 30 7 40 $L,$L,$AB+PMENV_RELAY_LEAD=4096,$AB+PMENV_RELAY_LEAD=16384 two_launch,relay,relay,relay
ab 2048 30 7 40 $L,$L,$L two_launch,relay,auto
ab 16384 30 5 20 $L,$L,$L,$AB+PMENV_RELAY_LEAD=4096 two_launch,relay,flat,relay
ab 65536 30 3 10 $L,$L,$L,$AB+PMENV_RELAY_LEAD=8192 flat,relay,two_launch,relay
ab 8192 500 3 6 $L,$L,$AB+PMENV_RELAY_LEAD=65536 two_launch,relay,relay "--reward diff_sharpe"
ab 8192 30 5 40 $L,$L two_launch,relay --out
grep "^#" gpurun_out/ab_relay2_$TAG.err
