# round 4: step_relay_kernel's scalar-block lead (tiles), tools build (PMENV_RELAY_LEAD read at
# create), in-process interleaved against the product two-launch path
set -u
export TMPDIR=/tmp
TAG=${1:-r04l}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps libs paths [extra]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $5 --path $6 --envs $1 --assets $2 --rounds $3 --steps $4 ${7:-} \
    > gpurun_out/ab_lead_${TAG}_$1x$2.json 2>> gpurun_out/ab_lead_$TAG.err || { tail -5 gpurun_out/ab_lead_$TAG.err; exit 1; }
}
ab 8192 30 5 40 $L,$AB+PMENV_RELAY_LEAD=2048,$AB+PMENV_RELAY_LEAD=4096,$AB+PMENV_RELAY_LEAD=8192,$AB+PMENV_RELAY_LEAD=16384 two_launch,relay,relay,relay,relay
ab 4096 30 5 40 $L,$AB+PMENV_RELAY_LEAD=2048,$AB+PMENV_RELAY_LEAD=4096,$AB+PMENV_RELAY_LEAD=8192 two_launch,relay,relay,relay
ab 65536 30 3 10 $L,$AB+PMENV_RELAY_LEAD=2048,$AB+PMENV_RELAY_LEAD=4096,$L flat,relay,relay,two_launch
ab 8192 500 3 6 $L,$AB+PMENV_RELAY_LEAD=8192,$AB+PMENV_RELAY_LEAD=32768 two_launch,relay,relay "--reward diff_sharpe"
grep "^#" gpurun_out/ab_lead_$TAG.err
