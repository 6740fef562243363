# round 4: the relayed one-launch step (step_relay_kernel) — its GPU tests, then in-process
# interleaved A/B against the two-launch path (and the flat step where AUTO takes it)
set -u
export TMPDIR=/tmp
TAG=${1:-r04r}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relay.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_relay_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_relay_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_relay_$TAG.log
L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps paths [extra]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $5 --path $6 --envs $1 --assets $2 --rounds $3 --steps $4 ${7:-} \
    > gpurun_out/ab_relay_${TAG}_$1x$2.json 2>> gpurun_out/ab_relay_$TAG.err || { tail -5 gpurun_out/ab_relay_$TAG.err; exit 1; }
}
ab 8192 30 7 40 $L,$L two_launch,relay
ab 4096 30 7 40 $L,$L two_launch,relay
ab 2048 30 7 40 $L,$L,$L two_launch,relay,auto
ab 16384 30 5 20 $L,$L,$L two_launch,relay,flat
ab 65536 30 3 10 $L,$L,$L two_launch,relay,flat
ab 8192 500 3 6 $L,$L two_launch,relay "--reward diff_sharpe"
ab 8192 30 5 40 $L,$L two_launch,relay --out
grep "^#" gpurun_out/ab_relay_$TAG.err
