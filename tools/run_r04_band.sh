# round 4: where the relay step (scalar blocks first) wins — in-process interleaved against
# AUTO's current choice and the two-launch path, in place and double-buffered, over window
# sizes from 31 MB to 1 GB and N = 8 .. 64, plus config 5
set -u
export TMPDIR=/tmp
TAG=${1:-r04b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relay.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_relay_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_relay_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_relay_$TAG.log
L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps [extra]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$L,$L --path auto,relay,two_launch --envs $1 --assets $2 \
    --rounds $3 --steps $4 ${5:-} > gpurun_out/ab_band_${TAG}_$1x$2.json 2>> gpurun_out/ab_band_$TAG.err \
    || { tail -5 gpurun_out/ab_band_$TAG.err; exit 1; }
}
for B in 1024 2048 3072 4096 6144 8192 12288 16384; do ab $B 30 5 30; done
ab 4096 8 5 30; ab 8192 8 5 30; ab 16384 8 5 30
ab 4096 16 5 30; ab 8192 16 5 30
ab 2048 64 5 30; ab 4096 64 5 30
ab 8192 30 5 30 "--commission 0.0025"
for B in 2048 4096 8192; do ab $B 30 5 30 --out; done
ab 32768 30 3 10; ab 65536 30 3 10
ab 8192 500 3 6 "--reward diff_sharpe"
grep "^#" gpurun_out/ab_band_$TAG.err
