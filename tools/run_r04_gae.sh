# round 4: the one-pass look-back GAE horizon split against the round-3 maps + apply split;
# the GAE GPU tests
set -u
export TMPDIR=/tmp
TAG=${1:-r04e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k gae --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_gae_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_gae_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_gae_$TAG.log
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
timeout -k 10 300 python3 tools/ab_gae2.py --shapes ${SHAPES:-4096x512,16384x64,512x64,1000x200,5000x3,700x4099,2048x4096} \
  > gpurun_out/ab_gae2_$TAG.json 2> gpurun_out/ab_gae2_$TAG.err || { tail -5 gpurun_out/ab_gae2_$TAG.err; exit 1; }
grep "^#" gpurun_out/ab_gae2_$TAG.err
