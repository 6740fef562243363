# round 4: the paired look-back GAE (tools: PMENV_GAE=lb2, 2 x 64-day chunks per workgroup;
# lb2x16, 2 x 128 days) against the product (single 128-day chunks where they pay)
set -u
export TMPDIR=/tmp
TAG=${1:-r04q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k gae --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_gae_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_gae_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_gae_$TAG.log
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
for V in lb2 lb2x16; do
timeout -k 10 300 python3 tools/ab_gae2.py --variant $V --shapes 4096x512,16384x64,2048x4096,700x4099,8192x256,2048x1024,1024x2048,1000x200 \
  > gpurun_out/ab_gae4_${TAG}_$V.json 2>> gpurun_out/ab_gae4_$TAG.err || { tail -5 gpurun_out/ab_gae4_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_gae4_$TAG.err
