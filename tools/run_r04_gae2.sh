# round 4: look-back GAE geometries (8 x 8 product against 8 x 16, 4 x 16, 16 x 4 in the tools build)
set -u
export TMPDIR=/tmp
TAG=${1:-r04h}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
for V in ${VARIANTS:-lb16 lb4x16 lb16x4}; do
timeout -k 10 300 python3 tools/ab_gae2.py --variant $V --shapes 4096x512,16384x64,1000x200,2048x4096 \
  > gpurun_out/ab_gae3_${TAG}_$V.json 2>> gpurun_out/ab_gae3_$TAG.err || { tail -5 gpurun_out/ab_gae3_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_gae3_$TAG.err
