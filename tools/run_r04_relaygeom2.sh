# round 4: the relay step's tile geometry at the cache-resident shapes: the product's 256 x 2
# against 128 x 2, 128 x 4, 256 x 4, 256 x 1 (tools build, PMENV_RELAY_GEOM)
set -u
export TMPDIR=/tmp
TAG=${1:-r04j}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
for B in 4096 8192; do
timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_RELAY_GEOM=128x2,$AB+PMENV_RELAY_GEOM=128x4,$AB+PMENV_RELAY_GEOM=256x4,$AB+PMENV_RELAY_GEOM=256x1 \
  --path relay,relay,relay,relay,relay --envs $B --assets 30 --rounds 7 --steps 40 \
  > gpurun_out/ab_rgeom_${TAG}_$B.json 2>> gpurun_out/ab_rgeom_$TAG.err || { tail -5 gpurun_out/ab_rgeom_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_rgeom_$TAG.err
