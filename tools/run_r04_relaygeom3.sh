# round 4: the relay step's tile geometry across the relay band: the product's 256 x 2 against
# 256 x 4, 256 x 8, 512 x 4, 128 x 4 (tools build, PMENV_RELAY_GEOM), in place and double-buffered
set -u
export TMPDIR=/tmp
TAG=${1:-r04k}
mkdir -p gpurun_out
timeout -k 10 400 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
LIBS=$L,$AB+PMENV_RELAY_GEOM=256x4,$AB+PMENV_RELAY_GEOM=256x8,$AB+PMENV_RELAY_GEOM=512x4,$AB+PMENV_RELAY_GEOM=128x4
for S in 2048x30 6144x30 8192x30 8192x8 16384x8 8192x16 2048x64 4096x64 4096x30/out 8192x30/out; do
  B=${S%%x*}; R=${S#*x}; N=${R%%/*}; O=""; [ "$R" != "$N" ] && O="--out"
  timeout -k 10 300 python3 tools/ab_libs.py --libs $LIBS --path relay,relay,relay,relay,relay --envs $B --assets $N $O \
    --rounds 5 --steps 40 > gpurun_out/ab_rgeom3_${TAG}_${B}_$N.json 2>> gpurun_out/ab_rgeom3_$TAG.err || { tail -5 gpurun_out/ab_rgeom3_$TAG.err; exit 1; }
done
grep "^#" gpurun_out/ab_rgeom3_$TAG.err
