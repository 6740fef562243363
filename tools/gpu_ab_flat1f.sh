# Cache-resident in-place windows (BASELINE config 2 = 4,096 envs, config 4's per-GPU
# share = 8,192): step_flat_kernel geometries against the two-launch stream.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
F=stream+PMENV_FLAT1=1+PMENV_FLAT1_GEOM
V="stream,$F=256x4,$F=128x8,$F=512x2,$F=128x4,$F=256x2,$F=256x8"
for B in 4096 8192; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --rounds 9 --variants "$V" > $OUT/flat1f_ip_$B.json 2> $OUT/flat1f_ip_$B.err || exit 1
done
