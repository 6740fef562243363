# step_flat_kernel geometries (threads x chunks per lane) and the persistent form
# against the two-launch stream and the one-workgroup-per-env step (in place).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
F=stream+PMENV_FLAT1=1
V="stream,$F,$F+PMENV_FLAT1_GEOM=512x4,$F+PMENV_FLAT1_GEOM=256x4,$F+PMENV_FLAT1_GEOM=1024x2,$F+PMENV_FLAT1_GRID=4,$F+PMENV_FLAT1_GEOM=512x4+PMENV_FLAT1_GRID=2,stream+PMENV_ONE=all"
for B in 65536 16384 4096; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > $OUT/flat1b_ip_$B.json 2> $OUT/flat1b_ip_$B.err || exit 1
done
timeout -k 10 300 python tools/ab_advance.py --assets 8 --envs 262144 --steps 60 --rounds 5 --variants "$V" > $OUT/flat1b_n8.json 2> $OUT/flat1b_n8.err || exit 1
