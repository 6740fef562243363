# step_flat_kernel at smaller workgroups (threads x chunks per lane) against the
# two-launch stream and the one-workgroup-per-env step (in place).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
F=stream+PMENV_FLAT1=1+PMENV_FLAT1_GEOM
V="stream,$F=256x4,$F=256x8,$F=256x2,$F=128x8,$F=128x4,stream+PMENV_ONE=all"
for B in 65536 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > $OUT/flat1c_ip_$B.json 2> $OUT/flat1c_ip_$B.err || exit 1
done
for NB in "8 262144" "16 131072" "64 32768"; do
  set -- $NB
  timeout -k 10 300 python tools/ab_advance.py --assets $1 --envs $2 --steps 60 --rounds 5 --variants "$V" > $OUT/flat1c_n$1.json 2> $OUT/flat1c_n$1.err || exit 1
done
