# Cache-resident in-place windows (BASELINE configs 2 and 4's share): the two-launch
# stream's geometry (threads x chunks per thread) and the scalar-step form.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
S=stream+PMENV_FLAT_IP_BLOCK
V="stream,$S=256+PMENV_FLAT_IP_VEC=2,$S=256+PMENV_FLAT_IP_VEC=4,$S=512+PMENV_FLAT_IP_VEC=1,$S=1024+PMENV_FLAT_IP_VEC=1,stream+PMENV_K1=16x2,stream+PMENV_ONE=ip"
for B in 4096 8192; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --rounds 9 --variants "$V" > $OUT/smallip_$B.json 2> $OUT/smallip_$B.err || exit 1
done
