# step_flat_kernel 128 x 8 against 256 x 4 at N = 30 by env count (where does 128 x 8 start to win).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1_GEOM=128x8"
for B in 16384 32768 49152 65536 98304; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 11 --variants "$V" > $OUT/flat1l_ip_$B.json 2> $OUT/flat1l_ip_$B.err || exit 1
done
