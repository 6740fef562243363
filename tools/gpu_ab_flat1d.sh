# step_flat_kernel (256 x 4) against the two-launch stream and the one-workgroup-per-env
# step by env count, in place and double-buffered: where AUTO switches.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1=1+PMENV_FLAT1_GEOM=256x4,stream+PMENV_ONE=all"
VO="o,o+PMENV_FLAT1=1+PMENV_FLAT1_GEOM=256x4,o+PMENV_ONE=all"
for B in 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > $OUT/flat1d_ip_$B.json 2> $OUT/flat1d_ip_$B.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$VO" > $OUT/flat1d_db_$B.json 2> $OUT/flat1d_db_$B.err || exit 1
done
for NB in "24 87381" "40 52428" "48 43690"; do
  set -- $NB
  timeout -k 10 300 python tools/ab_advance.py --assets $1 --envs $2 --steps 60 --rounds 5 --variants "$V" > $OUT/flat1d_n$1.json 2> $OUT/flat1d_n$1.err || exit 1
done
