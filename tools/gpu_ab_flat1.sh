# The flat one-launch step (step_flat_kernel) against the two-launch stream and the
# one-workgroup-per-env step, in place and double-buffered, across env counts and
# asset counts (interleaved rounds in one process per shape).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1=1,stream+PMENV_ONE=all"
VO="o,o+PMENV_FLAT1=1,o+PMENV_ONE=all"
for B in 65536 16384 8192 4096 1024; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > $OUT/flat1_ip_$B.json 2> $OUT/flat1_ip_$B.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$VO" > $OUT/flat1_db_$B.json 2> $OUT/flat1_db_$B.err || exit 1
done
# ~2 GB windows at other asset counts (the one-workgroup-per-env geometry loses 4-15 % there)
for NB in "8 262144" "16 131072" "64 32768"; do
  set -- $NB
  timeout -k 10 300 python tools/ab_advance.py --assets $1 --envs $2 --steps 60 --rounds 5 --variants "$V" > $OUT/flat1_n$1.json 2> $OUT/flat1_n$1.err || exit 1
done
