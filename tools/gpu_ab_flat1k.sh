# step_flat_kernel 128 x 8 (2 waves, 16 KiB tiles) against 256 x 4 where env windows have
# 1,023 .. 2,047 chunks (two envs per tile at most for both), ~2 GB windows.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1_GEOM=128x8"
for NB in "30 65536" "24 81920" "32 61440" "20 98304" "28 70000"; do
  set -- $NB
  timeout -k 10 300 python tools/ab_advance.py --assets $1 --envs $2 --steps 80 --rounds 11 --variants "$V" > $OUT/flat1k_n$1.json 2> $OUT/flat1k_n$1.err || exit 1
done
timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 80 --rounds 11 --variants "o,o+PMENV_FLAT1_GEOM=128x8" > $OUT/flat1k_db_n30.json 2> $OUT/flat1k_db_n30.err || exit 1
