# step_flat_kernel: sc1 nt on the window loads and stores against nt, more rounds.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 100 --rounds 15 --variants "stream,stream+PMENV_FLAT1_POL=6" > $OUT/flat1j_ip_$rep.json 2> $OUT/flat1j_ip_$rep.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 100 --rounds 15 --variants "o,o+PMENV_FLAT1_POL=6" > $OUT/flat1j_db_$rep.json 2> $OUT/flat1j_db_$rep.err || exit 1
done
