# With commission > 0 (the capped fixed point per env) and other reward kinds: the flat
# one-launch step against the two-launch stream and the one-workgroup-per-env step.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream+PMENV_FLAT1=0,stream,stream+PMENV_FLAT1=0+PMENV_ONE=all"
for B in 65536 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --commission 0.0025 --steps 100 --rounds 7 --variants "$V" > $OUT/flat1e_comm_$B.json 2> $OUT/flat1e_comm_$B.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs $B --reward diff_sharpe --steps 100 --rounds 7 --variants "$V" > $OUT/flat1e_dsr_$B.json 2> $OUT/flat1e_dsr_$B.err || exit 1
done
timeout -k 10 300 python tools/ab_advance.py --envs 65536 --commission 0.01 --steps 100 --rounds 7 --variants "$V" > $OUT/flat1e_comm1_65536.json 2> $OUT/flat1e_comm1_65536.err || exit 1
