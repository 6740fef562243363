# Where the one-launch step loses (asset counts other than 30): its stream alone (a128: no
# scalar step) and other chunks-per-lane, against the two-launch path.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream,a128+PMENV_ONE=all,stream+PMENV_ONE_V=2,stream+PMENV_ONE_V=3,stream+PMENV_ONE_V=8"
for NW in 16x50 40x50 32x50 30x50; do
  N=${NW%x*}; W=${NW#*x}
  B=$(python -c "print(max(1024, round(1.97e9 / ($N * $W * 20) / 64) * 64))")
  timeout -k 10 300 python tools/ab_advance.py --envs $B --assets $N --window $W --steps 60 --rounds 7 --variants "$V" > gpurun_out/ab_$TAG/shape2_n${N}_w${W}.json 2> gpurun_out/ab_$TAG/shape2_n${N}_w${W}.err || exit 1
done
