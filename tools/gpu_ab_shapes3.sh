# One-launch step with idle blocks skipped (default) vs issued (a144), chunks per lane 4 / 8, vs two launches.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream,a144+PMENV_ONE=all,stream+PMENV_ONE_V=8"
for NW in 16x50 40x50 32x50 30x50 8x50; do
  N=${NW%x*}; W=${NW#*x}
  B=$(python -c "print(max(1024, round(1.97e9 / ($N * $W * 20) / 64) * 64))")
  timeout -k 10 300 python tools/ab_advance.py --envs $B --assets $N --window $W --steps 60 --rounds 7 --variants "$V" > gpurun_out/ab_$TAG/shape3_n${N}_w${W}.json 2> gpurun_out/ab_$TAG/shape3_n${N}_w${W}.err || exit 1
done
