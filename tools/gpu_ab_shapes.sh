# One-launch vs two-launch across asset counts and windows at ~2 GB windows (in place).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream"
for NW in 30x50 32x50 32x32 31x50 33x50 16x50 24x50 40x50 48x50 60x50 64x40 8x50 30x32 30x64; do
  N=${NW%x*}; W=${NW#*x}
  B=$(python -c "print(max(1024, round(1.97e9 / ($N * $W * 20) / 64) * 64))")
  timeout -k 10 300 python tools/ab_advance.py --envs $B --assets $N --window $W --steps 60 --rounds 7 --variants "$V" > gpurun_out/ab_$TAG/shape_n${N}_w${W}.json 2> gpurun_out/ab_$TAG/shape_n${N}_w${W}.err || exit 1
done
