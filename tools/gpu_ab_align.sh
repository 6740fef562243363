# One-launch vs two-launch when env windows are 128-B multiples (N = 32: 32,000 B) vs not (N = 30: 30,000 B).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream"
for N in 32 30 28; do
  timeout -k 10 300 python tools/ab_advance.py --envs 65536 --assets $N --steps 100 --rounds 9 --variants "$V" > gpurun_out/ab_$TAG/align_ip_n$N.json 2> gpurun_out/ab_$TAG/align_ip_n$N.err || exit 1
done
