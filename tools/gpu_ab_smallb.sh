# One-launch vs two-launch at small env counts across asset counts (in place and double-buffered).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for N in 8 16 32 64; do
  for B in 256 1024 2048 4096; do
    timeout -k 10 300 python tools/ab_advance.py --envs $B --assets $N --window 40 --steps 100 --rounds 7 --variants "stream+PMENV_ONE=0,stream+PMENV_ONE=all" > gpurun_out/ab_$TAG/smallb_ip_n${N}_b$B.json 2> gpurun_out/ab_$TAG/smallb_ip_n${N}_b$B.err || exit 1
    timeout -k 10 300 python tools/ab_advance.py --envs $B --assets $N --window 40 --steps 100 --rounds 7 --variants "o+PMENV_ONE=0,o+PMENV_ONE=all" > gpurun_out/ab_$TAG/smallb_db_n${N}_b$B.json 2> gpurun_out/ab_$TAG/smallb_db_n${N}_b$B.err || exit 1
  done
done
