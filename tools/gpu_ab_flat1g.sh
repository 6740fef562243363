# step_flat_kernel: XCD-contiguous tile ranges (straddling envs' scalar inputs stay in
# one XCD's L2) against the default round-robin, and the two-launch path.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1_XCD=1,stream+PMENV_FLAT1=0"
for B in 65536 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 9 --variants "$V" > $OUT/flat1g_ip_$B.json 2> $OUT/flat1g_ip_$B.err || exit 1
done
