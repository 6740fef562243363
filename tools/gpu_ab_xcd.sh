# step_env_kernel: XCD-contiguous env ranges, default-policy loads; vs the two-launch path.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream,a132,a136,a140,stream+PMENV_ONE=0+PMENV_FLAT_S80=1"
for B in 65536 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 9 --variants "$V" > gpurun_out/ab_$TAG/xcd_ip_$B.json 2> gpurun_out/ab_$TAG/xcd_ip_$B.err || exit 1
done
