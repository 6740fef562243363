# step_env_kernel geometry (chunks per lane) and its stream alone (no scalar step) vs the two-launch default.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream,stream+PMENV_ONE=all+PMENV_ONE_V=4,stream+PMENV_ONE=all+PMENV_ONE_V=6,stream+PMENV_ONE=all+PMENV_ONE_V=8,a128+PMENV_ONE=all+PMENV_ONE_V=4,a128+PMENV_ONE=all+PMENV_ONE_V=8"
for B in 65536 4096; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > gpurun_out/ab_$TAG/one2_ip_$B.json 2> gpurun_out/ab_$TAG/one2_ip_$B.err || exit 1
done
