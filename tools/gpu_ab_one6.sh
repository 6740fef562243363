# Where the one-launch step (step_env_kernel) beats the fused row kernel / the two-launch path, by env count.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream,stream+PMENV_FUSED=0,stream+PMENV_ONE=all+PMENV_ONE_V=4"
VO="o,o+PMENV_FUSED=0,o+PMENV_ONE=all+PMENV_ONE_V=4"
for B in 64 256 1024 2048 4096 8192 32768; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --rounds 9 --variants "$V" > gpurun_out/ab_$TAG/one6_ip_$B.json 2> gpurun_out/ab_$TAG/one6_ip_$B.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --rounds 9 --variants "$VO" > gpurun_out/ab_$TAG/one6_db_$B.json 2> gpurun_out/ab_$TAG/one6_db_$B.err || exit 1
done
