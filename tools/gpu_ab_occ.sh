# step_env_kernel: workgroups per CU (LDS padding) and the flat stream's own occupancy (80-SGPR twin).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
V="stream+PMENV_ONE=0,stream,stream+PMENV_ONE_LDS_PAD=24000,stream+PMENV_ONE_LDS_PAD=48000,stream+PMENV_ONE_S80=1,stream+PMENV_ONE_S80=1+PMENV_ONE_LDS_PAD=8000,stream+PMENV_ONE_V=8+PMENV_ONE_S80=1"
timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 100 --rounds 9 --variants "$V" > gpurun_out/ab_$TAG/occ_ip_65536.json 2> gpurun_out/ab_$TAG/occ_ip_65536.err || exit 1
