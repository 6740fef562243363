# step_env_kernel: conditional vs unconditional bar / w' LDS reads; vs the two-launch default.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -k "one_launch" \
    --timeout 120 --timeout-method thread > gpurun_out/ab_$TAG/one_tests.log 2>&1 || { tail -30 gpurun_out/ab_$TAG/one_tests.log; exit 1; }
tail -2 gpurun_out/ab_$TAG/one_tests.log
V="stream,stream+PMENV_ONE=all+PMENV_ONE_V=4,a130+PMENV_ONE=all+PMENV_ONE_V=4,stream+PMENV_ONE=all+PMENV_ONE_V=4+PMENV_ONE_S80=1,stream+PMENV_ONE=all+PMENV_ONE_V=8"
for B in 65536 4096 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 9 --variants "$V" > gpurun_out/ab_$TAG/one5_ip_$B.json 2> gpurun_out/ab_$TAG/one5_ip_$B.err || exit 1
done
