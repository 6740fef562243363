# step_env_kernel with 1 KiB-aligned block mapping: parity tests, then A/B vs the two-launch default.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -k "one_launch" \
    --timeout 120 --timeout-method thread > gpurun_out/ab_$TAG/one_tests.log 2>&1 || { tail -30 gpurun_out/ab_$TAG/one_tests.log; exit 1; }
tail -2 gpurun_out/ab_$TAG/one_tests.log
V="stream,stream+PMENV_ONE=all+PMENV_ONE_V=2,stream+PMENV_ONE=all+PMENV_ONE_V=3,stream+PMENV_ONE=all+PMENV_ONE_V=4,stream+PMENV_ONE=all+PMENV_ONE_V=8,a128+PMENV_ONE=all+PMENV_ONE_V=4"
VO="o,o+PMENV_ONE=all+PMENV_ONE_V=3,o+PMENV_ONE=all+PMENV_ONE_V=4"
for B in 65536 4096 16384; do
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$V" > gpurun_out/ab_$TAG/one3_ip_$B.json 2> gpurun_out/ab_$TAG/one3_ip_$B.err || exit 1
  timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 100 --rounds 7 --variants "$VO" > gpurun_out/ab_$TAG/one3_db_$B.json 2> gpurun_out/ab_$TAG/one3_db_$B.err || exit 1
done
