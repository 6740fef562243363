# the register steps with thousands of envs against the oracle
set -u
export TMPDIR=/tmp
TAG=${1:-r05v}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "many_envs" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/${TAG}_tests.log | cut -c1-300 | head -30
exit $rc
