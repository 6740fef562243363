#!/bin/bash
# Round 6: the resident host-I/O step — its tests, then the reference driver's per-step time.
#   bash tools/r06_hostio.sh TAG
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dropin.py \
    tests/test_gpu_parity.py -k "host or dropin or driver" > $O/hostio_tests.log 2>&1 \
    || { echo "host-I/O tests failed"; tail -30 $O/hostio_tests.log; exit 1; }
tail -1 $O/hostio_tests.log
timeout -k 10 400 python -u tools/bench_hostio.py > $O/hostio.json 2> $O/hostio.err || { echo "bench failed"; tail -20 $O/hostio.err; exit 1; }
cat $O/hostio.json
