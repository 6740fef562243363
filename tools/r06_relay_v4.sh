#!/bin/bash
# Round 6: 256 x 4 relay tiles for the 192-256 MiB in-place windows (config 4's share): the relay,
# configs and deferral tests, the in-process A/B against the 256 x 2 tiles (tools build,
# PMENV_RELAY_GEOM=256x2), and bench.py at the share.
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_relay.py tests/test_gpu_relay_deferral.py tests/test_gpu_configs.py > $O/v4_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $O/v4_tests.log; exit 1; }
tail -n 1 $O/v4_tests.log
timeout -k 10 300 python -u tools/ab_libs.py --envs 8192 --assets 30 --rounds 9 --steps 40 \
    --libs pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_ab.so+PMENV_RELAY_GEOM=256x2 > $O/v4_ab.json 2> $O/v4_ab.err || { tail -20 $O/v4_ab.err; exit 1; }
grep "^# [0-9]" $O/v4_ab.err
for i in 1 2; do
  timeout -k 10 300 python bench.py --envs-per-gpu 8192 --steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 0 > $O/v4_share_$i.json 2> $O/v4_share_$i.err || exit 1
  python -c "import json; d=json.loads(open('$O/v4_share_$i.json').read().strip().splitlines()[-1]); print('share', round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']/1e6,1), 'M')"
done
