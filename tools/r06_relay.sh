#!/bin/bash
# (tools/libpmenv_base.so: the round-5 library, pm-rl_amd/csrc of commit fc5c583 built with build.py's flags;
#  removed from the tree after round 6's A/B runs — rebuild it from that commit to re-run)
# Round 6: the relay step's forward-progress deferral and the F <= 16 generic stream on the GPU box.
#   bash tools/r06_relay.sh TAG [quick]
# 1. the relay GPU tests and the generic-stream / register-step parity tests on the product
# library; 2. in-process A/B of the round-5 library (tools/libpmenv_base.so) and the product on
# the cache-resident relay shapes; 3. the deferral forced through the tools build — tiles first
# (every tile precedes every scalar block) and / or spin 0 — against the product, bit for bit, at
# every scalar-step form.
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_relay.py \
    tests/test_gpu_parity.py -k "relay or generic or register_step or auto_rule or golden" \
    > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for S in 4096x30 8192x30; do
  B=${S%x*}; N=${S#*x}
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds 9 --steps 40 \
      --libs tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so \
      > $O/ab_$S.json 2> $O/ab_$S.err || { echo "ab $S failed"; tail -20 $O/ab_$S.err; exit 1; }
  grep "^# [0-9]" $O/ab_$S.err
done
[ "$2" = quick ] && exit 0
for S in 512x30 4096x30 8192x30 4096x8 2048x64 1024x100; do
  B=${S%x*}; N=${S#*x}
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds 2 --steps 5 --path relay --attribute \
      --libs pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_ab.so+PMENV_RELAY_SPIN=0,tools/libpmenv_ab.so+PMENV_RELAY_TILES_FIRST=1,tools/libpmenv_ab.so+PMENV_RELAY_TILES_FIRST=1+PMENV_RELAY_SPIN=0 \
      > $O/fb_$S.json 2> $O/fb_$S.err || { echo "deferral $S failed"; tail -20 $O/fb_$S.err; exit 1; }
  grep "^# [0-9]" $O/fb_$S.err
done
