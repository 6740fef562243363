#!/bin/bash
# (tools/libpmenv_base.so: the round-5 library, pm-rl_amd/csrc of commit fc5c583 built with build.py's flags;
#  removed from the tree after round 6's A/B runs — rebuild it from that commit to re-run)
# Round 6: the surface stream with staged counters and the F <= 16 generic stream, against the
# round-5 library (tools/libpmenv_base.so), one process per comparison, bits compared.
#   bash tools/r06_streams.sh TAG
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "surface" > $O/surface_tests.log 2>&1 || { echo "surface tests failed"; tail -30 $O/surface_tests.log; exit 1; }
tail -1 $O/surface_tests.log
SURF_LIBS=tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so SURF_SHAPES=65536x30x50x5,16384x30x50x5,16384x30x50x8 \
    timeout -k 10 300 python -u tools/bench_surface.py > $O/surface.json 2> $O/surface.err || { echo "surface bench failed"; tail -20 $O/surface.err; exit 1; }
python -c "import json; d=json.load(open('$O/surface.json')); print(json.dumps(d)[:3000])"
for S in 65536x30x12 65536x30x16 16384x30x12; do
  B=$(echo $S | cut -dx -f1); N=$(echo $S | cut -dx -f2); F=$(echo $S | cut -dx -f3)
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --features $F --rounds 5 --steps 10 \
      --libs tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so > $O/gen_$S.json 2> $O/gen_$S.err || { echo "gen $S failed"; tail -20 $O/gen_$S.err; exit 1; }
  grep "^# [0-9]" $O/gen_$S.err
done
