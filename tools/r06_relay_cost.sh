#!/bin/bash
# Round 6: where the relay deferral's cost sits, in process against the product (bits compared):
#   libpmenv_va.so — the scalar wave's list read after its tail instead of before it
#   libpmenv_vb.so — timing probe: the tile's vote ignored (no deferral; the compiler drops the path)
#   libpmenv_vd.so — one list read per scalar block (thread 0 after a barrier) instead of per wave
#   (LIBS overrides the list)
# Both built from the working tree by an edit script (profiles/r06/relay/cost_edits/), removed after.
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
for S in 8192x30 4096x30; do
  B=${S%x*}; N=${S#*x}
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds 9 --steps 40 --path relay \
      --libs ${LIBS:-pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_va.so,tools/libpmenv_vb.so} \
      > $O/cost_$S.json 2> $O/cost_$S.err || { echo "ab $S failed"; tail -20 $O/cost_$S.err; exit 1; }
  grep "^# [0-9]" $O/cost_$S.err
done
