#!/bin/bash
# (the edit: profiles/r06/relay_stamps/compose_branchfree_edit.py, applied by a variant build;
#  the variant library was removed after the run, r06o)
# Round 6: compose2's last-day / slot patch written with bitwise selects instead of short-circuit
# conditions (no exec-mask branches; the same values) — tools/libpmenv_vcompose.so, built from the
# working tree with that edit — against the product, in process, bits compared.
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
L=pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_vcompose.so
for S in 8192x30 4096x30 65536x30; do
  B=${S%x*}; N=${S#*x}; R=9; K=40; [ $B = 65536 ] && { R=5; K=10; }
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds $R --steps $K --libs $L \
      > $O/compose_$S.json 2> $O/compose_$S.err || { echo "ab $S failed"; tail -20 $O/compose_$S.err; exit 1; }
  grep "^# [0-9]" $O/compose_$S.err
done
