#!/bin/bash
# (tools/libpmenv_base.so: the round-5 library, pm-rl_amd/csrc of commit fc5c583 built with build.py's flags;
#  removed from the tree after round 6's A/B runs — rebuild it from that commit to re-run)
# Round 6: attribute the relay fallback's cost (in-process A/B; the fallback is not exercised)
set -o pipefail
T=${1:-r06}
LIBS=${2:-tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
for S in 8192x30 4096x30; do
  B=${S%x*}; N=${S#*x}
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds 9 --steps 40 --libs $LIBS \
      > $O/ab_$S.json 2> $O/ab_$S.err || { echo "ab $S failed"; tail -20 $O/ab_$S.err; exit 1; }
  grep "^# [0-9]" $O/ab_$S.err
done
