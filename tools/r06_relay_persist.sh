#!/bin/bash
# (measured once, r06n: the kernel form is profiles/r06/relay_stamps/persist_tiles_step_relay.patch,
#  removed after the run — apply it and the PMENV_RELAY_PERSIST launcher to re-run)
# Round 6: persistent tile workers for the relay step (tools build, PMENV_RELAY_PERSIST = workers
# per CU: step_relay_kernel<..., ANY = 3>) against the product, in process, bits compared.
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
L=pm-rl_amd/pmenv/libpmenv.so
A=tools/libpmenv_ab.so
for S in 8192x30 4096x30; do
  B=${S%x*}; N=${S#*x}
  timeout -k 10 300 python -u tools/ab_libs.py --envs $B --assets $N --rounds 7 --steps 40 --path relay \
      --libs $L,$A+PMENV_RELAY_PERSIST=4,$A+PMENV_RELAY_PERSIST=6,$A+PMENV_RELAY_PERSIST=8,$A+PMENV_RELAY_PERSIST=12 \
      > $O/persist_$S.json 2> $O/persist_$S.err || { echo "ab $S failed"; tail -20 $O/persist_$S.err; exit 1; }
  grep "^# [0-9]" $O/persist_$S.err
done
