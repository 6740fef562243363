#!/bin/bash
# Round 6: the relay tiles' geometry at the cache-resident shares (the stamps showed ~4.6 tiles
# in flight per CU against 8 the registers and LDS allow: the workgroup dispatch rate), in-process
# A/B of the product against the tools build's other tile sizes (PMENV_RELAY_GEOM), bits compared.
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
      --libs $L,$A+PMENV_RELAY_GEOM=256x4,$A+PMENV_RELAY_GEOM=512x4,$A+PMENV_RELAY_GEOM=256x8,$A+PMENV_RELAY_GEOM=128x4 \
      > $O/geom_$S.json 2> $O/geom_$S.err || { echo "ab $S failed"; tail -20 $O/geom_$S.err; exit 1; }
  grep "^# [0-9]" $O/geom_$S.err
done
