#!/bin/bash
# (tools/libpmenv_r05.so was removed from the tree after the run, r06p: rebuild it from fc5c583 to re-run)
# Round 6: the cache-resident shares through bench.py itself, the round-6 product against the
# round-5 library (tools/libpmenv_r05.so: pm-rl_amd/csrc of commit fc5c583 built with build.py's
# flags), alternating on one box (the box copy's libpmenv.so swapped between runs, restored at
# the end), then the same two in one process (tools/ab_libs.py).
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
cp pm-rl_amd/pmenv/libpmenv.so /tmp/libpmenv_r06.so
for i in 1 2; do
  for L in r06 r05; do
    if [ $L = r05 ]; then cp tools/libpmenv_r05.so pm-rl_amd/pmenv/libpmenv.so; else cp /tmp/libpmenv_r06.so pm-rl_amd/pmenv/libpmenv.so; fi
    for B in 8192 4096; do
      timeout -k 10 300 python bench.py --envs-per-gpu $B --steps 200 --warmup 20 --cpu-baseline 0 --alt-steps 0 \
          > $O/share_${B}_${L}_$i.json 2> $O/share_${B}_${L}_$i.err || { cp /tmp/libpmenv_r06.so pm-rl_amd/pmenv/libpmenv.so; exit 1; }
      python -c "import json; d=json.loads(open('$O/share_${B}_${L}_$i.json').read().strip().splitlines()[-1]); print('$B $L $i', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_avg_us'],2), d['library']['sha256'][:12] if 'library' in d else '')"
    done
  done
done
cp /tmp/libpmenv_r06.so pm-rl_amd/pmenv/libpmenv.so
for S in 8192 4096; do
  timeout -k 10 300 python -u tools/ab_libs.py --envs $S --assets 30 --rounds 9 --steps 40 \
      --libs tools/libpmenv_r05.so,pm-rl_amd/pmenv/libpmenv.so > $O/ab_$S.json 2> $O/ab_$S.err || exit 1
  grep "^# [0-9]" $O/ab_$S.err
done
