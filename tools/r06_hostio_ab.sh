#!/bin/bash
# (tools/libpmenv_base.so: the round-5 library, pm-rl_amd/csrc of commit fc5c583 built with build.py's flags;
#  removed from the tree after round 6's A/B runs — rebuild it from that commit to re-run)
# Round 6: the host-I/O step per library (PMENV_LIB): the reference driver's loop and the raw C ABI call
set -o pipefail
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1 HOSTIO_T=${HOSTIO_T:-600} HOSTIO_REPS=${HOSTIO_REPS:-3}
for L in ${2:-tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so}; do :; done
IFS=, read -ra LIBS <<< "${2:-tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so}"
for L in "${LIBS[@]}"; do
  n=$(basename $L .so)
  PMENV_LIB=$PWD/$L timeout -k 10 300 python -u tools/bench_hostio.py > $O/hostio_$n.json 2> $O/hostio_$n.err || { echo "$n failed"; tail -20 $O/hostio_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/hostio_$n.json')); print('$n', {k: (round(v['direct']['us_per_step_median'],2), round(v['c_abi_us_per_step'],2)) for k, v in d.items() if isinstance(v, dict)})"
done
