#!/bin/bash
# Round 6's final lease on ONE product library (no rebuild between the parts; every record
# carries the library's sha256): bash tools/r06_final.sh PART TAG
#   tests   — the -m gpu suite in one process, then smoke() (tools/gpu_tests.sh)
#   bench   — bench.py default + short form, rocprofv3 kernel trace, FETCH_SIZE / WRITE_SIZE
#             passes (tools/gpu_bench_prof.sh), summarised by tools/pmc_summary.py on the host
#   configs — bench.py once more (traffic from the PMC passes just committed), the BASELINE
#             configs through bench.py (tools/bench_configs.sh) and the §8f rows
#             (tools/bench_rows.py on the product library)
set -o pipefail
PART=$1
T=${2:-r06end}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
sha256sum pm-rl_amd/pmenv/libpmenv.so | tee gpurun_out/lib_sha_${PART}_$T.txt
case $PART in
tests) bash tools/gpu_tests.sh $T ;;
bench) bash tools/gpu_bench_prof.sh $T ;;
configs)
  # the headline again, now that profiles/pmc_traffic.json carries this library's PMC passes
  timeout -k 10 600 python bench.py > gpurun_out/bench_final_$T.json 2> gpurun_out/bench_final_$T.err || exit $?
  tail -c 700 gpurun_out/bench_final_$T.json
  bash tools/bench_configs.sh $T || exit $?
  PMENV_LIB=$PWD/pm-rl_amd/pmenv/libpmenv.so timeout -k 10 300 python3 tools/bench_rows.py --reps 5 \
      --out gpurun_out/rows_$T.json > gpurun_out/rows_$T.log 2>&1 || { tail -20 gpurun_out/rows_$T.log; exit 1; }
  tail -c 1500 gpurun_out/rows_$T.json ;;
*) echo "unknown part $PART"; exit 2 ;;
esac
