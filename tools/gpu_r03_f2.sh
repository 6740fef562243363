# round 3: the f2 forward with kind / norm specialised records — trainer tests, then the rows bench
set -u
export TMPDIR=/tmp
TAG=${1:-r03v}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_on_policy.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_f2_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_f2_$TAG.log; [ $rc -eq 0 ] || exit $rc
# the previous library first (the r03 pre-split tree: all-candidate records), then this one
PMENV_LIB=tools/libpmenv_prev.so timeout -k 10 300 python tools/bench_rows.py --only f2 --reps 7 \
    --out gpurun_out/rows_f2_prev_$TAG.json > gpurun_out/rows_f2_prev_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_rows.py --only f2 --reps 7 --out gpurun_out/rows_f2_$TAG.json > gpurun_out/rows_f2_$TAG.log 2>&1 || exit $?
python - <<PY
import json
for f in ("rows_f2_prev_$TAG", "rows_f2_$TAG"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    for r in d["cases"]:
        print(f, r.get("case"), r.get("B"), r.get("N"), r.get("us"), r.get("same_bits", ""))
PY
