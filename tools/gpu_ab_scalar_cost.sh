# What the scalar step costs the one-workgroup-per-env step on cache-resident windows:
# step_env_kernel with (ABLATE=128) and without (129, constant w' / bar) its scalar step,
# both nt policy, against AUTO (two launches) and the flat step
set -u
mkdir -p gpurun_out
for B in 4096 8192 16384; do
  timeout -k 10 300 python3 tools/ab_advance.py --envs $B --rounds 7 --steps 40 \
    --variants "stream,stream+PMENV_ONE=all,stream+PMENV_ONE=all+PMENV_ABLATE=128,stream+PMENV_ONE=all+PMENV_ABLATE=129,stream+PMENV_ONE=all+PMENV_ABLATE=136" \
    > gpurun_out/ab_scalar_cost_$B.json 2> gpurun_out/ab_scalar_cost_$B.err || { tail -5 gpurun_out/ab_scalar_cost_$B.err; exit 1; }
  python3 - gpurun_out/ab_scalar_cost_$B.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["variants"].items():
    print(d["B"], "%-55s %8.2f" % (k, v["median_us"]))
PY
done
