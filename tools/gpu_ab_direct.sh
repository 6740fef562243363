# step_env_kernel without the LDS window image (PMENV_ONE_DIRECT: each lane loads its
# shifted source straight from memory) against the LDS form, AUTO and the flat step
set -u
mkdir -p gpurun_out
for B in 4096 8192 16384 65536; do
  for o in "" "o"; do
    timeout -k 10 300 python3 tools/ab_advance.py --envs $B --rounds 7 --steps 40 \
      --variants "stream$o+PMENV_ONE=all,stream$o+PMENV_ONE=all+PMENV_ONE_DIRECT=1,stream$o,stream$o+PMENV_FLAT1=1" \
      > gpurun_out/ab_direct_${B}$o.json 2> gpurun_out/ab_direct_${B}$o.err || { tail -5 gpurun_out/ab_direct_${B}$o.err; exit 1; }
    python3 - gpurun_out/ab_direct_${B}$o.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["variants"].items():
    print(d["B"], "%-50s %8.2f" % (k, v["median_us"]))
PY
  done
done
