# Occupancy probe of the flat one-launch step at the BASELINE shape: extra LDS per
# workgroup (PMENV_FLAT1_LDS_PAD) takes 128 x 8 from 8 workgroups per CU down to 7, 6, 5, 4
set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_advance.py --envs 65536 --rounds 7 --steps 40 \
  --variants "stream,stream+PMENV_FLAT1_LDS_PAD=4000,stream+PMENV_FLAT1_LDS_PAD=8000,stream+PMENV_FLAT1_LDS_PAD=13000,stream+PMENV_FLAT1_LDS_PAD=21000" \
  > gpurun_out/ab_flat_occ.json 2> gpurun_out/ab_flat_occ.err || { tail -5 gpurun_out/ab_flat_occ.err; exit 1; }
python3 - gpurun_out/ab_flat_occ.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["variants"].items():
    print(d["B"], "%-50s %8.2f" % (k, v["median_us"]))
PY
