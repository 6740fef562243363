# A/B of the window stream's workgroup size, unit size and cache policy (advance_rows_kernel)
set -u
mkdir -p gpurun_out
V="o,o+PMENV_STREAM_POL=1,o+PMENV_STREAM_POL=2"
V="$V,o+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=4+PMENV_STREAM_POL=2,o+PMENV_STREAM_BLOCK=128+PMENV_UNIT_ROWS=2+PMENV_STREAM_POL=2"
V="$V,o+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=8+PMENV_STREAM_POL=2,o+PMENV_STREAM_BLOCK=512+PMENV_UNIT_ROWS=8+PMENV_STREAM_POL=2"
V="$V,o+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=4,o+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=4+PMENV_STREAM_POL=1"
V="$V,stream,stream+PMENV_STREAM_POL=2,stream+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=4+PMENV_STREAM_POL=2"
V="$V,stream+PMENV_STREAM_BLOCK=128+PMENV_UNIT_ROWS=2+PMENV_STREAM_POL=2,stream+PMENV_STREAM_BLOCK=256+PMENV_UNIT_ROWS=8+PMENV_STREAM_POL=2"
timeout -k 10 600 python tools/ab_advance.py --rounds ${ROUNDS:-7} --steps 40 --variants "${1:-$V}" > gpurun_out/ab_pol.log 2>gpurun_out/ab_pol.err; rc=$?
grep -v amdgpu.ids gpurun_out/ab_pol.err | tail -20
python -c "
import json; t=open('gpurun_out/ab_pol.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print(f\"{k:72s} {v['median_us']:8.1f} us  {v['GBs']:7.1f} GB/s  frac {v['frac_8TBs']:.3f}\")
"; exit $rc
