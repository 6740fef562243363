set -u
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_advance.py --variants ${1} > gpurun_out/ab.log 2>gpurun_out/ab.err; rc=$?; grep -v amdgpu.ids gpurun_out/ab.err | tail -3; python -c "
import json; t=open('gpurun_out/ab.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print(f\"{k:10s} {v['median_us']:8.1f} us  {v['GBs']:7.1f} GB/s  frac {v['frac_8TBs']:.3f}\")
"; exit $rc
