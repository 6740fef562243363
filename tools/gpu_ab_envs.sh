set -u
mkdir -p gpurun_out
for B in 4096 16384 1024; do
timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --variants "o+PMENV_FUSED=0,o,stream,stream+PMENV_FUSED=all" > gpurun_out/ab_$B.log 2>gpurun_out/ab_$B.err || exit 1
python -c "
import json; t=open('gpurun_out/ab_$B.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print($B, f\"{k:24s} {v['median_us']:8.1f} us  {v['GBs']:7.1f} GB/s\")
"
done
