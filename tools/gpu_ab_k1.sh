# K1 (scalar_step_reg_kernel) alone: env groups per wave, B = 65536 and 16384
set -u
mkdir -p gpurun_out
for B in 65536 16384; do
timeout -k 10 300 python tools/ab_advance.py --envs $B --steps 200 --phases 1 --variants "stream+PMENV_K1_GROUPS=1,stream+PMENV_K1_GROUPS=2,stream+PMENV_K1_GROUPS=4" > gpurun_out/abk1_$B.log 2>gpurun_out/abk1_$B.err || exit 1
python -c "
import json; t=open('gpurun_out/abk1_$B.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print($B, f\"{k:28s} {v['median_us']:8.2f} us\")
"
done
