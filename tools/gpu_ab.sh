set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
PMENV_ADVANCE=lds timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "goldens or modes or shapes" > gpurun_out/gpu_tests_lds.log 2>&1
rc=$?; echo "lds pytest rc=$rc"; tail -2 gpurun_out/gpu_tests_lds.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/ab_advance.py --variants ${1:-lds,stream,u2,u4,u6} > gpurun_out/ab.log 2>gpurun_out/ab.err; rc=$?; cat gpurun_out/ab.err | grep -v amdgpu.ids; python -c "
import json; t=open('gpurun_out/ab.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print(f\"{k:10s} {v['median_us']:8.1f} us  {v['GBs']:7.1f} GB/s  frac {v['frac_8TBs']:.3f}\")
"; exit $rc
