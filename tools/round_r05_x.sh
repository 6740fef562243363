# the generic stream's cache policy and geometry
set -u
export TMPDIR=/tmp
TAG=${1:-r05x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "generic or goldens" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
PMENV_GEN_POL0=1 AB_R=3 timeout -k 10 300 python tools/ab_gen.py > gpurun_out/${TAG}_pol.json 2> gpurun_out/${TAG}_pol.err || { tail -5 gpurun_out/${TAG}_pol.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_pol.err | python3 -c "
import sys,json
for l in sys.stdin:
    k,_,j=l.partition(' ')
    try: o=json.loads(j)
    except Exception: continue
    print(k, round(o['gen']['us'],1), round(o['small']['us'],1), round(o['gen']['frac'],3), o['windows_equal'], o['rewards_equal'])
"
for g in 512x2 256x2; do
PMENV_GEN_GEOM=$g PMENV_GEN_PERELEM=1 AB_R=3 timeout -k 10 300 python tools/ab_gen.py > gpurun_out/${TAG}_geom_$g.json 2> gpurun_out/${TAG}_geom_$g.err || { tail -5 gpurun_out/${TAG}_geom_$g.err; exit 1; }
done
for g in 512x2 256x2; do
grep -v "^[WE]2" gpurun_out/${TAG}_geom_$g.err | python3 -c "
import sys,json
for l in sys.stdin:
    k,_,j=l.partition(' ')
    try: o=json.loads(j)
    except Exception: continue
    print('$g', k, round(o['gen']['us'],1), round(o['small']['us'],1), o['windows_equal'])
"
done
