# the generic stream with its side data sized by rows (dynamic LDS) against the previous build
set -u
export TMPDIR=/tmp
TAG=${1:-r05y}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "generic or goldens" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
AB_GEN_BASE=tools/libpmenv_r05x.so AB_R=5 timeout -k 10 400 python tools/ab_gen.py > gpurun_out/${TAG}_base.json 2> gpurun_out/${TAG}_base.err || { tail -5 gpurun_out/${TAG}_base.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_base.err | python3 -c "
import sys,json
for l in sys.stdin:
    k,_,j=l.partition(' ')
    try: o=json.loads(j)
    except Exception: continue
    print(k, round(o['gen']['us'],1), round(o['small']['us'],1), round(o['gen']['frac'],3), o['windows_equal'], o['rewards_equal'])
"
